"""fp64 numpy ALS with the semantics of Spark's ``ml.recommendation.ALS`` — the path the
reference keeps for explicit feedback (and every case its platform check rejects):
mllib-dal/src/main/scala/org/apache/spark-3.1.1/ml/recommendation/ALS.scala:922-932.

Per half-iteration each destination row solves the regularised normal equations of
``computeFactors`` (:1718-1800): implicit ``A = YtY + sum c1 y y^T + lambda n_u I`` with
``c1 = alpha |r|``, ``b = sum_{r>0} (1 + c1) y``; explicit ``A = sum y y^T + lambda n_u I``,
``b = sum r y``.  Cholesky for the unconstrained case (CholeskySolver, :757-788); non-negative
least squares on the same normal equations for ``nonnegative=True`` (NNLSSolver, :791-844).
Items are solved from users first, then users from items (:1036-1062).  Initial user factors
come from the same counter-based hash as the native engines (csrc/kernels/rng.h), so all three
engines start from identical factors.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def init_factors(ids: np.ndarray, rank: int, seed: int) -> np.ndarray:
    """Unit-norm Gaussian rows keyed by (seed, id, feature) — csrc/kernels/rng.h."""
    ids = np.asarray(ids, dtype=np.int64).astype(np.uint32).astype(np.uint64)
    f = np.arange(rank, dtype=np.uint64)
    with np.errstate(over="ignore"):
        key = ids[:, None] * np.uint64(0x9E3779B97F4A7C15) + f[None, :] * np.uint64(
            0xD1B54A32D192ED03)
        h1 = _splitmix64(np.uint64(seed & 0xFFFFFFFFFFFFFFFF) ^ _splitmix64(key))
        h2 = _splitmix64(h1)
    u1 = ((h1 >> np.uint64(11)).astype(np.float64) + 1.0) * (1.0 / 9007199254740992.0)
    u2 = (h2 >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    g = np.sqrt(-2.0 * np.log(u1)) * np.cos(6.283185307179586 * u2)
    return (g / np.linalg.norm(g, axis=1, keepdims=True)).astype(np.float32)


@dataclass
class ALSResult:
    user_ids: np.ndarray
    item_ids: np.ndarray
    user_factors: np.ndarray
    item_factors: np.ndarray


def _nnls(A: np.ndarray, b: np.ndarray) -> np.ndarray:
    """argmin_{x >= 0} 1/2 x^T A x - b^T x via scipy's NNLS on the Cholesky factor."""
    from scipy.optimize import nnls

    L = np.linalg.cholesky(A)
    return nnls(L.T, np.linalg.solve(L, b))[0]


def _solve_side(ptr, cols, vals, src, rank, reg, implicit, alpha, nonnegative):
    n = len(ptr) - 1
    out = np.zeros((n, rank), dtype=np.float32)
    Y = src.astype(np.float64)
    yty = Y.T @ Y if implicit else None
    for u in range(n):
        lo, hi = ptr[u], ptr[u + 1]
        Ys = Y[cols[lo:hi]]
        r = vals[lo:hi].astype(np.float64)
        if implicit:
            c1 = alpha * np.abs(r)
            A = yty + (Ys * c1[:, None]).T @ Ys
            b = ((r > 0) * (1.0 + c1)) @ Ys
            nexp = int((r > 0).sum())
        else:
            A = Ys.T @ Ys
            b = r @ Ys
            nexp = hi - lo
        A = A + reg * nexp * np.eye(rank)
        try:
            x = _nnls(A, b) if nonnegative else np.linalg.solve(A, b)
            np.linalg.cholesky(A)  # Spark's dppsv refuses non-SPD systems
        except np.linalg.LinAlgError:
            x = np.zeros(rank)
        out[u] = x
    return out


def _csr(rows: np.ndarray, cols: np.ndarray, vals: np.ndarray, n: int):
    order = np.lexsort((cols, rows))
    rows, cols, vals = rows[order], cols[order], vals[order]
    ptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(ptr, rows + 1, 1)
    return np.cumsum(ptr), cols, vals


def fit(users, items, ratings, rank=10, max_iter=10, reg=0.1, implicit=False, alpha=1.0,
        nonnegative=False, seed=0) -> ALSResult:
    users = np.asarray(users, dtype=np.int64)
    items = np.asarray(items, dtype=np.int64)
    ratings = np.asarray(ratings, dtype=np.float32)
    uid, ui = np.unique(users, return_inverse=True)
    iid, ii = np.unique(items, return_inverse=True)
    X = init_factors(uid, rank, seed)
    Y = np.zeros((len(iid), rank), dtype=np.float32)
    ucsr = _csr(ui, ii, ratings, len(uid))
    icsr = _csr(ii, ui, ratings, len(iid))
    for _ in range(max_iter):
        Y = _solve_side(*icsr, X, rank, reg, implicit, alpha, nonnegative)
        X = _solve_side(*ucsr, Y, rank, reg, implicit, alpha, nonnegative)
    return ALSResult(uid.astype(np.int32), iid.astype(np.int32), X, Y)
