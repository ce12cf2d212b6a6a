"""Vanilla (pure numpy, fp64) K-Means — the analog of the reference's Spark fallback path.

The reference dispatches to upstream Spark MLlib whenever its native path does not apply
(``trainWithML``, spark-3.1.1/ml/clustering/KMeans.scala:441-457: cosine distance or a weightCol).
This module re-implements the upstream semantics in numpy — Lloyd iterations with weighted sums,
"empty clusters keep their center", convergence when every moved center shifts by <= tol
(mllib/clustering/KMeans.scala:275-335), k-means|| and random initialisation (:354-432) and
``LocalKMeans.kMeansPlusPlus`` — including the cosine distance measure.  It is also the fp64
numerical oracle the native engine is tested against.  Random streams are our own (exact RNG
parity with Spark's XORShiftRandom is not a goal: "parity unpinned" for seeded draws).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

EUCLIDEAN = "euclidean"
COSINE = "cosine"


@dataclass
class VanillaKMeansResult:
    centers: np.ndarray
    cost: float
    num_iter: int
    converged: bool
    cost_history: list = field(default_factory=list)


def _normalize(x: np.ndarray) -> np.ndarray:
    n = np.linalg.norm(x, axis=1, keepdims=True)
    n[n == 0] = 1.0
    return x / n


def pairwise_cost(x: np.ndarray, c: np.ndarray, measure: str) -> np.ndarray:
    """(n, k) point-to-center costs (squared euclidean, or 1 - cosine similarity)."""
    if measure == COSINE:
        return 1.0 - _normalize(x) @ _normalize(c).T
    d = (x * x).sum(1)[:, None] - 2.0 * x @ c.T + (c * c).sum(1)[None, :]
    # exact refinement where the expansion may have cancelled
    return np.maximum(d, 0.0)


def find_closest(x: np.ndarray, c: np.ndarray, measure: str = EUCLIDEAN,
                 chunk: int = 65536) -> tuple[np.ndarray, np.ndarray]:
    labels = np.empty(len(x), dtype=np.int32)
    costs = np.empty(len(x))
    for s in range(0, len(x), chunk):
        xs = x[s:s + chunk]
        if measure == EUCLIDEAN:
            # exact fp64 distances (no expansion) to match Spark's precise fallback
            small = c.shape[0] * xs.shape[1] <= 4096
            d = ((xs[:, None, :] - c[None, :, :]) ** 2).sum(-1) if small \
                else pairwise_cost(xs, c, measure)
        else:
            d = pairwise_cost(xs, c, measure)
        labels[s:s + chunk] = np.argmin(d, axis=1)
        costs[s:s + chunk] = d[np.arange(len(xs)), labels[s:s + chunk]]
    return labels, costs


def _rng(seed: int) -> np.random.Generator:
    return np.random.default_rng(np.uint64(seed & 0xFFFFFFFFFFFFFFFF))


def _distinct(rows: np.ndarray) -> np.ndarray:
    seen, out = set(), []
    for r in rows:
        key = tuple((r + 0.0).tolist())
        if key not in seen:
            seen.add(key)
            out.append(r)
    return np.array(out).reshape(-1, rows.shape[1]) if out else rows[:0]


def _kmeans_pp_once(points, weights, k, max_iter, rng, measure):
    n = len(points)

    def pick(mass):
        r = rng.random() * mass.sum()
        return min(int(np.searchsorted(np.cumsum(mass), r, side="left")), n - 1) if r > 0 else 0

    centers = [points[pick(weights)]]
    cost = pairwise_cost(points, np.array(centers), measure)[:, 0]
    trials = 2 + int(np.log(k))
    for _ in range(1, k):
        best = None
        for _t in range(trials):
            cand = pick(weights * cost)
            tc = np.minimum(cost, pairwise_cost(points, points[cand:cand + 1], measure)[:, 0])
            pot = float((weights * tc).sum())
            if best is None or pot < best[0]:
                best = (pot, cand, tc)
        centers.append(points[best[1]])
        cost = best[2]
    centers = np.array(centers, dtype=np.float64)
    old = np.full(n, -1)
    for _ in range(max_iter):
        lab = np.argmin(pairwise_cost(points, centers, measure), axis=1)
        moved = bool((lab != old).any())
        old = lab
        for j in range(k):
            m = lab == j
            wj = weights[m].sum()
            if wj == 0:
                centers[j] = points[rng.integers(0, n)]
            else:
                centers[j] = (weights[m, None] * points[m]).sum(0) / wj
        if not moved:
            break
    total = float((weights * pairwise_cost(points, centers, measure).min(axis=1)).sum())
    return total, centers


def kmeans_pp(points: np.ndarray, weights: np.ndarray, k: int, max_iter: int, seed: int,
              measure: str = EUCLIDEAN) -> np.ndarray:
    """Weighted greedy k-means++ + weighted Lloyd, best of 3 restarts (same algorithm as the
    native ``local_kmeans_pp``; Spark's LocalKMeans.kMeansPlusPlus is the single-run variant)."""
    rng = _rng(seed)
    best = None
    for _ in range(3):
        c, centers = _kmeans_pp_once(points, weights, k, max_iter, rng, measure)
        if best is None or c < best[0]:
            best = (c, centers)
    return best[1]


def init_random(x: np.ndarray, k: int, seed: int) -> np.ndarray:
    idx = _rng(seed).choice(len(x), size=min(k, len(x)), replace=False)
    return _distinct(x[idx])


def init_parallel(x: np.ndarray, k: int, steps: int, seed: int, weights: np.ndarray | None,
                  measure: str = EUCLIDEAN) -> np.ndarray:
    rng = _rng(seed)
    n = len(x)
    centers = [x[rng.integers(0, n)]]
    new = np.array(centers)
    costs = np.full(n, np.inf)
    for _ in range(steps):
        costs = np.minimum(costs, pairwise_cost(x, new, measure).min(axis=1))
        s = costs.sum()
        if s <= 0:
            break
        chosen = x[rng.random(n) < 2.0 * costs * k / s]
        new = chosen
        centers.extend(list(chosen))
        if len(chosen) == 0:
            break
    cand = _distinct(np.array(centers))
    if len(cand) <= k:
        return cand
    lab, _ = find_closest(x, cand, measure)
    w = np.bincount(lab, weights=weights, minlength=len(cand)).astype(np.float64)
    return kmeans_pp(cand, w, k, 30, seed ^ 0x5A5A, measure)


def fit(x: np.ndarray, k: int, max_iter: int = 20, tol: float = 1e-4,
        init_mode: str = "k-means||", init_steps: int = 2, seed: int = 1,
        measure: str = EUCLIDEAN, weights: np.ndarray | None = None,
        init_centers: np.ndarray | None = None, allreduce=None) -> VanillaKMeansResult:
    """Lloyd iterations.  `allreduce(arr) -> arr` makes it distributed (x = local rows)."""
    x = np.asarray(x, dtype=np.float64)
    w = np.ones(len(x)) if weights is None else np.asarray(weights, dtype=np.float64)
    if init_centers is not None:
        centers = np.array(init_centers, dtype=np.float64)
    elif init_mode == "random":
        centers = init_random(x, k, seed)
    else:
        centers = init_parallel(x, k, init_steps, seed, w, measure)
    kk, d = centers.shape
    cost, it, converged, hist = 0.0, 0, False, []
    while it < max_iter and not converged:
        lab, c = find_closest(x, centers, measure)
        sums = np.zeros((kk, d))
        np.add.at(sums, lab, w[:, None] * x)
        wsum = np.bincount(lab, weights=w, minlength=kk).astype(np.float64)
        cst = float((c * w).sum())
        if allreduce is not None:
            packed = allreduce(np.concatenate([sums.ravel(), wsum, [cst]]))
            sums, wsum, cst = packed[:kk * d].reshape(kk, d), packed[kk * d:kk * d + kk], \
                float(packed[-1])
        converged = True
        for j in range(kk):
            if wsum[j] <= 0:
                continue
            nc = sums[j] / wsum[j]
            if measure == COSINE:
                nrm = np.linalg.norm(nc)
                nc = nc / nrm if nrm > 0 else nc
                # CosineDistanceMeasure: converged when distance(old, new) <= tol
                moved = 1.0 - float(np.dot(_normalize(centers[j:j + 1])[0], nc)) > tol
            else:
                moved = float(((nc - centers[j]) ** 2).sum()) > tol * tol
            if moved:
                converged = False
            centers[j] = nc
        cost = cst
        hist.append(cst)
        it += 1
    return VanillaKMeansResult(centers, cost, it, converged, hist)
