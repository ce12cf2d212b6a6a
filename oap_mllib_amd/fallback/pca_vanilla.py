"""fp64 numpy PCA with the semantics of Spark's ``mllib.feature.PCA`` — the path the reference
falls back to when ``numFeatures >= 65535`` or the platform check fails
(mllib-dal/src/main/scala/org/apache/spark-3.1.1/ml/feature/PCA.scala:103-116), i.e.
``RowMatrix.computePrincipalComponentsAndExplainedVariance``: sample covariance (/(n-1)), its
spectral decomposition, top-k vectors, explained variance = top-k / sum over all d.
"""
from __future__ import annotations

import numpy as np


def normalize_signs(pc: np.ndarray) -> np.ndarray:
    """Largest-magnitude component of every column positive (the native engine's convention)."""
    pc = np.array(pc, dtype=np.float64, copy=True)
    for j in range(pc.shape[1]):
        i = int(np.argmax(np.abs(pc[:, j])))
        if pc[i, j] < 0:
            pc[:, j] = -pc[:, j]
    return pc


def covariance(X: np.ndarray, allreduce=None) -> tuple[np.ndarray, np.ndarray, int]:
    """(cov, mean, n) with an optional sum-allreduce across ranks (shifted one-pass form)."""
    X = np.asarray(X, dtype=np.float64)
    d = X.shape[1]
    shift = X[: min(len(X), 256)].sum(axis=0)
    cnt = np.array([min(len(X), 256)], dtype=np.float64)
    if allreduce is not None:
        shift = allreduce(shift)
        cnt = allreduce(cnt)
    shift = shift / cnt[0] if cnt[0] > 0 else np.zeros(d)
    Y = X - shift
    S = Y.T @ Y
    c = Y.sum(axis=0)
    n = np.array([float(len(X))])
    if allreduce is not None:
        S, c, n = allreduce(S), allreduce(c), allreduce(n)
    n = int(n[0])
    if n <= 1:
        raise ValueError("Cannot compute the covariance of a matrix with <= 1 row")
    cov = (S - np.outer(c, c) / n) / (n - 1)
    return cov, shift + c / n, n


def fit(X: np.ndarray, k: int, allreduce=None) -> tuple[np.ndarray, np.ndarray]:
    """(pc d x k, explainedVariance k)."""
    cov, _, _ = covariance(X, allreduce)
    w, V = np.linalg.eigh(cov)
    order = np.argsort(-np.abs(w), kind="stable")
    w, V = np.abs(w[order]), V[:, order]
    tot = w.sum()
    ev = w[:k] / tot if tot > 0 else np.zeros(k)
    return normalize_signs(V[:, :k]), ev
