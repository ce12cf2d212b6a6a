"""CPU comparison baselines for the BASELINE.json configs (BASELINE.md "What this repo will
measure instead": vanilla Spark MLlib when Spark is present, otherwise a clearly labelled fp64
CPU proxy of the same algorithm on the GPU host's cores).  Spark is not installed on the GPU
hosts, so these are the proxies; each returns a labelled dict with the host threads it used and
the per-row (per-rating) rate it measured on a subsample, so a benchmark can scale it to the
configuration's size and report ``vs_baseline`` = GPU rate / CPU rate.

* K-Means: scikit-learn ``KMeans(algorithm="lloyd")`` (fp64, OpenMP + BLAS GEMM distance
  blocks — the same structure as oneDAL's batch step that the reference calls,
  mllib-dal/src/main/native/KMeansDALImpl.cpp:70-77), per-iteration time from the difference of a
  1- and a (1 + iters)-iteration fit from the same centers (input validation excluded).
* PCA: numpy fp64 covariance (BLAS SYRK-shaped X^T X) + ``numpy.linalg.eigh``: the reference's
  oneDAL covariance + eigen step (PCADALImpl.cpp:63-69,127-150).
* ALS: this framework's fp64 host engine (``Context(-1)``, thread pool, per-row Cholesky) on a
  ratings subsample — the reference's oneDAL implicit ALS is likewise a CPU per-row solver.
"""
from __future__ import annotations

import os
import time

import numpy as np


def host_threads() -> int:
    """Host cores this process may use (the GPU box grants a share, not the machine)."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        return os.cpu_count() or 1


def kmeans_proxy(X: np.ndarray, init: np.ndarray, iters: int = 2) -> dict:
    """Lloyd iterations of scikit-learn's KMeans on fp64 rows X from centers init."""
    from sklearn.cluster import KMeans

    X = np.ascontiguousarray(X, dtype=np.float64)
    init = np.ascontiguousarray(init, dtype=np.float64)
    k = init.shape[0]

    def fit(n_iter):
        t0 = time.perf_counter()
        m = KMeans(n_clusters=k, init=init, n_init=1, max_iter=n_iter, tol=0.0,
                   algorithm="lloyd", copy_x=False).fit(X)
        return time.perf_counter() - t0, int(m.n_iter_)

    fit(1)  # (warm: thread pool, BLAS)
    t1, _ = fit(1)
    tn, n_done = fit(1 + iters)
    per_iter = max(tn - t1, 1e-9) / max(n_done - 1, 1)
    return {"engine": "scikit-learn KMeans(algorithm='lloyd') fp64, OpenMP + BLAS",
            "threads": host_threads(), "rows": int(X.shape[0]), "dim": int(X.shape[1]), "k": k,
            "iters_timed": n_done - 1, "ms_per_iter": per_iter * 1e3,
            "samples_per_sec": X.shape[0] / per_iter,
            "note": "CPU proxy (no Spark on the GPU host): per-iteration time on a row "
                    "subsample, rate scales linearly with rows"}


def pca_proxy(X: np.ndarray, k: int, full_rows: int) -> dict:
    """fp64 covariance + eigh on rows X; the fit time scaled to full_rows rows."""
    X = np.ascontiguousarray(X, dtype=np.float64)
    n, d = X.shape
    t0 = time.perf_counter()
    mu = X.mean(axis=0)
    Xc = X - mu
    S = Xc.T @ Xc
    cov = S / (n - 1)
    t1 = time.perf_counter()
    w, _ = np.linalg.eigh(cov)
    t2 = time.perf_counter()
    stats_s = (t1 - t0) * (full_rows / n)
    return {"engine": "numpy fp64 covariance (BLAS) + numpy.linalg.eigh",
            "threads": host_threads(), "rows_measured": int(n), "dim": int(d), "k": int(k),
            "stats_s_measured": t1 - t0, "eigh_s": t2 - t1,
            "fit_s_scaled": stats_s + (t2 - t1), "rows_scaled_to": int(full_rows),
            "top_eigenvalue": float(w[-1]),
            "note": "CPU proxy (no Spark on the GPU host): covariance time scaled linearly "
                    "from the subsample to the configuration's rows, eigensolver as measured"}


def als_proxy(N, users: np.ndarray, items: np.ndarray, ratings: np.ndarray, rank: int,
              alpha: float, reg: float, full_ratings: int, iters: int = 1) -> dict:
    """This framework's fp64 host ALS engine on a ratings subsample; per-iteration time scaled
    to full_ratings ratings (the per-row solves dominate: linear in ratings and rows)."""
    threads = host_threads()
    ctx = N.Context(-1, 0.5, threads)
    comm = N.LocalComm(False)
    t0 = time.perf_counter()
    r = N.als_fit(ctx, comm, users, items, ratings, rank=rank, max_iter=iters, reg=reg,
                  alpha=alpha, implicit=True, seed=0)
    wall = time.perf_counter() - t0
    it_ms = float(np.mean(r["iter_ms"])) if len(r["iter_ms"]) else wall * 1e3 / iters
    nnz = int(len(ratings))
    return {"engine": "oap_mllib_amd fp64 host ALS engine (thread pool, per-row Cholesky)",
            "threads": threads, "ratings_measured": nnz, "rank": rank,
            "ms_per_iter_measured": it_ms,
            "s_per_iter_scaled": it_ms * 1e-3 * (full_ratings / max(nnz, 1)),
            "ratings_scaled_to": int(full_ratings),
            "note": "CPU proxy (no Spark on the GPU host): per-iteration time scaled linearly "
                    "from the ratings subsample"}
