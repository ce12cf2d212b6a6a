"""Dataset readers for the example/benchmark formats (native parallel parsers).

* ``read_csv``      — dense numeric CSV (examples/data/pca_data.csv)
* ``read_libsvm``   — LIBSVM "label idx:val ..." (examples/data/sample_kmeans_data.txt), as a
                      dense matrix or as SparseVector rows, with Spark's one-based indices
* ``read_ratings``  — "user<sep>item<sep>rating" lines (examples/data/onedal_als_csr_ratings.txt)

Counterparts of the reference's service.cpp readers (mllib-dal/src/main/native/
service.cpp:26-146) and of the Spark data sources its examples use.
"""
from __future__ import annotations

import os

import numpy as np

from .. import _loader
from ..linalg import SparseVector


def _threads() -> int:
    return max(1, min(16, os.cpu_count() or 1))


def read_csv(path: str, sep: str = ",") -> np.ndarray:
    return _loader.load().read_csv(path, sep, _threads())


def read_libsvm(path: str, num_features: int | None = None, dense: bool = True):
    """(labels, features): features is an (n, d) float64 array or a list of SparseVector."""
    labels, indptr, indices, values, max_index = _loader.load().read_libsvm(path, _threads())
    d = int(num_features) if num_features else int(max_index)
    if dense:
        X = np.zeros((len(labels), d), dtype=np.float64)
        rows = np.repeat(np.arange(len(labels)), np.diff(indptr))
        X[rows, indices] = values
        return np.asarray(labels), X
    vecs = [SparseVector(d, indices[indptr[i]:indptr[i + 1]].tolist(),
                         values[indptr[i]:indptr[i + 1]].tolist()) for i in range(len(labels))]
    return np.asarray(labels), vecs


def read_ratings(path: str, sep: str = "::") -> dict:
    """{"user", "item", "rating"} column arrays (int32, int32, float32)."""
    u, i, r = _loader.load().read_ratings(path, sep, _threads())
    return {"user": np.asarray(u), "item": np.asarray(i), "rating": np.asarray(r)}
