"""Minimal ``pyspark.ml.linalg`` counterparts (DenseVector, SparseVector, DenseMatrix).

They exist so that model attributes and persisted data have the same shapes and semantics as
Spark's (``KMeansModel.clusterCenters: Array[Vector]``, ``PCAModel.pc: DenseMatrix`` stored
column-major, ``explainedVariance: DenseVector``), and so that datasets holding Spark-style
vectors (dense or sparse) can be ingested.  Sparse vectors are densified at ingestion exactly
as the reference does (OneDAL.scala:126-139 calls ``toArray`` on every row).
"""
from __future__ import annotations

from typing import Iterable, Sequence

import numpy as np


class Vector:
    def toArray(self) -> np.ndarray:  # noqa: N802 (Spark API name)
        raise NotImplementedError

    @property
    def size(self) -> int:
        return len(self.toArray())

    def __len__(self) -> int:
        return self.size


class DenseVector(Vector):
    def __init__(self, values: Iterable[float]):
        self.values = np.asarray(list(values) if not isinstance(values, np.ndarray) else values,
                                 dtype=np.float64).reshape(-1)

    def toArray(self) -> np.ndarray:  # noqa: N802
        return self.values

    @property
    def size(self) -> int:
        return int(self.values.shape[0])

    def norm(self, p: float = 2.0) -> float:
        return float(np.linalg.norm(self.values, p))

    def dot(self, other) -> float:
        return float(np.dot(self.values, _arr(other)))

    def squared_distance(self, other) -> float:
        d = self.values - _arr(other)
        return float(np.dot(d, d))

    def __getitem__(self, i):
        return self.values[i]

    def __iter__(self):
        return iter(self.values)

    def __eq__(self, other) -> bool:
        if isinstance(other, Vector):
            a, b = self.toArray(), other.toArray()
            return a.shape == b.shape and bool(np.all(a == b))
        return NotImplemented

    def __hash__(self) -> int:
        return hash(tuple(self.values.tolist()))

    def __repr__(self) -> str:
        return f"DenseVector({self.values.tolist()})"


class SparseVector(Vector):
    def __init__(self, size: int, indices: Sequence[int], values: Sequence[float]):
        self._size = int(size)
        self.indices = np.asarray(indices, dtype=np.int32)
        self.values = np.asarray(values, dtype=np.float64)
        if self.indices.shape != self.values.shape:
            raise ValueError("indices and values must have the same length")
        if len(self.indices) and (self.indices.min() < 0 or self.indices.max() >= self._size):
            raise ValueError("index out of range")

    @property
    def size(self) -> int:
        return self._size

    def toArray(self) -> np.ndarray:  # noqa: N802
        a = np.zeros(self._size)
        a[self.indices] = self.values
        return a

    def __eq__(self, other) -> bool:
        if isinstance(other, Vector):
            return self.size == other.size and bool(np.all(self.toArray() == other.toArray()))
        return NotImplemented

    def __hash__(self) -> int:
        return hash(tuple(self.toArray().tolist()))

    def __repr__(self) -> str:
        return f"SparseVector({self._size}, {self.indices.tolist()}, {self.values.tolist()})"


class DenseMatrix:
    """Column-major dense matrix (Spark layout); ``toArray`` returns the numRows x numCols array."""

    def __init__(self, numRows: int, numCols: int, values: Iterable[float],  # noqa: N803
                 isTransposed: bool = False):  # noqa: N803
        self.numRows = int(numRows)
        self.numCols = int(numCols)
        self.values = np.asarray(list(values) if not isinstance(values, np.ndarray) else values,
                                 dtype=np.float64).reshape(-1)
        self.isTransposed = bool(isTransposed)
        if self.values.shape[0] != self.numRows * self.numCols:
            raise ValueError("values length must be numRows * numCols")

    @staticmethod
    def from_array(a: np.ndarray) -> "DenseMatrix":
        a = np.asarray(a, dtype=np.float64)
        return DenseMatrix(a.shape[0], a.shape[1], a.reshape(-1, order="F"))

    def toArray(self) -> np.ndarray:  # noqa: N802
        if self.isTransposed:
            return self.values.reshape(self.numRows, self.numCols)
        return self.values.reshape(self.numCols, self.numRows).T

    def __eq__(self, other) -> bool:
        return isinstance(other, DenseMatrix) and np.array_equal(self.toArray(), other.toArray())

    def __repr__(self) -> str:
        return f"DenseMatrix({self.numRows}, {self.numCols}, ...)"


class Vectors:
    @staticmethod
    def dense(*values) -> DenseVector:
        if len(values) == 1 and not np.isscalar(values[0]):
            return DenseVector(values[0])
        return DenseVector(values)

    @staticmethod
    def sparse(size: int, *args) -> SparseVector:
        if len(args) == 1:
            items = args[0].items() if isinstance(args[0], dict) else args[0]
            items = sorted(items)
            return SparseVector(size, [i for i, _ in items], [v for _, v in items])
        return SparseVector(size, args[0], args[1])

    @staticmethod
    def zeros(size: int) -> DenseVector:
        return DenseVector(np.zeros(size))

    @staticmethod
    def norm(v, p: float = 2.0) -> float:
        return float(np.linalg.norm(_arr(v), p))

    @staticmethod
    def squared_distance(a, b) -> float:
        d = _arr(a) - _arr(b)
        return float(np.dot(d, d))


class Matrices:
    @staticmethod
    def dense(numRows: int, numCols: int, values) -> DenseMatrix:  # noqa: N803
        return DenseMatrix(numRows, numCols, values)


def _arr(v) -> np.ndarray:
    if isinstance(v, Vector):
        return v.toArray()
    return np.asarray(v, dtype=np.float64)
