"""Dataset adapters: numpy / pandas / pyarrow / vector lists <-> dense row matrices.

Plays the part of the reference's RDD -> numeric-table marshalling
(OneDAL.vectorsToMergedNumericTables, mllib-dal/src/main/scala/org/apache/spark/ml/util/
OneDAL.scala:92-166) on the Python side: it produces ONE contiguous row-major block per rank that
the native ingestion streams to HBM in a single pipelined pass (no per-row JNI call).

Accepted datasets (the "DataFrame" of this framework):
  * ``np.ndarray`` of shape (n, d)
  * ``pandas.DataFrame`` whose ``featuresCol`` column holds arrays/lists/Vectors
  * ``pyarrow.Table`` with a list<double> (or Spark VectorUDT struct) features column
  * a list of Vectors / sequences
Outputs of ``transform`` are pandas DataFrames (the input columns plus the new column).
"""
from __future__ import annotations

from typing import Any

import numpy as np

from .linalg import DenseVector, SparseVector, Vector


def _row_to_array(v: Any) -> np.ndarray:
    if isinstance(v, Vector):
        return v.toArray()
    if isinstance(v, dict) and "type" in v:  # Spark VectorUDT struct (e.g. from parquet)
        if v["type"] == 1:
            return np.asarray(v["values"], dtype=np.float64)
        a = np.zeros(v["size"])
        a[np.asarray(v["indices"], dtype=np.int64)] = v["values"]
        return a
    return np.asarray(v, dtype=np.float64)


def _columns_to_frame(dataset: Any) -> Any:
    """A {column: values} mapping is accepted wherever a DataFrame is."""
    if isinstance(dataset, dict):
        import pandas as pd

        return pd.DataFrame({k: list(v) for k, v in dataset.items()})
    return dataset


def to_matrix(dataset: Any, features_col: str = "features",
              dtype=np.float64) -> np.ndarray:
    """Returns a C-contiguous (n, d) matrix for `dataset`."""
    dataset = _columns_to_frame(dataset)
    if isinstance(dataset, np.ndarray):
        m = dataset
        if m.ndim == 1:
            m = m.reshape(-1, 1)
        if m.ndim != 2:
            raise ValueError("feature matrix must be 2-D")
        if m.dtype not in (np.float32, np.float64):
            m = m.astype(dtype)
        return np.ascontiguousarray(m)
    try:
        import pandas as pd
    except ImportError:  # pragma: no cover
        pd = None
    if pd is not None and isinstance(dataset, pd.DataFrame):
        if features_col not in dataset.columns:
            raise ValueError(f"featuresCol '{features_col}' not in columns {list(dataset.columns)}")
        col = dataset[features_col].tolist()
        return _stack(col, dtype)
    try:
        import pyarrow as pa
    except ImportError:  # pragma: no cover
        pa = None
    if pa is not None and isinstance(dataset, pa.Table):
        return _stack(dataset.column(features_col).to_pylist(), dtype)
    if isinstance(dataset, (list, tuple)):
        return _stack(list(dataset), dtype)
    raise TypeError(f"unsupported dataset type {type(dataset).__name__}")


def _stack(rows: list, dtype) -> np.ndarray:
    if not rows:
        return np.zeros((0, 0), dtype=dtype)
    arrs = [_row_to_array(r) for r in rows]
    d = arrs[0].shape[0]
    for a in arrs:
        if a.shape[0] != d:
            raise ValueError("all feature vectors must have the same size")
    return np.ascontiguousarray(np.stack(arrs).astype(dtype, copy=False))


def as_frame(dataset: Any, features_col: str = "features"):
    """pandas view of a dataset (numpy matrices become a single vector column)."""
    import pandas as pd

    dataset = _columns_to_frame(dataset)
    if isinstance(dataset, pd.DataFrame):
        return dataset.copy()
    if isinstance(dataset, np.ndarray):
        m = dataset if dataset.ndim == 2 else dataset.reshape(-1, 1)
        return pd.DataFrame({features_col: [DenseVector(r) for r in m]})
    try:
        import pyarrow as pa

        if isinstance(dataset, pa.Table):
            df = dataset.to_pandas()
            df[features_col] = [DenseVector(_row_to_array(v)) for v in df[features_col]]
            return df
    except ImportError:  # pragma: no cover
        pass
    if isinstance(dataset, (list, tuple)):
        return pd.DataFrame({features_col: [v if isinstance(v, Vector) else DenseVector(v)
                                            for v in dataset]})
    raise TypeError(f"unsupported dataset type {type(dataset).__name__}")


def column(dataset: Any, name: str) -> np.ndarray:
    import pandas as pd

    dataset = _columns_to_frame(dataset)
    if isinstance(dataset, pd.DataFrame):
        return dataset[name].to_numpy()
    try:
        import pyarrow as pa

        if isinstance(dataset, pa.Table):
            return np.asarray(dataset.column(name).to_pylist())
    except ImportError:  # pragma: no cover
        pass
    raise TypeError(f"cannot read column '{name}' from {type(dataset).__name__}")


def is_sparse_rows(dataset: Any, features_col: str = "features") -> bool:
    try:
        import pandas as pd

        if isinstance(dataset, pd.DataFrame) and len(dataset):
            return isinstance(dataset[features_col].iloc[0], SparseVector)
    except ImportError:  # pragma: no cover
        pass
    return False
