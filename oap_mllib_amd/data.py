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
        ser = dataset[features_col]
        if isinstance(ser.dtype, pd.ArrowDtype):  # Arrow-backed vector column: zero-copy
            import pyarrow as pa

            m = _arrow_matrix(pa.array(ser), dtype)
            if m is not None:
                return m
        return _stack(ser.tolist(), dtype)
    try:
        import pyarrow as pa
    except ImportError:  # pragma: no cover
        pa = None
    if pa is not None and isinstance(dataset, pa.Table):
        m = _arrow_matrix(dataset.column(features_col), dtype)
        if m is not None:
            return m
        return _stack(dataset.column(features_col).to_pylist(), dtype)
    if isinstance(dataset, (list, tuple)):
        return _stack(list(dataset), dtype)
    raise TypeError(f"unsupported dataset type {type(dataset).__name__}")


def _arrow_matrix(col: Any, dtype) -> np.ndarray | None:
    """(n, d) matrix from an Arrow vector column without per-row Python objects: a
    fixed_size_list or (equal-length) list of floats, or Spark's VectorUDT struct when every row
    is dense (type 1).  None when the column needs the per-row path (sparse rows, ragged)."""
    import pyarrow as pa

    if isinstance(col, pa.ChunkedArray):
        col = col.combine_chunks() if col.num_chunks != 1 else col.chunk(0)
    n = len(col)
    if col.null_count:
        return None
    t = col.type
    if pa.types.is_struct(t) and {"type", "values"} <= {f.name for f in t}:
        kinds = col.field("type").to_numpy(zero_copy_only=False)
        if n and not np.all(kinds == 1):
            return None
        return _arrow_matrix(col.field("values"), dtype)
    if pa.types.is_fixed_size_list(t):
        d = t.list_size
        vals = col.values.slice(col.offset * d, n * d)
    elif pa.types.is_list(t) or pa.types.is_large_list(t):
        off = col.offsets.to_numpy(zero_copy_only=False)
        lens = np.diff(off)
        if n == 0:
            return np.zeros((0, 0), dtype=dtype)
        d = int(lens[0])
        if not np.all(lens == d):
            raise ValueError("all feature vectors must have the same size")
        vals = col.values.slice(int(off[0]), n * d)
    else:
        return None
    if not (pa.types.is_floating(vals.type) or pa.types.is_integer(vals.type)) or vals.null_count:
        return None
    m = vals.to_numpy(zero_copy_only=False).reshape(n, d)
    if m.dtype not in (np.float32, np.float64):
        m = m.astype(dtype)
    return np.ascontiguousarray(m)


def vector_column(m: np.ndarray):
    """(n, d) matrix -> pandas Series of vectors backed by ONE Arrow fixed_size_list buffer
    (zero-copy; no per-row Python objects — rows read back as lists / through to_matrix)."""
    import pandas as pd
    import pyarrow as pa

    m = np.ascontiguousarray(m)
    if m.ndim == 1:
        m = m.reshape(-1, 1)
    arr = pa.FixedSizeListArray.from_arrays(pa.array(m.reshape(-1)), int(m.shape[1]))
    return pd.Series(pd.arrays.ArrowExtensionArray(arr))


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
        return pd.DataFrame({features_col: vector_column(m)})
    try:
        import pyarrow as pa

        if isinstance(dataset, pa.Table):
            m = _arrow_matrix(dataset.column(features_col), np.float64)
            rest = dataset.drop_columns([features_col]) if m is not None else dataset
            df = rest.to_pandas()
            if m is not None:
                df.insert(dataset.schema.get_field_index(features_col), features_col,
                          vector_column(m))
            else:
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
            return dataset.column(name).to_numpy()
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
