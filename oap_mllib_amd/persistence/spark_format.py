"""Spark-ML on-disk model format (``MLWritable`` / ``MLReadable``), written with pyarrow.

Drop-in compatibility with ``org.apache.spark.ml`` is part of the reference's contract (its
shadow classes keep Spark's writers/readers: KMeans.scala:184-264, PCA.scala:205-249,
ALS.scala:522-553).  Spark is not available here, so the layout is produced
directly:

  <path>/metadata/part-00000   one-line JSON: class, timestamp, sparkVersion, uid, paramMap,
                               defaultParamMap (+ extra fields, e.g. ALS "rank")
  <path>/metadata/_SUCCESS
  <path>/data/part-00000-<uuid>-c000.snappy.parquet  (+ _SUCCESS)

Vectors and matrices use Spark's UDT struct encodings (VectorUDT: type/size/indices/values;
MatrixUDT: type/numRows/numCols/colPtrs/rowIndices/values/isTransposed) and the parquet footer
carries ``org.apache.spark.sql.parquet.row.metadata`` with the UDT-annotated schema, so Spark's
own ``KMeansModel.load`` / ``PCAModel.load`` / ``ALSModel.load`` can read the directories.
"""
from __future__ import annotations

import json
import os
import time
import uuid
from typing import Any

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

SPARK_VERSION = "3.1.1"  # default unless Config.spark_version or pyspark says otherwise
#: Spark versions the reference ships shadow sources for (mllib-dal/pom.xml:151-224)
SUPPORTED_SPARK_VERSIONS = ("3.0.0", "3.0.1", "3.0.2", "3.1.1")


def spark_version() -> str:
    """Version stamped into written models: Config.spark_version, else pyspark's, else 3.1.1."""
    from ..config import get_config

    v = get_config().spark_version
    if v:
        return v
    try:
        import pyspark

        return str(pyspark.__version__)
    except ImportError:
        return SPARK_VERSION


def major_version(v: str) -> int:
    """Spark's VersionUtils.majorVersion ("1.6.3" -> 1); used by the readers to pick the
    on-disk layout (Spark <= 1.6 stored K-Means centers in one row, PCA without variances)."""
    try:
        return int(str(v).split(".")[0])
    except ValueError as e:
        raise ValueError(f"Spark version {v!r} is not of the form major.minor[.patch]") from e
ROW_METADATA_KEY = b"org.apache.spark.sql.parquet.row.metadata"

VECTOR_SQL = {"type": "struct", "fields": [
    {"name": "type", "type": "byte", "nullable": False, "metadata": {}},
    {"name": "size", "type": "integer", "nullable": True, "metadata": {}},
    {"name": "indices", "type": {"type": "array", "elementType": "integer", "containsNull": False},
     "nullable": True, "metadata": {}},
    {"name": "values", "type": {"type": "array", "elementType": "double", "containsNull": False},
     "nullable": True, "metadata": {}}]}
VECTOR_UDT = {"type": "udt", "class": "org.apache.spark.ml.linalg.VectorUDT",
              "pyClass": "pyspark.ml.linalg.VectorUDT", "sqlType": VECTOR_SQL}
MATRIX_SQL = {"type": "struct", "fields": [
    {"name": "type", "type": "byte", "nullable": False, "metadata": {}},
    {"name": "numRows", "type": "integer", "nullable": False, "metadata": {}},
    {"name": "numCols", "type": "integer", "nullable": False, "metadata": {}},
    {"name": "colPtrs", "type": {"type": "array", "elementType": "integer", "containsNull": False},
     "nullable": True, "metadata": {}},
    {"name": "rowIndices", "type": {"type": "array", "elementType": "integer",
                                    "containsNull": False}, "nullable": True, "metadata": {}},
    {"name": "values", "type": {"type": "array", "elementType": "double", "containsNull": False},
     "nullable": True, "metadata": {}},
    {"name": "isTransposed", "type": "boolean", "nullable": False, "metadata": {}}]}
MATRIX_UDT = {"type": "udt", "class": "org.apache.spark.ml.linalg.MatrixUDT",
              "pyClass": "pyspark.ml.linalg.MatrixUDT", "sqlType": MATRIX_SQL}

VECTOR_ARROW = pa.struct([
    pa.field("type", pa.int8(), nullable=False), pa.field("size", pa.int32()),
    pa.field("indices", pa.list_(pa.field("element", pa.int32(), nullable=False))),
    pa.field("values", pa.list_(pa.field("element", pa.float64(), nullable=False)))])
MATRIX_ARROW = pa.struct([
    pa.field("type", pa.int8(), nullable=False), pa.field("numRows", pa.int32(), nullable=False),
    pa.field("numCols", pa.int32(), nullable=False),
    pa.field("colPtrs", pa.list_(pa.field("element", pa.int32(), nullable=False))),
    pa.field("rowIndices", pa.list_(pa.field("element", pa.int32(), nullable=False))),
    pa.field("values", pa.list_(pa.field("element", pa.float64(), nullable=False))),
    pa.field("isTransposed", pa.bool_(), nullable=False)])


def dense_vector_struct(v) -> dict:
    return {"type": 1, "size": None, "indices": None,
            "values": [float(x) for x in np.asarray(v, dtype=np.float64).ravel()]}


def dense_matrix_struct(a: np.ndarray) -> dict:
    a = np.asarray(a, dtype=np.float64)
    return {"type": 1, "numRows": int(a.shape[0]), "numCols": int(a.shape[1]), "colPtrs": None,
            "rowIndices": None, "values": a.reshape(-1, order="F").tolist(),
            "isTransposed": False}


def vector_from_struct(s: dict) -> np.ndarray:
    if s["type"] == 1:
        return np.asarray(s["values"], dtype=np.float64)
    out = np.zeros(int(s["size"]))
    out[np.asarray(s["indices"], dtype=np.int64)] = s["values"]
    return out


def matrix_from_struct(s: dict) -> np.ndarray:
    r, c = int(s["numRows"]), int(s["numCols"])
    if s["type"] == 1:
        v = np.asarray(s["values"], dtype=np.float64)
        return v.reshape(r, c) if s["isTransposed"] else v.reshape(c, r).T
    # sparse CSC (or CSR when transposed)
    out = np.zeros((r, c))
    ptr, idx, val = s["colPtrs"], s["rowIndices"], s["values"]
    outer = r if s["isTransposed"] else c
    for j in range(outer):
        for p in range(ptr[j], ptr[j + 1]):
            if s["isTransposed"]:
                out[j, idx[p]] = val[p]
            else:
                out[idx[p], j] = val[p]
    return out


def _json_value(v: Any) -> Any:
    if isinstance(v, (np.integer,)):
        return int(v)
    if isinstance(v, (np.floating,)):
        return float(v)
    return v


def _write_text_dir(path: str, line: str) -> None:
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "part-00000"), "w") as f:
        f.write(line + "\n")
    open(os.path.join(path, "_SUCCESS"), "w").close()


def prepare_dir(path: str, overwrite: bool) -> None:
    if os.path.exists(path):
        if not overwrite:
            raise IOError(f"Path {path} already exists. To overwrite it, please use "
                          f"write.overwrite().save(path).")
        import shutil

        shutil.rmtree(path)
    os.makedirs(path)


def write_metadata(path: str, class_name: str, uid: str, param_map: dict, default_map: dict,
                   extra: dict | None = None) -> dict:
    meta = {"class": class_name, "timestamp": int(time.time() * 1000),
            "sparkVersion": spark_version(), "uid": uid,
            "paramMap": {k: _json_value(v) for k, v in param_map.items()},
            "defaultParamMap": {k: _json_value(v) for k, v in default_map.items()}}
    if extra:
        meta.update({k: _json_value(v) for k, v in extra.items()})
    _write_text_dir(os.path.join(path, "metadata"), json.dumps(meta, separators=(",", ":")))
    return meta


def read_metadata(path: str, expected_class: str | None = None) -> dict:
    mdir = os.path.join(path, "metadata")
    files = sorted(f for f in os.listdir(mdir) if f.startswith("part-"))
    if not files:
        raise IOError(f"no metadata part file under {mdir}")
    with open(os.path.join(mdir, files[0])) as f:
        meta = json.loads(f.readline())
    if expected_class is not None and meta.get("class") != expected_class:
        raise ValueError(f"Error loading metadata: Expected class name {expected_class} but "
                         f"found class name {meta.get('class')}")
    return meta


def write_parquet(dir_path: str, table: pa.Table, spark_schema: dict) -> str:
    os.makedirs(dir_path, exist_ok=True)
    md = dict(table.schema.metadata or {})
    md[ROW_METADATA_KEY] = json.dumps(spark_schema, separators=(",", ":")).encode()
    md[b"org.apache.spark.version"] = spark_version().encode()
    table = table.replace_schema_metadata(md)
    fname = f"part-00000-{uuid.uuid4()}-c000.snappy.parquet"
    pq.write_table(table, os.path.join(dir_path, fname), compression="snappy")
    open(os.path.join(dir_path, "_SUCCESS"), "w").close()
    return fname


def read_parquet_dir(dir_path: str) -> pa.Table:
    files = sorted(f for f in os.listdir(dir_path) if f.endswith(".parquet"))
    if not files:
        raise IOError(f"no parquet files under {dir_path}")
    return pa.concat_tables([pq.read_table(os.path.join(dir_path, f)) for f in files])


def spark_schema(fields: list[tuple[str, Any, bool]]) -> dict:
    return {"type": "struct", "fields": [
        {"name": n, "type": t, "nullable": nullable, "metadata": {}} for n, t, nullable in fields]}
