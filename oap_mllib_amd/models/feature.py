"""PCA estimator / model with the ``org.apache.spark.ml.feature`` contract.

Mirrors the reference's shadow ``PCA`` (mllib-dal/src/main/scala/org/apache/spark-3.1.1/ml/
feature/PCA.scala:38-256): Param ``k`` (> 0) plus inputCol/outputCol; ``fit`` requires
k <= numFeatures (:96-97) and takes the accelerated path iff numFeatures < 65535 (:103;
configurable as ``Config.pca_max_features``), otherwise the vanilla fp64 path; the model holds
``pc`` (d x k DenseMatrix, column-major) and ``explainedVariance`` (k), ``transform`` is
pc^T v (:168-175), and persistence writes one parquet row (pc: Matrix, explainedVariance:
Vector) next to DefaultParamsWriter metadata (:205-249).

The native path (csrc/drivers/pca.cpp) replaces PCADALImpl.scala/PCADALImpl.cpp: one fused
shifted-SYRK pass over the HBM-resident rows (kernels/pca.hip), one allreduce of
[S | column sums], fp64 covariance and the hand-written symmetric eigensolver.
"""
from __future__ import annotations

import time
from typing import Any

import numpy as np

from .. import _loader
from ..data import as_frame, to_matrix, vector_column
from ..fallback import pca_vanilla as vanilla
from ..linalg import DenseMatrix, DenseVector
from ..params import Param, gt, to_int, to_str
from ..parallel.world import get_world
from ..persistence import spark_format as sf
from ..utils.logging import Instrumentation
from .base import (DefaultParamsPersistence, Estimator, MLReadable, MLWritable, Model,
                   choose_engine)


class _PCAParams:
    inputCol = Param("inputCol", "input column name", converter=to_str)
    outputCol = Param("outputCol", "output column name", converter=to_str)
    k = Param("k", "the number of principal components (> 0)", validator=gt(0), converter=to_int)


class PCA(_PCAParams, Estimator, DefaultParamsPersistence):
    """Principal component analysis (top-k eigenvectors of the sample covariance)."""

    _uid_prefix = "pca"
    _spark_class = "org.apache.spark.ml.feature.PCA"

    def __init__(self, **kwargs):
        super().__init__(kwargs.pop("uid", None))
        self._setDefault(outputCol=self.uid + "__output")
        if kwargs:
            self._set(**kwargs)

    def setParams(self, **kwargs) -> "PCA":  # noqa: N802
        return self._set(**kwargs)

    def _fit(self, dataset: Any) -> "PCAModel":
        instr = Instrumentation(self)
        instr.logParams(self.extractParamMap())
        w = get_world()
        X = to_matrix(dataset, self.getOrDefault("inputCol"))
        if X.ndim != 2 or X.shape[0] == 0:
            raise ValueError("PCA needs a non-empty dataset")
        d = X.shape[1]
        if not self.isDefined("k"):
            raise ValueError("Param k must be set")
        k = self.getOrDefault("k")
        if k > d:
            raise ValueError(f"source vector size {d} must be no less than k={k}")
        native_ok = d < w.config.pca_max_features
        engine = choose_engine(native_ok, w)
        t0 = time.time()
        extra: dict = {"engine": engine}
        if engine == "vanilla":
            allreduce = (lambda a: w.allreduce_np(a)) if w.distributed else None
            pc, ev = vanilla.fit(X, k, allreduce)
        else:
            from .clustering import upload_table

            N = _loader.load()
            exact = w.config.pca_precision != "fast"
            # f32 rows whatever storage_dtype says; exact mode keeps f64 input rows f64 while
            # they fit the HBM budget (upload_table), else uploads them as f32
            table = upload_table(w, X, layout="pca_exact" if exact else "pca")
            r = N.pca_fit(w.ctx, w.comm, table, k, False, exact=exact)
            precision = "exact" if exact else "fast"
            if exact and X.dtype == np.float64 and table.dtype != "f64":
                # f64 input beyond the HBM budget went up as f32 rows: the statistics are exact
                # fp64 products of ROUNDED rows (~1e-7 relative input error) — say so
                precision = "exact_f32_rows"
                import warnings

                warnings.warn("PCA exact mode: the float64 rows exceed the HBM budget and were "
                              "rounded to float32 on upload (fit_info['precision'] = "
                              "'exact_f32_rows')", RuntimeWarning, stacklevel=2)
            extra["precision"] = precision
            extra["device_rows_dtype"] = table.dtype
            pc, ev = np.asarray(r["pc"]), np.asarray(r["explained_variance"])
            extra.update({k_: r[k_] for k_ in ("stats_ms", "allreduce_ms", "eig_ms", "total_ms",
                                               "err_bound")})
            extra["stats_engine"] = r["engine"]  # int8_digits | fp64_mfma | bf16_split
        model = PCAModel(uid=self.uid, pc=DenseMatrix.from_array(pc),
                         explainedVariance=DenseVector(ev))
        self._copyValues(model)
        model.setParent(self)
        model.fit_info = {"fit_seconds": time.time() - t0, **extra}
        instr.logNamedValue("engine", engine)
        instr.finish()
        return model


class PCAModel(_PCAParams, Model, MLWritable, MLReadable):
    _uid_prefix = "pca"
    _spark_class = "org.apache.spark.ml.feature.PCAModel"

    def __init__(self, uid: str | None = None, pc: DenseMatrix | None = None,
                 explainedVariance: DenseVector | None = None):  # noqa: N803
        super().__init__(uid)
        self._setDefault(outputCol=self.uid + "__output")
        self.pc = pc if pc is not None else DenseMatrix(0, 0, [])
        self.explainedVariance = (explainedVariance if explainedVariance is not None
                                  else DenseVector([]))
        self.fit_info: dict = {}

    def project(self, X: np.ndarray) -> np.ndarray:
        """Rows of X projected onto the components: X pc (n x k)."""
        return np.asarray(X, dtype=np.float64) @ self.pc.toArray()

    def _transform(self, dataset):
        import pandas as pd

        df = as_frame(dataset, self.getOrDefault("inputCol"))
        X = to_matrix(dataset, self.getOrDefault("inputCol"))
        Y = self.project(X) if len(X) else np.zeros((0, self.pc.numCols))
        if isinstance(df[self.getOrDefault("inputCol")].dtype, pd.ArrowDtype):
            # matrix / Arrow input: the projections stay one Arrow buffer (no per-row objects)
            df[self.getOrDefault("outputCol")] = vector_column(Y)
        else:
            df[self.getOrDefault("outputCol")] = [DenseVector(r) for r in Y]
        return df

    def copy(self, extra: dict | None = None) -> "PCAModel":
        m = super().copy(extra)
        m.pc = DenseMatrix.from_array(self.pc.toArray())
        m.explainedVariance = DenseVector(self.explainedVariance.toArray())
        return m

    def _save_impl(self, path: str, fmt: str) -> None:
        import os

        import pyarrow as pa

        sf.write_metadata(path, self._spark_class, self.uid, self._paramMap,
                          self.defaultParamMap())
        row = {"pc": sf.dense_matrix_struct(self.pc.toArray()),
               "explainedVariance": sf.dense_vector_struct(self.explainedVariance.toArray())}
        table = pa.Table.from_pylist([row], schema=pa.schema([
            pa.field("pc", sf.MATRIX_ARROW), pa.field("explainedVariance", sf.VECTOR_ARROW)]))
        sf.write_parquet(os.path.join(path, "data"), table, sf.spark_schema(
            [("pc", sf.MATRIX_UDT, True), ("explainedVariance", sf.VECTOR_UDT, True)]))

    @classmethod
    def _load_impl(cls, path: str) -> "PCAModel":
        import os

        meta = sf.read_metadata(path, cls._spark_class)
        rows = sf.read_parquet_dir(os.path.join(path, "data")).to_pylist()
        pc = sf.matrix_from_struct(rows[0]["pc"])
        if sf.major_version(meta.get("sparkVersion", "3.1.1")) >= 2:
            ev = sf.vector_from_struct(rows[0]["explainedVariance"])
        else:  # Spark <= 1.6 stored no explained variance (PCA.scala:234-245)
            ev = np.zeros(0)
        m = cls(uid=meta["uid"], pc=DenseMatrix.from_array(pc), explainedVariance=DenseVector(ev))
        for k, v in meta.get("paramMap", {}).items():
            if m.hasParam(k):
                m._set(**{k: v})
        return m
