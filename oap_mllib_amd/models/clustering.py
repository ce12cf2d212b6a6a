"""K-Means estimator / model / summary with the ``org.apache.spark.ml.clustering`` contract.

Mirrors the reference's shadow ``KMeans`` (mllib-dal/src/main/scala/org/apache/spark-3.1.1/ml/
clustering/KMeans.scala): same Params and defaults (k=2, maxIter=20, initMode="k-means||",
initSteps=2, tol=1e-4, distanceMeasure="euclidean", seed = hash of the class name; :90-91), same
dispatch rule — native engine iff platform OK AND euclidean AND no weightCol (:349-351), else the
vanilla path — and the same post-fit summary built from ``model.transform(dataset)``
(:359-368).  The native path runs the whole fit (init + Lloyd) in C++/HIP
(csrc/drivers/kmeans.cpp); the model persists in Spark's "internal" parquet format or PMML
(:168,188-222).
"""
from __future__ import annotations

import time
from typing import Any

import numpy as np

from .. import _loader
from ..data import as_frame, column, to_matrix
from ..fallback import kmeans_vanilla as vanilla
from ..linalg import DenseVector
from ..params import (Param, gt, in_array, to_float, to_int, to_str)
from ..parallel.world import get_world
from ..persistence import spark_format as sf
from ..utils import checkpoint
from ..utils.logging import Instrumentation
from .base import (Estimator, HasTrainingSummary, MLReadable, MLWritable, Model,
                   DefaultParamsPersistence, choose_engine, java_string_hash)

K_MEANS_PARALLEL = "k-means||"
RANDOM = "random"


class _KMeansParams:
    featuresCol = Param("featuresCol", "features column name", "features", converter=to_str)
    predictionCol = Param("predictionCol", "prediction column name", "prediction",
                          converter=to_str)
    k = Param("k", "The number of clusters to create. Must be > 1.", 2, gt(1), to_int)
    maxIter = Param("maxIter", "maximum number of iterations (>= 0)", 20,
                    lambda v: v >= 0, to_int)
    tol = Param("tol", "the convergence tolerance for iterative algorithms (>= 0)", 1e-4,
                lambda v: v >= 0, to_float)
    initMode = Param("initMode", "The initialization algorithm. Supported options: 'random' and "
                     "'k-means||'.", K_MEANS_PARALLEL, in_array([RANDOM, K_MEANS_PARALLEL]),
                     to_str)
    initSteps = Param("initSteps", "The number of steps for k-means|| initialization mode. "
                      "Must be > 0.", 2, gt(0), to_int)
    distanceMeasure = Param("distanceMeasure", "the distance measure. Supported options: "
                            "'euclidean' and 'cosine'", vanilla.EUCLIDEAN,
                            in_array([vanilla.EUCLIDEAN, vanilla.COSINE]), to_str)
    seed = Param("seed", "random seed",
                 java_string_hash("org.apache.spark.ml.clustering.KMeans"), converter=to_int)
    weightCol = Param("weightCol", "weight column name. If this is not set or empty, we treat "
                      "all instance weights as 1.0", converter=to_str)


class KMeansSummary:
    """Training summary (``ml.clustering.KMeansSummary``).

    Spark builds it from ``model.transform(dataset)`` (KMeans.scala:359-368).  Here the fit hands
    over the labels of the final model straight from the device pass over the still-resident
    rows, and the counts it made (``clusterSizes``, global over the ranks); the ``predictions``
    frame is only assembled when it is read, so a fit on 100M rows creates no per-row objects.

    ``trainingCost`` accuracy class (GPU engine): the cost of the last assignment, either summed
    from the rows' exact-assignment fp32 distances in fp64 or — when the last pass computed none
    (row-scan fits) — from the fit's own statistics, ``sum|x|^2 - 2 sum c.S + sum n |c|^2``, taken
    only when its rigorous error bound (fp32 row norms, fixed-point sums, fp64 rounding) is within
    1e-5 of the result (drivers/kmeans.cpp kStatsCostRel); otherwise one exact pass over the rows
    runs.  Both are within 1e-5 relative of the fp64 cost Spark reports (typically ~1e-8).
    """

    def __init__(self, predictions, predictionCol: str, featuresCol: str, k: int,  # noqa: N803
                 numIter: int, trainingCost: float, labels: np.ndarray | None = None,  # noqa: N803
                 clusterSizes: list[int] | None = None):  # noqa: N803
        self._predictions = predictions  # a frame, or a zero-argument builder of one
        self.predictionCol = predictionCol
        self.featuresCol = featuresCol
        self.k = k
        self.numIter = numIter
        self.trainingCost = trainingCost
        self._labels = labels
        self._sizes = clusterSizes

    @property
    def predictions(self):
        if callable(self._predictions):
            self._predictions = self._predictions()
        return self._predictions

    @property
    def cluster(self):
        if self._labels is not None:
            import pandas as pd

            return pd.DataFrame({self.predictionCol: self._labels})
        return self.predictions[[self.predictionCol]]

    @property
    def clusterSizes(self) -> list[int]:  # noqa: N802
        if self._sizes is not None:
            return list(self._sizes)
        lab = (self._labels if self._labels is not None else
               np.asarray(self.predictions[self.predictionCol].to_numpy(), dtype=np.int64))
        return np.bincount(lab, minlength=self.k)[: max(self.k, 0)].tolist()


def _with_predictions(dataset, features_col: str, prediction_col: str, labels: np.ndarray):
    df = as_frame(dataset, features_col)
    df[prediction_col] = np.asarray(labels, dtype=np.int32)
    return df


class KMeans(_KMeansParams, Estimator, DefaultParamsPersistence):
    """K-means clustering with k-means|| initialisation (Bahmani et al., VLDB 2012)."""

    _uid_prefix = "KMeans"
    _spark_class = "org.apache.spark.ml.clustering.KMeans"

    def __init__(self, **kwargs):
        super().__init__(kwargs.pop("uid", None))
        if kwargs:
            self._set(**kwargs)

    def setParams(self, **kwargs) -> "KMeans":  # noqa: N802
        return self._set(**kwargs)

    def _use_native(self) -> bool:
        has_w = self.isSet("weightCol") and self.getOrDefault("weightCol") != ""
        return self.getOrDefault("distanceMeasure") == vanilla.EUCLIDEAN and not has_w

    def _fit(self, dataset: Any) -> "KMeansModel":
        instr = Instrumentation(self)
        instr.logParams(self.extractParamMap())
        w = get_world()
        engine = choose_engine(self._use_native(), w)
        X = to_matrix(dataset, self.getOrDefault("featuresCol"))
        instr.logNumFeatures(X.shape[1] if X.ndim == 2 else 0)
        k, max_iter, tol = self.getOrDefault("k"), self.getOrDefault("maxIter"), \
            self.getOrDefault("tol")
        seed = self.getOrDefault("seed") & 0xFFFFFFFFFFFFFFFF
        t0 = time.time()
        streamed = streamed_decision(w, X, engine)
        if engine == "vanilla":
            weights = None
            if self.isSet("weightCol") and self.getOrDefault("weightCol"):
                weights = np.asarray(column(dataset, self.getOrDefault("weightCol")),
                                     dtype=np.float64)
                if (weights < 0).any():
                    raise ValueError("Weights MUST NOT be negative")
            allreduce = (lambda a: w.allreduce_np(a)) if w.distributed else None
            r = vanilla.fit(X, k, max_iter, tol, self.getOrDefault("initMode"),
                            self.getOrDefault("initSteps"), seed,
                            self.getOrDefault("distanceMeasure"), weights, None, allreduce)
            centers, cost, n_iter = r.centers, r.cost, r.num_iter
            extra = {"engine": "vanilla"}
        elif streamed:
            r, centers, cost, n_iter = self._fit_streamed(w, X, k, max_iter, tol, seed)
            extra = {"engine": engine, "streamed": True, "init_seconds": r["init_seconds"],
                     "iter_seconds": r["iter_seconds"], "global_rows": r["global_rows"]}
        else:
            N = _loader.load()
            t_up = time.time()
            table = upload_table(w, X)
            upload_s = time.time() - t_up
            ck = checkpoint.for_fit(w, self, X.shape)
            if ck is None:
                r = N.kmeans_fit(w.ctx, w.comm, table, None, k, max_iter, tol,
                                 self.getOrDefault("initMode"), self.getOrDefault("initSteps"),
                                 seed)
                centers, cost, n_iter = r["centers"], r["cost"], r["num_iter"]
            else:
                r, centers, cost, n_iter = self._fit_segmented(N, w, table, ck, k, max_iter, tol,
                                                                seed)
            # the summary pass (model.transform in KMeans.scala:359-368) over the SAME resident
            # table: labels under the final centers + per-cluster counts, one device pass
            t_lab = time.time()
            labels, sizes = N.kmeans_labels(w.ctx, table, np.asarray(centers))
            del table
            extra = {"engine": engine, "init_seconds": r["init_seconds"],
                     "iter_seconds": r["iter_seconds"], "global_rows": r["global_rows"],
                     "upload_seconds": upload_s, "summary_seconds": time.time() - t_lab}
        model = KMeansModel(uid=self.uid, centers=np.asarray(centers), trainingCost=float(cost),
                            numIter=int(n_iter), distanceMeasure=self.getOrDefault(
                                "distanceMeasure"))
        self._copyValues(model)
        model.setParent(self)
        if "summary_seconds" not in extra:  # vanilla / streamed: predict in row chunks
            labels, _ = model.predict_matrix(X)
            labels = np.asarray(labels, dtype=np.int32)
            sizes = np.bincount(labels, minlength=k)[:k]
        if w.distributed:  # the summary covers the whole (distributed) dataset
            sizes = w.allreduce_np(np.asarray(sizes, dtype=np.int64))
        model.fit_info = {"fit_seconds": time.time() - t0, **extra}
        fcol, pcol = model.getOrDefault("featuresCol"), model.getOrDefault("predictionCol")
        summary = KMeansSummary(lambda: _with_predictions(dataset, fcol, pcol, labels), pcol, fcol,
                                k, model.numIter, model.trainingCost, labels=labels,
                                clusterSizes=[int(v) for v in np.asarray(sizes)[:k]])
        model.setSummary(summary)
        instr.logNamedValue("clusterSizes", summary.clusterSizes)
        instr.logNamedValue("engine", extra["engine"])
        instr.finish()
        return model


    def _fit_streamed(self, w, X, k, max_iter, tol, seed):
        """Rows beyond the HBM budget: k-means|| (or random) init on a uniform sample uploaded to
        HBM, then Lloyd with the rows streamed from host memory each iteration
        (drivers/kmeans.cpp kmeans_fit_streamed)."""
        N = _loader.load()
        t0 = time.time()
        rng = np.random.default_rng(seed)
        m = min(len(X), max(64 * k, 1 << 20))
        sample = X[np.sort(rng.choice(len(X), m, replace=False))] if m < len(X) else X
        st = upload_table(w, np.ascontiguousarray(sample))
        init = N.kmeans_init(w.ctx, w.comm, st, k, self.getOrDefault("initMode"),
                             self.getOrDefault("initSteps"), seed)
        del st
        init_s = time.time() - t0
        r = N.kmeans_fit_streamed(w.ctx, w.comm, np.ascontiguousarray(X, dtype=np.float32),
                                  np.asarray(init), max_iter, tol,
                                  int(w.config.stream_chunk_rows))
        r = dict(r)
        r["init_seconds"] = init_s
        return r, r["centers"], r["cost"], r["num_iter"]

    def _fit_segmented(self, N, w, table, ck, k, max_iter, tol, seed):
        """Lloyd in checkpoint_interval-sized segments, resuming from a saved state."""
        interval = max(1, int(w.config.checkpoint_interval))
        state = ck.load()
        centers, done, cost = None, 0, 0.0
        if state is not None:
            meta, arrays = state
            centers, done, cost = arrays["centers"], int(meta["num_iter"]), float(meta["cost"])
            if meta.get("converged"):
                return {"init_seconds": 0.0, "iter_seconds": 0.0,
                        "global_rows": meta["global_rows"]}, centers, cost, done
        r = {"init_seconds": 0.0, "iter_seconds": 0.0, "global_rows": 0}
        while True:
            seg = min(interval, max_iter - done)
            if seg <= 0 and centers is not None:
                break
            r = N.kmeans_fit(w.ctx, w.comm, table, centers, k, max(seg, 0), tol,
                             self.getOrDefault("initMode"), self.getOrDefault("initSteps"), seed)
            centers, cost = np.asarray(r["centers"]), float(r["cost"])
            done += int(r["num_iter"])
            conv = bool(r["converged"]) or done >= max_iter
            ck.save({"num_iter": done, "cost": cost, "converged": bool(r["converged"]),
                     "global_rows": r["global_rows"]}, {"centers": centers})
            if conv or seg == 0:
                break
            k = centers.shape[0]
        return r, centers, cost, done


def streamed_decision(w, X: np.ndarray, engine: str) -> bool:
    """Whether this fit streams its rows from host memory — the same answer on every rank: the
    streamed and resident fits issue different collective sequences, so one rank over its HBM
    budget (uneven Spark partitions) makes every rank stream."""
    if engine != "gpu":
        return False
    streamed = _streamed(w, X)
    if w.distributed:
        streamed = bool(w.allreduce_np(np.array([float(streamed)]), "max")[0] > 0)
    return streamed


def hbm_budget(w) -> int:
    """Bytes of rows a rank may keep resident (Config.hbm_budget_bytes; automatic: 60% of the
    device memory)."""
    budget = int(w.config.hbm_budget_bytes)
    return budget if budget > 0 else int(0.6 * w.ctx.info["total_mem"])


def _streamed(w, X: np.ndarray) -> bool:
    """K-Means rows of this rank exceed the HBM budget (Config.hbm_budget_bytes, automatic:
    60% of the device memory): stream them from host memory instead of uploading."""
    if X.ndim != 2 or w.config.storage_dtype != "f32":
        return False
    ld = (X.shape[1] + 3) // 4 * 4
    return X.shape[0] * ld * 4 > hbm_budget(w)


def upload_table(w, X: np.ndarray, layout: str = "kmeans"):
    """Rank-local matrix -> native DenseTable on the world's backend.  layout "pca": f32 rows
    ("pca_exact": f64 input rows stay f64, the exact-mode kernel reads them as they are)."""
    N = _loader.load()
    d = X.shape[1]
    if w.is_gpu:
        st = w.config.storage_dtype
        if layout == "kmeans":
            ld = N.kmeans_ld(d, st)
        elif layout == "pca_exact" and X.dtype == np.float64 and X.nbytes <= hbm_budget(w):
            # (f64 rows take twice the HBM of f32 ones; beyond the budget the rows go up as
            # f32 and the exact kernel still forms fp64 products of them)
            st, ld = "f64", d
        else:
            st, ld = "f32", d  # PCA reads f32 rows
        src = X if X.dtype in (np.float32, np.float64) else X.astype(np.float64)
        return N.upload_dense(w.ctx, np.ascontiguousarray(src), st, ld)
    return N.upload_dense(w.ctx, np.ascontiguousarray(X, dtype=np.float64), "f64", d)


class KMeansModel(_KMeansParams, Model, HasTrainingSummary, MLWritable, MLReadable):
    _uid_prefix = "KMeans"
    _spark_class = "org.apache.spark.ml.clustering.KMeansModel"

    def __init__(self, uid: str | None = None, centers: np.ndarray | None = None,
                 trainingCost: float = 0.0, numIter: int = 0,  # noqa: N803
                 distanceMeasure: str = vanilla.EUCLIDEAN):  # noqa: N803
        super().__init__(uid)
        self._centers = np.zeros((0, 0)) if centers is None else np.asarray(centers, np.float64)
        self.trainingCost = trainingCost
        self.numIter = numIter
        if distanceMeasure != vanilla.EUCLIDEAN:
            self._set(distanceMeasure=distanceMeasure)
        self.fit_info: dict = {}

    # ---- attributes --------------------------------------------------------------------
    def clusterCenters(self) -> list[np.ndarray]:  # noqa: N802
        return [c.copy() for c in self._centers]

    @property
    def numFeatures(self) -> int:  # noqa: N802
        return int(self._centers.shape[1]) if self._centers.size else 0

    @property
    def k_(self) -> int:
        return int(self._centers.shape[0])

    # ---- inference ---------------------------------------------------------------------
    def predict(self, value) -> int:
        v = value.toArray() if hasattr(value, "toArray") else np.asarray(value, np.float64)
        lab, _ = vanilla.find_closest(v.reshape(1, -1), self._centers,
                                      self.getOrDefault("distanceMeasure"))
        return int(lab[0])

    def predict_matrix(self, X: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
        """Labels and costs for a row matrix (native when possible)."""
        w = get_world()
        engine = choose_engine(self.getOrDefault("distanceMeasure") == vanilla.EUCLIDEAN, w)
        if engine == "vanilla" or len(X) == 0 or self._centers.shape[0] == 0:
            return vanilla.find_closest(X, self._centers, self.getOrDefault("distanceMeasure"))
        N = _loader.load()
        if engine == "gpu" and _streamed(w, X):  # beyond the HBM budget: predict in row chunks
            step = max(1, int(w.config.stream_chunk_rows))
            labs, costs = [], []
            for r0 in range(0, len(X), step):
                lb, cs = N.kmeans_predict(w.ctx, upload_table(w, X[r0:r0 + step]), self._centers)
                labs.append(np.asarray(lb))
                costs.append(np.asarray(cs))
            return np.concatenate(labs), np.concatenate(costs)
        table = upload_table(w, X)
        return N.kmeans_predict(w.ctx, table, self._centers)

    def _transform(self, dataset):
        df = as_frame(dataset, self.getOrDefault("featuresCol"))
        X = to_matrix(dataset, self.getOrDefault("featuresCol"))
        lab, _ = self.predict_matrix(X)
        df[self.getOrDefault("predictionCol")] = np.asarray(lab, dtype=np.int32)
        return df

    def copy(self, extra: dict | None = None) -> "KMeansModel":
        m = super().copy(extra)
        m._centers = self._centers.copy()
        return m

    # ---- persistence -------------------------------------------------------------------
    def _save_impl(self, path: str, fmt: str) -> None:
        import os

        import pyarrow as pa

        if fmt == "pmml":
            write_pmml(self, path)
            return
        if fmt not in ("internal", "org.apache.spark.ml.clustering.InternalKMeansModelWriter"):
            raise ValueError(f"unsupported format '{fmt}' (use 'internal' or 'pmml')")
        sf.write_metadata(path, self._spark_class, self.uid, self._paramMap,
                          self.defaultParamMap())
        rows = [{"clusterIdx": i, "clusterCenter": sf.dense_vector_struct(c)}
                for i, c in enumerate(self._centers)]
        table = pa.Table.from_pylist(rows, schema=pa.schema([
            pa.field("clusterIdx", pa.int32(), nullable=False),
            pa.field("clusterCenter", sf.VECTOR_ARROW)]))
        sf.write_parquet(os.path.join(path, "data"), table, sf.spark_schema(
            [("clusterIdx", "integer", False), ("clusterCenter", sf.VECTOR_UDT, True)]))

    @classmethod
    def _load_impl(cls, path: str) -> "KMeansModel":
        import os

        meta = sf.read_metadata(path, cls._spark_class)
        t = sf.read_parquet_dir(os.path.join(path, "data")).to_pylist()
        if sf.major_version(meta.get("sparkVersion", "3.1.1")) >= 2:
            t.sort(key=lambda r: r["clusterIdx"])
            centers = np.array([sf.vector_from_struct(r["clusterCenter"]) for r in t])
        else:  # Spark <= 1.6: one row holding every center (KMeans.scala:253-257)
            centers = np.array([sf.vector_from_struct(v) for v in t[0]["clusterCenters"]])
        m = cls(uid=meta["uid"], centers=centers)
        for k, v in meta.get("paramMap", {}).items():
            if m.hasParam(k):
                m._set(**{k: v})
        return m


def write_pmml(model: KMeansModel, path: str) -> None:
    """PMML 4.2 ClusteringModel, as Spark's KMeansPMMLModelExport writes it."""
    import os
    from xml.sax.saxutils import escape

    c = model._centers
    k, d = c.shape
    fields = [f"field_{i}" for i in range(d)]
    ts = time.strftime("%Y-%m-%dT%H:%M:%S")
    lines = ['<?xml version="1.0" encoding="UTF-8" standalone="yes"?>',
             '<PMML version="4.2" xmlns="http://www.dmg.org/PMML-4_2">',
             '    <Header description="k-means clustering">',
             f'        <Application name="Apache Spark MLlib" version="{sf.spark_version()}"/>',
             f'        <Timestamp>{escape(ts)}</Timestamp>', '    </Header>',
             f'    <DataDictionary numberOfFields="{d}">']
    lines += [f'        <DataField name="{f}" optype="continuous" dataType="double"/>'
              for f in fields]
    lines += ['    </DataDictionary>',
              f'    <ClusteringModel modelName="k-means" functionName="clustering" '
              f'modelClass="centerBased" numberOfClusters="{k}">', '        <MiningSchema>']
    lines += [f'            <MiningField name="{f}" usageType="active"/>' for f in fields]
    lines += ['        </MiningSchema>', '        <ComparisonMeasure kind="distance">',
              '            <squaredEuclidean/>', '        </ComparisonMeasure>']
    lines += [f'        <ClusteringField field="{f}" compareFunction="absDiff"/>' for f in fields]
    for i in range(k):
        vals = " ".join(repr(float(v)) for v in c[i])
        lines += [f'        <Cluster name="cluster_{i}">',
                  f'            <Array n="{d}" type="real">{vals}</Array>', '        </Cluster>']
    lines += ['    </ClusteringModel>', '</PMML>']
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "part-00000"), "w") as f:
        f.write("\n".join(lines) + "\n")
    open(os.path.join(path, "_SUCCESS"), "w").close()


def kmeans_center_vectors(model: KMeansModel) -> list[DenseVector]:
    return [DenseVector(c) for c in model._centers]
