"""``mllib.clustering.KMeans`` / ``KMeansModel`` — the RDD-based API.

The reference ships a shadow copy of Spark's ``mllib.clustering.KMeans``
(mllib-dal/src/main/scala/org/apache/spark-3.1.1/mllib/clustering/KMeans.scala:41-530) whose
only change is widening ``initRandom`` / ``initKMeansParallel`` so the ml-level estimator can
call them.  Here the same entry points run on the native engine: ``KMeans.train`` mirrors
``pyspark.mllib.clustering.KMeans.train`` (maxIterations, initializationMode,
initializationSteps, epsilon, initialModel, distanceMeasure), and ``KMeansModel`` offers
``predict`` / ``computeCost`` / ``save`` / ``load`` in the mllib on-disk layout (metadata JSON
with class/version/k/distanceMeasure/trainingCost + parquet rows ``(id: int, point: Vector)``).
"""
from __future__ import annotations

import json
import os
import time

import numpy as np

from .. import _loader
from ..data import to_matrix
from ..fallback import kmeans_vanilla as vanilla
from ..models.base import choose_engine
from ..parallel.world import get_world
from ..persistence import spark_format as sf

_CLASS = "org.apache.spark.mllib.clustering.KMeansModel"


class KMeansModel:
    def __init__(self, centers, distanceMeasure: str = vanilla.EUCLIDEAN,  # noqa: N803
                 trainingCost: float = 0.0, numIter: int = 0):  # noqa: N803
        self.centers = np.asarray(centers, dtype=np.float64)
        self.distanceMeasure = distanceMeasure
        self.trainingCost = float(trainingCost)
        self.numIter = int(numIter)

    @property
    def clusterCenters(self) -> list[np.ndarray]:  # noqa: N802
        return [c.copy() for c in self.centers]

    @property
    def k(self) -> int:
        return int(self.centers.shape[0])

    def _assign(self, X: np.ndarray):
        w = get_world()
        engine = choose_engine(self.distanceMeasure == vanilla.EUCLIDEAN, w)
        if engine == "vanilla" or len(X) == 0:
            return vanilla.find_closest(X, self.centers, self.distanceMeasure)
        from ..models.clustering import upload_table

        N = _loader.load()
        return N.kmeans_predict(w.ctx, upload_table(w, X), self.centers)

    def predict(self, x):
        """Cluster index of one vector, or an array of indices for a batch of rows."""
        arr = x.toArray() if hasattr(x, "toArray") else x
        a = np.asarray(arr, dtype=np.float64) if not isinstance(arr, list) or not arr or \
            np.isscalar(arr[0]) else to_matrix(arr)
        if a.ndim == 1:
            return int(self._assign(a.reshape(1, -1))[0][0])
        return np.asarray(self._assign(a)[0], dtype=np.int64)

    def computeCost(self, data) -> float:  # noqa: N802
        """Sum of squared distances of the rows to their nearest center."""
        X = to_matrix(data)
        _, cost = self._assign(X)
        total = float(np.sum(cost))
        w = get_world()
        if w.distributed:
            total = float(w.allreduce_np(np.array([total]))[0])
        return total

    def save(self, sc, path: str) -> None:  # sc kept for API parity (unused)
        import pyarrow as pa

        os.makedirs(path, exist_ok=True)
        meta = {"class": _CLASS, "version": "2.0", "k": self.k,
                "distanceMeasure": self.distanceMeasure, "trainingCost": self.trainingCost}
        sf._write_text_dir(os.path.join(path, "metadata"), json.dumps(meta, separators=(",", ":")))
        rows = [{"id": i, "point": sf.dense_vector_struct(c)} for i, c in enumerate(self.centers)]
        t = pa.Table.from_pylist(rows, schema=pa.schema([pa.field("id", pa.int32(),
                                                                   nullable=False),
                                                          pa.field("point", sf.VECTOR_ARROW)]))
        sf.write_parquet(os.path.join(path, "data"), t, sf.spark_schema(
            [("id", "integer", False), ("point", sf.VECTOR_UDT, True)]))

    @classmethod
    def load(cls, sc, path: str) -> "KMeansModel":
        meta = sf.read_metadata(path, _CLASS)
        rows = sorted(sf.read_parquet_dir(os.path.join(path, "data")).to_pylist(),
                      key=lambda r: r["id"])
        centers = np.array([sf.vector_from_struct(r["point"]) for r in rows])
        if len(centers) != int(meta["k"]):
            raise ValueError("KMeansModel requires k centers, found %d" % len(centers))
        return cls(centers, meta.get("distanceMeasure", vanilla.EUCLIDEAN),
                   meta.get("trainingCost", 0.0))


class KMeans:
    K_MEANS_PARALLEL = "k-means||"
    RANDOM = "random"

    @classmethod
    def train(cls, rdd, k: int, maxIterations: int = 100,  # noqa: N803
              initializationMode: str = "k-means||", seed: int | None = None,  # noqa: N803
              initializationSteps: int = 2, epsilon: float = 1e-4,  # noqa: N803
              initialModel: KMeansModel | None = None,  # noqa: N803
              distanceMeasure: str = "euclidean") -> KMeansModel:  # noqa: N803
        if k < 1:
            raise ValueError(f"Number of clusters must be positive but got {k}")
        if maxIterations < 0:
            raise ValueError("Maximum of iterations must be nonnegative")
        if initializationMode not in (cls.K_MEANS_PARALLEL, cls.RANDOM):
            raise ValueError(f"Invalid initialization mode: {initializationMode}")
        X = to_matrix(rdd)
        seed = int(seed if seed is not None else np.random.SeedSequence().entropy % (2 ** 63))
        seed &= 0xFFFFFFFFFFFFFFFF
        init = None
        if initialModel is not None:
            init = np.asarray(initialModel.centers, dtype=np.float64)
            if init.shape[0] != k:
                raise ValueError("mismatched cluster count")
        w = get_world()
        engine = choose_engine(distanceMeasure == vanilla.EUCLIDEAN, w)
        t0 = time.time()
        if engine == "vanilla":
            allreduce = (lambda a: w.allreduce_np(a)) if w.distributed else None
            r = vanilla.fit(X, k, maxIterations, epsilon, initializationMode, initializationSteps,
                            seed, distanceMeasure, None, init, allreduce)
            centers, cost, n_iter = r.centers, r.cost, r.num_iter
        else:
            from ..models.clustering import upload_table

            N = _loader.load()
            r = N.kmeans_fit(w.ctx, w.comm, upload_table(w, X), init, k, maxIterations, epsilon,
                             initializationMode, initializationSteps, seed)
            centers, cost, n_iter = r["centers"], r["cost"], r["num_iter"]
        m = KMeansModel(centers, distanceMeasure, cost, n_iter)
        m.fit_seconds = time.time() - t0
        return m
