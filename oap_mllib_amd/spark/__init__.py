"""Running the estimators inside a Spark job (one rank per GPU executor task).

The reference's JVM glue (KMeansDALImpl.scala / PCADALImpl.scala / ALSDALImpl.scala) coalesces
the cached input to one partition per executor (ExecutorInProcessCoalescePartitioner.scala:
25-58), resolves a KVS ip:port (Utils.scala:60-96), runs one native task per executor and
hopes all of them are scheduled together (no barrier mode).  Here:

* ``fit(estimator, df, num_ranks)`` repartitions ``df`` to ``num_ranks`` partitions and runs a
  Spark **barrier stage** (gang scheduling: all ranks start together or the stage is retried as
  a whole);
* every task derives RANK / WORLD_SIZE / LOCAL_RANK from the BarrierTaskContext, rank 0
  publishes a free port through ``allGather``, and ``init_world`` forms the gloo rendezvous
  plus the RCCL communicator (unique id broadcast) — no ports are guessed in advance;
* the local partition is converted to a numpy matrix (or rating columns) and the estimator's
  normal ``fit`` runs on it; rank 0 returns the fitted model as ``.npy`` payloads (loaded on
  the driver with ``allow_pickle=False``).

pyspark is optional: everything except ``fit`` is importable and testable without it.
"""
from __future__ import annotations

import io
import json
import socket
from typing import Any

import numpy as np


def spark_available() -> bool:
    try:
        import pyspark  # noqa: F401

        return True
    except ImportError:
        return False


def local_ranks(addresses: list[str]) -> list[int]:
    """Local rank of each task = its index among the tasks on the same host."""
    seen: dict[str, int] = {}
    out = []
    for a in addresses:
        host = a.rsplit(":", 1)[0] if ":" in a else a
        out.append(seen.get(host, 0))
        seen[host] = seen.get(host, 0) + 1
    return out


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("", 0))
        return int(s.getsockname()[1])


# ---- model payloads (numpy, pickle-free) ----------------------------------------------------
def export_model(model) -> dict[str, bytes]:
    """Arrays + JSON metadata describing a fitted model."""
    from ..models.clustering import KMeansModel
    from ..models.feature import PCAModel
    from ..models.recommendation import ALSModel

    arrays: dict[str, np.ndarray] = {}
    meta: dict[str, Any] = {"uid": model.uid, "params": model._paramMap}
    if isinstance(model, KMeansModel):
        meta["kind"] = "kmeans"
        meta.update(trainingCost=model.trainingCost, numIter=model.numIter)
        arrays["centers"] = model._centers
    elif isinstance(model, PCAModel):
        meta["kind"] = "pca"
        arrays["pc"] = model.pc.toArray()
        arrays["explainedVariance"] = model.explainedVariance.toArray()
    elif isinstance(model, ALSModel):
        meta["kind"] = "als"
        meta["rank"] = model.rank
        for name, which in (("user", "user"), ("item", "item")):
            ids, F = model._mat(which)
            arrays[name + "_ids"] = ids.astype(np.int32)
            arrays[name + "_factors"] = F
    else:
        raise TypeError(f"cannot export {type(model).__name__}")
    out = {"__meta__": json.dumps(meta).encode()}
    for k, v in arrays.items():
        buf = io.BytesIO()
        np.save(buf, np.asarray(v), allow_pickle=False)
        out[k] = buf.getvalue()
    return out


def import_model(payload: dict[str, bytes]):
    from ..linalg import DenseMatrix, DenseVector
    from ..models.clustering import KMeansModel
    from ..models.feature import PCAModel
    from ..models.recommendation import ALSModel, _factor_frame

    meta = json.loads(payload["__meta__"].decode())
    arr = {k: np.load(io.BytesIO(v), allow_pickle=False) for k, v in payload.items()
           if k != "__meta__"}
    kind = meta["kind"]
    if kind == "kmeans":
        m = KMeansModel(uid=meta["uid"], centers=arr["centers"],
                        trainingCost=meta["trainingCost"], numIter=meta["numIter"])
    elif kind == "pca":
        m = PCAModel(uid=meta["uid"], pc=DenseMatrix.from_array(arr["pc"]),
                     explainedVariance=DenseVector(arr["explainedVariance"]))
    else:
        m = ALSModel(uid=meta["uid"], rank=meta["rank"],
                     userFactors=_factor_frame(arr["user_ids"], arr["user_factors"]),
                     itemFactors=_factor_frame(arr["item_ids"], arr["item_factors"]))
    for k, v in meta["params"].items():
        if m.hasParam(k):
            m._set(**{k: v})
    return m


def _partition_to_input(estimator, rows: list):
    """Spark Rows of this partition -> what estimator.fit accepts."""
    from ..models.recommendation import ALS

    if isinstance(estimator, ALS):
        u, i, r = (estimator.getOrDefault(c) for c in ("userCol", "itemCol", "ratingCol"))
        return {"user": [row[u] for row in rows], "item": [row[i] for row in rows],
                "rating": [row[r] for row in rows] if r else [1.0] * len(rows)}
    col = (estimator.getOrDefault("inputCol") if estimator.hasParam("inputCol")
           else estimator.getOrDefault("featuresCol"))
    vecs = [row[col] for row in rows]
    return np.array([v.toArray() for v in vecs], dtype=np.float64) if vecs else np.zeros((0, 0))


def fit(estimator, df, num_ranks: int, spark_conf: dict | None = None):
    """Fits `estimator` on Spark DataFrame `df` with `num_ranks` gang-scheduled ranks."""
    if not spark_available():
        raise RuntimeError("pyspark is not installed")
    from pyspark import BarrierTaskContext

    est_cls = type(estimator)
    est_params = dict(estimator._paramMap)
    est_uid = estimator.uid
    conf = dict(spark_conf or {})

    def task(it):
        import os

        ctx = BarrierTaskContext.get()
        rank = ctx.partitionId()
        infos = ctx.getTaskInfos()
        addrs = [t.address for t in infos]
        port = str(free_port()) if rank == 0 else ""
        ports = ctx.allGather(port)
        os.environ.update(RANK=str(rank), WORLD_SIZE=str(len(infos)),
                          LOCAL_RANK=str(local_ranks(addrs)[rank]),
                          MASTER_ADDR=addrs[0].rsplit(":", 1)[0], MASTER_PORT=ports[0])
        import oap_mllib_amd as O
        from oap_mllib_amd.config import resolve

        O.init_world(resolve(spark_conf=conf))
        est = est_cls(uid=est_uid)
        est._set(**est_params)
        model = est.fit(_partition_to_input(est, list(it)))
        payload = export_model(model) if rank == 0 else None
        O.shutdown_world()
        ctx.barrier()
        if payload is not None:
            yield payload

    payloads = df.repartition(num_ranks).rdd.barrier().mapPartitions(task).collect()
    model = import_model(payloads[0])
    model.setParent(estimator)
    return model
