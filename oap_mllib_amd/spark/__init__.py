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
* only the input columns are shuffled; on Spark >= 3.5 the stage is ``mapInArrow(...,
  barrier=True)`` and each partition arrives as Arrow record batches that become the numpy
  matrix (or rating columns) column-at-a-time (``vectors_from_arrow``); older Spark uses the
  RDD barrier path with one numpy pass per column;
* the estimator's normal ``fit`` runs on it; rank 0 returns the fitted model as ``.npy``
  payloads (loaded on the driver with ``allow_pickle=False``).

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
    from ..models.recommendation import ALSModel

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
                     user_arrays=(arr["user_ids"], arr["user_factors"]),
                     item_arrays=(arr["item_ids"], arr["item_factors"]))
    for k, v in meta["params"].items():
        if m.hasParam(k):
            m._set(**{k: v})
    return m


def _input_columns(estimator) -> list[str]:
    """The DataFrame columns a fit reads (only these are shuffled into the barrier stage)."""
    from ..models.recommendation import ALS

    if isinstance(estimator, ALS):
        cols = [estimator.getOrDefault("userCol"), estimator.getOrDefault("itemCol")]
        r = estimator.getOrDefault("ratingCol")
        return cols + ([r] if r else [])
    return [estimator.getOrDefault("inputCol") if estimator.hasParam("inputCol")
            else estimator.getOrDefault("featuresCol")]


def vectors_from_arrow(col) -> np.ndarray:
    """A VectorUDT column in Arrow form (struct<type: int8, size: int32, indices: list<int32>,
    values: list<double>>, how Spark ships ml.linalg vectors to Python) -> dense float64 matrix.
    Column-at-a-time: dense rows are one reshape of the flattened values, sparse rows one
    scatter — no per-row Python objects (the reference coalesces partitions in the JVM and
    copies rows into oneDAL tables one by one, OneDAL.scala:69-101)."""
    import pyarrow as pa

    if isinstance(col, pa.ChunkedArray):
        col = col.combine_chunks()
    n = len(col)
    if n == 0:
        return np.zeros((0, 0))
    typ = col.field("type").to_numpy(zero_copy_only=False)
    vals = col.field("values")
    lens = vals.value_lengths().fill_null(0).to_numpy(zero_copy_only=False).astype(np.int64)
    flat = vals.flatten().to_numpy(zero_copy_only=False).astype(np.float64, copy=False)
    dense = typ == 1
    if dense.all():
        d = int(lens[0])
        if not np.all(lens == d):
            raise ValueError("dense vectors of different sizes in one column")
        return flat.reshape(n, d)
    size = col.field("size").fill_null(0).to_numpy(zero_copy_only=False).astype(np.int64)
    d = int(max(np.where(dense, lens, size).max(), 0))
    out = np.zeros((n, d))
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
    if dense.any():
        dl = lens[dense]
        if not np.all(dl == d):
            raise ValueError("dense vectors of different sizes in one column")
        idx = starts[dense][:, None] + np.arange(d)[None, :]
        out[dense] = flat[idx]
    sp = ~dense
    ind = col.field("indices")
    ilens = ind.value_lengths().fill_null(0).to_numpy(zero_copy_only=False).astype(np.int64)
    iflat = ind.flatten().to_numpy(zero_copy_only=False)
    istarts = np.concatenate([[0], np.cumsum(ilens)[:-1]])
    rows_sp = np.nonzero(sp)[0]
    cnt = ilens[rows_sp]
    r_rep = np.repeat(rows_sp, cnt)
    off = np.arange(cnt.sum()) - np.repeat(np.cumsum(cnt) - cnt, cnt)
    out[r_rep, iflat[np.repeat(istarts[rows_sp], cnt) + off]] = \
        flat[np.repeat(starts[rows_sp], cnt) + off]
    return out


def table_to_input(estimator, table):
    """An Arrow table of this partition's input columns -> what estimator.fit accepts."""
    from ..models.recommendation import ALS

    cols = _input_columns(estimator)
    if isinstance(estimator, ALS):
        get = lambda c: table.column(c).to_numpy()  # noqa: E731
        n = table.num_rows
        return {"user": get(cols[0]), "item": get(cols[1]),
                "rating": get(cols[2]) if len(cols) > 2 else np.ones(n)}
    return vectors_from_arrow(table.column(cols[0]))


def batches_to_input(estimator, batches) -> Any:
    """This partition's Arrow record batches (mapInArrow) -> what estimator.fit accepts.  An
    empty partition (no batches at all, e.g. after repartition(num_ranks) of a small frame)
    yields an empty input instead of failing in Table.from_batches."""
    import pyarrow as pa

    batches = list(batches)
    if not batches:
        return _partition_to_input(estimator, [])
    return table_to_input(estimator, pa.Table.from_batches(batches))


def _agree_on_width(ctx, estimator, data):
    """Vector estimators: a rank with no rows learns the feature count from its peers (barrier
    allGather), so every rank enters the fit with the same d."""
    from ..models.recommendation import ALS

    if isinstance(estimator, ALS):
        return data
    d_local = int(data.shape[1]) if getattr(data, "ndim", 0) == 2 and len(data) else 0
    d = max(int(v) for v in ctx.allGather(str(d_local)))
    if len(data) == 0:
        return np.zeros((0, d))
    return data


def _partition_to_input(estimator, rows: list):
    """Spark Rows of this partition (the pre-3.5 RDD barrier path) -> what estimator.fit
    accepts, column-wise through numpy (one pass over the rows per column)."""
    from ..models.recommendation import ALS

    cols = _input_columns(estimator)
    n = len(rows)
    if isinstance(estimator, ALS):
        u = np.fromiter((row[cols[0]] for row in rows), dtype=np.int64, count=n)
        i = np.fromiter((row[cols[1]] for row in rows), dtype=np.int64, count=n)
        r = (np.fromiter((row[cols[2]] for row in rows), dtype=np.float64, count=n)
             if len(cols) > 2 else np.ones(n))
        return {"user": u, "item": i, "rating": r}
    if n == 0:
        return np.zeros((0, 0))
    first = rows[0][cols[0]]
    out = np.empty((n, first.size))
    for j, row in enumerate(rows):
        out[j] = row[cols[0]].toArray()
    return out


def _arrow_barrier_supported(df) -> bool:
    """mapInArrow(..., barrier=True) exists from pyspark 3.5 on."""
    import inspect

    f = getattr(df, "mapInArrow", None)
    return f is not None and "barrier" in inspect.signature(f).parameters


def fit(estimator, df, num_ranks: int, spark_conf: dict | None = None):
    """Fits `estimator` on Spark DataFrame `df` with `num_ranks` gang-scheduled ranks."""
    if not spark_available():
        raise RuntimeError("pyspark is not installed")
    from pyspark import BarrierTaskContext

    est_cls = type(estimator)
    est_params = dict(estimator._paramMap)
    est_uid = estimator.uid
    conf = dict(spark_conf or {})

    def run_rank(make_input):
        """Rendezvous through the barrier context, fit this rank's shard, return rank 0's
        payload (None elsewhere)."""
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
        model = est.fit(_agree_on_width(ctx, est, make_input(est)))
        payload = export_model(model) if rank == 0 else None
        O.shutdown_world()
        ctx.barrier()
        return payload

    def task(it):  # RDD barrier path: Row objects
        rows = list(it)
        payload = run_rank(lambda est: _partition_to_input(est, rows))
        if payload is not None:
            yield payload

    def arrow_task(batches):  # Arrow barrier path: record batches
        import pyarrow as pa

        batches = list(batches)
        payload = run_rank(lambda est: batches_to_input(est, batches))
        if payload is not None:
            keys = list(payload)
            yield pa.RecordBatch.from_arrays(
                [pa.array(keys), pa.array([payload[k] for k in keys], type=pa.binary())],
                names=["key", "value"])

    src = df.select(*_input_columns(estimator)).repartition(num_ranks)
    if _arrow_barrier_supported(src):
        # Spark >= 3.5: partitions arrive as Arrow record batches (no Row objects at all)
        rows = src.mapInArrow(arrow_task, "key string, value binary", barrier=True).collect()
        payloads = [{r["key"]: bytes(r["value"]) for r in rows}]
    else:
        payloads = src.rdd.barrier().mapPartitions(task).collect()
    model = import_model(payloads[0])
    model.setParent(estimator)
    return model
