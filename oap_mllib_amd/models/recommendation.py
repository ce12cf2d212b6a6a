"""ALS estimator / model with the ``org.apache.spark.ml.recommendation`` contract.

Mirrors the reference's shadow ``ALS`` (mllib-dal/src/main/scala/org/apache/spark-3.1.1/ml/
recommendation/ALS.scala): Params and defaults (:241-245, blockSize :130), integer-id checks
(``checkedCast``, :89-113), dispatch (the reference accelerates only ``implicitPrefs``,
:922-926, and falls back to Spark's distributed ALS otherwise, :971-1114; here every
configuration runs natively with the ratings sharded — see below), ``ALSModel.transform`` with
``coldStartStrategy`` nan/drop (:303-334), ``recommendForAll*`` / ``recommendFor*Subset``
(:365-505) and persistence: metadata with an extra ``rank`` field plus ``userFactors`` /
``itemFactors`` parquet of (id: int, features: array<float>) (:522-553).

The native path (csrc/drivers/als.cpp) replaces ALSDALImpl.scala + ALSShuffle.cpp +
ALSDALImpl.cpp: id-owner alltoallv shuffle with dense re-indexing, replicated fp32 factors in
HBM, MFMA Gramian + allreduce, per-row normal equations + Cholesky on the GPU
(kernels/als.hip), one allgather per half-iteration.

Explicit feedback takes the same GPU kernels (``A = sum y y^T + lambda n I``, Spark's
``computeFactors`` semantics, ALS.scala:1777-1795).  Ranks beyond the GPU kernels
(``als_max_rank()``) and ``nonnegative=True`` run the driver's fp64 host solver over the same
distributed shuffle (per-row Cholesky; Lawson-Hanson NNLS for non-negative factors — the
minimiser Spark's NNLS converges to; the reference's oneDAL path silently ignored
``nonnegative``).  Only the ``vanilla`` backend (no native library) runs the single-process
numpy fallback.
"""
from __future__ import annotations

import time
from typing import Any

import numpy as np

from .. import _loader
from ..fallback import als_vanilla as vanilla
from ..params import Param, gt_eq, in_array, to_bool, to_float, to_int, to_str
from ..parallel.world import get_world
from ..persistence import spark_format as sf
from ..utils import checkpoint
from ..utils.logging import Instrumentation
from .base import (DefaultParamsPersistence, Estimator, MLReadable, MLWritable, Model,
                   choose_engine, java_string_hash)

_INT_MAX = 2 ** 31 - 1


def _lower(v):
    return to_str(v).lower()


class _ALSModelParams:
    userCol = Param("userCol", "column name for user ids. Ids must be within the integer value "
                    "range.", "user", converter=to_str)
    itemCol = Param("itemCol", "column name for item ids. Ids must be within the integer value "
                    "range.", "item", converter=to_str)
    predictionCol = Param("predictionCol", "prediction column name", "prediction",
                          converter=to_str)
    coldStartStrategy = Param("coldStartStrategy", "strategy for dealing with unknown or new "
                              "users/items at prediction time. Supported values: nan, drop.",
                              "nan", in_array(["nan", "drop"]), _lower)
    blockSize = Param("blockSize", "block size for stacking input data in matrices.", 4096,
                      gt_eq(1), to_int)


class _ALSParams(_ALSModelParams):
    rank = Param("rank", "rank of the factorization", 10, gt_eq(1), to_int)
    numUserBlocks = Param("numUserBlocks", "number of user blocks", 10, gt_eq(1), to_int)
    numItemBlocks = Param("numItemBlocks", "number of item blocks", 10, gt_eq(1), to_int)
    implicitPrefs = Param("implicitPrefs", "whether to use implicit preference", False,
                          converter=to_bool)
    alpha = Param("alpha", "alpha for implicit preference", 1.0, gt_eq(0), to_float)
    ratingCol = Param("ratingCol", "column name for ratings", "rating", converter=to_str)
    nonnegative = Param("nonnegative", "whether to use nonnegative constraint for least squares",
                        False, converter=to_bool)
    maxIter = Param("maxIter", "maximum number of iterations (>= 0)", 10, gt_eq(0), to_int)
    regParam = Param("regParam", "regularization parameter (>= 0)", 0.1, gt_eq(0), to_float)
    checkpointInterval = Param("checkpointInterval", "set checkpoint interval (>= 1) or disable "
                               "checkpoint (-1)", 10, lambda v: v == -1 or v >= 1, to_int)
    seed = Param("seed", "random seed",
                 java_string_hash("org.apache.spark.ml.recommendation.ALS"), converter=to_int)
    intermediateStorageLevel = Param("intermediateStorageLevel", "StorageLevel for intermediate "
                                     "datasets. Cannot be 'NONE'.", "MEMORY_AND_DISK",
                                     lambda v: v != "NONE", to_str)
    finalStorageLevel = Param("finalStorageLevel", "StorageLevel for ALS model factors.",
                              "MEMORY_AND_DISK", converter=to_str)


def _frame(dataset: Any):
    import pandas as pd

    if isinstance(dataset, pd.DataFrame):
        return dataset
    if isinstance(dataset, dict):
        return pd.DataFrame({k: list(v) if not isinstance(v, np.ndarray) else v
                             for k, v in dataset.items()})
    try:
        import pyarrow as pa

        if isinstance(dataset, pa.Table):
            return dataset.to_pandas()
    except ImportError:  # pragma: no cover
        pass
    if isinstance(dataset, np.ndarray) and dataset.dtype.names:
        return pd.DataFrame({n: dataset[n] for n in dataset.dtype.names})
    raise TypeError(f"unsupported dataset type {type(dataset).__name__}")


def checked_cast(values, name: str) -> np.ndarray:
    """Spark's checkedCast: integral values within the Int range, else an error."""
    v = np.asarray(values)
    if v.dtype.kind in "iu":
        if len(v) and (v.min() < -_INT_MAX - 1 or v.max() > _INT_MAX):
            raise ValueError(f"ALS only supports values in Integer range for column {name}")
        return v.astype(np.int32)
    if v.dtype.kind == "f":
        if len(v) and (not np.all(np.isfinite(v)) or np.any(v != np.floor(v)) or
                       v.min() < -_INT_MAX - 1 or v.max() > _INT_MAX):
            raise ValueError(f"ALS only supports values in Integer range and without fractional "
                             f"part for column {name}")
        return v.astype(np.int32)
    raise TypeError(f"Column {name} must be of numeric type, got {v.dtype}")


class ALS(_ALSParams, Estimator, DefaultParamsPersistence):
    """Alternating least squares matrix factorisation (explicit or implicit feedback)."""

    _uid_prefix = "als"
    _spark_class = "org.apache.spark.ml.recommendation.ALS"

    def __init__(self, **kwargs):
        super().__init__(kwargs.pop("uid", None))
        if kwargs:
            self._set(**kwargs)

    def setParams(self, **kwargs) -> "ALS":  # noqa: N802
        return self._set(**kwargs)

    def setNumBlocks(self, value: int) -> "ALS":  # noqa: N802
        return self._set(numUserBlocks=value, numItemBlocks=value)

    def _ratings(self, dataset):
        df = _frame(dataset)
        u = checked_cast(df[self.getOrDefault("userCol")].to_numpy(), self.getOrDefault("userCol"))
        i = checked_cast(df[self.getOrDefault("itemCol")].to_numpy(), self.getOrDefault("itemCol"))
        rc = self.getOrDefault("ratingCol")
        r = (np.ones(len(u), dtype=np.float32) if rc == "" else
             np.asarray(df[rc].to_numpy(), dtype=np.float32))
        return u, i, r

    def _fit(self, dataset: Any) -> "ALSModel":
        instr = Instrumentation(self)
        instr.logParams(self.extractParamMap())
        w = get_world()
        u, i, r = self._ratings(dataset)
        rank = self.getOrDefault("rank")
        implicit = self.getOrDefault("implicitPrefs")
        nonneg = self.getOrDefault("nonnegative")
        # every configuration runs natively and distributed (ratings stay sharded): explicit and
        # implicit feedback on the GPU kernels; ranks beyond them and non-negative factors
        # (NNLS) on the fp64 host solver of the same driver, over the same world
        engine = choose_engine(True, w)
        host_solver = engine == "gpu" and (nonneg or rank > _loader.load().als_max_rank())
        seed = self.getOrDefault("seed") & 0xFFFFFFFFFFFFFFFF
        t0 = time.time()
        extra: dict = {"engine": engine, "host_solver": host_solver or engine == "cpu"}
        if engine == "vanilla":
            if w.distributed:  # the fallback is single-process: gather every rank's ratings
                parts = w.allgather_obj((u, i, r))
                u = np.concatenate([p[0] for p in parts])
                i = np.concatenate([p[1] for p in parts])
                r = np.concatenate([p[2] for p in parts])
            res = vanilla.fit(u, i, r, rank, self.getOrDefault("maxIter"),
                              self.getOrDefault("regParam"), implicit,
                              self.getOrDefault("alpha"), self.getOrDefault("nonnegative"), seed)
            uid, uf, iid, itf = res.user_ids, res.user_factors, res.item_ids, res.item_factors
        else:
            N = _loader.load()
            ck = checkpoint.for_fit(w, self, (len(u),)) \
                if self.getOrDefault("checkpointInterval") > 0 else None
            out = self._fit_native(N, w, u, i, r, rank, implicit, seed, ck, host_solver, nonneg)
            uid, uf = np.asarray(out["user_ids"]), np.asarray(out["user_factors"])
            iid, itf = np.asarray(out["item_ids"]), np.asarray(out["item_factors"])
            extra.update({k: out[k] for k in ("nnz", "setup_ms", "train_ms", "iter_ms", "gram_ms",
                                              "solve_ms", "comm_ms", "failed_rows")})
        model = ALSModel(uid=self.uid, rank=rank, user_arrays=(uid, uf), item_arrays=(iid, itf))
        self._copyValues(model)
        model.setParent(self)
        model.fit_info = {"fit_seconds": time.time() - t0, **extra}
        instr.logNamedValue("engine", engine)
        instr.finish()
        return model


    def _fit_native(self, N, w, u, i, r, rank, implicit, seed, ck, host_solver=False,
                    nonneg=False):
        """Native fit; with a checkpointer, in checkpointInterval-sized segments that save
        (and resume from) the user factors."""
        max_iter = self.getOrDefault("maxIter")
        args = (self.getOrDefault("regParam"), self.getOrDefault("alpha"), implicit, seed)
        kw = {"host_engine": host_solver, "nonnegative": nonneg}
        if ck is None:
            return N.als_fit(w.ctx, w.comm, u, i, r, rank, max_iter, *args, **kw)
        interval = self.getOrDefault("checkpointInterval")
        done, ids, fac = 0, None, None
        state = ck.load()
        if state is not None:
            meta, arrays = state
            done, ids, fac = int(meta["num_iter"]), arrays["user_ids"], arrays["user_factors"]
        out = None
        while out is None or done < max_iter:
            seg = min(interval, max_iter - done)
            out = N.als_fit(w.ctx, w.comm, u, i, r, rank, max(seg, 0), *args, ids, fac, **kw)
            done += max(seg, 0)
            ids = np.asarray(out["user_ids"])
            order = np.argsort(ids, kind="stable")
            ids, fac = ids[order], np.asarray(out["user_factors"])[order]
            ck.save({"num_iter": done}, {"user_ids": ids, "user_factors": fac})
            if seg <= 0:
                break
        return out


def _factor_frame(ids: np.ndarray, factors: np.ndarray):
    """(id, features) frame of a factor matrix, sorted by id; the features column is one Arrow
    fixed_size_list<float> buffer (no per-row Python objects)."""
    import pandas as pd

    from ..data import vector_column

    ids, F = _sorted_factors(ids, factors)
    return pd.DataFrame({"id": ids.astype(np.int32), "features": vector_column(F)})


def _sorted_factors(ids, factors, rank: int | None = None) -> tuple[np.ndarray, np.ndarray]:
    ids = np.asarray(ids)
    F = np.asarray(factors, dtype=np.float32)
    if F.ndim != 2:
        F = F.reshape(len(ids), -1 if rank is None else rank)
    if len(ids) > 1 and np.any(ids[1:] < ids[:-1]):
        order = np.argsort(ids, kind="stable")
        ids, F = ids[order], F[order]
    return ids.astype(np.int64), np.ascontiguousarray(F)


def _frame_factors(df, rank: int) -> tuple[np.ndarray, np.ndarray]:
    from ..data import to_matrix

    if len(df) == 0:
        return np.zeros(0, np.int64), np.zeros((0, rank), np.float32)
    return _sorted_factors(df["id"].to_numpy(), to_matrix(df, "features", np.float32), rank)


class ALSModel(_ALSModelParams, Model, MLWritable, MLReadable):
    """Factors live as two contiguous (sorted ids, [n][rank] float32) pairs; the Spark-shaped
    ``userFactors`` / ``itemFactors`` frames are views built on first access."""

    _uid_prefix = "als"
    _spark_class = "org.apache.spark.ml.recommendation.ALSModel"

    def __init__(self, uid: str | None = None, rank: int = 0, userFactors=None,
                 itemFactors=None, user_arrays=None, item_arrays=None):  # noqa: N803
        super().__init__(uid)
        self.rank = int(rank)
        empty = (np.zeros(0, np.int64), np.zeros((0, self.rank), np.float32))
        self._fac = {"user": empty, "item": empty}
        self._frames: dict = {}
        for which, frame, arrays in (("user", userFactors, user_arrays),
                                     ("item", itemFactors, item_arrays)):
            if arrays is not None:
                self._fac[which] = _sorted_factors(arrays[0], arrays[1], self.rank)
            elif frame is not None:
                self._fac[which] = _frame_factors(frame, self.rank)
        self.fit_info: dict = {}

    def _frame(self, which: str):
        if which not in self._frames:
            self._frames[which] = _factor_frame(*self._fac[which])
        return self._frames[which]

    @property
    def userFactors(self):  # noqa: N802
        return self._frame("user")

    @userFactors.setter
    def userFactors(self, df):  # noqa: N802
        self._fac["user"] = _frame_factors(df, self.rank)
        self._frames.pop("user", None)

    @property
    def itemFactors(self):  # noqa: N802
        return self._frame("item")

    @itemFactors.setter
    def itemFactors(self, df):  # noqa: N802
        self._fac["item"] = _frame_factors(df, self.rank)
        self._frames.pop("item", None)

    # ---- factor access -----------------------------------------------------------------
    def _mat(self, which: str) -> tuple[np.ndarray, np.ndarray]:
        return self._fac[which]

    def _lookup(self, which: str, keys: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
        ids, F = self._mat(which)
        pos = np.searchsorted(ids, keys)
        pos = np.clip(pos, 0, max(len(ids) - 1, 0))
        found = (len(ids) > 0) & (ids[pos] == keys) if len(ids) else np.zeros(len(keys), bool)
        return found, (F[pos] if len(ids) else np.zeros((len(keys), self.rank), np.float32))

    # ---- transform ---------------------------------------------------------------------
    def _transform(self, dataset):
        df = _frame(dataset).copy()
        u = np.asarray(df[self.getOrDefault("userCol")].to_numpy(), dtype=np.float64)
        it = np.asarray(df[self.getOrDefault("itemCol")].to_numpy(), dtype=np.float64)
        ok_u = np.isfinite(u) & (u == np.floor(u)) & (np.abs(u) <= _INT_MAX)
        ok_i = np.isfinite(it) & (it == np.floor(it)) & (np.abs(it) <= _INT_MAX)
        fu, Fu = self._lookup("user", np.where(ok_u, u, -1).astype(np.int64))
        fi, Fi = self._lookup("item", np.where(ok_i, it, -1).astype(np.int64))
        pred = np.einsum("ij,ij->i", Fu.astype(np.float32), Fi.astype(np.float32),
                         dtype=np.float32)
        valid = fu & fi & ok_u & ok_i
        pred = np.where(valid, pred, np.float32(np.nan)).astype(np.float32)
        df[self.getOrDefault("predictionCol")] = pred
        if self.getOrDefault("coldStartStrategy") == "drop":
            df = df[~np.isnan(pred)].reset_index(drop=True)
        return df

    def predict(self, user: int, item: int) -> float:
        fu, Fu = self._lookup("user", np.array([user]))
        fi, Fi = self._lookup("item", np.array([item]))
        return float(np.dot(Fu[0], Fi[0])) if fu[0] and fi[0] else float("nan")

    # ---- recommendations ---------------------------------------------------------------
    def _topk(self, src_ids, S, dst_ids, D, num: int, dst_col: str, src_col: str,
              replicated: bool = True):
        import pandas as pd

        import pyarrow as pa

        num = max(0, min(int(num), len(dst_ids)))
        recs_idx, recs_val = _blocked_topk(S, D, num, replicated=replicated)
        # array<struct<dst: int, rating: float>> per source row, as ONE Arrow list array
        dst = np.asarray(dst_ids, dtype=np.int32)[recs_idx.reshape(-1)] if recs_idx.size else \
            np.zeros(0, np.int32)
        st = pa.StructArray.from_arrays(
            [pa.array(dst, pa.int32()), pa.array(recs_val.reshape(-1), pa.float32())],
            names=[dst_col, "rating"])
        offsets = pa.array(np.arange(len(recs_idx) + 1, dtype=np.int32) * num, pa.int32())
        recs = pa.ListArray.from_arrays(offsets, st)
        return pd.DataFrame({src_col: np.asarray(src_ids, dtype=np.int32),
                             "recommendations": pd.arrays.ArrowExtensionArray(recs)})

    def recommendForAllUsers(self, numItems: int):  # noqa: N802,N803
        uids, U = self._mat("user")
        iids, I = self._mat("item")
        return self._topk(uids, U, iids, I, numItems, self.getOrDefault("itemCol"),
                          self.getOrDefault("userCol"))

    def recommendForAllItems(self, numUsers: int):  # noqa: N802,N803
        uids, U = self._mat("user")
        iids, I = self._mat("item")
        return self._topk(iids, I, uids, U, numUsers, self.getOrDefault("userCol"),
                          self.getOrDefault("itemCol"))

    def recommendForUserSubset(self, dataset, numItems: int):  # noqa: N802,N803
        keys = np.unique(checked_cast(_frame(dataset)[self.getOrDefault("userCol")].to_numpy(),
                                      self.getOrDefault("userCol")).astype(np.int64))
        found, U = self._lookup("user", keys)
        iids, I = self._mat("item")
        return self._topk(keys[found], U[found], iids, I, numItems, self.getOrDefault("itemCol"),
                          self.getOrDefault("userCol"), replicated=False)

    def recommendForItemSubset(self, dataset, numUsers: int):  # noqa: N802,N803
        keys = np.unique(checked_cast(_frame(dataset)[self.getOrDefault("itemCol")].to_numpy(),
                                      self.getOrDefault("itemCol")).astype(np.int64))
        found, I = self._lookup("item", keys)
        uids, U = self._mat("user")
        return self._topk(keys[found], I[found], uids, U, numUsers, self.getOrDefault("userCol"),
                          self.getOrDefault("itemCol"), replicated=False)

    def copy(self, extra: dict | None = None) -> "ALSModel":
        m = super().copy(extra)
        m._fac = {w: (ids.copy(), F.copy()) for w, (ids, F) in self._fac.items()}
        m._frames = {}
        return m

    # ---- persistence -------------------------------------------------------------------
    def _save_impl(self, path: str, fmt: str) -> None:
        import os

        import pyarrow as pa

        sf.write_metadata(path, self._spark_class, self.uid, self._paramMap,
                          self.defaultParamMap(), extra={"rank": self.rank})
        schema = pa.schema([pa.field("id", pa.int32(), nullable=False),
                            pa.field("features", pa.list_(pa.field("element", pa.float32(),
                                                                   nullable=False)))])
        spark = sf.spark_schema([("id", "integer", False),
                                 ("features", {"type": "array", "elementType": "float",
                                               "containsNull": False}, True)])
        for name, which in (("userFactors", "user"), ("itemFactors", "item")):
            ids, F = self._mat(which)
            offsets = pa.array(np.arange(len(ids) + 1, dtype=np.int32) * self.rank, pa.int32())
            feats = pa.ListArray.from_arrays(offsets, pa.array(F.reshape(-1), pa.float32()),
                                             type=schema.field("features").type)
            t = pa.Table.from_arrays([pa.array(ids.astype(np.int32), pa.int32()), feats],
                                     schema=schema)
            sf.write_parquet(os.path.join(path, name), t, spark)

    @classmethod
    def _load_impl(cls, path: str) -> "ALSModel":
        import os

        meta = sf.read_metadata(path, cls._spark_class)
        from ..data import _arrow_matrix

        rank = int(meta["rank"])
        arrays = []
        for name in ("userFactors", "itemFactors"):
            t = sf.read_parquet_dir(os.path.join(path, name))
            ids = t.column("id").to_numpy()
            F = (_arrow_matrix(t.column("features"), np.float32) if len(ids)
                 else np.zeros((0, rank), np.float32))
            if F is None:  # (null / ragged entries: the per-row reader)
                F = np.asarray(t.column("features").to_pylist(), dtype=np.float32)
            arrays.append((ids, F.reshape(len(ids), rank)))
        m = cls(uid=meta["uid"], rank=rank, user_arrays=arrays[0], item_arrays=arrays[1])
        for k, v in meta.get("paramMap", {}).items():
            if m.hasParam(k):
                m._set(**{k: v})
        return m


def _blocked_topk(S: np.ndarray, D: np.ndarray, num: int, block: int = 4096,
                  replicated: bool = True):
    """Top-`num` (index, score) per row of S @ D^T, descending; ties by lower index.

    ``replicated`` (recommendForAll*: S is the model's factor matrix, the same on every rank):
    sharded by rank as Spark's blocked recommendForAll is over the source blocks
    (ALS.scala:365-505) — each rank takes a contiguous slab of S, then the slabs are
    allgathered as typed int32 / fp32 row slabs.  Otherwise (the subset calls: S comes from this
    rank's own dataset shard) every row is scored locally and nothing is exchanged.  On a GPU
    world the scoring runs through the fused score + top-k kernel (kernels/als_recommend.hip:
    split-fp16 MFMA scores kept in registers, no score matrix anywhere), numpy on CPU.
    """
    n = len(S)
    w = get_world()
    if not replicated or w.size == 1:
        return _local_topk(S, D, num, w, block)
    bounds = [(n * r) // w.size for r in range(w.size + 1)]
    counts = [bounds[r + 1] - bounds[r] for r in range(w.size)]
    idx, val = _local_topk(S[bounds[w.rank]:bounds[w.rank + 1]], D, num, w, block)
    idx = w.allgather_rows(idx.astype(np.int32), counts).astype(np.int64)
    val = w.allgather_rows(val.astype(np.float32), counts)
    return idx, val


def _local_topk(S: np.ndarray, D: np.ndarray, num: int, w, block: int):
    n = len(S)
    idx = np.zeros((n, num), dtype=np.int64)
    val = np.zeros((n, num), dtype=np.float32)
    if n == 0 or num == 0:
        return idx, val
    if w.is_gpu:
        # the fused score + top-k kernel for every num it holds (LDS lists up to ~24, HBM
        # candidate buffers up to 4088: kernels/als_recommend.hip); beyond that, and for ranks
        # above 256, the host loop below (said out loud: it is not the GPU path)
        N = _loader.load()
        rank = S.shape[1] if S.ndim == 2 else 0
        if 1 <= rank and num <= N.als_recommend_max_num(rank) and len(D) > 0:
            i32, v, _ = N.als_recommend(w.ctx, np.ascontiguousarray(S, dtype=np.float32),
                                        np.ascontiguousarray(D, dtype=np.float32), num)
            return i32.astype(np.int64), v
        import warnings

        warnings.warn(f"recommendForAll*: num={num} at rank {rank} is beyond the GPU kernel "
                      f"(num <= {N.als_recommend_max_num(max(rank, 1))}, rank <= 256); "
                      "scoring on the host", RuntimeWarning, stacklevel=3)
    for b in range(0, n, block):
        sc = S[b:b + block].astype(np.float32) @ D.astype(np.float32).T
        part = np.argpartition(-sc, num - 1, axis=1)[:, :num] if num < sc.shape[1] else \
            np.tile(np.arange(sc.shape[1]), (len(sc), 1))
        pv = np.take_along_axis(sc, part, axis=1)
        order = np.lexsort((part, -pv), axis=1)
        idx[b:b + block] = np.take_along_axis(part, order, axis=1)
        val[b:b + block] = np.take_along_axis(pv, order, axis=1)
    return idx, val
