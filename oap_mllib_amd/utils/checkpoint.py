"""Periodic training snapshots and resume (SURVEY.md §5 "checkpoint / resume").

The reference's accelerated paths have none; upstream Spark's ALS fallback checkpoints factor
RDDs every ``checkpointInterval`` iterations when ``sc.checkpointDir`` is set
(spark-3.1.1/ml/recommendation/ALS.scala:1023-1079).  Here a fit whose
``Config.checkpoint_dir`` is set runs in segments; after each segment rank 0 writes the whole
iteration state — K-Means centers, ALS user factors (the only state: item factors are recomputed
from them first) — atomically to ``<dir>/<key>/``, where the key hashes the estimator uid,
params and data shape.  A later fit with the same key resumes from the snapshot; because one
Lloyd / ALS iteration is a function of that state alone, the resumed result equals an
uninterrupted run.  Snapshots are .npy files read with ``allow_pickle=False``.
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import tempfile

import numpy as np


class Checkpointer:
    def __init__(self, directory: str, key: dict, rank: int = 0):
        digest = hashlib.sha1(json.dumps(key, sort_keys=True, default=str).encode()).hexdigest()
        self.path = os.path.join(directory, digest[:16])
        self.rank = rank
        self.key = key

    def load(self) -> tuple[dict, dict] | None:
        meta_p = os.path.join(self.path, "state.json")
        if not os.path.exists(meta_p):
            return None
        with open(meta_p) as f:
            meta = json.load(f)
        arrays = {name: np.load(os.path.join(self.path, name + ".npy"), allow_pickle=False)
                  for name in meta.get("arrays", [])}
        return meta, arrays

    def save(self, meta: dict, arrays: dict[str, np.ndarray]) -> None:
        if self.rank != 0:
            return
        os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
        tmp = tempfile.mkdtemp(prefix=".ckpt-", dir=os.path.dirname(self.path) or ".")
        for name, a in arrays.items():
            np.save(os.path.join(tmp, name + ".npy"), np.asarray(a), allow_pickle=False)
        with open(os.path.join(tmp, "state.json"), "w") as f:
            json.dump({**meta, "arrays": sorted(arrays), "key": self.key}, f, default=str)
        old = self.path + ".old"
        if os.path.exists(self.path):
            os.replace(self.path, old)
        os.replace(tmp, self.path)
        shutil.rmtree(old, ignore_errors=True)

    def clear(self) -> None:
        if self.rank == 0:
            shutil.rmtree(self.path, ignore_errors=True)


def for_fit(world, estimator, shape: tuple, extra: dict | None = None) -> Checkpointer | None:
    d = world.config.checkpoint_dir
    if not d:
        return None
    key = {"uid": estimator.uid, "class": type(estimator).__name__,
           "params": estimator.extractParamMap(), "shape": list(shape), "world": world.size,
           **(extra or {})}
    return Checkpointer(d, key, world.rank)
