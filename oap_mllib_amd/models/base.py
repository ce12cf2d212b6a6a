"""Estimator / Model / persistence base classes (``pyspark.ml`` contract) and engine dispatch.

Every estimator picks its engine the way the reference's shadow classes do (native path when the
platform check passes and the parameters are supported, otherwise the vanilla path:
KMeans.scala:349-351, PCA.scala:103, ALS.scala:922-926), with the platform check being
"a visible MI355X + the native engine loaded" instead of ``daal_check_is_intel_cpu()``
(OneDAL.cpp:96-102).
"""
from __future__ import annotations

import os
from typing import Any

from ..params import Params
from ..parallel.world import World, get_world
from ..utils.logging import get_logger

log = get_logger("oap_mllib_amd.models")


def java_string_hash(s: str) -> int:
    """java.lang.String#hashCode (Spark's default seed is getClass.getName.hashCode)."""
    h = 0
    for ch in s:
        h = (31 * h + ord(ch)) & 0xFFFFFFFF
    return h - (1 << 32) if h >= (1 << 31) else h


def choose_engine(native_supported: bool, world: World | None = None) -> str:
    """'gpu' | 'cpu' | 'vanilla' for this call."""
    w = world or get_world()
    if not native_supported or w.backend == "vanilla":
        return "vanilla"
    return w.backend


class Estimator(Params):
    def fit(self, dataset: Any, params: dict | None = None):
        if params:
            return self.copy(params)._fit(dataset)
        return self._fit(dataset)

    def _fit(self, dataset: Any):  # pragma: no cover - abstract
        raise NotImplementedError


class Transformer(Params):
    def transform(self, dataset: Any, params: dict | None = None):
        if params:
            return self.copy(params)._transform(dataset)
        return self._transform(dataset)

    def _transform(self, dataset: Any):  # pragma: no cover - abstract
        raise NotImplementedError


class Model(Transformer):
    parent: Any = None

    def setParent(self, parent) -> "Model":  # noqa: N802
        self.parent = parent
        return self

    def hasParent(self) -> bool:  # noqa: N802
        return self.parent is not None


class HasTrainingSummary:
    _summary = None

    @property
    def hasSummary(self) -> bool:  # noqa: N802
        return self._summary is not None

    @property
    def summary(self):
        if self._summary is None:
            raise RuntimeError(f"No training summary available for this {type(self).__name__}")
        return self._summary

    def setSummary(self, summary):  # noqa: N802
        self._summary = summary
        return self


class MLWriter:
    def __init__(self, instance: Any):
        self.instance = instance
        self._overwrite = False
        self._format = "internal"

    def overwrite(self) -> "MLWriter":
        self._overwrite = True
        return self

    def format(self, source: str) -> "MLWriter":
        self._format = source
        return self

    def save(self, path: str) -> None:
        from ..persistence.spark_format import prepare_dir

        path = os.fspath(path)
        w = get_world()
        # like Spark, the driver (rank 0) writes; other ranks only synchronise
        if w.rank == 0:
            prepare_dir(path, self._overwrite)
            self.instance._save_impl(path, self._format)
        w.barrier()


class MLWritable:
    def write(self) -> MLWriter:
        return MLWriter(self)

    def save(self, path: str) -> None:
        self.write().save(path)

    def _save_impl(self, path: str, fmt: str) -> None:  # pragma: no cover - abstract
        raise NotImplementedError


class MLReader:
    def __init__(self, cls):
        self.cls = cls

    def load(self, path: str):
        return self.cls._load_impl(os.fspath(path))


class MLReadable:
    @classmethod
    def read(cls) -> MLReader:
        return MLReader(cls)

    @classmethod
    def load(cls, path: str):
        return cls.read().load(path)

    @classmethod
    def _load_impl(cls, path: str):  # pragma: no cover - abstract
        raise NotImplementedError


class DefaultParamsPersistence(MLWritable, MLReadable):
    """Estimators persist only metadata (DefaultParamsWriter / DefaultParamsReader)."""

    _spark_class: str = ""

    def _save_impl(self, path: str, fmt: str) -> None:
        from ..persistence.spark_format import write_metadata

        write_metadata(path, self._spark_class, self.uid, self._paramMap, self.defaultParamMap())

    @classmethod
    def _load_impl(cls, path: str):
        from ..persistence.spark_format import read_metadata

        meta = read_metadata(path, cls._spark_class)
        inst = cls()
        inst.uid = meta["uid"]
        for k, v in meta.get("paramMap", {}).items():
            if inst.hasParam(k):
                inst._set(**{k: v})
        return inst
