"""Spark-ML style Param system (``org.apache.spark.ml.param``) for the estimators.

Same contract as Spark's: every Param has a name, doc, optional default and validator; values
are validated when set; ``explainParams``, ``extractParamMap``, ``copy(extra)`` behave as in
Spark; ``setX``/``getX`` accessors are generated for every declared Param (``setK``,
``getMaxIter``...).  Param names and defaults of the three estimators mirror the reference's
shadow classes (e.g. KMeans: spark-3.1.1/ml/clustering/KMeans.scala:90-91, ALS: ALS.scala:241-245).
"""
from __future__ import annotations

import copy as _copy
import uuid
from typing import Any, Callable


class _NoDefault:
    def __repr__(self) -> str:
        return "<undefined>"


NO_DEFAULT = _NoDefault()


class Param:
    def __init__(self, name: str, doc: str, default: Any = NO_DEFAULT,
                 validator: Callable[[Any], bool] | None = None,
                 converter: Callable[[Any], Any] | None = None):
        self.name = name
        self.doc = doc
        self.default = default
        self.validator = validator
        self.converter = converter

    def validate(self, value: Any) -> Any:
        if self.converter is not None and value is not None:
            value = self.converter(value)
        if self.validator is not None and not self.validator(value):
            raise ValueError(f"{self.name} given invalid value {value!r}: {self.doc}")
        return value

    def __repr__(self) -> str:
        return f"Param({self.name})"


# ---- validators (ParamValidators) --------------------------------------------------------
def gt(lo):
    return lambda v: v is not None and v > lo


def gt_eq(lo):
    return lambda v: v is not None and v >= lo


def in_range(lo, hi, lower_inclusive=True, upper_inclusive=True):
    def f(v):
        if v is None:
            return False
        a = v >= lo if lower_inclusive else v > lo
        b = v <= hi if upper_inclusive else v < hi
        return a and b
    return f


def in_array(allowed):
    return lambda v: v in allowed


def to_int(v):
    if isinstance(v, bool) or int(v) != v:
        raise TypeError(f"expected an integer, got {v!r}")
    return int(v)


def to_float(v):
    return float(v)


def to_str(v):
    if not isinstance(v, str):
        raise TypeError(f"expected a string, got {v!r}")
    return v


def to_bool(v):
    if not isinstance(v, bool):
        raise TypeError(f"expected a bool, got {v!r}")
    return v


def _cap(name: str) -> str:
    return name[0].upper() + name[1:]


class Params:
    """Base class: collects the class-level ``Param`` declarations and manages values."""

    _uid_prefix = "Params"

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        for p in cls._param_decls().values():
            pname = p.name
            setter, getter = "set" + _cap(pname), "get" + _cap(pname)
            if not hasattr(cls, setter):
                def _set(self, value, _n=pname):
                    return self._set(**{_n: value})
                _set.__name__ = setter
                setattr(cls, setter, _set)
            if not hasattr(cls, getter):
                def _get(self, _n=pname):
                    return self.getOrDefault(_n)
                _get.__name__ = getter
                setattr(cls, getter, _get)

    def __init__(self, uid: str | None = None):
        self.uid = uid or f"{self._uid_prefix}_{uuid.uuid4().hex[-12:]}"
        self._paramMap: dict[str, Any] = {}
        self._defaults: dict[str, Any] = {}  # per-instance defaults (e.g. outputCol = uid__output)

    def _setDefault(self, **kw) -> "Params":  # noqa: N802
        for name, value in kw.items():
            self.getParam(name)
            self._defaults[name] = value
        return self

    def _default_of(self, name: str) -> Any:
        if name in getattr(self, "_defaults", {}):
            return self._defaults[name]
        return self.getParam(name).default

    # -- introspection -----------------------------------------------------------------
    @classmethod
    def _param_decls(cls) -> dict[str, Param]:
        out: dict[str, Param] = {}
        for klass in reversed(cls.__mro__):
            for v in vars(klass).values():
                if isinstance(v, Param):
                    out[v.name] = v
        return out

    @property
    def params(self) -> list[Param]:
        return sorted(self._param_decls().values(), key=lambda p: p.name)

    def getParam(self, name: str) -> Param:  # noqa: N802
        try:
            return self._param_decls()[name]
        except KeyError:
            raise ValueError(f"{type(self).__name__} has no param '{name}'") from None

    def hasParam(self, name: str) -> bool:  # noqa: N802
        return name in self._param_decls()

    def isSet(self, name: str) -> bool:  # noqa: N802
        return name in self._paramMap

    def hasDefault(self, name: str) -> bool:  # noqa: N802
        return self._default_of(name) is not NO_DEFAULT

    def isDefined(self, name: str) -> bool:  # noqa: N802
        return self.isSet(name) or self.hasDefault(name)

    def getOrDefault(self, name: str) -> Any:  # noqa: N802
        if name in self._paramMap:
            return self._paramMap[name]
        v = self._default_of(name)
        if v is NO_DEFAULT:
            raise KeyError(f"Failed to find a default value for {name}")
        return v

    def getDefault(self, name: str) -> Any:  # noqa: N802
        return self._default_of(name)

    def _set(self, **kw) -> "Params":
        for name, value in kw.items():
            p = self.getParam(name)
            self._paramMap[name] = p.validate(value)
        return self

    def set(self, name: str, value: Any) -> "Params":
        return self._set(**{name: value})

    def clear(self, name: str) -> "Params":
        self._paramMap.pop(name, None)
        return self

    def extractParamMap(self, extra: dict | None = None) -> dict[str, Any]:  # noqa: N802
        out = self.defaultParamMap()
        out.update(self._paramMap)
        out.update(extra or {})
        return out

    def defaultParamMap(self) -> dict[str, Any]:  # noqa: N802
        out = {}
        for p in self.params:
            v = self._default_of(p.name)
            if v is not NO_DEFAULT:
                out[p.name] = v
        return out

    def explainParam(self, name: str) -> str:  # noqa: N802
        p = self.getParam(name)
        parts = []
        if self._default_of(name) is not NO_DEFAULT:
            parts.append(f"default: {self._default_of(name)}")
        if name in self._paramMap:
            parts.append(f"current: {self._paramMap[name]}")
        extra = f" ({', '.join(parts)})" if parts else " (undefined)"
        return f"{name}: {p.doc}{extra}"

    def explainParams(self) -> str:  # noqa: N802
        return "\n".join(self.explainParam(p.name) for p in self.params)

    def copy(self, extra: dict | None = None) -> "Params":
        that = _copy.copy(self)
        that._paramMap = dict(self._paramMap)
        that._defaults = dict(getattr(self, "_defaults", {}))
        for k, v in (extra or {}).items():
            that._set(**{k: v})
        return that

    def _copyValues(self, to: "Params", extra: dict | None = None) -> "Params":  # noqa: N802
        for name, value in {**self._paramMap, **(extra or {})}.items():
            if to.hasParam(name):
                to._paramMap[name] = value
        return to
