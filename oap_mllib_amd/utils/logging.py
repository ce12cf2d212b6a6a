"""Python-side structured logging that shares the native logger's JSON-lines format.

The reference logs through Spark ``logInfo`` and ``Instrumentation`` on the JVM side and raw
``cout`` in the natives (KMeansDALImpl.scala:89-95, KMeansDALImpl.cpp:202-222).  Here both sides
emit one JSON object per line (rank, device, phase, µs, bytes...).  ``Instrumentation`` mirrors
Spark's ``instr.logParams / logNamedValue`` fields (numIter, cost, clusterSizes...).
"""
from __future__ import annotations

import json
import logging
import os
import sys
import time
from typing import Any


class _JsonFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        payload = {"ts_us": int(record.created * 1e6), "rank": int(os.environ.get("RANK", 0)),
                   "level": record.levelname.lower(), "phase": record.name}
        extra = getattr(record, "fields", None)
        if extra:
            payload.update(extra)
        msg = record.getMessage()
        if msg:
            payload["msg"] = msg
        return json.dumps(payload, default=str)


def get_logger(name: str) -> logging.Logger:
    lg = logging.getLogger(name)
    if not lg.handlers and not logging.getLogger("oap_mllib_amd").handlers:
        root = logging.getLogger("oap_mllib_amd")
        h = logging.StreamHandler(sys.stderr)
        h.setFormatter(_JsonFormatter())
        root.addHandler(h)
        root.setLevel(os.environ.get("OAP_MLLIB_LOG_LEVEL", "warn").upper().replace("WARN",
                                                                                     "WARNING"))
        root.propagate = False
    return lg


class Instrumentation:
    """Spark-``Instrumentation``-style record of one fit (params, named values, timings)."""

    def __init__(self, estimator: Any):
        self.estimator = type(estimator).__name__
        self.uid = getattr(estimator, "uid", "")
        self.values: dict[str, Any] = {}
        self.t0 = time.time()
        self._log = get_logger(f"oap_mllib_amd.instr.{self.estimator}")

    def logParams(self, params: dict) -> None:  # noqa: N802
        self.values["params"] = {k: v for k, v in params.items()}

    def logNamedValue(self, name: str, value: Any) -> None:  # noqa: N802
        self.values[name] = value

    def logNumFeatures(self, n: int) -> None:  # noqa: N802
        self.values["numFeatures"] = int(n)

    def logNumExamples(self, n: int) -> None:  # noqa: N802
        self.values["numExamples"] = int(n)

    def finish(self) -> dict:
        self.values["fit_seconds"] = time.time() - self.t0
        self._log.info("", extra={"fields": {"uid": self.uid, **self.values}})
        return self.values
