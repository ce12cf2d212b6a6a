"""Loads the native engine (``_native*.so``) built in-tree by :mod:`oap_mllib_amd.build`.

torch is imported first on purpose: the extension links ``libamdhip64.so.7`` / ``librccl.so.1``
by SONAME, so with torch already loaded it binds to torch's copies and the process keeps ONE HIP
runtime (two runtimes in one process would not share device pointers).

The reference loads its natives by extracting ``.so`` files from the jar into a temp dir and
``System.load``-ing them in dependency order (mllib-dal/src/main/java/org/apache/spark/ml/util/
LibLoader.java:47-73); here the module sits in the package and is imported normally.  If it is
missing on a machine that HAS a GPU, importing raises — GPU code paths never silently fall back
to Python.
"""
from __future__ import annotations

import importlib
import os

import torch  # noqa: F401  (must precede the native import, see module docstring)

_native = None
_error: Exception | None = None


def _gpu_present() -> bool:
    try:
        return torch.cuda.device_count() > 0
    except Exception:  # pragma: no cover - driver probing failure
        return False


def load():
    """Returns the native module, raising ImportError when it is unavailable."""
    global _native, _error
    if _native is not None:
        return _native
    if _error is not None:
        raise ImportError(str(_error))
    try:
        _native = importlib.import_module("oap_mllib_amd._native")
        return _native
    except ImportError as e:  # pragma: no cover - exercised only on broken installs
        _error = ImportError(
            f"oap_mllib_amd native engine not built ({e}); run `python -m oap_mllib_amd.build`")
        raise _error


def available() -> bool:
    try:
        load()
        return True
    except ImportError:
        return False


def require_on_gpu_hosts() -> None:
    """Fails loudly when a GPU is visible but the native engine is missing."""
    if _gpu_present() and not available() and not os.environ.get("OAP_MLLIB_ALLOW_NO_NATIVE"):
        raise ImportError(str(_error))
