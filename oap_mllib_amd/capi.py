"""ctypes view of ``liboap_mllib.so`` — the C ABI (csrc/capi/oap_capi.h) that the JNI shim and
other non-Python hosts use.  Mainly a test harness for that ABI: the Python API itself goes
through the pybind11 module.  The library is built in-tree by ``python -m oap_mllib_amd.build``.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

_LIB = None
UNIQUE_ID_BYTES = 128


def lib_path() -> Path:
    return Path(__file__).resolve().parent / "liboap_mllib.so"


def load() -> C.CDLL:
    global _LIB
    if _LIB is not None:
        return _LIB
    p = lib_path()
    if not p.exists():
        raise ImportError(f"{p} is missing: run python -m oap_mllib_amd.build")
    L = C.CDLL(str(p))
    dp, ip, i64 = C.POINTER(C.c_double), C.POINTER(C.c_int32), C.c_int64
    sig = {
        "oap_capi_version": (C.c_int, []),
        "oap_last_error": (C.c_char_p, []),
        "oap_device_count": (C.c_int, []),
        "oap_check_platform": (C.c_int, [C.c_int]),
        "oap_ctx_create": (C.c_void_p, [C.c_int, C.c_double, C.c_int]),
        "oap_ctx_destroy": (None, [C.c_void_p]),
        "oap_rccl_unique_id": (C.c_int, [C.c_char_p]),
        "oap_ctx_join": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int, C.c_int, C.c_double]),
        "oap_ctx_world_size": (C.c_int, [C.c_void_p]),
        "oap_ctx_rank": (C.c_int, [C.c_void_p]),
        "oap_kmeans_fit": (C.c_int, [C.c_void_p, dp, i64, C.c_int, dp, C.c_int, C.c_int,
                                     C.c_double, C.c_int, dp, dp, C.POINTER(C.c_int)]),
        "oap_kmeans_init": (C.c_int, [C.c_void_p, dp, i64, C.c_int, C.c_int, C.c_char_p,
                                      C.c_int, C.c_uint64, dp, C.POINTER(C.c_int)]),
        "oap_kmeans_predict": (C.c_int, [C.c_void_p, dp, i64, C.c_int, dp, C.c_int, ip, dp]),
        "oap_pca_fit": (C.c_int, [C.c_void_p, dp, i64, C.c_int, C.c_int, dp, dp]),
        "oap_als_fit": (C.c_int, [C.c_void_p, ip, ip, C.POINTER(C.c_float), i64, C.c_int, C.c_int,
                                  C.c_double, C.c_double, C.c_int, C.c_uint64,
                                  C.POINTER(C.c_void_p)]),
        "oap_als_result_count": (C.c_int64, [C.c_void_p, C.c_int]),
        "oap_als_result_rank": (C.c_int, [C.c_void_p]),
        "oap_als_result_ids": (ip, [C.c_void_p, C.c_int]),
        "oap_als_result_factors": (C.POINTER(C.c_float), [C.c_void_p, C.c_int]),
        "oap_als_result_free": (None, [C.c_void_p]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    _LIB = L
    return L


class NativeError(RuntimeError):
    pass


def _check(rc: int) -> None:
    if rc < 0:
        raise NativeError(load().oap_last_error().decode())


def _d(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class Context:
    """One device (``device >= 0``) or the native CPU engine (``device = -1``)."""

    def __init__(self, device: int = -1, hbm_fraction: float = 0.5, cpu_threads: int = 0):
        L = load()
        self._h = L.oap_ctx_create(device, hbm_fraction, cpu_threads)
        if not self._h:
            raise NativeError(L.oap_last_error().decode())

    def close(self) -> None:
        if self._h:
            load().oap_ctx_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def join(self, unique_id: bytes, world: int, rank: int, timeout_s: float = 600.0) -> None:
        _check(load().oap_ctx_join(self._h, unique_id, world, rank, timeout_s))

    @property
    def world_size(self) -> int:
        return load().oap_ctx_world_size(self._h)

    def kmeans_fit(self, X, init_centers, max_iter=20, tol=1e-4, bf16=False):
        X = np.ascontiguousarray(X, dtype=np.float64)
        c0 = np.ascontiguousarray(init_centers, dtype=np.float64)
        k, d = c0.shape
        out = np.zeros((k, d))
        cost, iters = C.c_double(), C.c_int()
        _check(load().oap_kmeans_fit(self._h, _d(X), X.shape[0], d, _d(c0), k, max_iter, tol,
                                     int(bf16), _d(out), C.byref(cost), C.byref(iters)))
        return out, cost.value, iters.value

    def kmeans_init(self, X, k, mode="k-means||", steps=2, seed=1):
        X = np.ascontiguousarray(X, dtype=np.float64)
        out = np.zeros((k, X.shape[1]))
        keff = C.c_int()
        _check(load().oap_kmeans_init(self._h, _d(X), X.shape[0], X.shape[1], k, mode.encode(),
                                      steps, seed, _d(out), C.byref(keff)))
        return out[: keff.value]

    def kmeans_predict(self, X, centers):
        X = np.ascontiguousarray(X, dtype=np.float64)
        c = np.ascontiguousarray(centers, dtype=np.float64)
        lab = np.zeros(X.shape[0], dtype=np.int32)
        d2 = np.zeros(X.shape[0])
        _check(load().oap_kmeans_predict(self._h, _d(X), X.shape[0], X.shape[1], _d(c), c.shape[0],
                                         lab.ctypes.data_as(C.POINTER(C.c_int32)), _d(d2)))
        return lab, d2

    def pca_fit(self, X, k):
        X = np.ascontiguousarray(X, dtype=np.float64)
        pc = np.zeros((X.shape[1], k))
        ev = np.zeros(k)
        _check(load().oap_pca_fit(self._h, _d(X), X.shape[0], X.shape[1], k, _d(pc), _d(ev)))
        return pc, ev

    def als_fit(self, users, items, ratings, rank=10, max_iter=10, reg=0.1, alpha=1.0,
                implicit=True, seed=0):
        L = load()
        u = np.ascontiguousarray(users, dtype=np.int32)
        i = np.ascontiguousarray(items, dtype=np.int32)
        r = np.ascontiguousarray(ratings, dtype=np.float32)
        h = C.c_void_p()
        _check(L.oap_als_fit(self._h, u.ctypes.data_as(C.POINTER(C.c_int32)),
                             i.ctypes.data_as(C.POINTER(C.c_int32)),
                             r.ctypes.data_as(C.POINTER(C.c_float)), len(u), rank, max_iter, reg,
                             alpha, int(implicit), seed, C.byref(h)))
        try:
            out = {}
            rk = L.oap_als_result_rank(h)
            for which, name in ((0, "user"), (1, "item")):
                n = L.oap_als_result_count(h, which)
                ids = np.ctypeslib.as_array(L.oap_als_result_ids(h, which), (n,)).copy() \
                    if n else np.zeros(0, np.int32)
                f = np.ctypeslib.as_array(L.oap_als_result_factors(h, which), (n * rk,)).copy() \
                    if n else np.zeros(0, np.float32)
                out[name + "_ids"], out[name + "_factors"] = ids, f.reshape(n, rk)
            return out
        finally:
            L.oap_als_result_free(h)


def rccl_unique_id() -> bytes:
    buf = C.create_string_buffer(UNIQUE_ID_BYTES)
    _check(load().oap_rccl_unique_id(buf))
    return buf.raw
