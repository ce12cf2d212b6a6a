"""Platform compatibility check — the counterpart of the reference's
``Utils.checkClusterPlatformCompatibility`` (mllib-dal/src/main/scala/org/apache/spark/ml/util/
Utils.scala:98-132), which gated every accelerated path on CPU features.  Here the native
kernels are compiled for gfx950 (MI355X) only, so the GPU engine is eligible iff the native
extension loads and the selected device reports a gfx950 architecture; otherwise the native
CPU engine (or the vanilla path) is used.
"""
from __future__ import annotations

from dataclasses import dataclass, field

from .. import _loader

SUPPORTED_ARCH = "gfx950"


@dataclass
class PlatformReport:
    native: bool = False
    devices: list = field(default_factory=list)  # [(index, name, arch)]
    rccl: bool = False
    reason: str = ""

    def gpu_ok(self, device: int = 0) -> bool:
        return self.native and any(i == device and a.split(":")[0] == SUPPORTED_ARCH
                                   for i, _, a in self.devices)


_cache: PlatformReport | None = None


def check_platform_compatibility(refresh: bool = False) -> PlatformReport:
    global _cache
    if _cache is not None and not refresh:
        return _cache
    rep = PlatformReport()
    if not _loader.available():
        rep.reason = "native extension not built"
        _cache = rep
        return rep
    N = _loader.load()
    rep.native = True
    rep.rccl = bool(N.rccl_available())
    n = N.visible_device_count()
    if n:
        import torch

        for i in range(n):
            p = torch.cuda.get_device_properties(i)
            rep.devices.append((i, p.name, getattr(p, "gcnArchName", "")))
    if not rep.devices:
        rep.reason = "no HIP device visible"
    elif not any(a.split(":")[0] == SUPPORTED_ARCH for _, _, a in rep.devices):
        rep.reason = f"no {SUPPORTED_ARCH} device (found {[a for _, _, a in rep.devices]})"
    _cache = rep
    return rep
