"""Process world: one rank per GPU, its native execution Context and its communicator.

Replaces the reference's per-fit oneCCL bootstrap (``OneCCL.init`` -> ``c_init`` ->
``ccl::create_main_kvs`` + ``create_communicator``, mllib-dal/src/main/native/OneCCL.cpp:47-86,
torn down again after every fit, KMeansDALImpl.scala:50,73) with a persistent per-process world:

* rank / size / local_rank come from the launcher environment (``RANK``, ``WORLD_SIZE``,
  ``LOCAL_RANK`` — torchrun, our own :mod:`oap_mllib_amd.parallel.launcher`, or Spark barrier
  tasks via :mod:`oap_mllib_amd.spark`);
* GPU pinning: rank -> ``LOCAL_RANK % visible_gpus`` (the executor->GPU pinning of the north star);
* control plane: ``torch.distributed`` gloo group (rendezvous over MASTER_ADDR/MASTER_PORT, no
  port scan / KVS race as in OneCCL.cpp:207-247);
* data plane: a native RCCL communicator (unique id broadcast over the control plane) for GPU
  ranks, or the gloo host communicator for CPU ranks.
"""
from __future__ import annotations

import atexit
import os
from dataclasses import dataclass, field
from typing import Any

import numpy as np

from .. import _loader
from ..config import Config, get_config


@dataclass
class World:
    rank: int
    size: int
    local_rank: int
    device: int  # -1 => CPU engine
    backend: str  # "gpu" | "cpu" | "vanilla"
    config: Config
    ctx: Any = None  # native Context (None for vanilla)
    comm: Any = None  # native Comm (None for vanilla)
    _owns_pg: bool = False
    _extra: dict = field(default_factory=dict)

    @property
    def is_gpu(self) -> bool:
        return self.backend == "gpu"

    @property
    def distributed(self) -> bool:
        return self.size > 1

    # ---- python-side collectives (used by vanilla fallbacks and API glue) -----------------
    def allreduce_np(self, arr: np.ndarray, op: str = "sum") -> np.ndarray:
        if self.size == 1:
            return arr
        import torch
        import torch.distributed as dist

        a = np.ascontiguousarray(arr).copy()
        t = torch.from_numpy(a)
        opmap = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}
        dist.all_reduce(t, opmap[op])
        return a

    def allgather_obj(self, obj):
        if self.size == 1:
            return [obj]
        import torch.distributed as dist

        out = [None] * self.size
        dist.all_gather_object(out, obj)
        return out

    def allgather_rows(self, arr: np.ndarray, counts: list[int]) -> np.ndarray:
        """Concatenates every rank's ``arr`` (``counts[r]`` leading rows on rank r, same trailing
        shape and dtype everywhere) in rank order: one typed all_gather of row slabs padded to
        the largest count — no pickling, so the bytes moved are the arrays' own."""
        if self.size == 1:
            return arr
        import torch
        import torch.distributed as dist

        a = np.ascontiguousarray(arr)
        assert len(a) == counts[self.rank], (len(a), counts)
        cap = max(max(counts), 1)
        tail = a.shape[1:]
        pad = np.zeros((cap,) + tail, dtype=a.dtype)
        pad[:len(a)] = a
        outs = [torch.empty((cap,) + tail, dtype=torch.from_numpy(pad).dtype)
                for _ in range(self.size)]
        dist.all_gather(outs, torch.from_numpy(pad))
        return np.concatenate([o.numpy()[:c] for o, c in zip(outs, counts)])

    def barrier(self) -> None:
        if self.size == 1:
            return
        if self.comm is not None:
            self.comm.barrier()
        else:
            import torch.distributed as dist

            dist.barrier()


_world: World | None = None


def _env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def _choose_backend(cfg: Config) -> tuple[str, int]:
    dev = cfg.device
    if dev == "vanilla":
        return "vanilla", -1
    if not _loader.available():
        if dev in ("gpu", "cpu"):
            _loader.load()  # raises with the build hint
        return "vanilla", -1
    n = _loader.load().visible_device_count()
    if dev == "gpu" and n == 0:
        raise RuntimeError("config.device='gpu' but no HIP device is visible")
    if dev in ("auto", "gpu") and n > 0:
        local = _env_int("LOCAL_RANK", 0)
        device = cfg.device_id if cfg.device_id >= 0 else local % n
        from ..utils.platform import check_platform_compatibility

        rep = check_platform_compatibility()
        if rep.gpu_ok(device):
            return "gpu", device
        if dev == "gpu":
            raise RuntimeError(f"config.device='gpu' but the platform check failed: {rep.reason}")
    return "cpu", -1


def init_world(config: Config | None = None, rank: int | None = None,
               size: int | None = None, local_rank: int | None = None) -> World:
    """Creates (or returns) the process world.  Idempotent."""
    global _world
    if _world is not None:
        return _world
    cfg = config or get_config()
    rank = _env_int("RANK", 0) if rank is None else rank
    size = _env_int("WORLD_SIZE", 1) if size is None else size
    local_rank = _env_int("LOCAL_RANK", rank) if local_rank is None else local_rank
    backend, device = _choose_backend(cfg)
    owns_pg = False
    if size > 1:
        import datetime

        import torch.distributed as dist

        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", cfg.rendezvous_host)
            if cfg.rendezvous_port:
                os.environ.setdefault("MASTER_PORT", str(cfg.rendezvous_port))
            dist.init_process_group(
                "gloo", rank=rank, world_size=size,
                timeout=datetime.timedelta(seconds=max(cfg.comm_timeout_s, 30.0)))
            owns_pg = True
    w = World(rank=rank, size=size, local_rank=local_rank, device=device, backend=backend,
              config=cfg, _owns_pg=owns_pg)
    if backend != "vanilla":
        N = _loader.load()
        N.clear_knobs()
        for name, value in (cfg.native_knobs or {}).items():
            N.set_knob(str(name), str(value))
        N.configure_logging(rank, device, cfg.log_level, cfg.log_file)
        w.ctx = N.Context(device, cfg.hbm_fraction, cfg.cpu_threads)
        if size == 1 and not (backend == "gpu" and cfg.force_device_comm):
            w.comm = N.LocalComm(backend == "gpu")
        elif size == 1:  # forced 1-rank RCCL world (the device-collective paths on one GPU)
            if not (cfg.use_rccl and N.rccl_available()):
                raise RuntimeError("force_device_comm needs RCCL (use_rccl and librccl)")
            w.comm = N.RcclComm(N.rccl_unique_id(), 1, 0, device, cfg.comm_timeout_s)
        elif backend == "gpu" and cfg.use_rccl and N.rccl_available():
            import torch.distributed as dist

            box = [N.rccl_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(box, src=0)
            w.comm = N.RcclComm(box[0], size, rank, device, cfg.comm_timeout_s)
        else:
            from .host_comm import TorchHostComm

            w.comm = N.HostComm(TorchHostComm(), rank, size)
    _world = w
    return w


def get_world() -> World:
    return _world if _world is not None else init_world()


def shutdown_world() -> None:
    """Releases native resources in a safe order (tables first, then comm, then context)."""
    global _world
    w = _world
    _world = None
    if w is None:
        return
    import gc

    w._extra.clear()
    w.comm = None
    gc.collect()
    if w.ctx is not None:
        try:
            w.ctx.sync()
        except Exception:
            pass
    w.ctx = None
    gc.collect()
    if w._owns_pg:
        try:
            import torch.distributed as dist

            if dist.is_initialized():
                dist.destroy_process_group()
        except Exception:
            pass


atexit.register(shutdown_world)
