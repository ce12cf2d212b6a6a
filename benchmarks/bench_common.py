"""Shared pieces of the benchmark scripts: the ``--gpus N`` self-launch (one rank per GPU, started
before anything in this process touches a GPU — the same pattern as bench.py) and the world
setup (``OAP_BENCH_DEVICE=cpu`` runs the CPU engine: the multi-rank rehearsal of the tests).
"""
from __future__ import annotations

import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def self_launch(script: str, argv: list[str], gpus: int):
    """With ``gpus > 1`` and no launcher environment: start ``gpus`` rank processes of
    ``script`` (oap_mllib_amd/parallel/launcher.py: LOCAL_RANK pinning, gang kill) and return
    their exit code; None when this process is a rank itself.  Loads the launcher by path so
    the package (and HIP) is not initialised in the parent."""
    if gpus > 1 and "WORLD_SIZE" not in os.environ:
        spec = importlib.util.spec_from_file_location(
            "_oap_launcher", os.path.join(ROOT, "oap_mllib_amd", "parallel", "launcher.py"))
        launcher = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(launcher)
        return launcher.launch([sys.executable, os.path.abspath(script)] + list(argv), gpus)
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws != gpus:
        print(f"--gpus {gpus} but WORLD_SIZE={ws}", file=sys.stderr)
        return 2
    return None


def init_world(force_rccl: bool = False):
    import oap_mllib_amd as O

    dev = os.environ.get("OAP_BENCH_DEVICE", "gpu")
    return O.init_world(O.get_config().replace(device=dev,
                                               force_device_comm=force_rccl and dev == "gpu"))


def shard(total: int, rank: int, size: int) -> tuple[int, int]:
    """(local count, global offset) of a contiguous near-equal split."""
    base, rem = divmod(total, size)
    return base + (1 if rank < rem else 0), rank * base + min(rank, rem)
