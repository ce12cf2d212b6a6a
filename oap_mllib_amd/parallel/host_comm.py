"""Host-buffer collectives over ``torch.distributed`` (gloo) for the native engine.

An instance is wrapped by the native ``HostComm`` class: C++ drivers call back into
``allreduce/allgather/alltoallv/bcast/barrier`` with numpy views of their host buffers.  This is
the CPU path (and the fallback for GPU ranks when RCCL is unavailable, staged through pinned
memory by the native layer).  It plays the role the reference gives oneCCL-over-OFI-sockets
(mllib-dal/src/main/native/OneCCL.cpp:47-86), without serialised archives: every
call moves typed arrays in place.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

_OPS = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}


def _t(a: np.ndarray) -> torch.Tensor:
    if a.dtype == np.uint16:  # bf16 payloads travel as raw int16 bits (sum is not meaningful)
        return torch.from_numpy(a.view(np.int16))
    return torch.from_numpy(a)


class TorchHostComm:
    """Collectives on numpy arrays through the default torch.distributed process group."""

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)

    def allreduce(self, arr: np.ndarray, op: str = "sum") -> None:
        # int64 sums wrap around (two's complement), exactly what the fixed-point
        # centroid accumulators of the K-Means driver rely on
        dist.all_reduce(_t(arr), _OPS[op], group=self.group)

    def allgather(self, send: np.ndarray, recv: np.ndarray) -> None:
        s = _t(send)
        parts = list(_t(recv).chunk(self.world))
        dist.all_gather(parts, s.clone(), group=self.group)

    def alltoallv(self, send: np.ndarray, send_counts, recv: np.ndarray, recv_counts) -> None:
        s, r = _t(send), _t(recv)
        # every rank participates even with empty splits, so peers never hang
        dist.all_to_all_single(r, s, output_split_sizes=list(map(int, recv_counts)),
                               input_split_sizes=list(map(int, send_counts)), group=self.group)

    def bcast(self, arr: np.ndarray, root: int) -> None:
        dist.broadcast(_t(arr), src=root, group=self.group)

    def barrier(self) -> None:
        dist.barrier(group=self.group)
