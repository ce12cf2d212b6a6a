"""Array-level ops on torch tensors: the MI355X kernels without the Spark-style estimator layer.

GPU tensors are used in place (zero-copy table views over ``tensor.data_ptr()``; a padded copy is
made only when the row stride does not match the kernel layout), outputs are device tensors, and
every op orders itself after torch's current stream and finishes its own stream before returning.
CPU tensors (or a process without a GPU world) go through the native CPU engine.  All ops run on
the process world (``oap_mllib_amd.init_world``): with several ranks, every rank passes its own
row shard and collective ops (``kmeans_fit``, ``pca``) return the global result on every rank.

    import torch, oap_mllib_amd.ops as ops
    x = torch.randn(10_000_000, 50, device="cuda")
    centers, cost, iters = ops.kmeans_fit(x, k=200)
    labels, dist2 = ops.kmeans_assign(x, centers)     # int32 / float32 tensors on x.device
    pc, explained = ops.pca(x, k=10)
"""
from __future__ import annotations

import numpy as np

from .. import _loader

__all__ = ["kmeans_assign", "kmeans_fit", "pca"]


def _torch():
    import torch

    return torch


def _world():
    from ..parallel.world import get_world

    return get_world()


def _on_world_gpu(x, w) -> bool:
    return bool(getattr(x, "is_cuda", False)) and w.is_gpu and x.device.index in (None, w.device)


def _view(x, w, layout: str):
    """Zero-copy native table over a 2-D GPU tensor (padded copy if the stride does not fit).
    Returns (table, keepalive tensor)."""
    torch = _torch()
    N = _loader.load()
    if x.dim() != 2:
        raise ValueError(f"expected a 2-D tensor, got shape {tuple(x.shape)}")
    n, d = x.shape
    if x.dtype == torch.bfloat16 and layout == "kmeans":
        dt = "bf16"
    elif x.dtype == torch.float32:
        dt = "f32"
    else:
        x, dt = x.float(), "f32"
    ld = N.kmeans_ld(d, dt) if layout == "kmeans" else (d + 3) // 4 * 4
    # zero-copy only when the row IS the kernel layout: with ld > d the kernels read columns
    # [d, ld) as zero padding, and a column-sliced view would have real data there
    ok = (ld == d and x.stride(1) == 1 and x.stride(0) == ld and x.data_ptr() % 16 == 0)
    if not ok:
        xp = torch.zeros((n, ld), dtype=x.dtype, device=x.device)
        xp[:, :d] = x
        x = xp
    torch.cuda.current_stream(x.device).synchronize()  # producers of x are done
    t = N.table_view(w.ctx, x.data_ptr(), n, d, ld, dt)
    return t, x


def _host_table(x, w, layout: str):
    N = _loader.load()
    a = np.ascontiguousarray(x.detach().cpu().double().numpy() if hasattr(x, "detach") else x,
                             dtype=np.float64)
    from ..models.clustering import upload_table

    return upload_table(w, a, layout)


def kmeans_assign(x, centers):
    """Nearest center (Euclidean) per row: ``(labels int32, squared distances float32)`` on
    ``x``'s device.  Assignments equal an exact fp32 evaluation (tiered MFMA + refinement)."""
    torch = _torch()
    N = _loader.load()
    w = _world()
    c = np.ascontiguousarray(
        centers.detach().cpu().double().numpy() if hasattr(centers, "detach") else centers,
        dtype=np.float64)
    if _on_world_gpu(x, w):
        t, keep = _view(x, w, "kmeans")
        labels = torch.empty(x.shape[0], dtype=torch.int32, device=x.device)
        dist = torch.empty(x.shape[0], dtype=torch.float32, device=x.device)
        N.kmeans_predict_device(w.ctx, t, c, labels.data_ptr(), dist.data_ptr())
        del keep
        return labels, dist
    table = _host_table(x, w, "kmeans")
    lab, d2 = N.kmeans_predict(w.ctx, table, c)
    dev = getattr(x, "device", "cpu")
    return (torch.as_tensor(lab, dtype=torch.int32, device=dev),
            torch.as_tensor(d2, dtype=torch.float32, device=dev))


def kmeans_fit(x, k: int | None = None, init_centers=None, max_iter: int = 20,
               tol: float = 1e-4, seed: int = 1, init_mode: str = "k-means||",
               init_steps: int = 2):
    """Lloyd's algorithm on this rank's rows.  Returns ``(centers float64 [k, d] CPU tensor,
    cost, iterations)``; ``init_centers`` (k x d) or ``k`` with k-means|| / random init."""
    torch = _torch()
    N = _loader.load()
    w = _world()
    if init_centers is None and k is None:
        raise ValueError("give k or init_centers")
    init = None
    if init_centers is not None:
        init = np.ascontiguousarray(
            init_centers.detach().cpu().double().numpy() if hasattr(init_centers, "detach")
            else init_centers, dtype=np.float64)
        k = init.shape[0]
    keep = None
    if _on_world_gpu(x, w):
        table, keep = _view(x, w, "kmeans")
    else:
        table = _host_table(x, w, "kmeans")
    r = N.kmeans_fit(w.ctx, w.comm, table, init, int(k), max_iter, tol, init_mode, init_steps,
                     seed)
    del keep
    return torch.as_tensor(np.asarray(r["centers"])), float(r["cost"]), int(r["num_iter"])


def pca(x, k: int, precise: bool = False):
    """Top-k principal components of the (globally) mean-centred rows: ``(pc float64 [d, k],
    explained variance [k])`` as CPU tensors (Spark PCA semantics)."""
    torch = _torch()
    N = _loader.load()
    w = _world()
    keep = None
    if _on_world_gpu(x, w):
        table, keep = _view(x, w, "pca")
    else:
        table = _host_table(x, w, "pca")
    r = N.pca_fit(w.ctx, w.comm, table, int(k), precise)
    del keep
    return (torch.as_tensor(np.asarray(r["pc"])),
            torch.as_tensor(np.asarray(r["explained_variance"])))
