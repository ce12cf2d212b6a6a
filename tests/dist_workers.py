"""Worker functions executed inside multi-process test worlds (see mp_util.run_world)."""
import os

import numpy as np


def _blobs(n, d, k, seed, sigma=1.0):
    rng = np.random.default_rng(seed)
    c = rng.uniform(-10, 10, size=(k, d))
    return c[rng.integers(0, k, n)] + rng.normal(0, sigma, size=(n, d))


def _shard(X, rank, world):
    base, rem = divmod(len(X), world)
    lo = rank * base + min(rank, rem)
    return X[lo: lo + base + (1 if rank < rem else 0)]


def kmeans_native(n=4000, d=6, k=5, seed=7, device="cpu", use_rccl=True, init_mode="k-means||",
                  device_id=0):
    import oap_mllib_amd as O

    w = O.init_world(O.get_config().replace(device=device, use_rccl=use_rccl,
                                             device_id=device_id))
    X = _blobs(n, d, k, seed)
    local = _shard(X, w.rank, w.size)
    m = O.KMeans(k=k, seed=seed, maxIter=25, initMode=init_mode).fit(local)
    out = {"rank": w.rank, "size": w.size, "engine": m.fit_info["engine"],
           "comm": w.comm.name if w.comm is not None else None,
           "centers": np.array(m.clusterCenters()).tolist(), "cost": m.trainingCost,
           "iters": m.numIter}
    O.shutdown_world()
    return out


def kmeans_uneven(n=200000, d=16, k=20, seed=11, sigma=3.0, max_iter=12, tol=0.0,
                  empty_rank=-1, no_image_rank=-1, device="gpu", use_rccl=False):
    """Ranks that differ in what the row scan needs: one rank without rows (empty_rank) or one
    without the fp16 operand image (no_image_rank: OAP_KMEANS_IMAGE=0 there), with tol >= 0 (the
    batched form: a converged iteration halts the rest of its batch on the device) — every
    per-batch collective must pair up across ranks."""
    import oap_mllib_amd as O
    from oap_mllib_amd import _loader

    if no_image_rank >= 0 and int(os.environ.get("RANK", "0")) == no_image_rank:
        os.environ["OAP_KMEANS_IMAGE"] = "0"
    N = _loader.load()
    w = O.init_world(O.get_config().replace(device=device, use_rccl=use_rccl))
    X = _blobs(n, d, k, seed, sigma).astype(np.float32)
    if w.size == 1:
        local = X
    elif w.rank == empty_rank:
        local = X[:0]
    else:
        rest = [r for r in range(w.size) if r != empty_rank]
        local = _shard(X, rest.index(w.rank), len(rest))
    init = X[np.random.default_rng(seed).choice(n, k, replace=False)].astype(np.float64)
    t = N.upload_dense(w.ctx, np.ascontiguousarray(local), "f32", N.kmeans_ld(d))
    r = N.kmeans_fit(w.ctx, w.comm, t, init.ravel(), k, max_iter, tol)
    out = {"rank": w.rank, "centers": np.asarray(r["centers"]).tolist(), "cost": r["cost"],
           "iters": r["num_iter"], "comm": w.comm.name if w.comm is not None else None}
    del t
    O.shutdown_world()
    return out


def kmeans_vanilla(n=2000, d=4, k=3, seed=3):
    import oap_mllib_amd as O

    w = O.init_world(O.get_config().replace(device="vanilla"))
    X = _blobs(n, d, k, seed)
    local = _shard(X, w.rank, w.size)
    init = X[:k]
    from oap_mllib_amd.fallback import kmeans_vanilla as V

    r = V.fit(local, k, 10, 0.0, init_centers=init, allreduce=lambda a: w.allreduce_np(a))
    O.shutdown_world()
    return {"centers": r.centers.tolist(), "cost": r.cost}


def fault_injection(device="cpu"):
    """Rank 1 raises at iteration 0; rank 0 must not hang (gloo timeout / error)."""
    import oap_mllib_amd as O

    w = O.init_world(O.get_config().replace(device=device, comm_timeout_s=30.0))
    X = _shard(_blobs(2000, 4, 3, 1), w.rank, w.size)
    try:
        O.KMeans(k=3, seed=1, maxIter=10, tol=0.0).fit(X)
        status = "finished"
    except Exception as e:  # noqa: BLE001
        status = type(e).__name__
    os._exit(3 if status != "finished" else 0)


def host_comm_collectives():
    """Exercises every HostComm collective through the native layer."""
    import oap_mllib_amd as O
    from oap_mllib_amd import _loader

    N = _loader.load()
    w = O.init_world(O.get_config().replace(device="cpu"))
    a = np.arange(5, dtype=np.float64) * (w.rank + 1)
    w.comm.allreduce_f64(w.ctx, a, "sum")
    b = np.array([float(w.rank)])
    w.comm.allreduce_f64(w.ctx, b, "max")
    t = N.upload_dense(w.ctx, np.ones((3 + w.rank, 2)), "f64", 2)
    N.assign_global_offsets(w.ctx, w.comm, t)
    out = {"sum": a.tolist(), "max": b.tolist(), "offset": t.global_offset,
           "total": t.global_rows}
    O.shutdown_world()
    return out


def pca_native(n=3000, d=12, k=4, seed=5, device="cpu", use_rccl=True, device_id=0):
    import oap_mllib_amd as O

    w = O.init_world(O.get_config().replace(device=device, use_rccl=use_rccl,
                                             device_id=device_id))
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, d)) @ rng.normal(size=(d, d)) + 50.0
    local = _shard(X, w.rank, w.size)
    m = O.PCA(k=k, inputCol="features").fit(local)
    out = {"rank": w.rank, "engine": m.fit_info["engine"], "pc": m.pc.toArray().tolist(),
           "ev": m.explainedVariance.toArray().tolist()}
    O.shutdown_world()
    return out


def als_native(seed=3, device="cpu", use_rccl=True, rank=3, device_id=0, implicit=True,
               nonnegative=False):
    import oap_mllib_amd as O
    from test_als import gen_implicit

    w = O.init_world(O.get_config().replace(device=device, use_rccl=use_rccl,
                                             device_id=device_id))
    tr, _ = gen_implicit(30, 50, 2, 0.01, seed)
    mine = {k: v[w.rank::w.size] for k, v in tr.items()}  # a strided (non-range) partition
    if w.distributed:  # the native path never gathers the ratings (only the vanilla one did)
        w.allgather_obj = None
    m = O.ALS(rank=rank, maxIter=4, regParam=0.01, implicitPrefs=implicit, seed=0,
              nonnegative=nonnegative).fit(mine)
    out = {"engine": m.fit_info["engine"], "uid": m.userFactors["id"].tolist(),
           "uf": np.stack(m.userFactors["features"].to_list()).tolist(),
           "if": np.stack(m.itemFactors["features"].to_list()).tolist()}
    O.shutdown_world()
    return out


def recommend_sharded(n=301, m=57, rank=6, num=7, seed=9):
    """recommendForAllUsers on a 2-rank CPU world: each rank scores its own slab of users (the
    local top-k sees only its rows), then the slabs are allgathered in rank order."""
    import oap_mllib_amd as O
    from oap_mllib_amd.models import recommendation as rec

    w = O.init_world(O.get_config().replace(device="cpu"))
    rng = np.random.default_rng(seed)
    U = rng.normal(size=(n, rank)).astype(np.float32)
    V = rng.normal(size=(m, rank)).astype(np.float32)
    seen = []
    local = rec._local_topk

    def spy(S, D, k, world, block):
        seen.append(len(S))
        return local(S, D, k, world, block)

    rec._local_topk = spy
    try:
        idx, val = rec._blocked_topk(U, V, num)
    finally:
        rec._local_topk = local
    model = O.ALSModel(rank=rank, user_arrays=(np.arange(n), U), item_arrays=(np.arange(m), V))
    first = [r[0]["item"] for r in model.recommendForAllUsers(num)["recommendations"].tolist()]
    out = {"rank": w.rank, "rows_scored": seen, "idx": idx.tolist(), "val": val.tolist(),
           "first": first}
    O.shutdown_world()
    return out


def recommend_subset(n=120, m=40, rank=5, num=6, seed=4):
    """recommendForUserSubset with a DIFFERENT subset on each rank (each rank's own dataset
    shard): every rank gets the recommendations of its own users, computed locally."""
    import pandas as pd

    import oap_mllib_amd as O

    w = O.init_world(O.get_config().replace(device="cpu"))
    rng = np.random.default_rng(seed)
    U = rng.normal(size=(n, rank)).astype(np.float32)
    V = rng.normal(size=(m, rank)).astype(np.float32)
    model = O.ALSModel(rank=rank, user_arrays=(np.arange(n), U), item_arrays=(np.arange(m), V))
    mine = np.arange(w.rank, n, 7 + w.rank)  # uneven subsets, different sizes per rank
    out = model.recommendForUserSubset(pd.DataFrame({"user": mine}), num)
    recs = {int(u): [int(r["item"]) for r in rs] for u, rs in
            zip(out["user"].tolist(), out["recommendations"].tolist())}
    O.shutdown_world()
    return {"rank": w.rank, "users": mine.tolist(), "recs": {str(k): v for k, v in recs.items()}}


def tcp_alltoallv(port, piece=0):
    """Uneven alltoallv / allreduce / allgather over the KVS TcpComm (streamed star routing);
    piece > 0 forces several forwarding pieces per segment."""
    import numpy as np

    from oap_mllib_amd import _loader

    if piece:
        os.environ["OAP_TCP_PIECE_BYTES"] = str(piece)
    N = _loader.load()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    comm = N.TcpComm(f"127.0.0.1_{port}", world, rank, 60.0)
    ctx = N.Context(-1, 0.5, 1)

    def cnt(p, q):  # elements p sends q (uneven, some empty)
        return 0 if (p + q) % 4 == 3 else (p + 1) * (q + 2) * 7 + (5 if p == q else 0)

    def seg(p, q):
        return p * 1e6 + q * 1e3 + np.arange(cnt(p, q), dtype=np.float64)

    send = [cnt(rank, q) for q in range(world)]
    recv = [cnt(p, rank) for p in range(world)]
    data = np.concatenate([seg(rank, q) for q in range(world)])
    out = comm.exchange_f64(ctx, "alltoallv", data, send, recv)
    want = np.concatenate([seg(p, rank) for p in range(world)])
    red = comm.exchange_f64(ctx, "allreduce", np.full(5, float(rank + 1)))
    gat = comm.exchange_f64(ctx, "allgather", np.array([float(rank)]))
    return {"a2a": bool(np.array_equal(out, want)),
            "allreduce": bool(np.all(red == world * (world + 1) / 2)),
            "allgather": gat.tolist() == [float(p) for p in range(world)]}
