"""ALS benchmark: implicit-feedback ALS, rank 100, synthetic ratings.

Each rank generates its shard of (user, item, count) triples (uniform users, power-law item
popularity), then runs the native ALS fit.  Reported: seconds per iteration (both halves:
Gramian + normal equations/Cholesky + factor allgather), setup (shuffle + CSR) separately.
Run: python benchmarks/bench_als.py [--gpus N] [--ratings N] [--users U] [--items I] [--rank R]
     [--iters K]
With --gpus N (N > 1) and no launcher environment the script starts N rank processes itself
(bench_common.self_launch).  The ratings are ONE global synthetic set for any N — fixed blocks of
2^22 triples, each drawn from its own generator, each rank taking its contiguous share — so N
changes only the sharding (strong scaling).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def gen_ratings(lo, hi, total, users, items, seed=1000, block=1 << 22):
    """Triples [lo, hi) of the global synthetic set: uniform users, power-law item popularity
    (a Pareto transform, ids scrambled), counts 1-5; block b drawn by default_rng([seed, b])."""
    import numpy as np

    u = np.empty(hi - lo, np.int32)
    it = np.empty(hi - lo, np.int32)
    r = np.empty(hi - lo, np.float32)
    for b in range(lo // block, (hi - 1) // block + 1 if hi > lo else lo // block):
        b0 = b * block
        n = min(block, total - b0)
        rng = np.random.default_rng([seed, b])
        bu = rng.integers(0, users, n, dtype=np.int32)
        bi = np.minimum((rng.pareto(1.2, n) * items / 50).astype(np.int64), items - 1)
        bi = ((bi * 2654435761) % items).astype(np.int32)
        br = rng.integers(1, 6, n).astype(np.float32)
        s0, s1 = max(lo, b0) - b0, min(hi, b0 + n) - b0
        u[b0 + s0 - lo:b0 + s1 - lo] = bu[s0:s1]
        it[b0 + s0 - lo:b0 + s1 - lo] = bi[s0:s1]
        r[b0 + s0 - lo:b0 + s1 - lo] = br[s0:s1]
    return u, it, r


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--ratings", type=int, default=1_000_000_000)
    ap.add_argument("--users", type=int, default=20_000_000)
    ap.add_argument("--items", type=int, default=2_000_000)
    ap.add_argument("--rank", type=int, default=100)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--alpha", type=float, default=40.0)
    ap.add_argument("--reg", type=float, default=0.01)
    ap.add_argument("--cpu-ratings", type=int, default=2_000_000,
                    help="ratings of the fp64 host-engine CPU-proxy baseline (0: skip)")
    ap.add_argument("--force-rccl", action="store_true",
                    help="1 GPU: a real 1-rank RCCL communicator (device shuffle, comm-stream "
                    "Gramian allreduce, chunked factor broadcasts) instead of the local comm")
    a = ap.parse_args(argv)
    from bench_common import init_world, self_launch, shard

    rc = self_launch(__file__, argv, a.gpus)
    if rc is not None:
        return rc
    sys.stdout.flush()
    out_fd = os.dup(1)  # (native banners go to stderr; stdout carries the one JSON line)
    os.dup2(2, 1)
    import numpy as np

    import oap_mllib_amd as O
    from oap_mllib_amd import _loader

    N = _loader.load()
    w = init_world(a.force_rccl)
    n_loc, r0 = shard(a.ratings, w.rank, w.size)
    t0 = time.time()
    u, it, r = gen_ratings(r0, r0 + n_loc, a.ratings, a.users, a.items)
    gen_s = time.time() - t0
    w.barrier()
    t0 = time.time()
    out = N.als_fit(w.ctx, w.comm, u, it, r, a.rank, a.iters, a.reg, a.alpha, True, 0)
    w.barrier()
    wall = time.time() - t0
    cpu = None
    if w.rank == 0 and a.cpu_ratings > 0:
        # labelled CPU proxy — the fp64 host engine on a ratings subsample of the
        # same generator (users and items scaled down with it), scaled to the full ratings
        from cpu_baseline import als_proxy

        m = min(a.cpu_ratings, n_loc)
        fu = max(1, int(a.users * m / a.ratings))
        fi = max(1, int(a.items * m / a.ratings))
        cpu = als_proxy(N, (u[:m] % fu).astype(np.int32), (it[:m] % fi).astype(np.int32), r[:m],
                        a.rank, a.alpha, a.reg, a.ratings)
    if w.rank == 0:
        it_ms = list(out["iter_ms"])
        steady = it_ms[1:] if len(it_ms) > 1 else it_ms
        os.write(out_fd, (json.dumps({
            "metric": "als_iteration_s", "value": sum(steady) / len(steady) / 1e3, "unit": "s",
            "n_gpus": w.size, "higher_is_better": False,
            # CPU-proxy seconds per iteration over the GPU's (extra.cpu_baseline)
            "vs_baseline": (cpu["s_per_iter_scaled"] / (sum(steady) / len(steady) / 1e3)
                            if cpu else None),
            "dtype": ("fp32 factors; Gramian: fp32 MFMA (rows <= 64 ratings), split-fp16 "
                      "hi+lo MFMA with fp32 accumulation (longer rows); fp32 Cholesky"),
            "data": "synthetic implicit counts (uniform users, power-law items)",
            "config": {"model": "als implicit rank %d" % a.rank, "ratings": int(out["nnz"]),
                       "users": len(out["user_ids"]), "items": len(out["item_ids"]),
                       "parallelism": "dp%d" % w.size},
            "extra": {"iter_ms": it_ms, "setup_s": out["setup_ms"] / 1e3,
                      "fit_wall_s": wall, "gram_ms_total": out["gram_ms"],
                      "solve_ms_total": out["solve_ms"], "comm_ms_total": out["comm_ms"],
                      "failed_rows": out["failed_rows"], "datagen_s": gen_s,
                      "comm": w.comm.name, "world_size": w.size,
                      # factor exchange (chunked owner broadcasts on the comm stream)
                      "factor_bcast_ms_total": out["bcast_ms"],
                      "factor_bcast_recv_bytes": out["bcast_recv_bytes"],
                      "factor_bcast_gbps": (out["bcast_recv_bytes"] / out["bcast_ms"] / 1e6
                                            if out["bcast_ms"] > 0 else None),
                      "cpu_baseline": cpu,
                      # (for the world-size tests: the fit's factors, summarised)
                      "user_factor_sum": float(np.abs(np.asarray(out["user_factors"])).sum()),
                      "item_factor_sum": float(np.abs(np.asarray(out["item_factors"])).sum()),
                      "factor_head": np.asarray(out["user_factors"])[
                          np.argsort(np.asarray(out["user_ids"]))[:3], :4].tolist()}})
                      + "\n").encode())
    O.shutdown_world()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
