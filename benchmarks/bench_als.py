"""ALS benchmark: implicit-feedback ALS, rank 100, synthetic ratings.

Each rank generates its shard of (user, item, count) triples (uniform users, power-law item
popularity), then runs the native ALS fit.  Reported: seconds per iteration (both halves:
Gramian + normal equations/Cholesky + factor allgather), setup (shuffle + CSR) separately.
Run: python benchmarks/bench_als.py [--ratings N] [--users U] [--items I] [--rank R] [--iters K]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
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
    a = ap.parse_args()
    import numpy as np

    import oap_mllib_amd as O
    from oap_mllib_amd import _loader

    N = _loader.load()
    w = O.init_world(O.get_config().replace(device="gpu", force_device_comm=a.force_rccl))
    n_loc = a.ratings // w.size + (1 if w.rank < a.ratings % w.size else 0)
    t0 = time.time()
    rng = np.random.default_rng(1000 + w.rank)
    u = rng.integers(0, a.users, n_loc, dtype=np.int32)
    # power-law item popularity (Zipf-like via a Pareto transform), ids scrambled
    it = np.minimum((rng.pareto(1.2, n_loc) * a.items / 50).astype(np.int64), a.items - 1)
    it = ((it * 2654435761) % a.items).astype(np.int32)
    r = rng.integers(1, 6, n_loc).astype(np.float32)
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
        print(json.dumps({
            "metric": "als_iteration_s", "value": sum(steady) / len(steady) / 1e3, "unit": "s",
            "n_gpus": w.size, "higher_is_better": False,
            # CPU-proxy seconds per iteration over the GPU's (extra.cpu_baseline)
            "vs_baseline": (cpu["s_per_iter_scaled"] / (sum(steady) / len(steady) / 1e3)
                            if cpu else None),
            "dtype": ("fp32 factors; Gramian: fp32 MFMA (rows <= 64 ratings), split-fp16 "
                      "hi+lo MFMA with fp32 accumulation (longer rows); fp32 Cholesky"),
            "data": "synthetic implicit counts (uniform users, power-law items)",
            "config": {"model": "als implicit rank %d" % a.rank, "ratings": int(out["nnz"]),
                       "users": len(out["user_ids"]), "items": len(out["item_ids"])},
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
                      "cpu_baseline": cpu}}))
    O.shutdown_world()


if __name__ == "__main__":
    main()
