#!/usr/bin/env python
"""Headline benchmark: K-Means Lloyd iterations, k=200, 100M x 50 dense fp32 (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W]            # 1 GPU
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N --steps K --warmup W

A "step" is one full Lloyd iteration of the distributed fit (every local row gets its exact
assignment: exact Hamerly bounds prove most labels unchanged, a 16-byte-per-row scan lists the
tiles that may change, the fused MFMA assign kernel runs on those and adds the moved rows' deltas
to the fixed-point statistics; then one RCCL allreduce of the full statistics + the finalize
kernel + the convergence read-back; the fit's final exact-cost pass over all rows is inside the
timed region) — nothing is skipped: tol=-1 disables the convergence exit, so exactly K
iterations run, and the centers are bitwise those of the unpruned fit (asserted below).
Scaling is STRONG: the global dataset is 100M rows for every N, each rank generating its own
contiguous shard directly in HBM (synthetic Gaussian blobs, identical values for any N).
--config kmeans_bf16 is BASELINE config #5: k=1000, 1B x 100 bf16 (208 GB of rows on one GPU —
the 288 GB HBM partition sizing case), same protocol.
The timed region is bracketed by a barrier + device synchronize on both sides and the MAX over
ranks is reported.  `value` is whole-job samples/s = global_rows * K / t.  The end-to-end fit()
wall clock (k-means|| init + Lloyd to convergence, maxIter=20) is reported alongside.
Other BASELINE configs: --config pca | als | kmeans_bf16 (see bench/).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np


def _barrier_sync(w):
    import torch

    if w.size > 1:
        w.barrier()
    if w.device >= 0:
        torch.cuda.set_device(w.device)  # sync (and create torch's context on) OUR GPU only
    torch.cuda.synchronize()
    if w.ctx is not None:
        w.ctx.sync()


def bench_kmeans(args, w):
    from oap_mllib_amd import _loader

    N = _loader.load()
    rows_total, d, k = args.rows, args.dim, args.k
    base, rem = divmod(rows_total, w.size)
    local = base + (1 if w.rank < rem else 0)
    row0 = w.rank * base + min(w.rank, rem)
    st = args.dtype
    ld = N.kmeans_ld(d, st)
    t_ing = time.time()
    table = N.synth_blobs(w.ctx, local, d, ld, row0, k, 10.0, 1.0, 20240917, st)
    table.set_global(row0, rows_total)
    _barrier_sync(w)
    ingest_s = time.time() - t_ing
    # initial centers: k-means|| (identical for any world size), untimed
    t0 = time.time()
    init = N.kmeans_init(w.ctx, w.comm, table, k, "k-means||", 2, 7)
    init_s = time.time() - t0
    # warmup iterations
    if args.warmup > 0:
        N.kmeans_fit(w.ctx, w.comm, table, init, k, args.warmup, -1.0)
    _barrier_sync(w)
    t0 = time.perf_counter()
    r = N.kmeans_fit(w.ctx, w.comm, table, init, k, args.steps, -1.0, precise=args.precise,
                     prune=not args.no_prune)
    _barrier_sync(w)
    el = time.perf_counter() - t0
    el_max = float(w.allreduce_np(np.array([el]), "max")[0])
    assert r["num_iter"] == args.steps, r["num_iter"]
    # the same timed run with every distance evaluated (no bound-based pruning), for reference
    ms_unpruned = None
    if not args.no_prune and not args.precise and not args.skip_unpruned:
        _barrier_sync(w)
        t2 = time.perf_counter()
        ru = N.kmeans_fit(w.ctx, w.comm, table, init, k, args.steps, -1.0, prune=False)
        _barrier_sync(w)
        el_u = float(w.allreduce_np(np.array([time.perf_counter() - t2]), "max")[0])
        ms_unpruned = el_u / args.steps * 1e3
        assert np.array_equal(ru["centers"], r["centers"]), "pruning changed the result"
    # end-to-end fit(): init + Lloyd to convergence (maxIter 20, tol 1e-4)
    fit_s = None
    if not args.skip_fit:
        _barrier_sync(w)
        t1 = time.perf_counter()
        rf = N.kmeans_fit(w.ctx, w.comm, table, None, k, 20, 1e-4, "k-means||", 2, 7)
        _barrier_sync(w)
        fit_s = float(w.allreduce_np(np.array([time.perf_counter() - t1]), "max")[0])
        fit_iters = rf["num_iter"]
    m = w.ctx.metrics()["phases"]
    ak = m.get("kmeans/assign_kernel", {"total_us": 0, "count": 1})
    ar = m.get("kmeans/allreduce", {"total_us": 0, "count": 1})
    itr = m.get("kmeans/iteration", {"total_us": 0, "count": 1})
    samples = rows_total * args.steps / el_max
    flops = 2.0 * rows_total * k * d
    out = {
        "metric": "kmeans_samples_per_sec", "value": samples, "unit": "samples/s",
        "n_gpus": w.size, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": el_max / args.steps * 1e3, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "fp32" if st == "f32" else "bf16",
        "data": "synthetic (gaussian blobs, on-device)",
        "config": {"model": f"kmeans k={k} d={d} (Lloyd, euclidean)", "global_batch": rows_total,
                   "seq_len": d, "parallelism": f"dp{w.size}", "k": k,
                   "rows": rows_total, "dim": d},
        "extra": {"fit_wall_s_end_to_end": fit_s,
                  "fit_iters": fit_iters if fit_s is not None else None,
                  "init_kmeans_parallel_s": init_s, "ingest_synth_s": ingest_s,
                  "init_phases_ms": {kk.split("/")[-1]: round(vv["total_us"] / 1e3, 1)
                                     for kk, vv in m.items() if kk.startswith("kmeans/init/")},
                  "assign_kernel_ms": ak["total_us"] / max(ak["count"], 1) / 1e3,
                  "allreduce_us": ar["total_us"] / max(ar["count"], 1),
                  # device time of one whole iteration minus assign and allreduce: finalize,
                  # the flag/count read-back and launch gaps
                  "iteration_rest_us": (itr["total_us"] / max(itr["count"], 1)
                                        - ak["total_us"] / max(ak["count"], 1)
                                        - ar["total_us"] / max(ar["count"], 1)),
                  # dense-equivalent rate (2 n k d flops per iteration over the timed wall
                  # clock); pruning and delta accumulation skip most of that work, so this is
                  # NOT the MFMA throughput (see ms_per_step_unpruned for the unpruned run)
                  "dense_equiv_tflops": flops / (el_max / args.steps) / 1e12,
                  "refine_tiles_per_iter": r["refine_tiles"] / max(args.steps, 1),
                  "tier3_tiles_per_iter": r["tier3_tiles"] / max(args.steps, 1),
                  # 32-row tile passes whose distance work the exact bounds skipped (pruning:
                  # labels provably unchanged; with delta accumulation their rows are not even
                  # read — only the 16-byte per-row bounds scan runs)
                  "pruned_tiles_per_iter": r.get("pruned_tiles", 0) / max(args.steps, 1),
                  "tiles_per_pass": (rows_total + 31) // 32,
                  "ms_per_step_unpruned": ms_unpruned,
                  "storage": st,
                  "distance_path": "fp32-exact MFMA" if args.precise else
                  ("tiered bf16 MFMA (1 product, then bf16x3 split where unsure) + exact-fp32 "
                   "refinement (assignments identical to fp32)"
                   if st == "f32" else "bf16 rows x bf16-split centroids on MFMA + exact-fp32 "
                   "refinement (assignments identical to exact fp32 on the bf16 data)"),
                  "cost": r["cost"]},
    }
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="kmeans", choices=["kmeans", "kmeans_bf16"],
                    help="kmeans: k=200, 100M x 50 f32 (headline); kmeans_bf16: k=1000, "
                    "1B x 100 bf16")
    ap.add_argument("--rows", type=int, default=None)
    ap.add_argument("--dim", type=int, default=None)
    ap.add_argument("--k", type=int, default=None)
    ap.add_argument("--skip-fit", action="store_true")
    ap.add_argument("--no-prune", action="store_true",
                    help="evaluate every distance (disable the exact bound-based pruning)")
    ap.add_argument("--skip-unpruned", action="store_true",
                    help="do not repeat the timed run without pruning for reference")
    ap.add_argument("--precise", action="store_true",
                    help="exact-fp32 MFMA distances only (no bf16-split fast path)")
    args = ap.parse_args(argv)
    preset = {"kmeans": (100_000_000, 50, 200, "f32"),
              "kmeans_bf16": (1_000_000_000, 100, 1000, "bf16")}[args.config]
    args.rows = args.rows or preset[0]
    args.dim = args.dim or preset[1]
    args.k = args.k or preset[2]
    args.dtype = preset[3]

    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and ws != args.gpus:
        print(f"--gpus {args.gpus} requires a launcher with WORLD_SIZE={args.gpus} "
              f"(python -m torch.distributed.run --nproc-per-node {args.gpus} bench.py ...)",
              file=sys.stderr)
        return 2
    import oap_mllib_amd as O

    w = O.init_world(O.get_config().replace(device="gpu"))
    out = bench_kmeans(args, w)
    if w.rank == 0:
        print(json.dumps(out), flush=True)
    O.shutdown_world()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
