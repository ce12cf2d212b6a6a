#!/usr/bin/env python
"""Headline benchmark: K-Means Lloyd iterations, k=200, 100M x 50 dense fp32 (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W]

With ``--gpus N`` (N > 1) and no launcher environment, bench.py starts N rank processes itself
(oap_mllib_amd/parallel/launcher.py: one process per GPU, LOCAL_RANK pinning, gang kill) before
anything touches a GPU; under ``torchrun`` / ``torch.distributed.run`` it uses the given world.
Every rank forms the RCCL communicator; the JSON reports the world it actually formed
(``extra.comm``, ``extra.rccl_ranks``).

A "step" is one full Lloyd iteration of the distributed fit (every local row gets its exact
assignment: exact Hamerly bounds prove some labels unchanged, a 16-byte-per-row scan lists the
tiles that may change, the fused MFMA assign kernel runs on those and adds the moved rows' deltas
to the fixed-point statistics; then one RCCL allreduce of the full statistics + the finalize
kernel + the convergence read-back; the fit's final exact-cost pass over all rows is inside the
timed region) — nothing is skipped: tol=-1 disables the convergence exit, so exactly K
iterations run, and the centers are bitwise those of the unpruned fit (asserted below).

Data regime (the headline ``value``): synthetic Gaussian blobs whose per-cluster spread is
comparable to the distance between cluster centers (--sigma, default 8 with centers uniform in
[-10, 10]^50: cluster radius sqrt(50)*8 = 57, nearest center ~45-58 apart), so clusters overlap,
the centers still move at the last timed step (``extra.max_center_shift_last``) and most tiles
cannot be pruned (``extra.pruned_frac``).  The well-separated regime of round 1 (sigma 1: the fit
converges in 2 iterations and later iterations are almost all pruned) is reported as
``extra.separable_regime`` for reference only.
Scaling is STRONG: the global dataset is 100M rows for every N, each rank generating its own
contiguous shard directly in HBM (identical values for any N).
--config kmeans_bf16 is BASELINE config #5: k=1000, 1B x 100 bf16 (208 GB of rows on one GPU —
the 288 GB HBM partition sizing case), same protocol.
The timed region is bracketed by a barrier + device synchronize on both sides and the MAX over
ranks is reported.  The untimed warmup runs max(W, K) iterations of the same fit, so every kernel
variant the timed fit launches has had its code object loaded (HIP loads lazily, on first use).
`value` is whole-job samples/s = global_rows * K / t.  The end-to-end fit() wall clock
(k-means|| init + Lloyd to convergence, maxIter=20, tol=1e-4) is reported alongside.
Other BASELINE configs: benchmarks/bench_pca.py, benchmarks/bench_als.py.
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


def _timed_fit(args, w, N, table, init, steps, prune=True):
    _barrier_sync(w)
    t0 = time.perf_counter()
    # (one event pair per batch of iterations: per-phase events put ~10 us gaps in the stream)
    r = N.kmeans_fit(w.ctx, w.comm, table, init, args.k, steps, -1.0, precise=args.precise,
                     prune=prune, phase_events=False)
    _barrier_sync(w)
    el = float(w.allreduce_np(np.array([time.perf_counter() - t0]), "max")[0])
    assert r["num_iter"] == steps, r["num_iter"]
    return r, el


def _shard(args, w):
    base, rem = divmod(args.rows, w.size)
    local = base + (1 if w.rank < rem else 0)
    row0 = w.rank * base + min(w.rank, rem)
    return local, row0


def _estimator_fit(args, w, N):
    """The user-facing estimator end to end: ``KMeans(k, maxIter=20).fit(X)`` on this rank's
    rows as a HOST numpy array (the same synthetic blobs, made on the device and copied down
    untimed) — H2D ingestion, k-means|| init, Lloyd, and the summary pass (labels + clusterSizes)
    are all inside the timed call.  The native fit of the same rows (already resident) is timed
    alongside, so the estimator's overhead is visible."""
    import oap_mllib_amd as O

    rows_total, d, k = args.rows, args.dim, args.k
    local, row0 = _shard(args, w)
    t = N.synth_blobs(w.ctx, local, d, d, row0, k, args.box, args.sigma, 20240917, "f32")
    X = t.download_f32(w.ctx) if w.is_gpu else t.to_numpy(w.ctx).astype(np.float32)
    del t
    _barrier_sync(w)
    t0 = time.perf_counter()
    m = O.KMeans(k=k, maxIter=20, seed=7).fit(X)
    sizes = m.summary.clusterSizes
    _barrier_sync(w)
    est_s = float(w.allreduce_np(np.array([time.perf_counter() - t0]), "max")[0])
    assert sum(sizes) == rows_total and m.fit_info["engine"] == w.backend, m.fit_info
    fi = m.fit_info
    return {"estimator_fit_wall_s": est_s, "fit_iters": m.summary.numIter,
            "upload_s": fi.get("upload_seconds"), "init_s": fi.get("init_seconds"),
            "lloyd_s": fi.get("iter_seconds"), "summary_pass_s": fi.get("summary_seconds"),
            "host_rows_per_rank": int(local), "host_dtype": "float32",
            "call": f"oap_mllib_amd.KMeans(k={k}, maxIter=20).fit(ndarray[{local}, {d}])"}


def bench_kmeans(args, w):
    from oap_mllib_amd import _loader

    N = _loader.load()
    rows_total, d, k = args.rows, args.dim, args.k
    local, row0 = _shard(args, w)
    st = args.dtype
    ld = N.kmeans_ld(d, st)
    t_ing = time.time()
    table = N.synth_blobs(w.ctx, local, d, ld, row0, k, args.box, args.sigma, 20240917, st)
    table.set_global(row0, rows_total)
    _barrier_sync(w)
    ingest_s = time.time() - t_ing
    # initial centers: k-means|| (identical for any world size), untimed
    t0 = time.time()
    w.ctx.reset_metrics()
    init = N.kmeans_init(w.ctx, w.comm, table, k, "k-means||", 2, 7)
    init_s = time.time() - t0
    init_phases = {name.split("/")[-1]: round(v["total_us"] / 1e3, 2)
                   for name, v in w.ctx.metrics()["phases"].items()
                   if name.startswith("kmeans/init/")}
    # warmup iterations (same fit from the same init; results discarded).  At least as many as
    # the timed fit runs: HIP loads a kernel's code object on its first launch, and a fit of W
    # iterations does not launch every variant a K-iteration fit does (the row-scan pass, the
    # last iteration's cost, the final-cost helpers) — measured at the 12.5M-row shard: W = 3
    # put ~0.03-0.06 ms/step of one-time loading into the timed steps (0.67-0.70 vs 0.64).
    if args.warmup > 0:
        N.kmeans_fit(w.ctx, w.comm, table, init, k, max(args.warmup, args.steps), -1.0,
                     precise=args.precise, prune=not args.no_prune)
    r, el_max = _timed_fit(args, w, N, table, init, args.steps, prune=not args.no_prune)
    # the phase breakdown (assign / allreduce / rest per iteration): the same fit again with
    # per-phase events, untimed
    w.ctx.reset_metrics()
    N.kmeans_fit(w.ctx, w.comm, table, init, args.k, args.steps, -1.0, precise=args.precise,
                 prune=not args.no_prune, phase_events=True)
    m = w.ctx.metrics()["phases"]
    # the same timed run with every distance evaluated (no bound-based pruning), for reference
    ms_unpruned = None
    if not args.no_prune and not args.precise and not args.skip_unpruned:
        # (its own untimed warmup: the unpruned passes are other kernel variants)
        N.kmeans_fit(w.ctx, w.comm, table, init, k, args.steps, -1.0, prune=False)
        ru, el_u = _timed_fit(args, w, N, table, init, args.steps, prune=False)
        ms_unpruned = el_u / args.steps * 1e3
        assert np.array_equal(ru["centers"], r["centers"]), "pruning changed the result"
    # end-to-end fit(): init + Lloyd to convergence (maxIter 20, tol 1e-4)
    fit_s = fit_iters = tol_ms = None
    if not args.skip_fit:
        _barrier_sync(w)
        t1 = time.perf_counter()
        rf = N.kmeans_fit(w.ctx, w.comm, table, None, k, 20, 1e-4, "k-means||", 2, 7)
        _barrier_sync(w)
        fit_s = float(w.allreduce_np(np.array([time.perf_counter() - t1]), "max")[0])
        fit_iters = rf["num_iter"]
        # its Lloyd phase per iteration (tol >= 0: batched, a converged iteration halts the rest
        # of its batch on the device) — against the timed tol = -1 step
        tol_ms = float(w.allreduce_np(np.array([rf["iter_seconds"] / max(fit_iters, 1) * 1e3]),
                                      "max")[0])
    ak = m.get("kmeans/assign_kernel", {"total_us": 0, "count": 1})
    ar = m.get("kmeans/allreduce", {"total_us": 0, "count": 1})
    itr = m.get("kmeans/iteration", {"total_us": 0, "count": 1})
    tiles = (rows_total + 31) // 32
    pruned_g = float(w.allreduce_np(np.array([float(r.get("pruned_tiles", 0))]), "sum")[0])
    samples = rows_total * args.steps / el_max
    flops = 2.0 * rows_total * k * d
    comm_name = getattr(w.comm, "name", "none") if w.comm is not None else "none"
    # the label names the kernel path the timed fit's last iteration actually took
    # (kmeans_fit's assign_path), described for the record
    described = {
        "lean_fp16": "lean pass: one fp16 MFMA product per k-step (v_mfma_f32_32x32x16_f16) with "
                     "a rigorous error bound; rows inside it re-decided by the exact fp32 MFMA "
                     "argmin (assignments identical to exact fp32)",
        "lean_fp16_delta": "lean fp16 MFMA pass + exact fp32 re-decision; delta accumulation "
                           "of moved rows",
        "lean_fp16_delta_scan": "bound scan + lean fp16 MFMA pass over the listed tiles + exact "
                                "fp32 re-decision; delta accumulation of moved rows",
        "lean_fp16_image_delta": "lean fp16 MFMA pass streaming the resident fp16 operand image "
                                 "(written by the fit's first pass) + exact fp32 re-decision "
                                 "from the f32 rows; delta accumulation of moved rows",
        "lean_fp16_image_delta_scan": "bound scan + lean fp16 MFMA pass over the listed tiles' "
                                      "resident fp16 operand image + exact fp32 re-decision; "
                                      "delta accumulation of moved rows",
        "lean_fp16_centroid_chunked": "centroid-chunked lean fp16 MFMA pass (running top-2 keys "
                                      "across centroid chunks) + chunked exact fp32 re-decision; "
                                      "label-driven binned accumulation",
        "lean_fp16_centroid_chunked_delta": "centroid-chunked lean fp16 MFMA pass + chunked "
                                            "exact fp32 re-decision; binned accumulation of the "
                                            "moved rows only",
        "lean_img_kernel_delta": "dedicated steady-state image kernel (oap_kmeans_lean_img): "
                                 "lean fp16 MFMA pass over the resident operand image + exact "
                                 "fp32 re-decision; delta accumulation of moved rows",
        "lean_img_kernel_delta_rowscan": "row-level Hamerly scan + the image kernel over the rows "
                                         "it could not prune (gathered from the row-major "
                                         "operand image) + exact fp32 re-decision; delta "
                                         "accumulation of moved rows",
        "lean_img_kernel_delta_fused_rowscan_gated": "per iteration, a sample of the rows' "
                                                     "bounds picks (on the device) the image "
                                                     "kernel with the row-level Hamerly scan "
                                                     "fused in or the dense pipelined image "
                                                     "kernel; exact fp32 re-decision; delta "
                                                     "accumulation of moved rows",
        "lean_img_kernel_delta_fused_rowscan": "image kernel with the row-level Hamerly scan "
                                               "fused in (per-wave LDS ring of the rows it "
                                               "cannot prune) + exact fp32 re-decision; delta "
                                               "accumulation of moved rows",
        "tiered_bf16_mfma": "tiered bf16 MFMA distances (exact-fp32 re-decision of near ties)",
        "tiered_bf16_mfma_chunked": "centroid-chunked tiered bf16 MFMA distances",
        "exact_fp32_mfma": "fp32-exact MFMA (v_mfma_f32_32x32x2_f32)",
        "wide_mfma": "wide-row MFMA tier-1 + exact re-decision (d > 128)",
    }
    path = r.get("assign_path", "unknown")
    path_desc = described.get(path, path)
    extra = {"fit_wall_s_end_to_end": fit_s, "fit_iters": fit_iters,
             "fit_tol1e-4_lloyd_ms_per_iter": tol_ms,
             "init_kmeans_parallel_s": init_s, "init_phases_ms": init_phases,
             "ingest_synth_s": ingest_s,
             "data_sigma": args.sigma, "data_box": args.box,
             # centers still move at the last timed step (Lloyd not converged)
             "max_center_shift_last": r["shift_history"][-1],
             "center_shift_history": [round(v, 4) for v in r["shift_history"]],
             # share of (tile, iteration) pairs whose distance work the exact bounds skipped
             "pruned_frac": pruned_g / (tiles * args.steps),
             # share of (row, iteration) pairs the row-level scan proved unchanged
             "pruned_rows_frac": float(w.allreduce_np(np.array(
                 [float(r.get("pruned_rows", 0))]), "sum")[0]) / (rows_total * args.steps),
             "assign_kernel_ms": ak["total_us"] / max(ak["count"], 1) / 1e3,
             "allreduce_us": ar["total_us"] / max(ar["count"], 1),
             # device time of one whole iteration minus assign and allreduce: finalize,
             # the flag/count read-back and launch gaps
             "iteration_rest_us": (itr["total_us"] / max(itr["count"], 1)
                                   - ak["total_us"] / max(ak["count"], 1)
                                   - ar["total_us"] / max(ar["count"], 1)),
             # dense-equivalent rate (2 n k d flops per iteration over the timed wall clock)
             "dense_equiv_tflops": flops / (el_max / args.steps) / 1e12,
             # rows the tier-1 pass left to the exact fp32 MFMA re-decision (near ties)
             "deferred_rows_per_iter": r.get("deferred_rows", 0) / max(args.steps, 1),
             "moved_rows_per_iter": r.get("moved_rows", 0) / max(args.steps, 1),
             # Lloyd passes that streamed the fp16 operand image instead of the f32 rows
             "image_passes": r.get("image_passes", 0),
             "scale_source": r.get("scale_source"),
             "final_cost_path": r.get("final_cost_path"),
             "refine_tiles_per_iter": r["refine_tiles"] / max(args.steps, 1),
             "tiles_per_pass": tiles,
             "ms_per_step_unpruned": ms_unpruned,
             "storage": st,
             "comm": comm_name,
             "rccl_ranks": w.size if comm_name == "rccl" else 0,
             "world_size": w.size,
             "distance_path": path,
             "distance_path_desc": path_desc,
             "cost": r["cost"]}
    # CPU comparison (BASELINE.md protocol: no Spark on the GPU host -> a labelled fp64 CPU
    # proxy of the same Lloyd step on this host's cores, on a row subsample of the same data
    # and the same initial centers; the rate scales linearly with rows)
    cpu = None
    if args.cpu_rows > 0 and w.is_gpu:
        if w.rank == 0:
            sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                            "benchmarks"))
            from cpu_baseline import kmeans_proxy

            Xs = table.to_numpy(w.ctx, 0, min(args.cpu_rows, local))
            cpu = kmeans_proxy(Xs, np.asarray(init, dtype=np.float64).reshape(k, d),
                               iters=args.cpu_iters)
            del Xs
        w.barrier()
    if cpu is not None:
        extra["cpu_baseline"] = cpu
    del table
    if args.separable_extra and args.sigma != 1.0:
        # round-1 regime (well-separated blobs): converges in ~2 iterations, later iterations
        # are mostly pruned — reported for reference, NOT the headline
        t2 = N.synth_blobs(w.ctx, local, d, ld, row0, k, args.box, 1.0, 20240917, st)
        t2.set_global(row0, rows_total)
        init2 = N.kmeans_init(w.ctx, w.comm, t2, k, "k-means||", 2, 7)
        N.kmeans_fit(w.ctx, w.comm, t2, init2, k, 2, -1.0)
        r2, el2 = _timed_fit(args, w, N, t2, init2, args.steps)
        p2 = float(w.allreduce_np(np.array([float(r2.get("pruned_tiles", 0))]), "sum")[0])
        extra["separable_regime"] = {
            "data_sigma": 1.0, "samples_per_sec": rows_total * args.steps / el2,
            "ms_per_step": el2 / args.steps * 1e3, "pruned_frac": p2 / (tiles * args.steps),
            "max_center_shift_last": r2["shift_history"][-1]}
        del t2
    if args.estimator and st != "f32":
        # (the estimator call takes a host float32 array of the rows: 400 GB at config 5's
        # shape, beyond both HBM and host memory — its bf16 storage is exercised by the tests)
        extra["estimator"] = {"skipped": f"host float32 rows of a {st} configuration"}
    elif args.estimator:
        extra["estimator"] = _estimator_fit(args, w, N)
    out = {
        "metric": "kmeans_samples_per_sec", "value": samples, "unit": "samples/s",
        "n_gpus": w.size, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": el_max / args.steps * 1e3, "higher_is_better": True, "scaling": "strong",
        # whole-job GPU samples/s over the CPU proxy's samples/s on this host (extra.cpu_baseline)
        "vs_baseline": samples / cpu["samples_per_sec"] if cpu else None,
        "dtype": "fp32" if st == "f32" else "bf16",
        "data": f"synthetic (overlapping gaussian blobs sigma={args.sigma}, box={args.box}, "
                "generated on-device; random k-means|| init)",
        "config": {"model": f"kmeans k={k} d={d} (Lloyd, euclidean)", "global_batch": rows_total,
                   "seq_len": d, "parallelism": f"dp{w.size}", "k": k,
                   "rows": rows_total, "dim": d},
        "extra": extra,
    }
    return out


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="kmeans", choices=["kmeans", "kmeans_bf16"],
                    help="kmeans: k=200, 100M x 50 f32 (headline); kmeans_bf16: k=1000, "
                    "1B x 100 bf16")
    ap.add_argument("--rows", type=int, default=None)
    ap.add_argument("--dim", type=int, default=None)
    ap.add_argument("--k", type=int, default=None)
    ap.add_argument("--sigma", type=float, default=8.0,
                    help="per-feature spread of the synthetic blobs (centers in [-box, box]^d)")
    ap.add_argument("--box", type=float, default=10.0)
    ap.add_argument("--skip-fit", action="store_true")
    ap.add_argument("--no-prune", action="store_true",
                    help="evaluate every distance (disable the exact bound-based pruning)")
    ap.add_argument("--skip-unpruned", action="store_true",
                    help="do not repeat the timed run without pruning for reference")
    ap.add_argument("--no-separable-extra", dest="separable_extra", action="store_false",
                    help="skip the well-separated (sigma=1) reference run")
    ap.add_argument("--precise", action="store_true",
                    help="exact-fp32 MFMA distances only (no bf16-split fast path)")
    ap.add_argument("--no-estimator", dest="estimator", action="store_false",
                    help="skip the user-facing KMeans(...).fit(host ndarray) timing")
    ap.add_argument("--cpu-rows", type=int, default=2_000_000,
                    help="rows of the CPU-proxy baseline (scikit-learn fp64 Lloyd on this "
                    "host's cores; 0 skips it and vs_baseline is null)")
    ap.add_argument("--cpu-iters", type=int, default=2)
    ap.add_argument("--force-rccl", action="store_true",
                    help="N=1: form a real 1-rank RCCL communicator (the multi-GPU device "
                    "collective path) instead of the no-op local comm")
    args = ap.parse_args(argv)
    preset = {"kmeans": (100_000_000, 50, 200, "f32"),
              "kmeans_bf16": (1_000_000_000, 100, 1000, "bf16")}[args.config]
    args.rows = args.rows or preset[0]
    args.dim = args.dim or preset[1]
    args.k = args.k or preset[2]
    args.dtype = preset[3]

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # self-launch one rank per GPU BEFORE anything initialises a GPU in this process
        import importlib.util

        spec = importlib.util.spec_from_file_location(
            "_oap_launcher", os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                          "oap_mllib_amd", "parallel", "launcher.py"))
        launcher = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(launcher)
        return launcher.launch([sys.executable, os.path.abspath(__file__)] + argv, args.gpus)
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws != args.gpus:
        print(f"--gpus {args.gpus} but WORLD_SIZE={ws}", file=sys.stderr)
        return 2
    # native libraries write to fd 1 too (RCCL's version banner at communicator init): fd 1 goes
    # to stderr while the world runs, so rank 0's stdout carries exactly the one JSON line
    sys.stdout.flush()
    out_fd = os.dup(1)
    os.dup2(2, 1)
    import oap_mllib_amd as O

    dev = os.environ.get("OAP_BENCH_DEVICE", "gpu")  # "cpu": CPU-engine rehearsal (tests)
    w = O.init_world(O.get_config().replace(device=dev, force_device_comm=args.force_rccl))
    out = bench_kmeans(args, w)
    if w.rank == 0:
        os.write(out_fd, (json.dumps(out) + "\n").encode())
    O.shutdown_world()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
