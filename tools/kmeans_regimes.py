"""K-Means data-regime sweep (run on the GPU box): how the Lloyd loop behaves as the synthetic
blobs overlap more (sigma up, centers fixed in [-10, 10]^50, k=200, 100M rows by default).

Per sigma, one JSON line: ms/iteration of a 20-iteration fit from the k-means|| init with and
without pruning, pruned fraction, tier-3 / exact re-decision tiles per iteration, the center shift
history, and the full assign pass with timing ablations on the fit's final centers.

    python tools/kmeans_regimes.py [rows] [sigma,sigma,...] [iters]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: F401,E402

from oap_mllib_amd import _loader  # noqa: E402

N = _loader.load()
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
sigmas = [float(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 4, 6, 8, 12]
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
d, k = 50, 200
g = N.Context(0, 0.9, 0)
comm = N.LocalComm(True)
for sg in sigmas:
    t = N.synth_blobs(g, rows, d, N.kmeans_ld(d), 0, k, 10.0, sg, 20240917)
    t.set_global(0, rows)
    init = N.kmeans_init(g, comm, t, k, "k-means||", 2, 7)
    out = {"sigma": sg, "rows": rows}
    for prune in (True, False):
        N.kmeans_fit(g, comm, t, init, k, 2, -1.0, prune=prune)  # warm
        g.sync()
        t0 = time.perf_counter()
        r = N.kmeans_fit(g, comm, t, init, k, iters, -1.0, prune=prune)
        g.sync()
        el = time.perf_counter() - t0
        tag = "pruned" if prune else "unpruned"
        out[f"ms_per_iter_{tag}"] = round(el / iters * 1e3, 3)
        out[f"tier3_tiles_per_iter_{tag}"] = r["tier3_tiles"] / iters
        out[f"refine_tiles_per_iter_{tag}"] = r["refine_tiles"] / iters
        out[f"deferred_rows_per_iter_{tag}"] = r.get("deferred_rows", 0) / iters
        if prune:
            out["pruned_frac"] = r["pruned_tiles"] / (((rows + 31) // 32) * iters)
            out["shift_history"] = [round(v, 4) for v in r["shift_history"]]
            C = r["centers"]
    # full single pass on the final centers, with ablations (ms per 100M rows)
    abl = {}
    for v in (6, 8):
        N.kmeans_set_lean_variant(v)
        abl[f"lean_v{v}"] = round(N.kmeans_assign_timing(g, t, C, 5, False, 64) * 100e6 / rows, 3)
    for name, precise, ab in [("lean", False, 64), ("lean_no_acc", False, 65),
                              ("full", False, 0), ("tier3_only", False, 32),
                              ("no_accumulate", False, 1), ("no_acc_no_cost", False, 3),
                              ("no_distance", False, 8), ("loads_only", False, 11)]:
        abl[name] = round(N.kmeans_assign_timing(g, t, C, 5, precise, ab) * 100e6 / rows, 3)
        if ab & 64:
            abl[name + "_deferred_rows"] = N.kmeans_last_timing_deferred()
    out["assign_ms_per_100M"] = abl
    print(json.dumps(out), flush=True)
    del t
