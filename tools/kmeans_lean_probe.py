"""Lean K-Means pass probe (run on the GPU box): timings of the Lloyd fit's assign path (lean
tier-1 kernel + exact re-decision of deferred rows) with timing ablations, on synthetic blobs.

    python tools/kmeans_lean_probe.py [rows] [sigma] [reps] [variant] [ablations,...]

ablation bits (added to 64 = lean path): 1 no accumulate, 2 no cost, 8 no distance work.
Prints one JSON line (ms per 100M rows)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402

from oap_mllib_amd import _loader  # noqa: E402

N = _loader.load()
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000_000
sigma = float(sys.argv[2]) if len(sys.argv) > 2 else 8.0
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
variant = int(sys.argv[4]) if len(sys.argv) > 4 else 6  # (6 or 8)
abls = [int(v) for v in sys.argv[5].split(",")] if len(sys.argv) > 5 else [0, 1, 2, 3, 8, 11]
d, k = 50, 200
g = N.Context(0, 0.9, 0)
t = N.synth_blobs(g, rows, d, N.kmeans_ld(d), 0, k, 10.0, sigma, 20240917)
t.set_global(0, rows)
comm = N.LocalComm(True)
init = N.kmeans_init(g, comm, t, k, "k-means||", 2, 7)
C = N.kmeans_fit(g, comm, t, init, k, 3, -1.0, prune=False)["centers"]
N.kmeans_set_lean_variant(variant)
out = {"rows": rows, "sigma": sigma, "variant": variant}
for ab in abls:
    ms = N.kmeans_assign_timing(g, t, C, reps, False, 64 | ab)
    out[f"ablate{ab}"] = round(ms * 100e6 / rows, 3)
out["deferred_rows_per_pass"] = N.kmeans_last_timing_deferred()
print(json.dumps(out), flush=True)
