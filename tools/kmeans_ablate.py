"""Per-phase timing ablation of the fused K-Means assign kernel (run on the GPU box)."""
import json
import sys

import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402

from oap_mllib_amd import _loader

N = _loader.load()
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000_000
only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
d, k = 50, 200
g = N.Context(0, 0.9, 0)
t = N.synth_blobs(g, rows, d, N.kmeans_ld(d), 0, k, 10.0, 1.0, 20240917)
# centers as in the benchmark: k-means|| init + 2 Lloyd iterations (the fast path's refinement
# rate depends on them; raw data rows as centers would force near ties)
comm = N.LocalComm()
C = N.kmeans_fit(g, comm, t, None, k, 2, -1.0, "k-means||", 2, 7)["centers"]
out = {}
for name, precise, ab in [("full", False, 0), ("no_accumulate", False, 1), ("no_cost", False, 2),
                          ("no_acc_no_cost", False, 3), ("no_distance", False, 8),
                          ("loads_only", False, 11), ("precise_full", True, 0),
                          ("precise_no_acc_no_cost", True, 3), ("full_prefetch2", False, 16),
                          ("full_tier3_only", False, 32)]:
    if only and name not in only:
        continue
    ms = N.kmeans_assign_timing(g, t, C, reps, precise, ab)
    out[name] = round(ms * 100e6 / rows, 3)  # normalised to 100M rows
# bf16 rows (same data rounded), LDS-resident centroids
tb = N.synth_blobs(g, rows, d, N.kmeans_ld(d, "bf16"), 0, k, 10.0, 1.0, 20240917, "bf16")
for name, ab in [("bf16_full", 0), ("bf16_prefetch2", 16), ("bf16_no_acc_no_cost", 3),
                 ("bf16_tier3_only", 32)]:
    if only and name not in only:
        continue
    out[name] = round(N.kmeans_assign_timing(g, tb, C, reps, False, ab) * 100e6 / rows, 3)
print(json.dumps({"rows": rows, "ms_per_100M_rows": out}))
