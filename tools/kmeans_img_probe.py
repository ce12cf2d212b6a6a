"""Steady-state image-pass probe (run on the GPU box): one delta Lloyd pass over the resident
fp16 operand image, timed for the general lean kernel (kmeans_lloyd.hip, img_mode 2) and for
configurations of the dedicated image kernel (kmeans_lean_img.hip), on synthetic blobs at the
headline shape.  Centers A (after a few Lloyd steps) write the image and labels; every rep then
times the pass at centers B (one more step), so the moved-row share is a real Lloyd step's.

    python tools/kmeans_img_probe.py [rows] [sigma] [reps] [cfg,cfg,...]

cfg -1 = the dedicated kernel's default; 'old' = kmeans_lloyd.  Each line: ms for the lean pass
alone and with the exact re-decision (per 100M rows), deferred / moved rows, and whether labels
and statistics equal the general kernel's bitwise (ablation configurations differ by design)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: F401,E402

from oap_mllib_amd import _loader  # noqa: E402

N = _loader.load()
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
sigma = float(sys.argv[2]) if len(sys.argv) > 2 else 8.0
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
cfgs = sys.argv[4].split(",") if len(sys.argv) > 4 else ["old", "-1", "0", "1"]
d, k = int(os.environ.get("PROBE_D", "50")), int(os.environ.get("PROBE_K", "200"))
g = N.Context(0, 0.9, 0)
t = N.synth_blobs(g, rows, d, N.kmeans_ld(d), 0, k, 10.0, sigma, 20240917)
t.set_global(0, rows)
comm = N.LocalComm(True)
init = N.kmeans_init(g, comm, t, k, "k-means||", 2, 7)
steps = int(os.environ.get("PROBE_STEPS", "10"))
ca = np.asarray(N.kmeans_fit(g, comm, t, init, k, steps, -1.0)["centers"]).reshape(k, d)
cb = np.asarray(N.kmeans_fit(g, comm, t, ca, k, 1, -1.0)["centers"]).reshape(k, d)
ref = None
for c in cfgs:
    kernel, cfg = (0, -1) if c == "old" else (1, int(c))
    fb = os.environ.get("PROBE_FALLBACK", "1") == "1"
    r = N.kmeans_image_timing(g, t, ca, cb, reps, kernel, cfg, fb)
    out = {"cfg": c, "rows": rows, "sigma": sigma, "d": d, "k": k,
           "lean_ms_per_100M": round(r["lean_ms"] * 100e6 / rows, 4),
           "pass_ms_per_100M": round(r["pass_ms"] * 100e6 / rows, 4),
           "deferred_rows": r["deferred_rows"], "moved_rows": r["moved_rows"],
           "image_passes": r["image_passes"], "path": r["path"], "fallback_launch": fb}
    if ref is None and c == "old":
        ref = r
    elif ref is not None:
        out["bitwise_vs_old"] = bool(np.array_equal(r["labels"], ref["labels"]) and
                                     np.array_equal(r["stats"], ref["stats"]))
    print(json.dumps(out), flush=True)
