"""Wide-row K-Means probe (GPU box): ms per Lloyd iteration on the MFMA wide path vs the generic
VALU kernel (OAP_KMEANS_NO_WIDE=1 in the environment), synthetic blobs.

    python tools/kmeans_wide_probe.py [rows] [d] [k] [iters]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oap_mllib_amd import _loader  # noqa: E402

N = _loader.load()
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 784
k = int(sys.argv[3]) if len(sys.argv) > 3 else 256
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 5
g = N.Context(0, 0.9, 0)
t = N.synth_blobs(g, rows, d, N.kmeans_ld(d), 0, k, 1.0, 0.5, 20240917)
t.set_global(0, rows)
comm = N.LocalComm(True)
init = t.to_numpy(g, 0, k)
N.kmeans_fit(g, comm, t, init, k, 1, -1.0, prune=False)  # warm
t0 = time.perf_counter()
r = N.kmeans_fit(g, comm, t, init, k, iters, -1.0, prune=False)
ms = (time.perf_counter() - t0) * 1e3 / iters
print(json.dumps({"rows": rows, "d": d, "k": k, "iters": iters,
                  "path": "generic" if os.environ.get("OAP_KMEANS_NO_WIDE") else "wide",
                  "ms_per_iter": round(ms, 3), "cost": r["cost"],
                  "dense_tflops": round(2.0 * rows * k * d / (ms * 1e-3) / 1e12, 1)}), flush=True)
