"""The estimator's Lloyd phase vs the timed native fit (run on the GPU box): the headline rows as a
host array through ``KMeans(k=200, maxIter=20).fit`` twice (first = cold table and buffers),
then the native fit on the uploaded table with tol = -1 and tol = 1e-4 from the same init.

    python tools/estimator_probe.py [rows]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import oap_mllib_amd as O  # noqa: E402
from oap_mllib_amd import _loader  # noqa: E402

N = _loader.load()
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
d, k = 50, 200
w = O.init_world(O.get_config().replace(device="gpu", device_id=0))
t = N.synth_blobs(w.ctx, rows, d, d, 0, k, 10.0, 8.0, 20240917, "f32")
X = t.download_f32(w.ctx)
del t
out = {}
for rep in range(2):
    t0 = time.perf_counter()
    m = O.KMeans(k=k, maxIter=20, seed=7).fit(X)
    fi = m.fit_info
    out[f"estimator_{rep}"] = {"wall_s": round(time.perf_counter() - t0, 4),
                               "lloyd_ms_per_iter": fi["iter_seconds"] / m.summary.numIter * 1e3,
                               "iters": m.summary.numIter, "upload_s": fi.get("upload_seconds")}
table = N.upload_dense(w.ctx, X, "f32", N.kmeans_ld(d))
init = N.kmeans_init(w.ctx, w.comm, table, k, "k-means||", 2, 7)
for tol in (-1.0, 1e-4, -1.0, 1e-4):
    t0 = time.perf_counter()
    r = N.kmeans_fit(w.ctx, w.comm, table, init, k, 20, tol)
    el = time.perf_counter() - t0
    out.setdefault(f"native_tol{tol}", []).append(
        {"wall_ms_per_iter": el / r["num_iter"] * 1e3,
         "iter_ms_per_iter": r["iter_seconds"] / r["num_iter"] * 1e3, "iters": r["num_iter"]})
print(json.dumps(out, indent=1))
