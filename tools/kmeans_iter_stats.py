"""Per-iteration deferred / moved rows and assign time of the headline fit (run on the GPU box
with OAP_MLLIB_LOG_LEVEL=info OAP_MLLIB_LOG_FILE=...): tol = 0 makes every batch one iteration.

    python tools/kmeans_iter_stats.py [rows] [sigma] [iters]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402

from oap_mllib_amd import _loader  # noqa: E402

N = _loader.load()
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
sigma = float(sys.argv[2]) if len(sys.argv) > 2 else 8.0
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
d, k = 50, 200
g = N.Context(0, 0.9, 0)
t = N.synth_blobs(g, rows, d, N.kmeans_ld(d), 0, k, 10.0, sigma, 20240917)
t.set_global(0, rows)
comm = N.LocalComm(True)
init = N.kmeans_init(g, comm, t, k, "k-means||", 2, 7)
r = N.kmeans_fit(g, comm, t, init, k, iters, 0.0)
print("num_iter", r["num_iter"], "deferred", r["deferred_rows"], "moved", r["moved_rows"],
      flush=True)
