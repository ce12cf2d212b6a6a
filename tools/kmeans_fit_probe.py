"""Torch-free K-Means fit for profiler traces (rocprofv3 at exit crashes with torch loaded):
k-means|| init, then `reps` timed fits of `iters` iterations on synthetic overlapping blobs
(the headline's generator), printing ms per iteration.

    python tools/kmeans_fit_probe.py [rows] [iters] [reps] [local|rccl]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oap_mllib_amd as O  # noqa: E402
from oap_mllib_amd import _loader  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 12_500_000
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
which = sys.argv[4] if len(sys.argv) > 4 else "rccl"
N = _loader.load()
w = O.init_world(O.get_config().replace(device="gpu", device_id=0, hbm_fraction=0.9,
                                        force_device_comm=which == "rccl"),
                 rank=0, size=1, local_rank=0)
d, k = 50, 200
t = N.synth_blobs(w.ctx, rows, d, N.kmeans_ld(d), 0, k, 10.0, 8.0, 20240917)
t.set_global(0, rows)
init = N.kmeans_init(w.ctx, w.comm, t, k, "k-means||", 2, 7)
N.kmeans_fit(w.ctx, w.comm, t, init, k, iters, -1.0)  # warm (every kernel variant loaded)
for _ in range(reps):
    w.ctx.sync()
    t0 = time.perf_counter()
    r = N.kmeans_fit(w.ctx, w.comm, t, init, k, iters, -1.0)
    w.ctx.sync()
    print("ms/iter %.4f" % ((time.perf_counter() - t0) / r["num_iter"] * 1e3), flush=True)
O.shutdown_world()
