"""Timed headline fits (20 iterations, tol -1, one GPU) by scan / dense policy, same table and
init, alternating reps: prune=False (dense, no bounds), scan_min_prune 2.0 (always dense, bounds
kept), 0.0 (always scan), and the sampled gate at a few thresholds.

    python tools/kmeans_gate_probe.py [rows] [reps] [local|rccl]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402,F401

from oap_mllib_amd import _loader  # noqa: E402

N = _loader.load()
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
d, k = 50, 200
which = sys.argv[3] if len(sys.argv) > 3 else "local"
import oap_mllib_amd as O  # noqa: E402

w = O.init_world(O.get_config().replace(device="gpu", device_id=0, hbm_fraction=0.9,
                                        force_device_comm=which == "rccl"),
                 rank=0, size=1, local_rank=0)
g, comm = w.ctx, w.comm
t = N.synth_blobs(g, rows, d, N.kmeans_ld(d), 0, k, 10.0, 8.0, 20240917)
t.set_global(0, rows)
init = N.kmeans_init(g, comm, t, k, "k-means||", 2, 7)
policies = [("unpruned", dict(prune=False)), ("dense_bounds", dict(scan_min_prune=2.0)),
            ("scan_always", dict(scan_min_prune=0.0)), ("gate_0.10", dict(scan_min_prune=0.10)),
            ("gate_0.20", dict(scan_min_prune=0.20)), ("gate_0.30", dict(scan_min_prune=0.30)),
            ("gate_0.20_tol1e-4", dict(tol=1e-4))]
N.kmeans_fit(g, comm, t, init, k, 3, -1.0)  # warm
out = {name: [] for name, _ in policies}
for rep in range(reps):
    for name, kw in policies:
        t0 = time.perf_counter()
        kw = dict(kw)
        tol = kw.pop("tol", -1.0)
        r = N.kmeans_fit(g, comm, t, init, k, 20, tol, **kw)
        out[name].append((time.perf_counter() - t0) / r["num_iter"] * 1e3)
med = {n: round(sorted(v)[len(v) // 2], 4) for n, v in out.items()}
print(json.dumps({"rows": rows, "comm": comm.name, "ms_per_step_median": med,
                  "all": out}, indent=1))
