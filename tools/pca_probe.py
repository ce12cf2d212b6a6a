"""PCA statistics probe: the exact-mode covariance of a synthetic n x d f32 table (on-device
blobs, as benchmarks/bench_pca.py) on the int8-digit engine and the fp64-MFMA engine, for
rocprofv3 --kernel-trace runs (per-kernel times of each engine's passes).

    python tools/pca_probe.py [rows] [dim] [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "benchmarks"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
dim = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
from bench_common import init_world  # noqa: E402

from oap_mllib_amd import _loader  # noqa: E402

N = _loader.load()
w = init_world()
t = N.synth_blobs(w.ctx, rows, dim, N.kmeans_ld(dim), 0, 64, 10.0, 1.0, 1234)
t.set_global(0, rows)
out = {}
for eng in ("int8", "fp64"):
    N.set_knob("OAP_PCA_EXACT_ENGINE", eng)
    ms = [N.pca_covariance(w.ctx, w.comm, t, False, exact=True)["stats_ms"] for _ in range(reps)]
    out[eng] = ms
N.set_knob("OAP_PCA_EXACT_ENGINE", "")
print(json.dumps({"rows": rows, "dim": dim, "stats_ms": out}))
