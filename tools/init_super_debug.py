"""GPU debug: k-means|| init with the super-chunk path on cost updates only / counts only."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oap_mllib_amd import _loader  # noqa: E402

N = _loader.load()
rng = np.random.default_rng(5)
k0, d, n = 40, 100, 30000
c = rng.uniform(-10, 10, size=(k0, d))
X = (c[rng.integers(0, k0, n)] + rng.normal(0, 1.0, size=(n, d))).astype(np.float32)
X = X.astype(np.float64)
g, cc = N.Context(0, 0.5, 0), N.Context(-1)
tg = N.upload_dense(g, X, "f32", N.kmeans_ld(d))
tc = N.upload_dense(cc, X, "f64", d)
out = {}
for mode in ("0", "1", "2", "3"):
    os.environ["OAP_KMEANS_INIT_SUPER"] = mode
    out[mode] = N.kmeans_init(g, N.LocalComm(True), tg, 400, "k-means||", 2, 13)
ref = N.kmeans_init(cc, N.LocalComm(False), tc, 400, "k-means||", 2, 13)
for mode, v in out.items():
    print(mode, "eq_precise", bool(np.array_equal(v, out["0"])),
          "eq_cpu", bool(np.array_equal(v, ref)))
# the lean chunked pass's labels / distances against numpy for 800 centers
C = X[rng.choice(n, 800, replace=False)] + 1e-3
lab, dist = N.kmeans_predict(g, tg, C)
D = ((X[:2000, None, :] - C[None]) ** 2).sum(-1)
print("predict(general) lab ok", float(np.mean(np.argmin(D, 1) == lab[:2000])))
