"""How many rows could skip the distance work per Lloyd iteration if the Hamerly test ran per
ROW instead of per 32-row tile (run on the GPU box; diagnostic only).

For the headline data (100M x 50, k = 200, sigma 8, k-means|| init) it steps the fit one
iteration at a time and, with torch on the GPU, measures for every row: u = distance to its
center, l = distance to the second-nearest center (exact bounds as a full pass would leave them),
and whether the next iteration's test l - max drift > u + drift[label] holds — per row and for
whole 32-row tiles.

    python tools/kmeans_prune_potential.py [rows] [iters]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oap_mllib_amd import _loader  # noqa: E402

N = _loader.load()
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
d, k, sigma = 50, 200, 8.0
g = N.Context(0, 0.9, 0)
t = N.synth_blobs(g, rows, d, N.kmeans_ld(d), 0, k, 10.0, sigma, 20240917, "f32")
t.set_global(0, rows)
comm = N.LocalComm(True)
init = np.asarray(N.kmeans_init(g, comm, t, k, "k-means||", 2, 7)).reshape(k, d)
X = torch.from_numpy(t.download_f32(g)).cuda()
torch.backends.cuda.matmul.allow_tf32 = False
xn = (X.double() ** 2).sum(1)
C = [init]
for it in range(iters):
    C.append(np.asarray(N.kmeans_fit(g, comm, t, C[-1], k, 1, -1.0)["centers"]).reshape(k, d))
chunk = 10_000_000
for it in range(1, iters):
    c = torch.from_numpy(C[it]).cuda()  # centers the pass of iteration `it` assigns against
    cn = (c ** 2).sum(1)
    drift = torch.from_numpy(np.linalg.norm(C[it + 1] - C[it], axis=1)).cuda() if it + 1 < len(C) \
        else None
    if drift is None:
        break
    dmax = float(drift.max())
    ok_rows = 0
    ok_tiles = 0
    for r0 in range(0, rows, chunk):
        xb = X[r0:r0 + chunk].double()
        dist = (xn[r0:r0 + chunk, None] - 2.0 * xb @ c.T + cn[None, :]).clamp_min(0).sqrt()
        two = dist.topk(2, dim=1, largest=False)
        u, lo = two.values[:, 0], two.values[:, 1]
        lab = two.indices[:, 0]
        ok = (lo - dmax) > (u + drift[lab])
        ok_rows += int(ok.sum())
        ok_tiles += int(ok.view(-1, 32).all(1).sum())
    print(json.dumps({"iter": it, "max_drift": round(dmax, 4),
                      "mean_drift": round(float(drift.mean()), 4),
                      "row_prunable_frac": round(ok_rows / rows, 4),
                      "tile_prunable_frac": round(ok_tiles / (rows // 32), 4)}), flush=True)
