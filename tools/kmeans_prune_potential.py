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
chunk = 5_000_000
# center groups for the Yinyang-style variants: G contiguous index blocks of 32 (the MFMA chunks
# of the image kernel) and G groups from a k-means of the initial centers
G = (k + 31) // 32
gid_idx = torch.arange(k, device="cuda") // 32
cc = torch.from_numpy(init).cuda()
G2 = 16
gid_km = torch.arange(k, device="cuda") % G2
for _ in range(20):
    gc = torch.stack([cc[gid_km == j].mean(0) if (gid_km == j).any() else cc[j] for j in range(G2)])
    gid_km = torch.cdist(cc, gc).argmin(1)


def group_ok(dist, lab, u, drift, gid, ng):
    """rows whose every group's lower bound (min over the group's centers other than the label),
    less the group's largest drift, stays above u + drift[label]"""
    big = torch.finfo(dist.dtype).max
    dd = dist.clone()
    dd.scatter_(1, lab[:, None], big)
    ok = torch.ones(dist.shape[0], dtype=torch.bool, device=dist.device)
    thr = u + drift[lab]
    for j in range(ng):
        m = gid == j
        if not bool(m.any()):
            continue
        lb = dd[:, m].min(1).values
        ok &= (lb - drift[m].max()) > thr
    return ok


for it in range(1, iters):
    c = torch.from_numpy(C[it]).cuda()  # centers the pass of iteration `it` assigns against
    cn = (c ** 2).sum(1)
    drift = torch.from_numpy(np.linalg.norm(C[it + 1] - C[it], axis=1)).cuda() if it + 1 < len(C) \
        else None
    if drift is None:
        break
    dmax = float(drift.max())
    top2 = drift.topk(2).values
    cnt = dict(rows=0, tiles=0, excl=0, yy_idx=0, yy_km=0, elkan=0, pair_sorted=0, pairs=0)
    labs_all = []
    for r0 in range(0, rows, chunk):
        xb = X[r0:r0 + chunk].double()
        dist = (xn[r0:r0 + chunk, None] - 2.0 * xb @ c.T + cn[None, :]).clamp_min(0).sqrt()
        two = dist.topk(2, dim=1, largest=False)
        u, lo = two.values[:, 0], two.values[:, 1]
        lab = two.indices[:, 0]
        labs_all.append(lab)
        ok = (lo - dmax) > (u + drift[lab])
        cnt["rows"] += int(ok.sum())
        cnt["tiles"] += int(ok.view(-1, 32).all(1).sum())
        # Hamerly with the largest drift among the OTHER centers
        dx = torch.where(drift[lab] >= top2[0], top2[1], top2[0])
        cnt["excl"] += int(((lo - dx) > (u + drift[lab])).sum())
        cnt["yy_idx"] += int(group_ok(dist, lab, u, drift, gid_idx, G).sum())
        cnt["yy_km"] += int(group_ok(dist, lab, u, drift, gid_km, G2).sum())
        # per-center bounds (Elkan, the limit of any bound scheme without fresh distances)
        dd = dist - drift[None, :]
        dd.scatter_(1, lab[:, None], float("inf"))
        cnt["elkan"] += int((dd.min(1).values > (u + drift[lab])).sum())
        # label-sorted 32-row tiles x 32-center blocks: a pair is skippable when every row of the
        # tile keeps every center of the block (its own label aside) outside u + drift[label]
        order = lab.argsort()
        ds, ls, us = dd[order], lab[order], (u + drift[lab])[order]
        nt = ds.shape[0] // 32
        far = ds[:nt * 32] > us[:nt * 32, None]
        far = far.view(nt, 32, k)
        for b in range(G):
            blk = far[:, :, b * 32:(b + 1) * 32].all(2).all(1)
            cnt["pair_sorted"] += int(blk.sum())
        cnt["pairs"] += nt * G
        del dist, dd, ds, far
    print(json.dumps({"iter": it, "max_drift": round(dmax, 4),
                      "mean_drift": round(float(drift.mean()), 4),
                      "row_prunable_frac": round(cnt["rows"] / rows, 4),
                      "tile_prunable_frac": round(cnt["tiles"] / (rows // 32), 4),
                      "row_excl_own_frac": round(cnt["excl"] / rows, 4),
                      "yinyang_idx32_frac": round(cnt["yy_idx"] / rows, 4),
                      f"yinyang_km{G2}_frac": round(cnt["yy_km"] / rows, 4),
                      "elkan_limit_frac": round(cnt["elkan"] / rows, 4),
                      "sorted_tile_block_skip_frac": round(cnt["pair_sorted"] / cnt["pairs"], 4)}),
          flush=True)
