"""K-Means on the MI355X engine: HIP kernel numerics vs an fp64 oracle, engine equivalence,
determinism and the multi-rank paths.  Run on the GPU box: ``pytest -m gpu``."""
import numpy as np
import pytest

import oap_mllib_amd as O
from mp_util import run_world
from oap_mllib_amd.fallback import kmeans_vanilla as vanilla

pytestmark = pytest.mark.gpu


def f32_blobs(n, d, k, seed, sigma=0.5, box=10.0):
    rng = np.random.default_rng(seed)
    c = rng.uniform(-box, box, size=(k, d))
    X = c[rng.integers(0, k, n)] + rng.normal(0, sigma, size=(n, d))
    return X.astype(np.float32).astype(np.float64)  # exactly representable in fp32


@pytest.mark.parametrize("n,d,k", [(5000, 3, 4), (20000, 8, 33), (30000, 50, 200),
                                    (10000, 64, 17), (8000, 100, 40), (6000, 130, 9),
                                    (12000, 50, 500), (777, 26, 2)])
def test_assign_kernel_matches_fp64_oracle(gpu_world, native, n, d, k):
    X = f32_blobs(n, d, k, seed=d * 1000 + k, sigma=0.3)
    rng = np.random.default_rng(1)
    C = X[rng.choice(n, k, replace=False)] + 1e-3
    w = gpu_world
    t = native.upload_dense(w.ctx, X, "f32", native.kmeans_ld(d))
    lab, dist = native.kmeans_predict(w.ctx, t, C)
    ref_lab, ref_cost = vanilla.find_closest(X, C)
    # fp32 expansion vs exact fp64: allow label flips only where the top-2 gap is ~fp32 eps
    bad = np.nonzero(lab != ref_lab)[0]
    if len(bad):
        D = ((X[bad][:, None, :] - C[None]) ** 2).sum(-1)
        r = np.arange(len(bad))
        gap = np.abs(D[r, lab[bad]] - D[r, ref_lab[bad]])
        assert (gap <= 1e-4 * (1 + D.min(1))).all()
    assert len(bad) <= max(2, n // 2000)
    np.testing.assert_allclose(dist[lab == ref_lab], ref_cost[lab == ref_lab], rtol=2e-5,
                               atol=1e-4)


@pytest.mark.parametrize("d,k", [(8, 5), (50, 200), (100, 40), (130, 7)])
def test_gpu_fit_bitwise_equals_cpu_engine(native, d, k):
    """Same inputs, same assignments => identical fixed-point sums => identical centers."""
    rng = np.random.default_rng(k + d)
    C = rng.uniform(-10, 10, size=(k, d))
    X = (C[rng.integers(0, k, 20000)] + rng.normal(0, 0.2, size=(20000, d)))
    X = X.astype(np.float32).astype(np.float64)
    init = (C + rng.normal(0, 0.05, size=C.shape)).astype(np.float32).astype(np.float64)
    g = native.Context(0, 0.5, 0)
    c = native.Context(-1)
    tg = native.upload_dense(g, X, "f32", native.kmeans_ld(d))
    tc = native.upload_dense(c, X, "f64", d)
    rg = native.kmeans_fit(g, native.LocalComm(True), tg, init, k, 8, 0.0)
    rc = native.kmeans_fit(c, native.LocalComm(False), tc, init, k, 8, 0.0)
    assert rg["last_counts"] == rc["last_counts"]
    assert np.array_equal(rg["centers"], rc["centers"])
    np.testing.assert_allclose(rg["cost"], rc["cost"], rtol=1e-5)


def test_gpu_fit_deterministic(native):
    g = native.Context(0, 0.5, 0)
    t = native.synth_blobs(g, 2_000_000, 50, native.kmeans_ld(50), 0, 64, 10.0, 2.0, 5)
    init = t.to_numpy(g, 0, 64)
    r1 = native.kmeans_fit(g, native.LocalComm(True), t, init, 64, 5, 0.0)
    r2 = native.kmeans_fit(g, native.LocalComm(True), t, init, 64, 5, 0.0)
    assert np.array_equal(r1["centers"], r2["centers"]) and r1["cost"] == r2["cost"]


def test_gpu_init_matches_cpu_engine(native):
    X = f32_blobs(30000, 10, 12, seed=4, sigma=1.0)
    g, c = native.Context(0, 0.5, 0), native.Context(-1)
    tg = native.upload_dense(g, X, "f32", native.kmeans_ld(10))
    tc = native.upload_dense(c, X, "f64", 10)
    for mode in ("random", "k-means||"):
        cg = native.kmeans_init(g, native.LocalComm(True), tg, 12, mode, 2, 11)
        cc = native.kmeans_init(c, native.LocalComm(False), tc, 12, mode, 2, 11)
        np.testing.assert_array_equal(cg, cc)


def test_gpu_init_super_chunks(native, monkeypatch):
    """k-means|| with candidate sets beyond one LDS plan (d = 100, k = 400: 800 candidates a
    round, ~1600 counted) on super-chunks of the lean pass, merged by exact distance.  With ~40
    near-equidistant candidates per blob, exact-fp32 forms (direct vs expanded) and fp64 differ
    for a few rows' nearest candidate, so the inits are compared by what they must share:
    deterministic, the cost updates exactly the general chunked kernel's (OAP_KMEANS_INIT_SUPER=1
    uses the super-chunks for those only), and an init cost within 2% of the general path's."""
    X = f32_blobs(30000, 100, 40, seed=5, sigma=1.0)
    g = native.Context(0, 0.5, 0)
    t = native.upload_dense(g, X, "f32", native.kmeans_ld(100))

    def init():
        return native.kmeans_init(g, native.LocalComm(True), t, 400, "k-means||", 2, 13)

    def cost(C):
        return sum(float(((X[i:i + 2000, None, :] - C[None]) ** 2).sum(-1).min(1).sum())
                   for i in range(0, len(X), 2000))

    cs = init()
    assert np.array_equal(cs, init())
    monkeypatch.setenv("OAP_KMEANS_INIT_SUPER", "0")
    cp = init()
    monkeypatch.setenv("OAP_KMEANS_INIT_SUPER", "1")
    assert np.array_equal(init(), cp)
    assert abs(cost(cs) - cost(cp)) <= 0.02 * cost(cp)


def test_api_uses_gpu_engine(gpu_world):
    X = f32_blobs(10000, 16, 6, seed=9)
    m = O.KMeans(k=6, seed=3).fit(X)
    assert m.fit_info["engine"] == "gpu"
    ref = vanilla.fit(X, 6, 20, 1e-4, init_centers=None, seed=3)
    assert abs(m.summary.trainingCost - ref.cost) / ref.cost < 1e-3
    assert sum(m.summary.clusterSizes) == len(X)


def test_synth_blobs_shard_independent(native):
    g = native.Context(0, 0.5, 0)
    full = native.synth_blobs(g, 1000, 7, native.kmeans_ld(7), 0, 5, 10.0, 1.0, 3)
    part = native.synth_blobs(g, 400, 7, native.kmeans_ld(7), 600, 5, 10.0, 1.0, 3)
    np.testing.assert_array_equal(full.to_numpy(g, 600, 400), part.to_numpy(g))


def test_gpu_world_two_ranks_host_comm_bitwise():
    """Two ranks on GPU 0 with host (gloo) collectives staged through pinned memory."""
    rc, outs = run_world("dist_workers", "kmeans_native", nproc=2, device="gpu",
                         use_rccl=False, n=20000, d=12, k=7)
    assert rc == 0, outs
    from dist_workers import kmeans_native

    O.shutdown_world()
    ref = kmeans_native(device="gpu", n=20000, d=12, k=7)
    for o in outs:
        assert o["engine"] == "gpu" and o["comm"] == "host"
        assert np.array_equal(np.array(o["centers"]), np.array(ref["centers"]))
        # (the final cost's collectives: the statistics form allreduces sum |x|^2)
        assert abs(o["cost"] - ref["cost"]) <= 1e-9 * ref["cost"]


@pytest.mark.parametrize("case", [{"empty_rank": 1}, {"no_image_rank": 1},
                                  {"empty_rank": 1, "tol": 0.2, "max_iter": 40},
                                  {"no_image_rank": 1, "tol": 0.2, "max_iter": 40}])
def test_two_ranks_uneven_scan_state(case):
    """A rank without rows, or without room for the operand image, takes different per-row
    scan paths than its peer; the batch's collectives (its control tail included) must still
    pair up and the fit must equal the one-rank fit of the same rows.  With a tolerance the fit
    converges inside a batch: the iterations enqueued behind it stand down on the device on
    both ranks (halt), so the result is the converged iteration's."""
    from dist_workers import kmeans_uneven

    rc, outs = run_world("dist_workers", "kmeans_uneven", nproc=2, timeout=240, **case)
    assert rc == 0, outs
    O.shutdown_world()
    ref = kmeans_uneven(**{k: v for k, v in case.items() if k in ("tol", "max_iter")})
    if "tol" in case:
        assert 3 < ref["iters"] < case["max_iter"], ref["iters"]  # (early convergence)
    for o in outs:
        assert o["comm"] == "host" and o["iters"] == ref["iters"]
        assert np.array_equal(np.array(o["centers"]), np.array(ref["centers"]))
        assert abs(o["cost"] - ref["cost"]) <= 1e-9 * abs(ref["cost"])


@pytest.mark.parametrize("force_rccl", [False, True])
def test_tolerance_fit_batches_and_stands_down(native, force_rccl):
    """A fit with a tolerance enqueues its iterations in batches; the finalize of the converged
    iteration sets the device halt word and every kernel of the iterations behind it returns at
    once.  The result must be exactly the converged iteration's: the fit of exactly that many
    iterations (tol < 0) gives the same centers, counts and shifts bitwise, the shift history
    crosses the tolerance exactly there, no image pass ran past it, and the iteration count is
    the CPU engine's (fp64; the data overlap, so its near-tie labels may differ from fp32's)."""
    n, d, k = 300000, 12, 16
    rng = np.random.default_rng(21)
    C = rng.uniform(-10, 10, size=(k, d))
    X = (C[rng.integers(0, k, n)] + rng.normal(0, 2.0, size=(n, d)))
    X = X.astype(np.float32).astype(np.float64)
    init = X[rng.choice(n, k, replace=False)].copy()
    O.shutdown_world()
    w = O.init_world(O.get_config().replace(device="gpu", device_id=0,
                                            force_device_comm=force_rccl),
                     rank=0, size=1, local_rank=0)
    g, comm = w.ctx, w.comm
    assert (comm.name == "rccl") == force_rccl, comm.name
    t = native.upload_dense(g, X, "f32", native.kmeans_ld(d))
    c = native.Context(-1)
    tc = native.upload_dense(c, X, "f64", d)
    for tol in (1e-1, 1e-2):  # (CPU engine: 7 and 48 iterations)
        rg = native.kmeans_fit(g, comm, t, init, k, 60, tol)
        rc = native.kmeans_fit(c, native.LocalComm(False), tc, init, k, 60, tol)
        it = rg["num_iter"]
        assert rg["converged"] and 2 < it < 60, it
        assert it == rc["num_iter"]
        sh = rg["shift_history"]
        assert len(sh) == it and sh[-1] <= tol < min(sh[:-1]), sh
        rf = native.kmeans_fit(g, comm, t, init, k, it, -1.0)  # exactly `it` iterations
        assert rf["num_iter"] == it and not rf["converged"]
        assert rg["last_counts"] == rf["last_counts"]
        assert np.array_equal(rg["centers"], rf["centers"])
        assert rg["shift_history"] == rf["shift_history"]
        assert abs(rg["cost"] - rf["cost"]) <= 1e-6 * rf["cost"]
        assert rg["image_passes"] <= it
    del t
    O.shutdown_world()


@pytest.mark.parametrize("d,k", [(50, 200), (16, 64), (100, 30)])
def test_fast_path_bitwise_equals_precise(native, d, k):
    """bf16-split + refinement must reproduce the exact-fp32 kernel's assignments exactly."""
    X = f32_blobs(60000, d, k, seed=d + 7 * k, sigma=3.0, box=4.0)  # heavily overlapping
    init = X[np.random.default_rng(5).choice(len(X), k, replace=False)]
    g = native.Context(0, 0.5, 0)
    t = native.upload_dense(g, X, "f32", native.kmeans_ld(d))
    rf = native.kmeans_fit(g, native.LocalComm(True), t, init, k, 4, 0.0, precise=False)
    rp = native.kmeans_fit(g, native.LocalComm(True), t, init, k, 4, 0.0, precise=True)
    # overlapping data: tier 1 is unsure for many rows (lean pass defers them / tiles escalate)
    assert rf["tier3_tiles"] + rf["deferred_rows"] > 0
    assert rf["last_counts"] == rp["last_counts"]
    assert np.array_equal(rf["centers"], rp["centers"])
    # per-row fp32 costs (precise) vs the statistics identity of a costless last pass (within
    # 1e-9 of the fp64 cost): both within the fp32 per-row rounding of each other
    assert abs(rf["cost"] - rp["cost"]) <= 1e-7 * rp["cost"]


def test_refinement_triggers_on_near_ties(native):
    """Rows exactly between two centers must take the exact pass (and still match precise)."""
    rng = np.random.default_rng(0)
    d, k = 32, 8
    C = rng.uniform(-5, 5, size=(k, d))
    mids = 0.5 * (C[rng.integers(0, k, 5000)] + C[rng.integers(0, k, 5000)])
    X = np.concatenate([mids, C[rng.integers(0, k, 5000)] + rng.normal(0, 0.1, (5000, d))])
    X = X.astype(np.float32).astype(np.float64)
    g = native.Context(0, 0.5, 0)
    t = native.upload_dense(g, X, "f32", native.kmeans_ld(d))
    rf = native.kmeans_fit(g, native.LocalComm(True), t, C, k, 1, 0.0, precise=False)
    rp = native.kmeans_fit(g, native.LocalComm(True), t, C, k, 1, 0.0, precise=True)
    assert rf["refine_tiles"] > 0
    assert rf["last_counts"] == rp["last_counts"]
    assert np.array_equal(rf["centers"], rp["centers"])


def test_many_centroids_chunked_path(gpu_world, native):
    """k beyond one LDS plan: centroid chunks + merge + label-driven accumulation."""
    d, k = 50, 1500
    rng = np.random.default_rng(1)
    centers = rng.uniform(-10, 10, size=(k, d))
    X = (centers[rng.integers(0, k, 40000)] + rng.normal(0, 0.05, size=(40000, d)))
    X = X.astype(np.float32).astype(np.float64)
    C = (centers + rng.normal(0, 0.01, size=centers.shape)).astype(np.float32).astype(np.float64)
    t = native.upload_dense(gpu_world.ctx, X, "f32", native.kmeans_ld(d))
    lab, dist = native.kmeans_predict(gpu_world.ctx, t, C)
    ref_lab, ref_d = vanilla.find_closest(X, C)
    assert (lab == ref_lab).all()
    np.testing.assert_allclose(dist, ref_d, rtol=1e-4, atol=1e-5)
    r = native.kmeans_fit(gpu_world.ctx, gpu_world.comm, t, C, k, 2, 0.0)
    c = native.Context(-1)
    tc = native.upload_dense(c, X, "f64", d)
    rc = native.kmeans_fit(c, native.LocalComm(False), tc, C, k, 2, 0.0)
    assert r["last_counts"] == rc["last_counts"]
    assert np.array_equal(r["centers"], rc["centers"])


def bf16_round(X):
    """Round-to-nearest-even to bf16, returned as float64 (what a bf16 table stores)."""
    u = np.ascontiguousarray(X, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.astype(np.uint32).view(np.float32).astype(np.float64)


@pytest.mark.parametrize("d,k", [(50, 200), (100, 1000), (13, 9), (128, 40), (100, 64)])
def test_bf16_table_fit_bitwise_equals_cpu_engine(native, d, k):
    """bf16 storage: exact fp32 assignments of the bf16 values => the CPU engine's integers.
    Covers the LDS-resident path, the chunked large-k path (k=1000: balanced centroid chunks +
    cluster-range-owned LDS accumulation) and the non-bias / wide-row variants."""
    rng = np.random.default_rng(3 * d + k)
    C = rng.uniform(-10, 10, size=(k, d))
    n = 30000
    X = bf16_round(C[rng.integers(0, k, n)] + rng.normal(0, 0.3, size=(n, d)))
    init = bf16_round(C + rng.normal(0, 0.05, size=C.shape))
    g, c = native.Context(0, 0.5, 0), native.Context(-1)
    tg = native.upload_dense(g, X, "bf16", native.kmeans_ld(d, "bf16"))
    np.testing.assert_array_equal(tg.to_numpy(g, 0, 64), X[:64])  # rounding == device cast
    tc = native.upload_dense(c, X, "f64", d)
    rg = native.kmeans_fit(g, native.LocalComm(True), tg, init, k, 4, 0.0)
    rc = native.kmeans_fit(c, native.LocalComm(False), tc, init, k, 4, 0.0)
    assert rg["last_counts"] == rc["last_counts"]
    assert np.array_equal(rg["centers"], rc["centers"])
    np.testing.assert_allclose(rg["cost"], rc["cost"], rtol=1e-5)
    lab, dist = native.kmeans_predict(g, tg, rg["centers"])
    ref_lab, ref_d = vanilla.find_closest(X, rg["centers"])
    assert (lab == ref_lab).mean() > 0.9999
    np.testing.assert_allclose(dist[lab == ref_lab], ref_d[lab == ref_lab], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("d,k", [(50, 200), (100, 60)])
def test_bf16_fast_path_bitwise_equals_precise(native, d, k):
    X = bf16_round(f32_blobs(60000, d, k, seed=d + 3 * k, sigma=3.0, box=4.0))
    init = X[np.random.default_rng(6).choice(len(X), k, replace=False)]
    g = native.Context(0, 0.5, 0)
    t = native.upload_dense(g, X, "bf16", native.kmeans_ld(d, "bf16"))
    rf = native.kmeans_fit(g, native.LocalComm(True), t, init, k, 3, 0.0, precise=False)
    rp = native.kmeans_fit(g, native.LocalComm(True), t, init, k, 3, 0.0, precise=True)
    assert rf["last_counts"] == rp["last_counts"]
    assert np.array_equal(rf["centers"], rp["centers"])


def test_bf16_synth_matches_cpu_generator(native):
    g, c = native.Context(0, 0.5, 0), native.Context(-1)
    tg = native.synth_blobs(g, 3000, 100, native.kmeans_ld(100, "bf16"), 500, 11, 10.0, 1.0, 9,
                            "bf16")
    tc = native.synth_blobs(c, 3000, 100, 100, 500, 11, 10.0, 1.0, 9, "bf16")
    a, b = tg.to_numpy(g), tc.to_numpy(c)
    assert np.array_equal(bf16_round(a), a)
    # device and host libm may differ in the last float ulp before rounding to bf16
    assert np.mean(a == b) > 0.999
    np.testing.assert_allclose(a, b, rtol=1e-2, atol=1e-2)


def test_api_bf16_storage():
    """KMeans estimator with bf16 storage through the public API."""
    X = f32_blobs(20000, 24, 8, seed=12)
    O.shutdown_world()
    O.init_world(O.get_config().replace(device="gpu", device_id=0, storage_dtype="bf16"), rank=0,
                 size=1, local_rank=0)
    try:
        m = O.KMeans(k=8, seed=2).fit(X)
        assert m.fit_info["engine"] == "gpu"
        ref = vanilla.fit(bf16_round(X), 8, 20, 1e-4, init_centers=None, seed=2)
        assert abs(m.summary.trainingCost - ref.cost) / ref.cost < 1e-3
    finally:
        O.shutdown_world()


def test_batched_iterations_match_stepwise(native):
    """tol < 0 enqueues iterations in batches without host round trips: same result and cost
    history as the step-by-step loop (tol = 0 here never converges within 5 iterations)."""
    X = f32_blobs(40000, 20, 16, seed=21, sigma=1.5)
    init = X[:16]
    g = native.Context(0, 0.5, 0)
    t = native.upload_dense(g, X, "f32", native.kmeans_ld(20))
    a = native.kmeans_fit(g, native.LocalComm(True), t, init, 16, 11, -1.0)
    b = native.kmeans_fit(g, native.LocalComm(True), t, init, 16, 11, 0.0)
    assert a["num_iter"] == 11 and b["num_iter"] == 11
    assert np.array_equal(a["centers"], b["centers"])
    # scan (pruned) iterations report no cost (NaN); where the batched and the stepwise loop
    # chose them differs (adaptive per batch vs per iteration), every reported cost agrees
    ha, hb = np.array(a["cost_history"]), np.array(b["cost_history"])
    both = np.isfinite(ha) & np.isfinite(hb)
    assert both[0] and np.isfinite(ha[-1]) and np.isfinite(hb[-1])
    np.testing.assert_allclose(ha[both], hb[both], rtol=1e-12)
    assert a["last_counts"] == b["last_counts"]


@pytest.mark.parametrize("d,k,dtype,n", [(50, 200, "f32", 200000), (20, 16, "f32", 100000),
                                         (50, 1500, "f32", 60000), (100, 1000, "bf16", 60000),
                                         (100, 60, "bf16", 100000), (128, 40, "f32", 50000)])
def test_pruning_is_exact(native, monkeypatch, d, k, dtype, n):
    """Bound-based pruning skips distance work but never changes a label: centers, cost history
    and counts are bitwise those of the unpruned fit (single-launch and chunked large-k paths;
    k <= 1024 large-k fits otherwise take the centroid-chunked lean pass, without pruning)."""
    monkeypatch.setenv("OAP_KMEANS_NO_LEAN_CHUNKED", "1")
    rng = np.random.default_rng(d * 7 + k)
    C = rng.uniform(-10, 10, size=(k, d))
    X = C[rng.integers(0, k, n)] + rng.normal(0, 1.0, size=(n, d))
    X = bf16_round(X) if dtype == "bf16" else X.astype(np.float32).astype(np.float64)
    # start near the truth with a few centers misplaced: centers still move (and the largest
    # move shrinks as they settle), so pruning ramps up over the iterations
    init = C + rng.normal(0, 0.3, size=C.shape)
    init[:2] = X[rng.choice(n, 2, replace=False)]
    init = bf16_round(init) if dtype == "bf16" else init.astype(np.float32).astype(np.float64)
    g = native.Context(0, 0.5, 0)
    t = native.upload_dense(g, X, dtype, native.kmeans_ld(d, dtype))
    # (scan_min_prune 0: every row-scan iteration scans, whatever the sampled prunable share)
    rp = native.kmeans_fit(g, native.LocalComm(True), t, init, k, 10, -1.0, prune=True,
                           scan_min_prune=0.0)
    ru = native.kmeans_fit(g, native.LocalComm(True), t, init, k, 10, -1.0, prune=False)
    rn = native.kmeans_fit(g, native.LocalComm(True), t, init, k, 10, -1.0, prune=True,
                           delta=False)
    # (f32 fits with the operand image prune per row: the image kernel's fused row scan)
    assert ru["pruned_tiles"] == 0 and ru["pruned_rows"] == 0 and rn["pruned_tiles"] > 0
    assert rp["pruned_tiles"] + rp["pruned_rows"] > 0
    if dtype == "f32" and k == 200:  # the tile-level scan (OAP_KMEANS_ROW_SCAN=0) still exact
        monkeypatch.setenv("OAP_KMEANS_ROW_SCAN", "0")
        rt = native.kmeans_fit(g, native.LocalComm(True), t, init, k, 10, -1.0, prune=True)
        assert rt["pruned_rows"] == 0 and rt["pruned_tiles"] > 0 and rp["pruned_rows"] > 0
        assert rt["last_counts"] == ru["last_counts"]
        assert np.array_equal(rt["centers"], ru["centers"])
        monkeypatch.delenv("OAP_KMEANS_ROW_SCAN")
    for r in (rp, rn):
        assert r["last_counts"] == ru["last_counts"]
        assert np.array_equal(r["centers"], ru["centers"])
    hn, hu0 = np.array(rn["cost_history"]), np.array(ru["cost_history"])
    both = np.isfinite(hn) & np.isfinite(hu0)  # lean iterations report costs where needed
    assert both[0] and both[-1]
    np.testing.assert_allclose(hn[both], hu0[both], rtol=1e-12)
    # delta accumulation (single launch): per-iteration costs only on full passes, the final
    # cost from an exact pass over the labels (same per-row fp32 values, fp64 sum)
    hp, hu = np.array(rp["cost_history"]), np.array(ru["cost_history"])
    fin = np.isfinite(hp) & np.isfinite(hu)
    assert fin[0] and np.isfinite(hp[-1]) and np.isfinite(hu[-1])
    np.testing.assert_allclose(hp[fin][:-1], hu[fin][:-1], rtol=1e-12)
    # (a costless last pass takes its cost from the statistics, within 1e-9 of the fp64 cost;
    # the unpruned fit's last pass sums per-row fp32 costs)
    assert abs(hp[-1] - hu[-1]) <= 1e-7 * hu[-1]
    assert abs(rp["cost"] - ru["cost"]) <= 1e-7 * ru["cost"]


@pytest.mark.parametrize("d,k,sigma,dtype", [(50, 200, 8.0, "f32"), (20, 64, 6.0, "f32"),
                                             (100, 60, 10.0, "bf16"), (12, 7, 4.0, "f32")])
def test_lean_pass_bitwise_equals_precise_on_overlapping_data(native, d, k, sigma, dtype):
    """The lean tier-1 kernel + exact re-decision of its deferred rows (the Lloyd fit's path on
    overlapping clusters, with and without delta iterations) reproduces the exact-fp32 fit."""
    n = 120000
    t_g = native.Context(0, 0.5, 0)
    t = native.synth_blobs(t_g, n, d, native.kmeans_ld(d, dtype), 0, k, 10.0, sigma, 77, dtype)
    init = t.to_numpy(t_g, 0, k) + 0.25
    if dtype == "bf16":
        init = bf16_round(init)
    comm = native.LocalComm(True)
    rl = native.kmeans_fit(t_g, comm, t, init, k, 6, -1.0)  # lean + delta iterations
    rf = native.kmeans_fit(t_g, comm, t, init, k, 6, -1.0, prune=False)  # lean full passes
    rp = native.kmeans_fit(t_g, comm, t, init, k, 6, -1.0, precise=True)
    assert rl["deferred_rows"] > 0 and rf["deferred_rows"] > 0
    assert rl["moved_rows"] > 0 and rf["moved_rows"] > 0  # the staged delta accumulation ran
    assert rl["shift_history"][-1] > 0  # centers still move: the delta path carries state
    for r in (rl, rf):
        assert r["last_counts"] == rp["last_counts"]
        assert np.array_equal(r["centers"], rp["centers"])
    assert abs(rf["cost"] - rp["cost"]) <= 1e-12 * rp["cost"]
    assert abs(rl["cost"] - rp["cost"]) <= 1e-7 * rp["cost"]  # (statistics identity)
    # deterministic: the deferral list is filled in tile order per wave
    rf2 = native.kmeans_fit(t_g, comm, t, init, k, 6, -1.0, prune=False)
    assert rf2["cost"] == rf["cost"] and rf2["deferred_rows"] == rf["deferred_rows"]


@pytest.mark.parametrize("d,k,sigma,tol", [(50, 200, 8.0, -1.0), (20, 64, 6.0, -1.0),
                                           (12, 7, 4.0, 0.0), (124, 30, 5.0, -1.0)])
def test_operand_image_bitwise(native, monkeypatch, d, k, sigma, tol):
    """Delta passes that stream the resident fp16 operand image (instead of the f32 rows) give
    the f32-row fit and the exact-fp32 fit bitwise (batched and per-iteration loops)."""
    n = 150000
    g = native.Context(0, 0.5, 0)
    t = native.synth_blobs(g, n, d, native.kmeans_ld(d), 0, k, 10.0, sigma, 91)
    init = t.to_numpy(g, 0, k) + 0.25
    comm = native.LocalComm(True)
    ri = native.kmeans_fit(g, comm, t, init, k, 8, tol)
    monkeypatch.setenv("OAP_KMEANS_IMAGE", "0")
    rr = native.kmeans_fit(g, comm, t, init, k, 8, tol)
    rp = native.kmeans_fit(g, comm, t, init, k, 8, tol, precise=True)
    assert ri["image_passes"] > 0 and rr["image_passes"] == 0
    assert ri["num_iter"] == rr["num_iter"] == rp["num_iter"]
    for r in (ri, rr):
        assert r["last_counts"] == rp["last_counts"]
        assert np.array_equal(r["centers"], rp["centers"])
        assert abs(r["cost"] - rp["cost"]) <= 1e-7 * rp["cost"]


def test_final_cost_from_statistics(native, monkeypatch):
    """A last pass that computed no cost (row-scan fits) takes it from the fit's statistics:
    sum |x|^2 - 2 c.S + n |c|^2 (sum |x|^2 from the first pass's fp32 row norms) with a rigorous
    bound within 1e-5, the class of the per-row fp32 cost pass it replaces.  Checked against the
    fp64 cost of
    the nearest-center assignment to the previous fit's centers (the last assignment's), and
    the per-row pass taken instead for rows far from the origin (the bound fails)."""
    n, d, k, it = 150000, 50, 200, 8
    g = native.Context(0, 0.5, 0)
    t = native.synth_blobs(g, n, d, native.kmeans_ld(d), 0, k, 10.0, 8.0, 23)
    X = t.to_numpy(g)
    init = X[:k] + 0.25
    comm = native.LocalComm(True)
    r = native.kmeans_fit(g, comm, t, init, k, it, -1.0)
    assert r["final_cost_path"] == "stats"
    prev = native.kmeans_fit(g, comm, t, init, k, it - 1, -1.0)["centers"]
    C = prev.astype(np.float32).astype(np.float64)  # the fp32 centers the last pass used
    D = (X * X).sum(1)[:, None] + (C * C).sum(1)[None, :] - 2.0 * X @ C.T  # fp64
    oracle = np.maximum(D.min(1), 0.0).sum()
    assert abs(r["cost"] - oracle) <= 1e-7 * oracle  # (the rows path's own accuracy, below)
    monkeypatch.setenv("OAP_KMEANS_FINAL_COST", "rows")
    rr = native.kmeans_fit(g, comm, t, init, k, it, -1.0)
    assert rr["final_cost_path"] == "rows" and np.array_equal(rr["centers"], r["centers"])
    assert abs(rr["cost"] - oracle) <= 1e-7 * oracle
    monkeypatch.delenv("OAP_KMEANS_FINAL_COST")
    # rows far from the origin: the statistics bound fails (or the fit's last pass is costed
    # itself): never the identity
    t2 = native.upload_dense(g, X + 4096.0, "f32", native.kmeans_ld(d))
    r2 = native.kmeans_fit(g, comm, t2, init + 4096.0, k, it, -1.0)
    assert r2["final_cost_path"] != "stats" and np.isfinite(r2["cost"])


def test_operand_image_scale_fallback(native):
    """Initial centers far smaller than the data fix a large image scale; once the centers grow
    past its range (beta max|c| > 2^9) the passes read the f32 rows — still the exact fit."""
    n, d, k = 100000, 20, 40
    g = native.Context(0, 0.5, 0)
    t = native.synth_blobs(g, n, d, native.kmeans_ld(d), 0, k, 50.0, 2.0, 5)
    init = (t.to_numpy(g, 0, k) * 1e-3).astype(np.float32).astype(np.float64)
    comm = native.LocalComm(True)
    ri = native.kmeans_fit(g, comm, t, init, k, 6, -1.0)
    rp = native.kmeans_fit(g, comm, t, init, k, 6, -1.0, precise=True)
    print({key: ri[key] for key in ("image_passes", "image_bytes", "deferred_rows", "moved_rows",
                                    "assign_path", "num_iter")})
    # (image_passes counts the passes that actually read the image: the grown centers force
    # the f32 rows on at least one delta pass)
    assert ri["image_bytes"] > 0 and ri["image_passes"] < ri["num_iter"] - 1
    assert ri["last_counts"] == rp["last_counts"]
    assert np.array_equal(ri["centers"], rp["centers"])


@pytest.mark.parametrize("variant", [0, 3, 5, 7, 11])
def test_lean_variants_agree(native, monkeypatch, variant):
    """Every workgroup shape of the lean kernel gives the same fit (f32-row operands: the
    operand image's scale moves a few rows across the tier-1 bound, not any label)."""
    monkeypatch.setenv("OAP_KMEANS_IMAGE", "0")
    g = native.Context(0, 0.5, 0)
    t = native.synth_blobs(g, 200000, 50, native.kmeans_ld(50), 0, 100, 10.0, 8.0, 3)
    init = t.to_numpy(g, 0, 100)
    native.kmeans_set_lean_variant(0)
    ref = native.kmeans_fit(g, native.LocalComm(True), t, init, 100, 4, -1.0, prune=False)
    try:
        native.kmeans_set_lean_variant(variant)
        r = native.kmeans_fit(g, native.LocalComm(True), t, init, 100, 4, -1.0, prune=False)
    finally:
        native.kmeans_set_lean_variant(-1)  # back to the width rule
    assert np.array_equal(r["centers"], ref["centers"])
    assert r["deferred_rows"] == ref["deferred_rows"]


@pytest.mark.parametrize("d,k,sigma,dtype", [(784, 256, 0.3, "f32"), (300, 40, 3.0, "f32"),
                                             (200, 100, 1.0, "bf16")])
def test_wide_mfma_path_bitwise_equals_generic_and_cpu(native, monkeypatch, d, k, sigma, dtype):
    """d > 128 on the matrix cores (kmeans_wide.hip: fp16 tier 1 over 128-feature chunks + exact
    re-decision) gives the generic VALU kernel's labels, hence bitwise its centers, and the CPU
    engine's."""
    rng = np.random.default_rng(d + k)
    C = rng.uniform(-1, 1, size=(k, d))
    X = C[rng.integers(0, k, 8000)] + rng.normal(0, sigma / np.sqrt(d), size=(8000, d))
    X = X.astype(np.float32).astype(np.float64)
    if dtype == "bf16":
        X = bf16_round(X)
    init = X[rng.choice(len(X), k, replace=False)]
    g = native.Context(0, 0.5, 0)
    tg = native.upload_dense(g, X, dtype, native.kmeans_ld(d, dtype))
    rw = native.kmeans_fit(g, native.LocalComm(True), tg, init, k, 4, -1.0)
    monkeypatch.setenv("OAP_KMEANS_NO_WIDE", "1")
    rgen = native.kmeans_fit(g, native.LocalComm(True), tg, init, k, 4, -1.0)
    monkeypatch.delenv("OAP_KMEANS_NO_WIDE")
    assert rw["last_counts"] == rgen["last_counts"]
    assert np.array_equal(rw["centers"], rgen["centers"])
    np.testing.assert_allclose(rw["cost"], rgen["cost"], rtol=1e-6)
    if dtype == "f32":
        c = native.Context(-1)
        tc = native.upload_dense(c, X, "f64", d)
        rc = native.kmeans_fit(c, native.LocalComm(False), tc, init, k, 4, -1.0)
        assert np.array_equal(rw["centers"], rc["centers"])


def test_streamed_out_of_core_fit_bitwise_equals_resident(native):
    """Rows streamed from host memory through two HBM chunk buffers each iteration (the
    out-of-core path for shards beyond the HBM budget) give the resident fit's centers."""
    rng = np.random.default_rng(5)
    C = rng.uniform(-5, 5, size=(16, 24))
    X = (C[rng.integers(0, 16, 70001)] + rng.normal(0, 1.5, size=(70001, 24))).astype(np.float32)
    init = X[:16].astype(np.float64)
    g = native.Context(0, 0.5, 0)
    t = native.upload_dense(g, X.astype(np.float64), "f32", native.kmeans_ld(24))
    rr = native.kmeans_fit(g, native.LocalComm(True), t, init, 16, 6, -1.0)
    rs = native.kmeans_fit_streamed(g, native.LocalComm(True), X, init, 6, -1.0, 8192)
    assert rs["last_counts"] == rr["last_counts"]
    assert np.array_equal(rs["centers"], rr["centers"])
    # (the resident fit's last cost may come from its statistics: the per-row pass's accuracy)
    np.testing.assert_allclose(rs["cost"], rr["cost"], rtol=1e-7)


def test_estimator_streams_beyond_budget(gpu_world, monkeypatch):
    rng = np.random.default_rng(1)
    X = rng.normal(size=(50000, 8)) + rng.integers(0, 4, (50000, 1)) * 6.0
    monkeypatch.setattr(gpu_world.config, "hbm_budget_bytes", 1 << 20)
    monkeypatch.setattr(gpu_world.config, "stream_chunk_rows", 10000)
    m = O.KMeans(k=4, seed=1, maxIter=10).fit(X)
    assert m.fit_info.get("streamed") and m.fit_info["engine"] == "gpu"
    assert len(m.summary.clusterSizes) == 4 and sum(m.summary.clusterSizes) == len(X)


@pytest.mark.parametrize("d,k,sigma,dtype", [(100, 1000, 8.0, "bf16"), (60, 1000, 6.0, "f32"),
                                             (100, 700, 1.0, "bf16")])
def test_lean_chunked_large_k_bitwise(native, monkeypatch, d, k, sigma, dtype):
    """k beyond one LDS plan (<= 1024): the lean tier-1 kernel walks fp16 centroid chunks carrying
    each row's top-2 keys, the exact re-decision walks fp32 chunks carrying (best, index), labels
    drive the binned accumulation.  Bitwise the exact-fp32 fit, the previous chunked path and the
    CPU engine."""
    n = 60000
    g = native.Context(0, 0.5, 0)
    t = native.synth_blobs(g, n, d, native.kmeans_ld(d, dtype), 0, k, 10.0, sigma, 5, dtype)
    init = t.to_numpy(g, 0, k) + 0.25
    if dtype == "bf16":
        init = bf16_round(init)
    comm = native.LocalComm(True)
    rl = native.kmeans_fit(g, comm, t, init, k, 3, -1.0)
    rp = native.kmeans_fit(g, comm, t, init, k, 3, -1.0, precise=True)
    monkeypatch.setenv("OAP_KMEANS_NO_LEAN_CHUNKED", "1")
    ro = native.kmeans_fit(g, comm, t, init, k, 3, -1.0)
    monkeypatch.delenv("OAP_KMEANS_NO_LEAN_CHUNKED")
    c = native.Context(-1)
    X = t.to_numpy(g)
    rc = native.kmeans_fit(c, native.LocalComm(False), native.upload_dense(c, X, "f64", d), init,
                           k, 3, -1.0)
    if sigma > 2:
        assert rl["deferred_rows"] > 0  # near ties went through the chunked exact pass
    for r in (rp, ro, rc):
        assert r["last_counts"] == rl["last_counts"]
        assert np.array_equal(r["centers"], rl["centers"])
    assert abs(rl["cost"] - rp["cost"]) <= 1e-9 * rp["cost"]
    lab, dist = native.kmeans_predict(g, t, rl["centers"])
    ref_lab, ref_d = vanilla.find_closest(X, rl["centers"])
    assert (lab == ref_lab).mean() > 0.9999


def test_lean_chunked_cost_only_where_reported(native):
    """Chunked lean iterations compute the cost only at the first and a known last pass; with a
    tolerance (last pass unknown) the final cost comes from one exact pass over the labels after
    the loop.  Same centers either way, the final cost equal to the in-pass one (per-row fp32,
    summed in fp64 in another order) and to the exact-fp32 fit's."""
    n, d, k = 60000, 100, 1000
    g = native.Context(0, 0.5, 0)
    t = native.synth_blobs(g, n, d, native.kmeans_ld(d, "bf16"), 0, k, 10.0, 6.0, 9, "bf16")
    init = bf16_round(t.to_numpy(g, 0, k) + 0.25)
    comm = native.LocalComm(True)
    rf = native.kmeans_fit(g, comm, t, init, k, 4, -1.0)  # fixed count: last pass costed
    rt = native.kmeans_fit(g, comm, t, init, k, 4, 0.0)  # tol 0: final pass after the loop
    rp = native.kmeans_fit(g, comm, t, init, k, 4, -1.0, precise=True)
    assert rf["num_iter"] == rt["num_iter"] == 4
    for r in (rt, rp):
        assert np.array_equal(r["centers"], rf["centers"])
    hf = np.array(rf["cost_history"])
    assert np.isfinite(hf[0]) and np.isfinite(hf[-1]) and np.isnan(hf[1:-1]).all()
    assert np.isfinite(rt["cost"])
    assert abs(rt["cost"] - rf["cost"]) <= 1e-12 * rf["cost"]
    assert abs(rf["cost"] - rp["cost"]) <= 1e-9 * rp["cost"]



@pytest.mark.parametrize("d,k,sigma", [(50, 200, 8.0), (20, 37, 4.0), (12, 7, 4.0), (60, 100, 6.0),
                                       (100, 50, 5.0), (40, 230, 4.0), (26, 160, 3.0)])
def test_image_kernel_matches_lloyd_image_branch(native, d, k, sigma):
    """The dedicated steady-state image kernel (kmeans_lean_img.hip) gives the general lean
    kernel's image branch bitwise: labels, fixed-point statistics, deferred and moved rows (one
    delta pass at the next Lloyd step's centers; partial last chunks, one chunk, 12-wave rows),
    in both its configurations (0, 1), with and without the f32-row fallback launch."""
    n = 120000
    g = native.Context(0, 0.5, 0)
    t = native.synth_blobs(g, n, d, native.kmeans_ld(d), 0, k, 10.0, sigma, 17)
    comm = native.LocalComm(True)
    init = t.to_numpy(g, 0, k) + 0.125
    ca = np.asarray(native.kmeans_fit(g, comm, t, init, k, 3, -1.0)["centers"]).reshape(k, d)
    cb = np.asarray(native.kmeans_fit(g, comm, t, ca, k, 1, -1.0)["centers"]).reshape(k, d)
    ref = native.kmeans_image_timing(g, t, ca, cb, 1, 0, -1, True)
    assert ref["image_passes"] > 0 and ref["moved_rows"] > 0
    for cfg, fb in ((-1, True), (-1, False), (0, True), (1, False)):
        r = native.kmeans_image_timing(g, t, ca, cb, 1, 1, cfg, fb)
        assert r["path"].startswith("lean_img_kernel"), r["path"]
        assert r["image_passes"] == ref["image_passes"]
        assert r["deferred_rows"] == ref["deferred_rows"]
        assert r["moved_rows"] == ref["moved_rows"]
        assert np.array_equal(r["labels"], ref["labels"])
        assert np.array_equal(r["stats"], ref["stats"])


def test_image_kernel_scale_fallback(native):
    """An image written at a scale the next centers outgrow (beta max|c| > 2^9): the dedicated
    image kernel does nothing and its f32-row fallback launch takes the pass — labels and
    statistics equal the general kernel's (which falls back inside), and no pass reads the
    image."""
    n, d, k = 100000, 20, 40
    g = native.Context(0, 0.5, 0)
    t = native.synth_blobs(g, n, d, native.kmeans_ld(d), 0, k, 50.0, 2.0, 5)
    comm = native.LocalComm(True)
    cb = np.asarray(native.kmeans_fit(g, comm, t, t.to_numpy(g, 0, k), k, 2, -1.0)["centers"])
    cb = cb.reshape(k, d)
    ca = (cb * 1e-3).astype(np.float32).astype(np.float64)
    ref = native.kmeans_image_timing(g, t, ca, cb, 1, 0, -1, True)
    r = native.kmeans_image_timing(g, t, ca, cb, 1, 1, -1, True)
    assert ref["image_passes"] == 0 and r["image_passes"] == 0
    assert np.array_equal(r["labels"], ref["labels"]) and np.array_equal(r["stats"], ref["stats"])
    assert r["moved_rows"] == ref["moved_rows"] > 0



@pytest.mark.parametrize("case", ["centers", "centers_checked", "restart"])
def test_provisional_fixed_point_bounds(native, monkeypatch, case):
    """Fixed-point bounds from the initial centers (no column-maxima pass before the first
    iteration; its lean pass checks every value against them and sums |x|^2 for the final
    cost) — bounds that hold ("centers"), a value past the smallest bound but inside its own
    column's ("centers_checked": the maxima pass confirms), a value past its column's bound
    ("restart": the fit reruns with the maxima's scales).  The lazy check gives the fit of the
    same rule evaluated eagerly on the column maxima (OAP_KMEANS_ABSMAX_PASS=1) bitwise, and
    (bounds that hold, separated clusters) the CPU engine's, which evaluates the rule on its own
    maxima.  (The other cases' outliers can sit near a tie, where fp32 and fp64 may differ.)"""
    monkeypatch.setenv("OAP_KMEANS_PROVISIONAL_MIN", "0")
    n, d, k = 120000, 12, 24
    for sigma in (2.0, 0.3):  # overlapping (lazy vs eager), separated (vs the CPU engine)
        rng = np.random.default_rng(7)
        C = rng.uniform(-10, 10, size=(k, d))
        lab = rng.integers(0, k, n)
        X = C[lab] + rng.normal(0, sigma, size=(n, d))
        if case == "centers_checked":
            X[:, 0] *= 40.0  # column 0's bound is large, the smallest bound another column's
            X[5, 0] = np.abs(X[:, 0]).max() * 0.99
        X = X.astype(np.float32).astype(np.float64)
        if sigma > 1.0:
            init = X[rng.choice(n, k, replace=False)].copy()
        else:  # one seed per blob: no split blob, so no fp32/fp64 near-ties against the CPU
            init = X[[int(np.argmax(lab == j)) for j in range(k)]].copy()
        if case == "restart":
            X[17, 3] = 1e5  # far past every initial center's coordinate range
        g = native.Context(0, 0.5, 0)
        tg = native.upload_dense(g, X, "f32", native.kmeans_ld(d))
        for tol, it in ((-1.0, 9), (0.0, 6)):
            rg = native.kmeans_fit(g, native.LocalComm(True), tg, init, k, it, tol)
            assert rg["scale_source"] == case, rg["scale_source"]
            assert rg["num_iter"] == it or (tol == 0.0 and rg["num_iter"] < it)  # (converged)
            if sigma > 1.0 or case != "centers":
                monkeypatch.setenv("OAP_KMEANS_ABSMAX_PASS", "1")
                re = native.kmeans_fit(g, native.LocalComm(True), tg, init, k, it, tol)
                monkeypatch.delenv("OAP_KMEANS_ABSMAX_PASS")
                assert re["scale_source"] == ("absmax" if case == "restart"
                                              else "centers_checked")
            else:
                c = native.Context(-1)
                tc = native.upload_dense(c, X, "f64", d)
                re = native.kmeans_fit(c, native.LocalComm(False), tc, init, k, it, tol)
            assert re["num_iter"] == rg["num_iter"] and rg["last_counts"] == re["last_counts"]
            assert np.array_equal(rg["centers"], re["centers"])
            np.testing.assert_allclose(rg["cost"], re["cost"], rtol=1e-6)


def test_zero_center_column_takes_column_maxima(native, monkeypatch):
    """A feature that is 0 in every initial center has provisional bound 0, which no row can
    satisfy: the fit must take the column maxima up front (scale_source "absmax"), not flag
    every row and restart, and give the eager rule's and the CPU engine's fit bitwise."""
    monkeypatch.setenv("OAP_KMEANS_PROVISIONAL_MIN", "0")
    n, d, k = 60000, 10, 12
    rng = np.random.default_rng(11)
    C = rng.uniform(-10, 10, size=(k, d))
    lab = rng.integers(0, k, n)
    X = C[lab] + rng.normal(0, 0.3, size=(n, d))
    X[:, 4] = 0.0  # constant-zero column (one-hot / sparse features)
    X = X.astype(np.float32).astype(np.float64)
    init = X[[int(np.argmax(lab == j)) for j in range(k)]].copy()
    g = native.Context(0, 0.5, 0)
    tg = native.upload_dense(g, X, "f32", native.kmeans_ld(d))
    rg = native.kmeans_fit(g, native.LocalComm(True), tg, init, k, 8, -1.0)
    assert rg["scale_source"] == "absmax", rg["scale_source"]
    c = native.Context(-1)
    tc = native.upload_dense(c, X, "f64", d)
    rc = native.kmeans_fit(c, native.LocalComm(False), tc, init, k, 8, -1.0)
    assert rg["last_counts"] == rc["last_counts"]
    assert np.array_equal(rg["centers"], rc["centers"])
    assert np.all(np.asarray(rg["centers"]).reshape(k, d)[:, 4] == 0.0)


@pytest.mark.parametrize("d,k", [(50, 200), (20, 44)])
def test_scan_or_dense_gate_is_exact(native, d, k):
    """Row-scan iterations enqueue a scan pass and a dense pass; kmeans_scan_decide picks one on
    the device from a sample of the rows (scan_min_prune).  Either writes every label and bound,
    so always-scan (0), always-dense (2) and the sampled choice (0.2) give the unpruned fit's
    centers and counts bitwise, and the scan prunes rows only when it runs."""
    n = 1_500_000
    g = native.Context(0, 0.5, 0)
    t = native.synth_blobs(g, n, d, native.kmeans_ld(d), 0, k, 10.0, 8.0, 91)
    comm = native.LocalComm(True)
    init = native.kmeans_init(g, comm, t, k, "k-means||", 2, 3)
    ref = native.kmeans_fit(g, comm, t, init, k, 16, -1.0, prune=False)
    runs = {m: native.kmeans_fit(g, comm, t, init, k, 16, -1.0, scan_min_prune=m)
            for m in (0.0, 0.2, 2.0)}
    for m, r in runs.items():
        assert np.array_equal(r["centers"], ref["centers"]), m
        assert r["last_counts"] == ref["last_counts"], m
        assert abs(r["cost"] - ref["cost"]) <= 1e-7 * ref["cost"], m
    assert runs[2.0]["pruned_rows"] == 0
    assert runs[0.0]["pruned_rows"] >= runs[0.2]["pruned_rows"] > 0
    assert runs[0.0]["assign_path"] == "lean_img_kernel_delta_fused_rowscan"
    assert runs[0.2]["assign_path"] == "lean_img_kernel_delta_fused_rowscan_gated"


@pytest.mark.parametrize("d,k,sigma", [(50, 200, 8.0), (20, 24, 3.0), (44, 96, 12.0)])
def test_exact_candidates_equal_mfma_sweep(native, monkeypatch, d, k, sigma):
    """The exact re-decision by candidates (tier 1 again, fp32 fmaf chains for the centers within
    2 tt of the tier-1 best; kmeans_lloyd.hip oap_kmeans_exact_cand) decides every deferred row
    as the full f32 MFMA sweep does: centers, counts and cost history bitwise, with and without
    the bound-based pruning (whose lower bounds it writes differently: best + tt / alpha^2 for
    the centers it leaves out)."""
    n = 1_200_000
    g = native.Context(0, 0.5, 0)
    t = native.synth_blobs(g, n, d, native.kmeans_ld(d), 0, k, 10.0, sigma, 91)
    comm = native.LocalComm(True)
    init = native.kmeans_init(g, comm, t, k, "k-means||", 2, 5)
    out = {}
    for mode in ("cand", "mfma"):
        monkeypatch.setenv("OAP_KMEANS_EXACT", mode)
        out[mode] = [native.kmeans_fit(g, comm, t, init, k, 12, -1.0, prune=pr)
                     for pr in (True, False)]
    monkeypatch.delenv("OAP_KMEANS_EXACT")
    for a, b in zip(out["cand"], out["mfma"]):
        assert a["deferred_rows"] > 0
        assert np.array_equal(a["centers"], b["centers"])
        assert a["last_counts"] == b["last_counts"]
        np.testing.assert_array_equal(a["cost_history"], b["cost_history"])  # (NaN: costless)


@pytest.mark.parametrize("d,k,sigma,scale", [(50, 200, 8.0, 1.0), (20, 24, 3.0, 1e-3),
                                             (40, 96, 12.0, 300.0), (27, 64, 6.0, 1.0)])
def test_refined_deferral_is_exact(native, monkeypatch, d, k, sigma, scale):
    """The refined tier-1 deferral test of the image passes (each row's own fp16 rounding residual
    carried in a pad slot of the operand image, the plane's largest residual; kmeans_frag.h
    refined_tt) defers fewer rows than the worst-case bound and never changes a label: centers,
    counts and cost history bitwise those with it off, and the exact-fp32 fit's centers.  Scales
    1e-3 and 300 move the image scale by powers of two; d = 27 puts the residual's slot right
    after the last feature."""
    n = 600_000
    g = native.Context(0, 0.5, 0)
    t = native.synth_blobs(g, n, d, native.kmeans_ld(d), 0, k, 10.0 * scale, sigma * scale, 23)
    comm = native.LocalComm(True)
    init = native.kmeans_init(g, comm, t, k, "k-means||", 2, 7)
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("OAP_KMEANS_REFINE", mode)
        out[mode] = native.kmeans_fit(g, comm, t, init, k, 10, -1.0)
    monkeypatch.delenv("OAP_KMEANS_REFINE")
    rp = native.kmeans_fit(g, comm, t, init, k, 10, -1.0, precise=True)
    on, off = out["1"], out["0"]
    print({key: (on[key], off[key]) for key in ("deferred_rows", "image_passes", "moved_rows")})
    assert on["image_passes"] > 0
    assert on["deferred_rows"] < off["deferred_rows"]
    for r in (off, rp):
        assert np.array_equal(r["centers"], on["centers"])
        assert r["last_counts"] == on["last_counts"]
    np.testing.assert_array_equal(on["cost_history"], off["cost_history"])
