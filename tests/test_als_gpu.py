"""ALS on the MI355X: MFMA per-row Gramian + in-LDS Cholesky (kernels/als.hip) against the fp64
numpy oracle from the same initial factors."""
import numpy as np
import pytest

import oap_mllib_amd as O
from oap_mllib_amd.fallback import als_vanilla

pytestmark = pytest.mark.gpu


def _data(nu, ni, nnz, seed):
    rng = np.random.default_rng(seed)
    u = (rng.integers(0, nu, nnz) * 5 - 3).astype(np.int32)
    i = (rng.integers(0, ni, nnz) * 2 + 1).astype(np.int32)
    r = rng.integers(-1, 6, nnz).astype(np.float32)
    return u, i, r


@pytest.mark.parametrize("rank,alpha,iters", [(1, 1.0, 3), (5, 4.0, 3), (16, 1.0, 2),
                                              (33, 10.0, 2), (100, 1.0, 1), (128, 1.0, 1)])
def test_gpu_matches_oracle(native, gpu_world, rank, alpha, iters):
    u, i, r = _data(80, 60, 3000, rank)
    out = native.als_fit(gpu_world.ctx, gpu_world.comm, u, i, r, rank, iters, 0.1, alpha, True, 7)
    ref = als_vanilla.fit(u, i, r, rank, iters, 0.1, True, alpha, False, 7)
    assert out["failed_rows"] == 0
    assert np.array_equal(out["user_ids"], ref.user_ids)
    eu = np.abs(out["user_factors"] - ref.user_factors).max() / np.abs(ref.user_factors).max()
    ei = np.abs(out["item_factors"] - ref.item_factors).max() / np.abs(ref.item_factors).max()
    print(f"rank {rank}: max |gpu - fp64| / max |fp64|: users {eu:.2e} items {ei:.2e}")
    # measured on MI355X: <= 2.2e-5 (rank 33, alpha 10); fp32 Gramian + Cholesky vs fp64
    assert eu < 1e-4 and ei < 1e-4


def test_gpu_explicit_kernel_matches_oracle(native, gpu_world):
    u, i, r = _data(40, 30, 800, 3)
    out = native.als_fit(gpu_world.ctx, gpu_world.comm, u, i, r, 4, 2, 0.1, 1.0, False, 5)
    ref = als_vanilla.fit(u, i, r, 4, 2, 0.1, False, 1.0, False, 5)
    np.testing.assert_allclose(out["user_factors"], ref.user_factors,
                               atol=2e-3 * np.abs(ref.user_factors).max())


def test_gpu_long_rows_and_determinism(native, gpu_world):
    rng = np.random.default_rng(0)
    # power-law item popularity: a few rows with thousands of ratings
    i = (rng.zipf(1.3, 40000) % 500).astype(np.int32)
    u = rng.integers(0, 3000, 40000).astype(np.int32)
    r = rng.uniform(0.5, 5, 40000).astype(np.float32)
    a = native.als_fit(gpu_world.ctx, gpu_world.comm, u, i, r, 24, 2, 0.05, 2.0, True, 1)
    b = native.als_fit(gpu_world.ctx, gpu_world.comm, u, i, r, 24, 2, 0.05, 2.0, True, 1)
    assert np.array_equal(a["user_factors"], b["user_factors"])
    ref = als_vanilla.fit(u, i, r, 24, 2, 0.05, True, 2.0, False, 1)
    np.testing.assert_allclose(a["item_factors"], ref.item_factors,
                               atol=3e-3 * np.abs(ref.item_factors).max())


@pytest.mark.parametrize("rank,implicit,rmax", [(100, True, 5.0), (33, True, 3e4),
                                                (20, False, 5.0), (128, True, 1.0)])
def test_long_row_split_fp16_gramian(native, gpu_world, monkeypatch, rank, implicit, rmax):
    """Rows with > 4096 ratings take the split-fp16 (hi + lo, three MFMAs) chunk Gramian: it
    stays within fp32-path noise of the exact-fp32 MFMA products (OAP_ALS_GRAM=fp32) and of the
    fp64 oracle, over a large rating range (the power-of-two operand scale)."""
    rng = np.random.default_rng(rank)
    n = 60000
    i = (rng.zipf(1.3, n) % 300).astype(np.int32)
    u = rng.integers(0, 4000, n).astype(np.int32)
    r = (rng.uniform(0.5, 1.0, n) * rmax).astype(np.float32)
    assert np.bincount(i).max() > 2 * 4096  # several chunks of one long row
    def fit():
        return native.als_fit(gpu_world.ctx, gpu_world.comm, u, i, r, rank, 2, 0.05, 1.0,
                              implicit, 3)
    x3 = fit()
    monkeypatch.setenv("OAP_ALS_GRAM", "fp32")
    f32 = fit()
    assert x3["failed_rows"] == 0 and f32["failed_rows"] == 0
    ref = als_vanilla.fit(u, i, r, rank, 2, 0.05, implicit, 1.0, False, 3)
    for key, rk in (("item_factors", ref.item_factors), ("user_factors", ref.user_factors)):
        scale = np.abs(rk).max()
        d32 = np.abs(x3[key] - f32[key]).max() / scale
        d64 = np.abs(x3[key] - rk).max() / scale
        e64 = np.abs(f32[key] - rk).max() / scale
        print(f"{key}: x3-fp32 {d32:.2e}  x3-fp64 {d64:.2e}  fp32-fp64 {e64:.2e}")
        assert d64 <= max(3e-3, 2 * e64)
        assert d32 <= max(1e-3, 2 * e64)


def test_api_gpu_engine(gpu_world):
    rng = np.random.default_rng(2)
    U = rng.uniform(-1, 1, (30, 3))
    I = rng.uniform(-1, 1, (50, 3))
    R = U @ I.T
    uu, ii = np.nonzero(rng.random(R.shape) < 0.5)
    data = {"user": uu, "item": ii, "rating": R[uu, ii]}
    m = O.ALS(rank=3, maxIter=5, regParam=0.01, implicitPrefs=True, seed=0).fit(data)
    assert m.fit_info["engine"] == "gpu"
    recs = m.recommendForAllUsers(4)
    assert len(recs) == 30 and all(len(x) == 4 for x in recs["recommendations"])
    pred = m.transform(data)["prediction"].to_numpy()
    assert np.all(np.isfinite(pred))


def test_device_setup_matches_host_setup(native, gpu_world, monkeypatch):
    """The GPU re-indexing + radix-sort CSR build (kernels/als_setup.hip) gives the host
    setup's ids and factors; sparse ids (range >> ratings) fall back to the host setup."""
    u, i, r = _data(300, 200, 20000, 11)
    dev = native.als_fit(gpu_world.ctx, gpu_world.comm, u, i, r, 12, 2, 0.1, 3.0, True, 3)
    monkeypatch.setenv("OAP_ALS_HOST_SETUP", "1")
    host = native.als_fit(gpu_world.ctx, gpu_world.comm, u, i, r, 12, 2, 0.1, 3.0, True, 3)
    monkeypatch.delenv("OAP_ALS_HOST_SETUP")
    assert np.array_equal(dev["user_ids"], host["user_ids"])
    assert np.array_equal(dev["item_ids"], host["item_ids"])
    assert dev["nnz"] == host["nnz"] == len(r)
    np.testing.assert_allclose(dev["user_factors"], host["user_factors"], rtol=0,
                               atol=1e-4 * np.abs(host["user_factors"]).max())
    # sparse ids: (the dense index would need a 2^30-wide range)
    us = (u.astype(np.int64) * 3_000_000 % (1 << 30)).astype(np.int32)
    sp = native.als_fit(gpu_world.ctx, gpu_world.comm, us, i, r, 12, 2, 0.1, 3.0, True, 3)
    assert len(sp["user_ids"]) == len(np.unique(us))
    assert sp["failed_rows"] == 0


def test_gpu_two_ranks_host_comm_matches_single():
    """Two ranks on GPU 0 over host (gloo) collectives: the chunked solve + per-chunk owner
    broadcasts into the replicated factor slab (the overlapped multi-rank path) give the
    single-rank factors."""
    from mp_util import run_world

    from dist_workers import als_native

    rc, outs = run_world("dist_workers", "als_native", nproc=2, device="gpu", use_rccl=False)
    assert rc == 0, outs
    O.shutdown_world()
    ref = als_native(device="gpu")
    O.shutdown_world()
    for o in outs:
        assert o["engine"] == "gpu"
        assert o["uid"] == ref["uid"]
        np.testing.assert_allclose(o["uf"], ref["uf"], rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(o["if"], ref["if"], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("rank", [7, 33, 100])
def test_lowrank_path_matches_direct_and_oracle(native, gpu_world, monkeypatch, rank):
    """Rows with <= 64 ratings are solved by the Woodbury path in the eigenbasis of Y^T Y
    (kernels/als_lowrank.hip); it must agree with the direct r x r Cholesky and the fp64 oracle,
    across all four row classes (1-16, 17-32, 33-48, 49-64 ratings), rows above 64, and zero /
    negative ratings."""
    rng = np.random.default_rng(rank)
    lens = rng.integers(1, 91, 300)
    u = np.repeat(np.arange(300), lens).astype(np.int32)
    i = rng.integers(0, 250, len(u)).astype(np.int32)
    r = rng.integers(-1, 6, len(u)).astype(np.float32)
    args = (u, i, r, rank, 2, 0.05, 8.0, True, 4)
    monkeypatch.setenv("OAP_ALS_LOWRANK", "1")
    lr = native.als_fit(gpu_world.ctx, gpu_world.comm, *args)
    assert lr["eig_unconverged"] == 0  # the device Jacobi met its tolerance every time
    monkeypatch.setenv("OAP_ALS_LOWRANK", "0")
    direct = native.als_fit(gpu_world.ctx, gpu_world.comm, *args)
    monkeypatch.delenv("OAP_ALS_LOWRANK")
    ref = als_vanilla.fit(u, i, r, rank, 2, 0.05, True, 8.0, False, 4)
    assert lr["failed_rows"] == 0 and direct["failed_rows"] == 0
    for key, rk in (("user_factors", ref.user_factors), ("item_factors", ref.item_factors)):
        scale = np.abs(rk).max()
        np.testing.assert_allclose(lr[key], direct[key], atol=1e-3 * scale)
        np.testing.assert_allclose(lr[key], rk, atol=2e-3 * scale)


@pytest.mark.parametrize("r", [1, 2, 7, 33, 64, 100, 101, 128])
def test_device_gram_eig_matches_numpy(native, gpu_world, r):
    """kernels/als_eig.hip: the fp64 parallel Jacobi that feeds the low-rank solve (no host
    round trip) against numpy.linalg.eigh, including the V-in-global variant (r > 100)."""
    rng = np.random.default_rng(r)
    Y = rng.normal(size=(4 * r + 5, r)) * np.geomspace(10, 0.01, r)
    G = Y.T @ Y
    Q, QT, e = native.als_gram_eig(gpu_world.ctx, G)
    ld = Q.shape[0]
    Qr = Q[:r, :r].astype(np.float64)
    np.testing.assert_array_equal(Q, QT.T)
    np.testing.assert_allclose(Qr.T @ Qr, np.eye(r), atol=2e-6)
    recon = (Qr * e[:r].astype(np.float64)) @ Qr.T
    assert np.max(np.abs(recon - G)) < 2e-6 * np.max(np.abs(G))
    np.testing.assert_allclose(np.sort(e[:r]), np.sort(np.linalg.eigvalsh(G)),
                               rtol=0, atol=1e-6 * np.max(np.abs(G)))
    assert np.all(e[r:] == 1.0) and np.all(Q[r:, r:] == np.eye(ld - r))


def test_direct_split_fp16_rows_match_fp64_oracle(native, gpu_world):
    """Rows of 129-4096 ratings (the direct solve on the split-fp16 hi + lo Gramian, both halves
    of the iteration) stay within 1e-4 of the fp64 oracle, relative to the largest factor."""
    rng = np.random.default_rng(11)
    nu, ni, rank = 600, 900, 100
    per = rng.integers(150, 700, nu)
    u = np.repeat(np.arange(nu), per).astype(np.int32)
    i = np.concatenate([rng.choice(ni, p, replace=False) for p in per]).astype(np.int32)
    r = rng.integers(1, 6, len(u)).astype(np.float32)
    cu, ci = np.bincount(u), np.bincount(i, minlength=ni)
    assert cu.min() > 128 and cu.max() <= 4096 and ci.min() > 128 and ci.max() <= 4096
    out = native.als_fit(gpu_world.ctx, gpu_world.comm, u, i, r, rank, 1, 0.05, 2.0, True, 7)
    ref = als_vanilla.fit(u, i, r, rank, 1, 0.05, True, 2.0, False, 7)
    assert out["failed_rows"] == 0
    for key, rk in (("item_factors", ref.item_factors), ("user_factors", ref.user_factors)):
        err = np.abs(out[key] - rk).max() / np.abs(rk).max()
        print(f"{key}: max |gpu - fp64| / max |fp64| = {err:.2e}")
        assert err <= 1e-4


def test_every_configuration_runs_natively(native, gpu_world):
    """Explicit feedback takes the GPU kernels; a rank beyond them and nonnegative=True take the
    driver's fp64 host solver over the same world (equal to the CPU engine's fit)."""
    u, i, r = _data(60, 40, 1200, 4)
    data = {"user": u, "item": i, "rating": r}
    m = O.ALS(rank=4, maxIter=2, regParam=0.1, seed=0).fit(data)
    assert m.fit_info["engine"] == "gpu" and not m.fit_info["host_solver"]
    big = native.als_max_rank() + 22
    m = O.ALS(rank=big, maxIter=2, regParam=0.1, implicitPrefs=True, seed=0).fit(data)
    assert m.fit_info["engine"] == "gpu" and m.fit_info["host_solver"]
    ref = native.als_fit(native.Context(-1, 1.0, 4), native.LocalComm(), u, i, r, big, 2, 0.1,
                         1.0, True, 0)
    F = np.stack(m.userFactors["features"].to_list())
    order = np.argsort(np.asarray(ref["user_ids"]))
    np.testing.assert_allclose(F, np.asarray(ref["user_factors"])[order], rtol=1e-5, atol=1e-6)
    m = O.ALS(rank=3, maxIter=2, regParam=0.1, nonnegative=True, seed=0).fit(data)
    assert m.fit_info["host_solver"]
    assert np.stack(m.userFactors["features"].to_list()).min() >= 0
