"""PCA on the MI355X: the fused shifted-SYRK MFMA kernel (kernels/pca.hip) against an fp64
numpy oracle computed on the SAME fp32-rounded rows the GPU sees."""
import numpy as np
import pytest

import oap_mllib_amd as O

pytestmark = pytest.mark.gpu


def _f32(X):
    return np.asarray(X, np.float32).astype(np.float64)


def _cov_gpu(native, w, X, precise=False):
    from oap_mllib_amd.models.clustering import upload_table

    t = upload_table(w, np.asarray(X, np.float32))
    r = native.pca_covariance(w.ctx, w.comm, t, precise)
    return np.asarray(r["cov"]), np.asarray(r["mean"]), r


@pytest.mark.parametrize("n,d", [(5, 3), (31, 7), (1000, 50), (4099, 127), (3000, 128),
                                 (2500, 129), (2000, 300), (20000, 1000)])
def test_covariance_matches_fp64(native, gpu_world, n, d):
    rng = np.random.default_rng(n * 7 + d)
    X = _f32(rng.normal(size=(n, d)) @ (rng.normal(size=(d, d)) / np.sqrt(d)) + rng.normal(size=d))
    C, mu, _ = _cov_gpu(native, gpu_world, X)
    Cr = np.cov(X.T, ddof=1)
    scale = np.sqrt(np.outer(np.diag(Cr), np.diag(Cr))) + 1e-30
    assert np.max(np.abs(C - Cr) / scale) < 3e-5
    np.testing.assert_allclose(mu, X.mean(axis=0), atol=1e-6 * (1 + np.abs(X).max()))
    assert np.array_equal(C, C.T)


def test_precise_mode_tighter(native, gpu_world):
    rng = np.random.default_rng(11)
    X = _f32(rng.normal(size=(5000, 96)) * rng.uniform(0.1, 10, size=96))
    Cr = np.cov(X.T, ddof=1)
    scale = np.sqrt(np.outer(np.diag(Cr), np.diag(Cr)))
    C3, _, _ = _cov_gpu(native, gpu_world, X, precise=False)
    C4, _, _ = _cov_gpu(native, gpu_world, X, precise=True)
    e3 = np.max(np.abs(C3 - Cr) / scale)
    e4 = np.max(np.abs(C4 - Cr) / scale)
    assert e4 < 2e-6 and e4 <= e3 * 1.01


def test_large_offset_no_cancellation(native, gpu_world):
    rng = np.random.default_rng(5)
    X = _f32(rng.normal(size=(30000, 20)) * np.linspace(0.01, 1, 20) + 3e3)
    C, mu, _ = _cov_gpu(native, gpu_world, X)
    Cr = np.cov(X.T, ddof=1)
    scale = np.sqrt(np.outer(np.diag(Cr), np.diag(Cr)))
    assert np.max(np.abs(C - Cr) / scale) < 5e-5


def test_deterministic(native, gpu_world):
    rng = np.random.default_rng(2)
    X = rng.normal(size=(70000, 200)).astype(np.float32)
    a, _, _ = _cov_gpu(native, gpu_world, X)
    b, _, _ = _cov_gpu(native, gpu_world, X)
    assert np.array_equal(a, b)


def test_fit_api_gpu_engine(gpu_world):
    rng = np.random.default_rng(9)
    d, k = 40, 5
    lat = rng.normal(size=(20000, d)) * np.geomspace(10, 0.1, d)
    Q, _ = np.linalg.qr(rng.normal(size=(d, d)))
    X = _f32(lat @ Q.T + 7.0)
    m = O.PCA(k=k, inputCol="features").fit(X)
    assert m.fit_info["engine"] == "gpu"
    Cr = np.cov(X.T, ddof=1)
    wr, Vr = np.linalg.eigh(Cr)
    o = np.argsort(-wr)
    wr, Vr = wr[o], Vr[:, o]
    np.testing.assert_allclose(m.explainedVariance.toArray(), wr[:k] / wr.sum(), atol=1e-5)
    np.testing.assert_allclose(np.abs(m.pc.toArray()), np.abs(Vr[:, :k]), atol=1e-4)


def test_gpu_close_to_cpu_engine(native, gpu_world):
    from oap_mllib_amd.models.clustering import upload_table

    rng = np.random.default_rng(4)
    X = rng.normal(size=(8000, 33)).astype(np.float32) * np.arange(1, 34, dtype=np.float32)
    r_gpu = native.pca_fit(gpu_world.ctx, gpu_world.comm, upload_table(gpu_world, X), 6, False)
    cpu = native.Context(-1, 1.0, 4)
    lc = native.LocalComm()
    t = native.upload_dense(cpu, X.astype(np.float64), "f64", 33)
    r_cpu = native.pca_fit(cpu, lc, t, 6, False)
    np.testing.assert_allclose(r_gpu["explained_variance"], r_cpu["explained_variance"],
                               atol=2e-6)
    np.testing.assert_allclose(np.abs(r_gpu["pc"]), np.abs(r_cpu["pc"]), atol=1e-4)


# ---------------------------------------------------------------- exact (reference fp64) mode
def _cov_exact(native, w, X, layout="pca_exact"):
    from oap_mllib_amd.models.clustering import upload_table

    t = upload_table(w, X, layout=layout)
    r = native.pca_covariance(w.ctx, w.comm, t, False, exact=True)
    return np.asarray(r["cov"]), np.asarray(r["mean"])


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("n,d", [(5, 3), (37, 7), (1000, 50), (4099, 127), (3000, 128),
                                 (2500, 129), (2000, 301), (20000, 1000)])
def test_exact_mode_matches_np_cov(native, gpu_world, dtype, n, d):
    """fp64 products and sums on v_mfma_f64_16x16x4_f64: np.cov (fp64) of the same rows to
    1e-12, scale-normalised — the reference's oneDAL fp64 precision (PCADALImpl.cpp:31)."""
    rng = np.random.default_rng(n * 3 + d)
    X = (rng.normal(size=(n, d)) @ (rng.normal(size=(d, d)) / np.sqrt(d))
         + rng.normal(size=d) * 5).astype(dtype)
    C, mu = _cov_exact(native, gpu_world, X)
    X64 = X.astype(np.float64)
    Cr = np.cov(X64.T, ddof=1)
    assert np.max(np.abs(C - Cr)) / np.max(np.abs(Cr)) < 1e-12
    np.testing.assert_allclose(mu, X64.mean(axis=0), rtol=0, atol=1e-12 * (1 + np.abs(X64).max()))


def test_exact_mode_f64_rows_not_rounded(native, gpu_world):
    """f64 rows whose low bits fp32 would drop: the exact path keeps them."""
    rng = np.random.default_rng(8)
    base = rng.normal(size=(6000, 24))
    X = 1.0 + base * 1e-9  # fp32 rounding would erase the whole signal
    C, _ = _cov_exact(native, gpu_world, X)
    Cr = np.cov(X.T, ddof=1)
    assert np.max(np.abs(C - Cr)) / np.max(np.abs(Cr)) < 1e-9


def test_exact_is_default_and_fast_selectable(gpu_world):
    rng = np.random.default_rng(12)
    X = rng.normal(size=(20000, 64)) * np.geomspace(5, 0.2, 64) + 3.0
    m = O.PCA(k=4, inputCol="features").fit(X)
    assert m.fit_info["engine"] == "gpu" and m.fit_info["precision"] == "exact"
    wr = np.sort(np.linalg.eigvalsh(np.cov(X.T, ddof=1)))[::-1]
    np.testing.assert_allclose(m.explainedVariance.toArray(), wr[:4] / wr.sum(), rtol=1e-10)
    O.set_config(O.get_config().replace(pca_precision="fast"))
    try:
        O.shutdown_world()
        O.init_world(O.get_config().replace(device="gpu", device_id=0))
        f = O.PCA(k=4, inputCol="features").fit(X)
        assert f.fit_info["precision"] == "fast"
        np.testing.assert_allclose(f.explainedVariance.toArray(), wr[:4] / wr.sum(), atol=1e-5)
    finally:
        O.set_config(O.get_config().replace(pca_precision="exact"))


def test_exact_with_bf16_storage_config(gpu_world):
    """PCA uploads with its own layout: a bf16 K-Means storage config does not reach it."""
    O.set_config(O.get_config().replace(storage_dtype="bf16"))
    try:
        O.shutdown_world()
        O.init_world(O.get_config().replace(device="gpu", device_id=0))
        X = np.random.default_rng(1).normal(size=(3000, 20))
        m = O.PCA(k=3, inputCol="features").fit(X)
        assert m.fit_info["engine"] == "gpu"
    finally:
        O.set_config(O.get_config().replace(storage_dtype="f32"))


def test_exact_f64_rows_beyond_budget_go_up_as_f32(gpu_world):
    """f64 input rows take twice the HBM: within the budget they stay f64 on the device, beyond
    it (Config.hbm_budget_bytes) they are uploaded as f32 and the exact kernel still forms fp64
    products of them (the covariance of the f32-rounded rows, to fp64 accuracy)."""
    rng = np.random.default_rng(21)
    X = rng.normal(size=(8000, 32)) * np.geomspace(4, 0.3, 32) + 1.0
    m = O.PCA(k=3, inputCol="features").fit(X)
    assert m.fit_info["device_rows_dtype"] == "f64"
    O.set_config(O.get_config().replace(hbm_budget_bytes=X.nbytes // 2))
    try:
        O.shutdown_world()
        O.init_world(O.get_config().replace(device="gpu", device_id=0))
        with pytest.warns(RuntimeWarning, match="f32"):
            f = O.PCA(k=3, inputCol="features").fit(X)
        assert f.fit_info["device_rows_dtype"] == "f32"
        assert f.fit_info["precision"] == "exact_f32_rows"  # (said so, not called "exact")
        X32 = X.astype(np.float32).astype(np.float64)
        wr = np.sort(np.linalg.eigvalsh(np.cov(X32.T, ddof=1)))[::-1]
        np.testing.assert_allclose(f.explainedVariance.toArray(), wr[:3] / wr.sum(), rtol=1e-10)
    finally:
        O.set_config(O.get_config().replace(hbm_budget_bytes=0))


# ------------------------------------------------- exact mode on the int8 matrix cores (Ozaki)
def _cov_exact_full(native, w, X):
    from oap_mllib_amd.models.clustering import upload_table

    t = upload_table(w, X, layout="pca_exact")
    return native.pca_covariance(w.ctx, w.comm, t, False, exact=True)


@pytest.mark.parametrize("n,d,offset,spread", [(7, 3, 0.0, 1.0), (3001, 50, 5.0, 1.0),
                                               (4099, 129, 3e3, 1.0), (2500, 300, 0.0, 1e3),
                                               (20000, 1000, 1.0, 1.0), (150001, 70, 2.0, 10.0)])
def test_exact_int8_digits_within_bound(native, gpu_world, n, d, offset, spread):
    """f32 rows in exact mode run on the int8 digit products (kernels/pca_ozaki.hip): the error
    against np.cov of the same rows stays inside the bound the kernel reports, the bound itself
    is far below the 1e-12 the exact-mode tests ask for, and the fp64-MFMA engine agrees."""
    rng = np.random.default_rng(n + d)
    X = (rng.normal(size=(n, d)) * np.geomspace(1.0, spread, d) + offset).astype(np.float32)
    r = _cov_exact_full(native, gpu_world, X)
    assert r["engine"] == "int8_digits"
    C = np.asarray(r["cov"])
    Cr = np.cov(X.astype(np.float64).T, ddof=1)
    err = np.max(np.abs(C - Cr))
    scale = np.max(np.abs(Cr))
    assert err / scale < 1e-12, err / scale
    assert 0 < r["err_bound"] < 1e-10 * scale
    # np.cov's own rounding (fp64 sums of n products) is the slack next to the bound
    M = np.abs(X.astype(np.float64) - X.mean(0)).max()
    assert err <= r["err_bound"] + n * 2.0 ** -52 * M * M / (n - 1)
    native.set_knob("OAP_PCA_EXACT_ENGINE", "fp64")
    try:
        f = _cov_exact_full(native, gpu_world, X)
    finally:
        native.set_knob("OAP_PCA_EXACT_ENGINE", "")
    assert f["engine"] == "fp64_mfma"
    assert np.max(np.abs(np.asarray(f["cov"]) - C)) / scale < 1e-12
    assert np.array_equal(C, C.T)


def test_exact_int8_digits_row_chunks_and_determinism(native, gpu_world):
    """Several digit-plane row chunks (a small chunk budget) give the statistics of one chunk to
    fp64 rounding, and repeated fits are bitwise equal."""
    rng = np.random.default_rng(77)
    X = (rng.normal(size=(9000, 70)) * 3 + 2).astype(np.float32)
    one = _cov_exact_full(native, gpu_world, X)
    native.set_knob("OAP_PCA_DIGIT_CHUNK_BYTES", str(1 << 20))  # 1 MiB: 5 chunks of 2048 rows
    try:
        many = _cov_exact_full(native, gpu_world, X)
        again = _cov_exact_full(native, gpu_world, X)
    finally:
        native.set_knob("OAP_PCA_DIGIT_CHUNK_BYTES", "")
    a, b = np.asarray(one["cov"]), np.asarray(many["cov"])
    assert np.max(np.abs(a - b)) / np.max(np.abs(a)) < 1e-14
    assert np.array_equal(b, np.asarray(again["cov"]))
    np.testing.assert_allclose(many["mean"], X.astype(np.float64).mean(0), rtol=0, atol=1e-12 * 10)


def test_exact_int8_digits_constant_and_zero_columns(native, gpu_world):
    """A constant column (zero range: no exponent) and an all-zero column give exact zeros in
    their rows and columns of the covariance."""
    rng = np.random.default_rng(3)
    X = rng.normal(size=(5000, 40)).astype(np.float32)
    X[:, 5] = 7.25
    X[:, 17] = 0.0
    r = _cov_exact_full(native, gpu_world, X)
    C = np.asarray(r["cov"])
    assert np.all(C[5] == 0) and np.all(C[:, 17] == 0)
    Cr = np.cov(X.astype(np.float64).T, ddof=1)
    assert np.max(np.abs(C - Cr)) / np.max(np.abs(Cr)) < 1e-12


def test_exact_int8_digits_sampled_scales_redone_on_outlier(native, gpu_world):
    """Beyond 65536 rows the column scales come from an even row sample (one bit of margin); an
    outlier the sample misses overflows a digit, the pass is flagged and redone with scales from
    every row, and the result is the exact covariance all the same.  A far outlier (a column
    range 10^4 x its spread) leaves the digit bound above 1e-10 of the variance: the pass is then
    redone on the fp64 MFMA."""
    rng = np.random.default_rng(19)
    n = 200_000
    X = rng.normal(size=(n, 24)).astype(np.float32)
    for outlier, fallback in ((40.0, False), (1e4, True)):
        X[1, 7] = outlier  # (row 1 is not a sampled row: the sample stride is n // 65536 = 3)
        r = _cov_exact_full(native, gpu_world, X)
        assert r["scales_redone"] and r["fallback_fp64"] == fallback
        assert r["engine"] == ("fp64_mfma" if fallback else "int8_digits")
        Cr = np.cov(X.astype(np.float64).T, ddof=1)
        C = np.asarray(r["cov"])
        assert np.max(np.abs(C - Cr)) / np.max(np.abs(Cr)) < 1e-12
    X[1, 7] = 0.5
    r2 = _cov_exact_full(native, gpu_world, X)
    assert not r2["scales_redone"] and not r2["fallback_fp64"]
    Cr2 = np.cov(X.astype(np.float64).T, ddof=1)
    assert np.max(np.abs(np.asarray(r2["cov"]) - Cr2)) / np.max(np.abs(Cr2)) < 1e-12
