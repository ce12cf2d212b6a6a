"""Device collectives on ONE GPU: a real 1-rank RCCL communicator (``force_device_comm``) drives
every multi-GPU code path of the drivers — the K-Means grouped allreduce per iteration, the PCA
statistics allreduce under the watchdog wait, and ALS's device ratings shuffle (RCCL send/recv
to self), comm-stream Gramian allreduce and chunked owner broadcasts — and must reproduce the
no-comm (LocalComm) fits.  Reference exchanges: KMeansDALImpl.cpp:97-99, PCADALImpl.cpp:111-113,
ALSShuffle.cpp:62-127, ALSDALImpl.cpp:336-431."""
import numpy as np
import pytest

import oap_mllib_amd as O

pytestmark = pytest.mark.gpu


def _world(force: bool):
    O.shutdown_world()
    return O.init_world(O.get_config().replace(device="gpu", device_id=0,
                                               force_device_comm=force),
                        rank=0, size=1, local_rank=0)


def _blobs(n, d, k, seed, sigma=1.0):
    rng = np.random.default_rng(seed)
    c = rng.uniform(-10, 10, size=(k, d))
    return c[rng.integers(0, k, n)] + rng.normal(0, sigma, size=(n, d))


# ------------------------------------------------------------------------------ collectives
def test_rccl_one_rank_collectives(rccl1_world):
    w = rccl1_world
    a = np.arange(7, dtype=np.float64) * 1.5 - 2.0
    np.testing.assert_array_equal(w.comm.exchange_f64(w.ctx, "allreduce", a), a)
    np.testing.assert_array_equal(w.comm.exchange_f64(w.ctx, "allreduce_max", a), a)
    np.testing.assert_array_equal(w.comm.exchange_f64(w.ctx, "allgather", a), a)
    np.testing.assert_array_equal(w.comm.exchange_f64(w.ctx, "bcast", a, root=0), a)
    # alltoallv = grouped send/recv to self
    np.testing.assert_array_equal(
        w.comm.exchange_f64(w.ctx, "alltoallv", a, send_counts=[7], recv_counts=[7]), a)
    # an explicit group around a collective (ncclGroupStart/End)
    np.testing.assert_array_equal(w.comm.exchange_f64(w.ctx, "allreduce", a, grouped=True), a)
    big = np.random.default_rng(0).normal(size=1 << 20)
    np.testing.assert_array_equal(w.comm.exchange_f64(w.ctx, "allgather", big), big)
    with pytest.raises(Exception):
        w.comm.exchange_f64(w.ctx, "alltoallv", a, send_counts=[7, 0], recv_counts=[7, 0])
    w.comm.barrier()
    assert w.comm.name == "rccl" and not w.comm.trivial


def test_rccl_chunked_alltoallv_rounds(rccl1_world, monkeypatch):
    """The multi-round path of RcclComm::alltoallv (segments above the round size move in
    several grouped send/recv rounds, offsets advancing per round): a 24-byte round size makes
    a 1000-element exchange take 334 rounds; equal to the single-round result."""
    w = rccl1_world
    a = np.random.default_rng(3).normal(size=1000)
    one = w.comm.exchange_f64(w.ctx, "alltoallv", a, send_counts=[1000], recv_counts=[1000])
    monkeypatch.setenv("OAP_RCCL_A2A_CHUNK_BYTES", "24")
    many = w.comm.exchange_f64(w.ctx, "alltoallv", a, send_counts=[1000], recv_counts=[1000])
    np.testing.assert_array_equal(one, a)
    np.testing.assert_array_equal(many, a)


def test_local_comm_is_trivial(gpu_world):
    assert gpu_world.comm.trivial and gpu_world.comm.name == "local"


# ------------------------------------------------------------------------------ drivers
@pytest.mark.parametrize("n,d,k", [(60000, 12, 7), (200000, 50, 64)])
def test_kmeans_forced_rccl_bitwise(n, d, k):
    X = _blobs(n, d, k, 5, sigma=2.0)
    out = {}
    for force in (False, True):
        w = _world(force)
        m = O.KMeans(k=k, seed=3, maxIter=12, tol=0.0).fit(X)
        assert m.fit_info["engine"] == "gpu"
        out[force] = (np.array(m.clusterCenters()), m.summary.trainingCost, m.summary.numIter,
                      w.comm.name)
    O.shutdown_world()
    assert out[True][3] == "rccl" and out[False][3] == "local"
    # fixed-point statistics: the allreduce of one rank is exact, so the fits are bitwise equal
    assert np.array_equal(out[True][0], out[False][0])
    assert out[True][1] == out[False][1] and out[True][2] == out[False][2]


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_pca_forced_rccl_matches_local(dtype):
    """f64 rows: the fp64-MFMA statistics; f32 rows: the int8 digit engine, whose error bound
    rides in the one allreduce (an extra element after [S | c])."""
    rng = np.random.default_rng(9)
    X = (rng.normal(size=(40000, 40)) @ rng.normal(size=(40, 40)) + 20.0).astype(dtype)
    res = {}
    for force in (False, True):
        _world(force)
        m = O.PCA(k=6, inputCol="features").fit(X)
        assert m.fit_info["engine"] == "gpu"
        assert m.fit_info["stats_engine"] == ("int8_digits" if dtype == np.float32
                                              else "fp64_mfma")
        res[force] = (m.pc.toArray(), m.explainedVariance.toArray())
    O.shutdown_world()
    np.testing.assert_allclose(res[True][1], res[False][1], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(np.abs(res[True][0]), np.abs(res[False][0]), atol=1e-9)


def _ratings(nu, ni, nnz, seed):
    rng = np.random.default_rng(seed)
    u = (rng.integers(0, nu, nnz) * 3 + 1).astype(np.int32)
    i = (rng.integers(0, ni, nnz) * 2 + 5).astype(np.int32)
    keep = np.unique(u.astype(np.int64) * 1_000_003 + i, return_index=True)[1]  # no duplicates
    keep.sort()
    r = rng.integers(-1, 6, nnz).astype(np.float32)
    return u[keep], i[keep], r[keep]


@pytest.mark.parametrize("rank", [10, 100])
def test_als_forced_rccl_matches_local(native, monkeypatch, rank):
    """Device shuffle (3 send/recv exchanges) + dist CSR build, the comm-stream Gramian
    allreduce and C=4 chunked owner broadcasts on the comm stream, against the single-rank
    device setup and the host setup of the same 1-rank RCCL world."""
    u, i, r = _ratings(2000, 900, 60000, rank)
    args = (u, i, r, rank, 3, 0.05, 4.0, True, 7)
    w = _world(False)
    loc = native.als_fit(w.ctx, w.comm, *args)
    w = _world(True)
    assert w.comm.name == "rccl"
    dev = native.als_fit(w.ctx, w.comm, *args)
    monkeypatch.setenv("OAP_ALS_HOST_SETUP", "1")
    host = native.als_fit(w.ctx, w.comm, *args)
    monkeypatch.delenv("OAP_ALS_HOST_SETUP")
    O.shutdown_world()
    for o in (dev, host):
        assert np.array_equal(o["user_ids"], loc["user_ids"])
        assert np.array_equal(o["item_ids"], loc["item_ids"])
        assert o["nnz"] == loc["nnz"] == len(r) and o["failed_rows"] == 0
        for key in ("user_factors", "item_factors"):
            np.testing.assert_allclose(o[key], loc[key], rtol=0,
                                       atol=1e-5 * np.abs(loc[key]).max())


def test_als_dist_setup_sparse_ids_fall_back(native, rccl1_world):
    """Ids spread over a 2^30-wide range: the dist device setup declines (rank-uniformly) and
    the host shuffle runs over the RCCL comm (host-buffer alltoallv staged through HBM)."""
    u, i, r = _ratings(500, 300, 8000, 2)
    us = (u.astype(np.int64) * 2_000_003 % (1 << 30)).astype(np.int32)
    out = native.als_fit(rccl1_world.ctx, rccl1_world.comm, us, i, r, 8, 2, 0.1, 2.0, True, 1)
    assert len(out["user_ids"]) == len(np.unique(us)) and out["failed_rows"] == 0
