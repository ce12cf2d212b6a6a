"""Multi-process (gloo, world size 2-3) tests of the distributed paths on CPU.

The reference's only multi-rank coverage is a pseudo-YARN cluster that runs the examples without
assertions.  Here real multi-process worlds check that the distributed fit equals
the single-process fit: with fixed-point centroid accumulation the result is BITWISE identical
for any world size (the sums are integers), which is asserted directly."""
import numpy as np
import pytest

from mp_util import run_world


def _single(**kw):
    import oap_mllib_amd as O
    from dist_workers import kmeans_native

    O.shutdown_world()
    r = kmeans_native(**kw)
    O.shutdown_world()
    return r


@pytest.mark.parametrize("nproc", [2, 3])
def test_kmeans_native_cpu_world_matches_single_process(nproc):
    rc, outs = run_world("dist_workers", "kmeans_native", nproc=nproc, device="cpu")
    assert rc == 0, outs
    ref = _single(device="cpu")
    for o in outs:
        assert o["size"] == nproc and o["engine"] == "cpu" and o["comm"] == "host"
        assert o["iters"] == ref["iters"]
        assert np.array_equal(np.array(o["centers"]), np.array(ref["centers"]))
        np.testing.assert_allclose(o["cost"], ref["cost"], rtol=1e-12)


def test_kmeans_rank_without_rows_cpu():
    """A rank that holds no rows still joins every collective of the fit (tol >= 0)."""
    from dist_workers import kmeans_uneven

    kw = dict(n=30000, d=8, k=9, device="cpu")
    rc, outs = run_world("dist_workers", "kmeans_uneven", nproc=2, empty_rank=0, **kw)
    assert rc == 0, outs
    import oap_mllib_amd as O

    O.shutdown_world()
    ref = kmeans_uneven(**kw)
    O.shutdown_world()
    for o in outs:
        assert o["iters"] == ref["iters"]
        assert np.array_equal(np.array(o["centers"]), np.array(ref["centers"]))


def test_kmeans_random_init_world_size_independent():
    rc, outs = run_world("dist_workers", "kmeans_native", nproc=2, device="cpu",
                         init_mode="random")
    assert rc == 0
    ref = _single(device="cpu", init_mode="random")
    assert np.array_equal(np.array(outs[0]["centers"]), np.array(ref["centers"]))


def test_vanilla_distributed_allreduce():
    rc, outs = run_world("dist_workers", "kmeans_vanilla", nproc=2)
    assert rc == 0
    from dist_workers import _blobs
    from oap_mllib_amd.fallback import kmeans_vanilla as V

    X = _blobs(2000, 4, 3, 3)
    ref = V.fit(X, 3, 10, 0.0, init_centers=X[:3])
    np.testing.assert_allclose(np.array(outs[0]["centers"]), ref.centers, rtol=1e-10)


def test_host_comm_collectives():
    rc, outs = run_world("dist_workers", "host_comm_collectives", nproc=2)
    assert rc == 0
    assert outs[0]["sum"] == [0.0, 3.0, 6.0, 9.0, 12.0]
    assert outs[1]["max"] == [1.0]
    assert (outs[0]["offset"], outs[1]["offset"]) == (0, 3)
    assert outs[0]["total"] == outs[1]["total"] == 7


def test_fault_injection_no_hang():
    """A rank that fails mid-fit must not leave its peer hanging (launcher gang-kills)."""
    rc, _ = run_world("dist_workers", "fault_injection", nproc=2, timeout=120,
                      env={"OAP_MLLIB_FAULT": "1:kmeans_iter:0"})
    assert rc not in (0, 124), rc


@pytest.mark.parametrize("nproc,piece", [(3, 0), (4, 64), (2, 40)])
def test_tcp_comm_streamed_alltoallv(nproc, piece):
    """The KVS TcpComm (JNI / C ABI worlds) routes alltoallv through rank 0 one bounded piece at
    a time (never the world's whole exchange): uneven and empty segments, 2-4 ranks, pieces of
    a few elements, plus allreduce / allgather on the same sockets."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    rc, outs = run_world("dist_workers", "tcp_alltoallv", nproc=nproc, port=port, piece=piece)
    assert rc == 0, outs
    for o in outs:
        assert o == {"a2a": True, "allreduce": True, "allgather": True}, outs


def test_recommend_for_user_subset_per_rank():
    """Subset calls score each rank's own keys locally (no cross-rank slab exchange), so ranks
    with different subsets each get exactly their users' recommendations."""
    rc, outs = run_world("dist_workers", "recommend_subset", nproc=2)
    assert rc == 0, outs
    rng = np.random.default_rng(4)
    U = rng.normal(size=(120, 5)).astype(np.float32)
    V = rng.normal(size=(40, 5)).astype(np.float32)
    sc = U @ V.T
    for o in outs:
        assert sorted(int(u) for u in o["recs"]) == sorted(o["users"])
        for u, items in o["recs"].items():
            want = np.lexsort((np.arange(40), -sc[int(u)]))[:6].tolist()
            assert items == want, (u, items, want)


def test_recommend_for_all_sharded_by_rank():
    """Each rank of a 2-rank world scores only its own slab of users (the result is the
    single-process one on every rank)."""
    rc, outs = run_world("dist_workers", "recommend_sharded", nproc=2)
    assert rc == 0
    from oap_mllib_amd.models.recommendation import _local_topk

    rng = np.random.default_rng(9)
    U = rng.normal(size=(301, 6)).astype(np.float32)
    V = rng.normal(size=(57, 6)).astype(np.float32)

    class W:
        is_gpu = False

    idx, val = _local_topk(U, V, 7, W(), 4096)
    assert outs[0]["rows_scored"] == [150] and outs[1]["rows_scored"] == [151]
    for o in outs:
        assert np.array_equal(np.array(o["idx"]), idx)
        np.testing.assert_array_equal(np.array(o["val"], dtype=np.float32), val)
        assert o["first"] == idx[:, 0].tolist()
