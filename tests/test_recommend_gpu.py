"""Fused score + top-k kernel of recommendForAll* (csrc/kernels/als_recommend.hip) against an
fp64 numpy oracle of the same scores: the picks must be as good as the exact top-num (every
returned score within the split-fp16 tolerance of the exact num-th best, sorted, distinct),
the returned values the exact scores of the returned indices, and the index sets equal to the
oracle's wherever the oracle has no near-tie at its boundary."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def native():
    from oap_mllib_amd import _loader

    N = _loader.load()
    if N.visible_device_count() < 1:
        pytest.skip("no GPU")
    return N


@pytest.fixture(scope="module")
def ctx(native):
    return native.Context(0, 0.5, 0)


def _check(S, D, idx, val, num):
    S64, D64 = S.astype(np.float64), D.astype(np.float64)
    exact = S64 @ D64.T
    mag = np.abs(S64) @ np.abs(D64).T  # sum |s_k d_k|: the tolerance's scale
    tol = 4e-6 * mag.max(axis=1) + 1e-30
    order = np.argsort(-exact, axis=1, kind="stable")[:, :num]
    best = np.take_along_axis(exact, order, axis=1)
    assert idx.shape == (len(S), num) and val.shape == (len(S), num)
    assert (idx >= 0).all() and (idx < len(D)).all()
    for i in range(len(S)):
        assert len(set(idx[i].tolist())) == num
    got = np.take_along_axis(exact, idx.astype(np.int64), axis=1)
    lim = np.broadcast_to(tol[:, None], got.shape)
    np.testing.assert_array_less(np.abs(got - val), lim)  # values = the exact scores
    np.testing.assert_array_less(best - got, 2 * lim)  # as good as the exact top-num
    assert (np.diff(val, axis=1) <= 0).all()  # sorted descending
    # away from boundary near-ties the index sets are the oracle's
    nxt = np.sort(exact, axis=1)[:, ::-1][:, num] if exact.shape[1] > num else \
        np.full(len(S), -np.inf)
    clear = (best[:, -1] - nxt) > 4 * tol
    for i in np.nonzero(clear)[0]:
        assert set(idx[i].tolist()) == set(order[i].tolist())


@pytest.mark.parametrize("n,m,rank,num", [(1000, 777, 10, 10), (600, 300, 1, 5),
                                          (700, 1000, 100, 10), (513, 129, 64, 16),
                                          (300, 2000, 100, 24), (300, 500, 129, 10),
                                          (260, 400, 256, 16), (100, 64, 16, 17)])
def test_topk_matches_oracle(native, ctx, n, m, rank, num):
    rng = np.random.default_rng(n + m + rank)
    S = rng.normal(0, 1, size=(n, rank)).astype(np.float32)
    D = (rng.normal(0, 0.3, size=(m, rank)) + 0.1).astype(np.float32)
    idx, val, info = native.als_recommend(ctx, S, D, num)
    _check(S, D, idx, val, num)
    assert info["slabs"] == 1


@pytest.mark.parametrize("n,m,rank,num", [(300, 5000, 10, 100), (200, 3000, 64, 1000),
                                          (150, 1400, 129, 600), (70, 4500, 8, 3000),
                                          (97, 2100, 33, 1016)])
def test_large_num_matches_oracle(native, ctx, n, m, rank, num):
    """num beyond the LDS lists: the HBM candidate-buffer variant (4 waves up to num 1016, one
    wave with the 64 KiB sort buffer above), against the same fp64 oracle."""
    assert num > 24 and num <= native.als_recommend_max_num(rank)
    rng = np.random.default_rng(n + m + rank + num)
    S = rng.normal(0, 1, size=(n, rank)).astype(np.float32)
    D = (rng.normal(0, 0.3, size=(m, rank)) + 0.1).astype(np.float32)
    idx, val, info = native.als_recommend(ctx, S, D, num)
    _check(S, D, idx, val, num)
    assert info["slabs"] == 1


def test_large_num_ties_and_padding(native, ctx):
    """Duplicate destinations (exact ties: lower index first) and fewer destinations than num
    in the HBM-buffer variant."""
    rng = np.random.default_rng(5)
    S = rng.normal(size=(90, 16)).astype(np.float32)
    D = np.repeat(rng.normal(size=(40, 16)).astype(np.float32), 3, axis=0)  # 120 rows
    idx, val, _ = native.als_recommend(ctx, S, D, 100)
    _check(S, D, idx, val, 100)
    for i in range(len(S)):  # among equal scores, indices ascend
        same = np.nonzero(np.diff(val[i]) == 0)[0]
        assert (idx[i][same] < idx[i][same + 1]).all()
    idx, val, _ = native.als_recommend(ctx, S, D[:70], 100)
    assert (idx[:, 70:] == -1).all() and np.isneginf(val[:, 70:]).all()
    _check(S, D[:70], idx[:, :70], val[:, :70], 70)


def test_slabs_and_scale(native, ctx):
    """Several source slabs (each with its own fp16 scale) give the one-slab answer."""
    rng = np.random.default_rng(7)
    S = (rng.normal(0, 1, size=(3000, 40)) * np.exp(rng.normal(0, 2, size=(3000, 1))))
    S = S.astype(np.float32)
    D = rng.normal(0, 5e-3, size=(900, 40)).astype(np.float32)
    i1, v1, _ = native.als_recommend(ctx, S, D, 10)
    i2, v2, info = native.als_recommend(ctx, S, D, 10, slab_rows=512)
    assert info["slabs"] == 6
    _check(S, D, i2, v2, 10)
    assert (i1 == i2).all()


def test_fewer_destinations_than_num(native, ctx):
    rng = np.random.default_rng(3)
    S = rng.normal(size=(70, 8)).astype(np.float32)
    D = rng.normal(size=(5, 8)).astype(np.float32)
    idx, val, _ = native.als_recommend(ctx, S, D, 8)
    assert (idx[:, 5:] == -1).all() and np.isneginf(val[:, 5:]).all()
    _check(S, D, idx[:, :5], val[:, :5], 5)


def test_model_recommend_uses_kernel(native, gpu_world):
    """ALSModel.recommendForAllUsers on a GPU world goes through the kernel: the same picks as
    the oracle (sets away from near-ties), int64 indices, the frame's rows in user order."""
    import oap_mllib_amd as om
    from oap_mllib_amd.models import recommendation as rec

    assert gpu_world.is_gpu
    rng = np.random.default_rng(11)
    U = rng.normal(size=(400, 12)).astype(np.float32)
    V = rng.normal(size=(333, 12)).astype(np.float32)
    idx, val = rec._blocked_topk(U, V, 10)
    assert idx.dtype == np.int64
    _check(U, V, idx, val, 10)
    model = om.ALSModel(rank=12, user_arrays=(np.arange(400) * 3, U),
                        item_arrays=(np.arange(333) + 5, V))
    df = model.recommendForAllUsers(10)
    recs = df["recommendations"].tolist()
    assert [r[0]["item"] for r in recs] == [int(5 + j) for j in idx[:, 0]]


def test_model_recommend_large_num_on_kernel(native, gpu_world):
    """recommendForAllUsers(num=1000) stays on the kernel (no host-scoring warning)."""
    import warnings

    from oap_mllib_amd.models import recommendation as rec

    rng = np.random.default_rng(12)
    U = rng.normal(size=(150, 20)).astype(np.float32)
    V = rng.normal(size=(2500, 20)).astype(np.float32)
    with warnings.catch_warnings():
        warnings.simplefilter("error", RuntimeWarning)
        idx, val = rec._blocked_topk(U, V, 1000)
    _check(U, V, idx, val, 1000)
