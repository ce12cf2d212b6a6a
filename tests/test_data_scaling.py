"""Estimator-scale data handling: zero-copy Arrow / numpy adapters, a K-Means fit whose summary
comes from the fit's own labels (no per-row Python objects), contiguous ALS factors, and the
rank-uniform streamed-fit decision (the reference marshals rows through one JNI call per row,
OneDAL.scala:116-142; the summary is a second Spark pass, KMeans.scala:359-368)."""
import tracemalloc

import numpy as np
import pandas as pd
import pyarrow as pa
import pytest

import oap_mllib_amd as O
from oap_mllib_amd.data import as_frame, to_matrix, vector_column


def test_arrow_fixed_size_and_list_columns_zero_copy():
    X = np.random.default_rng(0).normal(size=(1000, 7))
    fsl = pa.FixedSizeListArray.from_arrays(pa.array(X.reshape(-1)), 7)
    t = pa.table({"id": np.arange(1000), "features": fsl})
    np.testing.assert_array_equal(to_matrix(t), X)
    # a sliced (offset) chunk and a chunked column
    t2 = pa.Table.from_batches(t.to_batches(max_chunksize=300))
    np.testing.assert_array_equal(to_matrix(t2), X)
    np.testing.assert_array_equal(to_matrix(t.slice(10, 50)), X[10:60])
    lst = pa.ListArray.from_arrays(pa.array(np.arange(1001, dtype=np.int32) * 7),
                                   pa.array(X.reshape(-1)))
    np.testing.assert_array_equal(to_matrix(pa.table({"features": lst})), X)
    ragged = pa.ListArray.from_arrays(pa.array([0, 2, 5], pa.int32()), pa.array(np.ones(5)))
    with pytest.raises(ValueError):
        to_matrix(pa.table({"features": ragged}))


def test_vector_udt_struct_dense_and_sparse():
    from oap_mllib_amd.persistence import spark_format as sf

    X = np.arange(12, dtype=np.float64).reshape(4, 3)
    rows = [sf.dense_vector_struct(r) for r in X]
    t = pa.table({"features": pa.array(rows, type=sf.VECTOR_ARROW)})
    np.testing.assert_array_equal(to_matrix(t), X)
    sp = {"type": 0, "size": 3, "indices": [1], "values": [5.0]}
    t2 = pa.table({"features": pa.array(rows[:2] + [sp], type=sf.VECTOR_ARROW)})
    np.testing.assert_array_equal(to_matrix(t2), np.array([X[0], X[1], [0, 5.0, 0]]))


def test_numpy_frame_is_one_arrow_buffer():
    X = np.random.default_rng(1).normal(size=(5000, 4))
    df = as_frame(X)
    assert isinstance(df["features"].dtype, pd.ArrowDtype)
    np.testing.assert_array_equal(to_matrix(df), X)
    s = vector_column(X.astype(np.float32))
    assert to_matrix(pd.DataFrame({"features": s})).dtype == np.float32


def test_kmeans_fit_10m_rows_allocates_no_per_row_objects(cpu_world):
    rng = np.random.default_rng(2)
    C = rng.uniform(-10, 10, (3, 4))
    X = (C[rng.integers(0, 3, 10_000_000)] + rng.normal(0, 0.5, (10_000_000, 4)))
    tracemalloc.start()
    snap0 = tracemalloc.take_snapshot()
    m = O.KMeans(k=3, maxIter=3, seed=1).fit(X)
    sizes = m.summary.clusterSizes
    snap1 = tracemalloc.take_snapshot()
    tracemalloc.stop()
    blocks = sum(s.count_diff for s in snap1.compare_to(snap0, "filename") if s.count_diff > 0)
    assert blocks < 50_000, blocks  # per-row objects would be >= 10M blocks
    assert sum(sizes) == len(X) and m.fit_info["engine"] == "cpu"
    assert len(m.summary.cluster) == len(X)
    # the lazily built predictions frame matches a transform
    pred = m.summary.predictions["prediction"].to_numpy()[:1000]
    np.testing.assert_array_equal(pred, m.transform(X[:1000])["prediction"].to_numpy())


def test_pca_transform_of_matrix_is_arrow(cpu_world):
    X = np.random.default_rng(3).normal(size=(2000, 6))
    m = O.PCA(k=2, inputCol="features", outputCol="out").fit(X)
    out = m.transform(X)
    assert isinstance(out["out"].dtype, pd.ArrowDtype)
    np.testing.assert_allclose(to_matrix(out, "out"), X @ m.pc.toArray(), atol=1e-12)


def test_als_model_contiguous_factors_roundtrip(cpu_world, tmp_path):
    rng = np.random.default_rng(4)
    u = rng.integers(0, 50, 2000)
    i = rng.integers(0, 40, 2000)
    r = rng.integers(1, 5, 2000).astype(np.float64)
    m = O.ALS(rank=4, maxIter=2, implicitPrefs=True, seed=0).fit(
        {"user": u, "item": i, "rating": r})
    ids, F = m._mat("user")
    assert F.flags.c_contiguous and F.dtype == np.float32 and np.all(np.diff(ids) > 0)
    uf = m.userFactors
    assert isinstance(uf["features"].dtype, pd.ArrowDtype) and len(uf) == len(ids)
    recs = m.recommendForAllUsers(3)
    first = list(recs["recommendations"])[0]
    assert len(first) == 3 and set(first[0]) == {"item", "rating"}
    m.save(str(tmp_path / "als"))
    m2 = O.ALSModel.load(str(tmp_path / "als"))
    for w in ("user", "item"):
        np.testing.assert_array_equal(m2._mat(w)[0], m._mat(w)[0])
        np.testing.assert_array_equal(m2._mat(w)[1], m._mat(w)[1])
    # a frame assigned by the user is taken over as arrays
    m2.userFactors = uf.iloc[:5]
    assert len(m2._mat("user")[0]) == 5


class _FakeWorld:
    """Two ranks; allreduce over both shards' values (the collective the decision uses)."""

    def __init__(self, peer_value):
        self.peer = peer_value
        self.distributed = True
        self.is_gpu = True

    def allreduce_np(self, a, op="sum"):
        return np.maximum(a, self.peer) if op == "max" else a + self.peer


def test_streamed_decision_is_rank_uniform(monkeypatch):
    """One shard over a small HBM budget: BOTH ranks take the streamed fit."""
    from oap_mllib_amd.models import clustering as C

    calls = []

    def fake_streamed(w, X):
        calls.append(len(X))
        return len(X) > 100

    monkeypatch.setattr(C, "_streamed", fake_streamed)
    small = np.zeros((10, 3))
    assert C.streamed_decision(_FakeWorld(np.array([1.0])), small, "gpu") is True
    assert C.streamed_decision(_FakeWorld(np.array([0.0])), small, "gpu") is False
    assert C.streamed_decision(_FakeWorld(np.array([1.0])), small, "cpu") is False
