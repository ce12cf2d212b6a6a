"""PCA tests on the CPU engines (native fp64 C++ path and the vanilla numpy path).

Model: the reference's IntelPCASuite (mllib-dal/src/test/scala/org/apache/spark/ml/feature/
IntelPCASuite.scala:31-104): params, the 3x5 toy fit compared with RowMatrix's
computePrincipalComponentsAndExplainedVariance (explained variance absTol 1e-5, components by
absolute value and only where the variance > 1e-5), PCA / PCAModel read-write.  RowMatrix is not
importable here, so the oracle is the same math in numpy fp64 (sample covariance + eigh);
"parity unpinned" against Spark's own LAPACK output, which the reference does not store.
"""
import os

import numpy as np
import pytest

import oap_mllib_amd as O
from oap_mllib_amd.fallback import pca_vanilla
from oap_mllib_amd.linalg import DenseMatrix, DenseVector, Vectors

REF_DATA = "/root/reference/examples/data/pca_data.csv"


def _oracle(X, k):
    X = np.asarray(X, np.float64)
    C = np.cov(X.T, ddof=1)
    w, V = np.linalg.eigh(C)
    o = np.argsort(-np.abs(w), kind="stable")
    w, V = np.abs(w[o]), V[:, o]
    return V[:, :k], w[:k] / w.sum()


def _check(model, X, k, atol=1e-5):
    pc_ref, ev_ref = _oracle(X, k)
    ev = model.explainedVariance.toArray()
    np.testing.assert_allclose(ev, ev_ref, atol=atol)
    pc = model.pc.toArray()
    assert pc.shape == (X.shape[1], k)
    for j in range(k):
        if ev_ref[j] > 1e-5:
            np.testing.assert_allclose(np.abs(pc[:, j]), np.abs(pc_ref[:, j]), atol=atol)


def test_params():
    p = O.PCA()
    assert p.uid.startswith("pca_")
    assert p.getOutputCol() == p.uid + "__output"
    assert not p.isDefined("k")
    with pytest.raises(ValueError):
        p.setK(0)
    p.setK(3).setInputCol("features")
    assert p.getK() == 3
    m = O.PCAModel("pca", DenseMatrix(2, 2, [0.0, 1.0, 2.0, 3.0]), DenseVector([0.5, 0.5]))
    assert m.uid == "pca" and m.pc.numRows == 2


SUITE_DATA = [Vectors.sparse(5, [(1, 1.0), (3, 7.0)]), Vectors.dense(2.0, 0.0, 3.0, 4.0, 5.0),
              Vectors.dense(4.0, 0.0, 0.0, 6.0, 7.0)]


@pytest.mark.parametrize("world", ["cpu_world", "vanilla_world"])
def test_suite_toy_data(world, request):
    request.getfixturevalue(world)
    X = np.array([v.toArray() for v in SUITE_DATA])
    m = O.PCA(k=3, inputCol="features", outputCol="pca_features").fit(
        {"features": SUITE_DATA})
    assert m.fit_info["engine"] == ("cpu" if world == "cpu_world" else "vanilla")
    _check(m, X, 3)
    out = m.transform({"features": SUITE_DATA})
    Y = np.array([v.toArray() for v in out["pca_features"]])
    np.testing.assert_allclose(Y, X @ m.pc.toArray(), atol=1e-12)


@pytest.mark.skipif(not os.path.exists(REF_DATA), reason="reference example data absent")
def test_reference_example_csv(cpu_world):
    X = np.loadtxt(REF_DATA, delimiter=",")
    m = O.PCA(k=3, inputCol="features").fit(X)
    _check(m, X, 3)


@pytest.mark.parametrize("n,d,k", [(500, 7, 3), (64, 130, 10), (40, 200, 60), (300, 129, 129)])
def test_native_cpu_matches_oracle(cpu_world, n, d, k):
    rng = np.random.default_rng(n + d)
    X = rng.normal(size=(n, d)) @ rng.normal(size=(d, d)) * 0.3 + rng.normal(size=d) * 100
    m = O.PCA(k=k, inputCol="features").fit(X)
    _check(m, X, k, atol=1e-7)


def test_native_equals_vanilla_signs(cpu_world):
    rng = np.random.default_rng(1)
    X = rng.normal(size=(400, 9)) * np.arange(1, 10)
    m = O.PCA(k=4, inputCol="features").fit(X)
    pc, ev = pca_vanilla.fit(X, 4)
    np.testing.assert_allclose(m.pc.toArray(), pc, atol=1e-9)
    np.testing.assert_allclose(m.explainedVariance.toArray(), ev, atol=1e-12)


def test_large_offset_no_cancellation(cpu_world):
    rng = np.random.default_rng(3)
    X = rng.normal(size=(2000, 5)) * [1.0, 0.5, 0.25, 0.1, 0.01] + 1e6
    m = O.PCA(k=5, inputCol="features").fit(X)
    _check(m, X, 5, atol=1e-6)


def test_k_larger_than_features_rejected(cpu_world):
    with pytest.raises(ValueError):
        O.PCA(k=6, inputCol="features").fit(np.ones((10, 5)))


def test_feature_cap_falls_back(cpu_world):
    cfg = cpu_world.config
    old = cfg.pca_max_features
    try:
        cfg.pca_max_features = 4
        m = O.PCA(k=2, inputCol="features").fit(np.random.default_rng(0).normal(size=(50, 6)))
        assert m.fit_info["engine"] == "vanilla"
    finally:
        cfg.pca_max_features = old


def test_sym_eig_direct(native):
    rng = np.random.default_rng(0)
    for n in (1, 2, 3, 17, 100):
        A = rng.normal(size=(n, n))
        A = A + A.T
        for k in (1, n):
            w, V = native.sym_eig(A, k)
            wr = np.linalg.eigvalsh(A)
            wr = wr[np.argsort(-np.abs(wr))]
            np.testing.assert_allclose(w, wr, atol=1e-11 * n)
            np.testing.assert_allclose(A @ V, V * np.asarray(w)[:k], atol=1e-10 * n)
            np.testing.assert_allclose(V.T @ V, np.eye(k), atol=1e-10)
    # rank-deficient covariance (many zero eigenvalues) and exact multiplicities
    X = rng.normal(size=(20, 60))
    C = np.cov(X.T)
    w, V = native.sym_eig(C, 30)
    np.testing.assert_allclose(C @ V, V * np.asarray(w)[:30], atol=1e-12)
    np.testing.assert_allclose(V.T @ V, np.eye(30), atol=1e-12)
    Q, _ = np.linalg.qr(rng.normal(size=(6, 6)))
    A = Q @ np.diag([3.0, 3.0, 3.0, 1.0, 1.0, 0.0]) @ Q.T
    w, V = native.sym_eig(A, 5)
    np.testing.assert_allclose(w, [3, 3, 3, 1, 1, 0], atol=1e-12)
    np.testing.assert_allclose(V.T @ V, np.eye(5), atol=1e-12)


def test_pca_read_write(tmp_path, cpu_world):
    t = O.PCA(inputCol="myInputCol", outputCol="myOutputCol", k=3)
    t.save(str(tmp_path / "est"))
    t2 = O.PCA.load(str(tmp_path / "est"))
    assert t2.uid == t.uid and t2.getK() == 3 and t2.getOutputCol() == "myOutputCol"
    inst = O.PCAModel("myPCAModel", DenseMatrix(2, 2, [0.0, 1.0, 2.0, 3.0]),
                      DenseVector([0.5, 0.5]))
    inst.save(str(tmp_path / "model"))
    m2 = O.PCAModel.load(str(tmp_path / "model"))
    assert m2.uid == "myPCAModel" and m2.pc == inst.pc
    np.testing.assert_array_equal(m2.explainedVariance.toArray(), [0.5, 0.5])
    meta = (tmp_path / "model" / "metadata" / "part-00000").read_text()
    assert '"class":"org.apache.spark.ml.feature.PCAModel"' in meta.replace(" ", "")
    import pyarrow.parquet as pq

    files = [f for f in os.listdir(tmp_path / "model" / "data") if f.endswith(".parquet")]
    tab = pq.read_table(str(tmp_path / "model" / "data" / files[0]))
    assert tab.column_names == ["pc", "explainedVariance"]


def test_pca_distributed_matches_single():
    from mp_util import run_world

    from dist_workers import pca_native

    rc, outs = run_world("dist_workers", "pca_native", nproc=2, device="cpu")
    assert rc == 0, outs
    O.shutdown_world()
    ref = pca_native(device="cpu")
    O.shutdown_world()
    for o in outs:
        assert o["engine"] == "cpu"
        np.testing.assert_allclose(o["ev"], ref["ev"], atol=1e-12)
        np.testing.assert_allclose(o["pc"], ref["pc"], atol=1e-9)
