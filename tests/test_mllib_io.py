"""RDD-style mllib KMeans API and the native text readers (CPU engines).

The reference's examples (examples/kmeans*, examples/data/*) train on
sample_kmeans_data.txt (LIBSVM), pca_data.csv and onedal_als_csr_ratings.txt; those files are
read here with the native parallel readers and the expected results are checked directly
(the reference holds no golden outputs for them: parity unpinned)."""
import os

import numpy as np
import pytest

import oap_mllib_amd as O
from oap_mllib_amd.mllib.clustering import KMeans, KMeansModel
from oap_mllib_amd.utils import io

DATA = "/root/reference/examples/data"
needs_data = pytest.mark.skipif(not os.path.isdir(DATA), reason="reference example data absent")


def _blobs(seed=0):
    rng = np.random.default_rng(seed)
    c = np.array([[0.0, 0.0], [10.0, 10.0], [-10.0, 10.0]])
    return c[rng.integers(0, 3, 600)] + rng.normal(0, 0.3, (600, 2))


@pytest.mark.parametrize("world", ["cpu_world", "vanilla_world"])
def test_train_predict_cost(world, request):
    request.getfixturevalue(world)
    X = _blobs()
    m = KMeans.train(X, 3, maxIterations=20, seed=7)
    assert m.k == 3 and len(m.clusterCenters) == 3
    lab = m.predict(X)
    assert lab.shape == (600,) and len(set(lab.tolist())) == 3
    assert m.predict(X[0]) == lab[0]
    cost = m.computeCost(X)
    assert cost == pytest.approx(m.trainingCost, rel=1e-9)
    assert cost / len(X) < 2 * 0.3 ** 2 * 1.5


def test_initial_model_and_random_init(cpu_world):
    X = _blobs(1)
    init = KMeansModel(np.array([[1.0, 1.0], [9.0, 9.0], [-9.0, 9.0]]))
    m = KMeans.train(X, 3, maxIterations=5, initialModel=init)
    order = np.argsort(m.centers[:, 0])
    np.testing.assert_allclose(m.centers[order], [[-10, 10], [0, 0], [10, 10]], atol=0.1)
    r = KMeans.train(X, 3, maxIterations=10, initializationMode="random", seed=3)
    assert r.k == 3
    with pytest.raises(ValueError):
        KMeans.train(X, 0)


def test_cosine_runs_vanilla(cpu_world):
    X = _blobs(2) + 20.0
    m = KMeans.train(X, 2, maxIterations=5, seed=1, distanceMeasure="cosine")
    assert m.distanceMeasure == "cosine" and m.k == 2


def test_mllib_save_load(tmp_path, cpu_world):
    m = KMeans.train(_blobs(), 3, maxIterations=10, seed=5)
    m.save(None, str(tmp_path / "m"))
    m2 = KMeansModel.load(None, str(tmp_path / "m"))
    np.testing.assert_array_equal(m2.centers, m.centers)
    assert m2.trainingCost == pytest.approx(m.trainingCost)
    meta = (tmp_path / "m" / "metadata" / "part-00000").read_text()
    assert '"class":"org.apache.spark.mllib.clustering.KMeansModel"' in meta


def test_readers_roundtrip(tmp_path, native):
    X = np.random.default_rng(0).normal(size=(1000, 7))
    p = tmp_path / "x.csv"
    np.savetxt(p, X, delimiter=",", fmt="%.17g")
    np.testing.assert_array_equal(io.read_csv(str(p)), X)
    lines = ["1 1:0.5 3:2", "", "# comment", "0 2:-1.25", "2"]
    (tmp_path / "s.txt").write_text("\n".join(lines) + "\n")
    lab, D = io.read_libsvm(str(tmp_path / "s.txt"))
    np.testing.assert_array_equal(lab, [1, 0, 2])
    np.testing.assert_array_equal(D, [[0.5, 0, 2], [0, -1.25, 0], [0, 0, 0]])
    _, S = io.read_libsvm(str(tmp_path / "s.txt"), num_features=5, dense=False)
    assert S[0].size == 5 and S[0].indices.tolist() == [0, 2]
    (tmp_path / "r.txt").write_text("1::2::3.5\n4::5::-1\n7::8\n")
    r = io.read_ratings(str(tmp_path / "r.txt"))
    assert r["user"].tolist() == [1, 4, 7] and r["rating"].tolist() == [3.5, -1.0, 1.0]
    (tmp_path / "bad.csv").write_text("1,2\n3\n")
    with pytest.raises(O._loader.load().OapError):
        io.read_csv(str(tmp_path / "bad.csv"))


@needs_data
def test_reference_examples_end_to_end(cpu_world):
    _, X = io.read_libsvm(os.path.join(DATA, "sample_kmeans_data.txt"))
    km = O.KMeans(k=2, seed=1).fit(X)
    c = np.sort(np.array(km.clusterCenters())[:, 0])
    np.testing.assert_allclose(c, [0.1, 9.1], atol=1e-9)
    P = io.read_csv(os.path.join(DATA, "pca_data.csv"))
    pca = O.PCA(k=3, inputCol="features").fit(P)
    assert pca.pc.numRows == 5 and pca.explainedVariance.size == 3
    r = io.read_ratings(os.path.join(DATA, "onedal_als_csr_ratings.txt"))
    assert len(r["user"]) == 167
    als = O.ALS(rank=10, maxIter=5, regParam=0.01, alpha=40.0, implicitPrefs=True).fit(r)
    assert als.fit_info["engine"] == "cpu" and len(als.userFactors) == len(set(r["user"]))
