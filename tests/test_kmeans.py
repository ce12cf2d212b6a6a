"""K-Means tests (CPU): the reference's IntelKMeansSuite semantics
(mllib-dal/src/test/scala/org/apache/spark/ml/clustering/IntelKMeansSuite.scala) on the native
CPU engine, plus engine-vs-fp64-oracle checks.  GPU variants live in test_kmeans_gpu.py."""
import numpy as np
import pandas as pd
import pytest

import oap_mllib_amd as O
from oap_mllib_amd import KMeans, KMeansModel, Vectors
from oap_mllib_amd.fallback import kmeans_vanilla as vanilla


def generate_kmeans_data(rows=50, dim=3, k=5):
    # KMeansSuite.generateKMeansData: row i (1-based) = Array.fill(dim)(i % k)
    return pd.DataFrame({"features": [Vectors.dense([float(i % k)] * dim)
                                      for i in range(1, rows + 1)]})


def blobs(n=3000, d=8, k=6, seed=0, sigma=0.3):
    rng = np.random.default_rng(seed)
    c = rng.uniform(-10, 10, size=(k, d))
    return c[rng.integers(0, k, n)] + rng.normal(0, sigma, size=(n, d)), c


# -------------------------------------------------------------------- params (:50-108)
def test_default_parameters(cpu_world):
    km = KMeans()
    assert km.getK() == 2
    assert km.getFeaturesCol() == "features"
    assert km.getPredictionCol() == "prediction"
    assert km.getMaxIter() == 20
    assert km.getInitMode() == "k-means||"
    assert km.getInitSteps() == 2
    assert km.getTol() == 1e-4
    assert km.getDistanceMeasure() == "euclidean"
    model = km.setMaxIter(1).fit(generate_kmeans_data())
    assert model.hasParent()
    assert model.numFeatures == 3


def test_set_and_validate_params():
    km = KMeans().setK(9).setFeaturesCol("test_feature").setPredictionCol("test_prediction") \
        .setMaxIter(33).setInitMode("random").setInitSteps(3).setSeed(123).setTol(1e-3) \
        .setDistanceMeasure("cosine")
    assert (km.getK(), km.getMaxIter(), km.getInitMode(), km.getInitSteps(), km.getSeed(),
            km.getTol(), km.getDistanceMeasure()) == (9, 33, "random", 3, 123, 1e-3, "cosine")
    for bad in (lambda: KMeans().setK(1), lambda: KMeans().setInitMode("no_such_a_mode"),
                lambda: KMeans().setInitSteps(0), lambda: KMeans().setDistanceMeasure("nope")):
        with pytest.raises(ValueError):
            bad()


# -------------------------------------------------------- fit/transform/summary (:110-145)
@pytest.mark.parametrize("world", ["cpu_world", "vanilla_world"])
def test_fit_transform_and_summary(world, request):
    request.getfixturevalue(world)
    df = generate_kmeans_data()
    model = KMeans().setK(5).setPredictionCol("kmeans_prediction").setSeed(1).fit(df)
    assert len(model.clusterCenters()) == 5
    out = model.transform(df)
    assert set(out["kmeans_prediction"]) == {0, 1, 2, 3, 4}
    s = model.summary
    assert s.predictionCol == "kmeans_prediction" and s.featuresCol == "features"
    assert len(s.predictions) == len(df)
    assert list(s.cluster.columns) == ["kmeans_prediction"]
    assert s.trainingCost < 0.1
    assert len(s.clusterSizes) == 5 and sum(s.clusterSizes) == len(df)
    assert s.numIter == 1
    model.setSummary(None)
    assert not model.hasSummary


def test_non_default_columns(cpu_world):
    df = generate_kmeans_data().rename(columns={"features": "kmeans_model_features"})
    model = KMeans(k=5, seed=1, featuresCol="kmeans_model_features",
                   predictionCol="kmeans_model_prediction").fit(df)
    out = model.transform(df)
    assert "kmeans_model_prediction" in out.columns


def test_cosine_uses_vanilla_path(cpu_world):
    df = pd.DataFrame({"features": [Vectors.dense(v) for v in
                                    [(1.0, 1.0), (10.0, 10.0), (1.0, 0.5), (10.0, 4.4),
                                     (-1.0, 1.0), (-100.0, 90.0)]]})
    model = KMeans(k=3, seed=1, distanceMeasure="cosine").fit(df)
    assert model.fit_info["engine"] == "vanilla"
    pred = model.transform(df)["prediction"].tolist()
    assert len(set(pred)) == 3
    assert pred[0] == pred[1] and pred[2] == pred[3] and pred[4] == pred[5]
    for c in model.clusterCenters():
        assert abs(np.linalg.norm(c) - 1.0) < 1e-10


def test_numpy_and_list_inputs(cpu_world):
    X, _ = blobs(400, 4, 3)
    m1 = KMeans(k=3, seed=5).fit(X)
    m2 = KMeans(k=3, seed=5).fit([Vectors.dense(r) for r in X])
    np.testing.assert_allclose(np.array(m1.clusterCenters()), np.array(m2.clusterCenters()))


def test_single_instance_prediction(cpu_world):
    df = generate_kmeans_data()
    model = KMeans(k=5, seed=1).fit(df)
    out = model.transform(df)
    for f, p in zip(out["features"], out["prediction"]):
        assert model.predict(f) == p


# ----------------------------------------------------------- four centers (:413-480)
FOUR = [(0.1, 0.1), (5.0, 0.2), (10.0, 0.0), (15.0, 0.5), (32.0, 18.0), (30.1, 20.0),
        (-6.0, -6.0), (-10.0, -10.0)]


def test_four_centers_native_equals_weighted_vanilla(cpu_world):
    df1 = pd.DataFrame({"features": [Vectors.dense(v) for v in FOUR]})
    m1 = KMeans(k=4, initMode="k-means||", maxIter=10).fit(df1)
    assert m1.fit_info["engine"] == "cpu"
    p1 = dict(zip(map(tuple, (f.toArray() for f in df1["features"])),
                  m1.transform(df1)["prediction"]))
    assert len(set(p1.values())) == 4
    for a, b in [(0, 1), (2, 3), (4, 5), (6, 7)]:
        assert p1[FOUR[a]] == p1[FOUR[b]]
    df2 = pd.DataFrame({"features": [Vectors.dense(v) for v in FOUR], "weightCol": [2.0] * 8})
    m2 = KMeans(k=4, initMode="k-means||", maxIter=10, weightCol="weightCol").fit(df2)
    assert m2.fit_info["engine"] == "vanilla"
    p2 = dict(zip(map(tuple, (f.toArray() for f in df2["features"])),
                  m2.transform(df2)["prediction"]))
    for a, b in [(0, 1), (2, 3), (4, 5), (6, 7)]:
        assert p2[FOUR[a]] == p2[FOUR[b]]
    # same partition of the points => same set of centers (label order may differ)
    c1 = sorted(map(tuple, np.round(np.array(m1.clusterCenters()), 10)))
    c2 = sorted(map(tuple, np.round(np.array(m2.clusterCenters()), 10)))
    np.testing.assert_allclose(np.array(c1), np.array(c2), atol=1e-9)


# ------------------------------------------------------------ oracle equivalence
def test_native_cpu_matches_fp64_oracle_given_init(cpu_world, native):
    X, _ = blobs(5000, 12, 7, seed=3, sigma=1.0)
    init = X[:7].copy()
    w = O.get_world()
    t = native.upload_dense(w.ctx, X, "f64", 12)
    r = native.kmeans_fit(w.ctx, w.comm, t, init, 7, 15, 0.0)
    ref = vanilla.fit(X, 7, 15, 0.0, init_centers=init)
    assert r["num_iter"] == ref.num_iter == 15
    np.testing.assert_allclose(r["centers"], ref.centers, rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(r["cost"], ref.cost, rtol=1e-9)


def test_empty_cluster_keeps_center(cpu_world, native):
    X = np.array([[0.0, 0.0], [0.1, 0.0], [10.0, 10.0]])
    init = np.array([[0.0, 0.0], [10.0, 10.0], [1000.0, 1000.0]])
    w = O.get_world()
    t = native.upload_dense(w.ctx, X, "f64", 2)
    r = native.kmeans_fit(w.ctx, w.comm, t, init, 3, 5, 1e-4)
    np.testing.assert_allclose(r["centers"][2], [1000.0, 1000.0])
    np.testing.assert_allclose(r["centers"][0], [0.05, 0.0])
    assert r["last_counts"] == [2, 1, 0]


def test_fewer_distinct_points_than_k(cpu_world):
    df = pd.DataFrame({"features": [Vectors.dense([1.0, 2.0])] * 5 +
                       [Vectors.dense([3.0, 4.0])] * 5})
    for mode in ("random", "k-means||"):
        m = KMeans(k=4, initMode=mode, seed=2).fit(df)
        assert len(m.clusterCenters()) == 2


def test_convergence_and_tol(cpu_world):
    X, _ = blobs(2000, 5, 4, seed=11, sigma=0.05)
    m = KMeans(k=4, seed=11, maxIter=50, tol=1e-4).fit(X)
    assert m.summary.numIter < 50
    m0 = KMeans(k=4, seed=11, maxIter=0).fit(X)
    assert m0.summary.numIter == 0


def test_deterministic_repeat(cpu_world, native):
    X, _ = blobs(3000, 6, 5, seed=2, sigma=2.0)
    a = KMeans(k=5, seed=9).fit(X)
    b = KMeans(k=5, seed=9).fit(X)
    assert np.array_equal(np.array(a.clusterCenters()), np.array(b.clusterCenters()))
    assert a.summary.trainingCost == b.summary.trainingCost


def test_init_world_size_independent_draws(cpu_world, native):
    """k-means|| picks the same candidates for any sharding (keyed by global row index)."""
    X, _ = blobs(3000, 6, 5, seed=4, sigma=1.0)
    w = O.get_world()
    t = native.upload_dense(w.ctx, X, "f64", 6)
    c1 = native.kmeans_init(w.ctx, w.comm, t, 5, "k-means||", 2, 3)
    t2 = native.upload_dense(w.ctx, X, "f64", 6)
    c2 = native.kmeans_init(w.ctx, w.comm, t2, 5, "k-means||", 2, 3)
    np.testing.assert_array_equal(c1, c2)


def test_init_identical_for_any_host_pool(native):
    """Local k-means++ (the k-means|| reduction: pool-parallel seeding trials and Lloyd sweeps,
    every reduction over points in point order) gives the same centers for any host pool size."""
    X, _ = blobs(4000, 12, 200, seed=5, sigma=1.5)
    out = []
    for threads in (1, 4):
        O.shutdown_world()
        w = O.init_world(O.get_config().replace(device="cpu", cpu_threads=threads), rank=0,
                         size=1, local_rank=0)
        t = native.upload_dense(w.ctx, X, "f64", 12)
        out.append(np.asarray(native.kmeans_init(w.ctx, w.comm, t, 200, "k-means||", 2, 3)))
        O.shutdown_world()
    assert out[0].shape == (200, 12)
    np.testing.assert_array_equal(out[0], out[1])


# ------------------------------------------------------------------- persistence
def test_read_write_all_params(cpu_world, tmp_path):
    df = generate_kmeans_data()
    km = KMeans(predictionCol="myPrediction", k=3, maxIter=2, tol=0.01,
                distanceMeasure="euclidean")
    m = km.fit(df)
    p = str(tmp_path / "model")
    m.write().overwrite().save(p)
    m2 = KMeansModel.load(p)
    assert m2.uid == m.uid
    for name in ("predictionCol", "k", "maxIter", "tol", "distanceMeasure"):
        assert m2.getOrDefault(name) == m.getOrDefault(name)
    np.testing.assert_array_equal(np.array(m2.clusterCenters()), np.array(m.clusterCenters()))
    est = str(tmp_path / "est")
    km.save(est)
    km2 = KMeans.load(est)
    assert km2.getK() == 3 and km2.getPredictionCol() == "myPrediction"
    with pytest.raises(IOError):
        m.save(p)  # exists, no overwrite


def test_pmml_export(cpu_world, tmp_path):
    import xml.etree.ElementTree as ET

    m = KMeans(k=5, seed=1).fit(generate_kmeans_data())
    p = str(tmp_path / "pmml")
    m.write().format("pmml").save(p)
    root = ET.parse(p + "/part-00000").getroot()
    ns = {"p": "http://www.dmg.org/PMML-4_2"}
    cm = root.find("p:ClusteringModel", ns)
    assert cm.get("numberOfClusters") == "5"
    assert len(cm.findall("p:Cluster", ns)) == 5


def test_spark_parquet_layout(cpu_world, tmp_path):
    import glob
    import json

    import pyarrow.parquet as pq

    m = KMeans(k=5, seed=1).fit(generate_kmeans_data())
    p = str(tmp_path / "m")
    m.save(p)
    meta = json.loads(open(p + "/metadata/part-00000").readline())
    assert meta["class"] == "org.apache.spark.ml.clustering.KMeansModel"
    assert {"timestamp", "sparkVersion", "uid", "paramMap", "defaultParamMap"} <= set(meta)
    t = pq.read_table(glob.glob(p + "/data/*.parquet")[0])
    assert t.column_names == ["clusterIdx", "clusterCenter"]
    row_md = json.loads(t.schema.metadata[b"org.apache.spark.sql.parquet.row.metadata"])
    assert row_md["fields"][1]["type"]["class"] == "org.apache.spark.ml.linalg.VectorUDT"
    first = t.to_pylist()[0]["clusterCenter"]
    assert first["type"] == 1 and first["size"] is None and len(first["values"]) == 3


@pytest.mark.parametrize("version", ["3.0.0", "3.0.2", "3.1.1"])
def test_spark_version_knob(cpu_world, tmp_path, version):
    """Config.spark_version is what saved models carry (the reference's per-Spark-profile jars,
    pom.xml:151-224, collapse into one knob); the reader accepts every 3.x layout."""
    import json

    from oap_mllib_amd.persistence import spark_format as sf

    old = cpu_world.config.spark_version
    O.set_config(spark_version=version)
    try:
        m = KMeans(k=2, seed=1).fit(generate_kmeans_data())
        p = str(tmp_path / "m")
        m.write().save(p)
        meta = json.loads(open(p + "/metadata/part-00000").read())
        assert meta["sparkVersion"] == version and sf.spark_version() == version
        np.testing.assert_array_equal(np.array(KMeansModel.load(p).clusterCenters()),
                                      np.array(m.clusterCenters()))
    finally:
        O.set_config(spark_version=old)


def test_load_spark_1x_layouts(cpu_world, tmp_path):
    """Models saved by Spark <= 1.6 (majorVersion < 2): K-Means centers in one row's
    `clusterCenters` array, PCA without `explainedVariance` (KMeans.scala:253-257,
    PCA.scala:234-245)."""
    import json
    import os

    import pyarrow as pa

    from oap_mllib_amd.models.feature import PCAModel
    from oap_mllib_amd.persistence import spark_format as sf

    def meta(path, cls):
        os.makedirs(path + "/metadata")
        with open(path + "/metadata/part-00000", "w") as f:
            f.write(json.dumps({"class": cls, "timestamp": 0, "sparkVersion": "1.6.3",
                                "uid": "old_uid", "paramMap": {"k": 2}}))

    centers = np.array([[1.0, 2.0], [3.0, -4.0]])
    p = str(tmp_path / "km16")
    meta(p, "org.apache.spark.ml.clustering.KMeansModel")
    t = pa.table({"clusterCenters": pa.array(
        [[sf.dense_vector_struct(c) for c in centers]], type=pa.list_(sf.VECTOR_ARROW))})
    sf.write_parquet(p + "/data", t, sf.spark_schema(
        [("clusterCenters", {"type": "array", "elementType": sf.VECTOR_UDT,
                             "containsNull": True}, True)]))
    m = KMeansModel.load(p)
    assert m.uid == "old_uid" and m.getK() == 2
    np.testing.assert_array_equal(np.array(m.clusterCenters()), centers)

    pc = np.array([[0.6, 0.8], [0.8, -0.6]])
    p = str(tmp_path / "pca16")
    meta(p, "org.apache.spark.ml.feature.PCAModel")
    t = pa.table({"pc": pa.array([sf.dense_matrix_struct(pc)], type=sf.MATRIX_ARROW)})
    sf.write_parquet(p + "/data", t, sf.spark_schema([("pc", sf.MATRIX_UDT, True)]))
    pm = PCAModel.load(p)
    np.testing.assert_allclose(pm.pc.toArray(), pc)
    assert pm.explainedVariance.toArray().shape == (0,)
