"""Spark glue (oap_mllib_amd.spark): the pyspark-independent pieces run here; the barrier-stage
fit itself needs pyspark, which is not installed in this environment (test skipped)."""
import numpy as np
import pytest

import oap_mllib_amd as O
from oap_mllib_amd import spark as S


def test_local_ranks():
    assert S.local_ranks(["h1:1", "h2:5", "h1:2", "h1:3", "h2:6"]) == [0, 0, 1, 2, 1]


def test_model_payload_roundtrip(cpu_world):
    rng = np.random.default_rng(0)
    X = rng.normal(size=(200, 4))
    km = O.KMeans(k=3, seed=1, predictionCol="p").fit(X)
    km2 = S.import_model(S.export_model(km))
    np.testing.assert_array_equal(km2._centers, km._centers)
    assert km2.getPredictionCol() == "p" and km2.uid == km.uid
    pca = O.PCA(k=2, inputCol="features").fit(X)
    p2 = S.import_model(S.export_model(pca))
    np.testing.assert_array_equal(p2.pc.toArray(), pca.pc.toArray())
    als = O.ALS(rank=2, maxIter=2, implicitPrefs=True).fit(
        {"user": [1, 2, 2, 3], "item": [1, 1, 2, 3], "rating": [1.0, 2.0, 1.0, 5.0]})
    a2 = S.import_model(S.export_model(als))
    assert a2.rank == 2 and a2.userFactors["id"].tolist() == als.userFactors["id"].tolist()


def test_partition_conversion():
    class Row(dict):
        def __getitem__(self, k):
            return dict.__getitem__(self, k)

    from oap_mllib_amd.linalg import DenseVector

    rows = [Row(features=DenseVector([1.0, 2.0])), Row(features=DenseVector([3.0, 4.0]))]
    X = S._partition_to_input(O.KMeans(), rows)
    np.testing.assert_array_equal(X, [[1, 2], [3, 4]])
    r = S._partition_to_input(O.ALS(), [Row(user=1, item=2, rating=3.0)])
    assert r["user"].tolist() == [1] and r["item"].tolist() == [2]
    assert r["rating"].tolist() == [3.0]


def test_arrow_vector_column_to_matrix():
    """VectorUDT columns as Spark ships them to Python in Arrow form: dense, sparse and mixed
    chunks become one dense matrix without per-row objects."""
    import pyarrow as pa

    from oap_mllib_amd.persistence.spark_format import VECTOR_ARROW

    rng = np.random.default_rng(1)
    X = rng.normal(size=(7, 5))
    X[X < 0.3] = 0.0
    recs = []
    for j, x in enumerate(X):
        if j % 2:  # sparse
            nz = np.nonzero(x)[0]
            recs.append({"type": 0, "size": 5, "indices": nz.tolist(), "values": x[nz].tolist()})
        else:
            recs.append({"type": 1, "size": None, "indices": None, "values": x.tolist()})
    col = pa.chunked_array([pa.array(recs[:3], type=VECTOR_ARROW),
                            pa.array(recs[3:], type=VECTOR_ARROW)])
    np.testing.assert_array_equal(S.vectors_from_arrow(col), X)
    dense = pa.array([{"type": 1, "size": None, "indices": None, "values": x.tolist()}
                      for x in X], type=VECTOR_ARROW)
    np.testing.assert_array_equal(S.vectors_from_arrow(dense), X)
    tbl = pa.table({"features": dense})
    np.testing.assert_array_equal(S.table_to_input(O.KMeans(), tbl), X)
    als_tbl = pa.table({"user": [1, 2], "item": [3, 4], "rating": [0.5, 2.0]})
    r = S.table_to_input(O.ALS(), als_tbl)
    assert r["user"].tolist() == [1, 2] and r["rating"].tolist() == [0.5, 2.0]
    assert S._input_columns(O.PCA(inputCol="v")) == ["v"]


def test_empty_arrow_partition():
    """mapInArrow hands an empty partition no record batches at all: the rank
    still gets a (0-row) input, and vector estimators learn d from their peers."""
    import pyarrow as pa

    X = S.batches_to_input(O.KMeans(), [])
    assert X.shape[0] == 0
    r = S.batches_to_input(O.ALS(), iter([]))
    assert len(r["user"]) == len(r["item"]) == len(r["rating"]) == 0
    b = pa.RecordBatch.from_pydict({"user": [1], "item": [2], "rating": [3.0]})
    assert S.batches_to_input(O.ALS(), [b])["item"].tolist() == [2]

    class Ctx:  # BarrierTaskContext.allGather of the peers' widths
        def allGather(self, v):
            return [v, "6"]

    assert S._agree_on_width(Ctx(), O.KMeans(), X).shape == (0, 6)
    full = np.ones((3, 6))
    assert S._agree_on_width(Ctx(), O.PCA(), full) is full


@pytest.mark.skipif(not S.spark_available(), reason="pyspark not installed")
def test_barrier_fit_local_spark():  # pragma: no cover - needs pyspark
    from pyspark.ml.linalg import Vectors as SV
    from pyspark.sql import SparkSession

    spark = SparkSession.builder.master("local[2]").getOrCreate()
    df = spark.createDataFrame([(SV.dense([float(i % 5), 1.0]),) for i in range(100)],
                               ["features"])
    m = S.fit(O.KMeans(k=5, seed=1), df, num_ranks=2, spark_conf={"spark.oap.mllib.device": "cpu"})
    assert len(m.clusterCenters()) == 5
