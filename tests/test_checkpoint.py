"""Checkpoint / resume: a fit interrupted after a snapshot and resumed gives the same model as
an uninterrupted fit (K-Means centers, ALS factors)."""
import numpy as np
import pytest

import oap_mllib_amd as O


def _blobs():
    rng = np.random.default_rng(0)
    c = rng.uniform(-10, 10, (6, 5))
    return c[rng.integers(0, 6, 3000)] + rng.normal(0, 6.0, (3000, 5))


def test_kmeans_segmented_equals_plain(tmp_path, cpu_world):
    X = _blobs()
    plain = O.KMeans(k=6, seed=3, maxIter=25, tol=0.0).fit(X)
    cfg = cpu_world.config
    cfg.checkpoint_dir, cfg.checkpoint_interval = str(tmp_path), 4
    try:
        est = O.KMeans(k=6, seed=3, maxIter=25, tol=0.0)
        seg = est.fit(X)
        np.testing.assert_array_equal(np.array(seg.clusterCenters()),
                                      np.array(plain.clusterCenters()))
        assert seg.numIter == plain.numIter and seg.trainingCost == plain.trainingCost
        # "crash" half way, then resume from the snapshot with the full budget
        half = plain.numIter // 2
        assert half >= 3
        est2 = O.KMeans(k=6, seed=3, maxIter=half, tol=0.0)
        est2.fit(X)
        est3 = est2.copy({"maxIter": 25})
        est3.uid = est2.uid
        from oap_mllib_amd.utils import checkpoint
        ck8 = checkpoint.for_fit(cpu_world, est2, X.shape)
        meta, arrays = ck8.load()
        assert meta["num_iter"] == half and not meta["converged"]
        ck25 = checkpoint.for_fit(cpu_world, est3, X.shape)
        ck25.save(meta, arrays)  # same run, larger budget: seed its snapshot
        resumed = est3.fit(X)
        np.testing.assert_array_equal(np.array(resumed.clusterCenters()),
                                      np.array(plain.clusterCenters()))
        assert resumed.numIter == plain.numIter
    finally:
        cfg.checkpoint_dir = ""


def test_als_segmented_equals_plain(tmp_path, cpu_world):
    rng = np.random.default_rng(1)
    data = {"user": rng.integers(0, 40, 800), "item": rng.integers(0, 30, 800),
            "rating": rng.integers(1, 5, 800).astype(float)}
    plain = O.ALS(rank=4, maxIter=7, implicitPrefs=True, seed=2, checkpointInterval=-1).fit(data)
    cfg = cpu_world.config
    cfg.checkpoint_dir = str(tmp_path)
    try:
        seg = O.ALS(rank=4, maxIter=7, implicitPrefs=True, seed=2, checkpointInterval=3).fit(data)
    finally:
        cfg.checkpoint_dir = ""
    for a, b in ((plain.userFactors, seg.userFactors), (plain.itemFactors, seg.itemFactors)):
        np.testing.assert_array_equal(np.stack(a["features"].to_list()),
                                      np.stack(b["features"].to_list()))
