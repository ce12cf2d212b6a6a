"""RCCL worlds on real GPUs: one process per GPU (LOCAL_RANK pinning), device collectives over
RCCL/xGMI, for K-Means, PCA and ALS against the single-GPU fit — the reference's per-iteration
cross-rank reductions (mllib-dal/src/main/native/KMeansDALImpl.cpp:97-99,201-223,
PCADALImpl.cpp:111-113, ALSDALImpl.cpp:336-431).  Skipped when fewer than 2 GPUs are visible
(RCCL cannot put two ranks on one device); the 1-GPU box covers the same drivers through the gloo
world in test_kmeans_gpu.py and the bench self-launch CPU test."""
import os
import subprocess
import sys

import numpy as np
import pytest

import oap_mllib_amd as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gpus():
    try:
        import torch

        return torch.cuda.device_count()  # (counting does not initialize HIP)
    except Exception:
        return 0


needs2 = pytest.mark.skipif("_gpus() < 2", reason="RCCL world needs >= 2 visible GPUs")


def _world(func, nproc, **kw):
    from mp_util import run_world

    return run_world("dist_workers", func, nproc=nproc, device="gpu", use_rccl=True,
                     device_id=-1, timeout=300, **kw)


def _nproc():
    return min(_gpus(), 4)


@needs2
def test_rccl_kmeans_matches_single_gpu():
    n = _nproc()
    rc, outs = _world("kmeans_native", n, n=40000, d=12, k=7)
    assert rc == 0, outs
    from dist_workers import kmeans_native

    O.shutdown_world()
    ref = kmeans_native(device="gpu", n=40000, d=12, k=7)
    O.shutdown_world()
    for o in outs:
        assert o["engine"] == "gpu" and o["comm"] == "rccl" and o["size"] == n
        # fixed-point statistics: bitwise equal for any world size
        assert np.array_equal(np.array(o["centers"]), np.array(ref["centers"]))


@needs2
def test_rccl_pca_matches_single_gpu():
    n = _nproc()
    rc, outs = _world("pca_native", n)
    assert rc == 0, outs
    from dist_workers import pca_native

    O.shutdown_world()
    ref = pca_native(device="gpu")
    O.shutdown_world()
    for o in outs:
        assert o["engine"] == "gpu"
        np.testing.assert_allclose(o["ev"], ref["ev"], rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(np.abs(o["pc"]), np.abs(ref["pc"]), atol=1e-7)


@needs2
def test_rccl_als_matches_single_gpu():
    n = _nproc()
    rc, outs = _world("als_native", n)
    assert rc == 0, outs
    from dist_workers import als_native

    O.shutdown_world()
    ref = als_native(device="gpu")
    O.shutdown_world()
    for o in outs:
        assert o["engine"] == "gpu"
        assert o["uid"] == ref["uid"]
        np.testing.assert_allclose(o["uf"], ref["uf"], rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(o["if"], ref["if"], rtol=1e-4, atol=1e-5)


@needs2
def test_bench_self_launch_rccl():
    """bench.py --gpus N starts N ranks itself and reports the RCCL world it formed."""
    import json

    n = _nproc()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n),
                        "--rows", "2000000", "--steps", "3", "--warmup", "1", "--skip-fit",
                        "--skip-unpruned", "--no-separable-extra"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    j = json.loads(line)
    assert j["n_gpus"] == n and j["extra"]["rccl_ranks"] == n and j["extra"]["comm"] == "rccl"
