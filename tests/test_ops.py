"""oap_mllib_amd.ops: array-level ops on torch tensors (zero-copy GPU views, CPU engine else)."""
import numpy as np
import pytest
import torch

import oap_mllib_amd as O
from oap_mllib_amd import ops
from oap_mllib_amd.fallback import kmeans_vanilla as vanilla


def _blobs(n, d, k, seed):
    rng = np.random.default_rng(seed)
    c = rng.uniform(-8, 8, size=(k, d))
    X = c[rng.integers(0, k, n)] + rng.normal(0, 0.4, size=(n, d))
    return X.astype(np.float32), c


def test_cpu_engine_ops(cpu_world):
    X, c = _blobs(3000, 6, 4, 0)
    x = torch.from_numpy(X)
    lab, d2 = ops.kmeans_assign(x, torch.from_numpy(c))
    ref_lab, ref_d = vanilla.find_closest(X.astype(np.float64), c)
    assert lab.dtype == torch.int32 and np.array_equal(lab.numpy(), ref_lab)
    np.testing.assert_allclose(d2.numpy(), ref_d, rtol=1e-5, atol=1e-5)
    centers, cost, iters = ops.kmeans_fit(x, init_centers=c + 0.1, max_iter=10, tol=0.0)
    ref = vanilla.fit(X.astype(np.float64), 4, 10, 0.0, init_centers=c + 0.1)
    np.testing.assert_allclose(centers.numpy(), ref.centers, rtol=1e-9, atol=1e-9)
    assert cost == pytest.approx(ref.cost, rel=1e-9)
    pc, ev = ops.pca(x, 2)
    w = np.linalg.eigvalsh(np.cov(X.astype(np.float64).T))[::-1]
    np.testing.assert_allclose(ev.numpy(), w[:2] / w.sum(), rtol=1e-6)
    assert pc.shape == (6, 2)


@pytest.mark.gpu
@pytest.mark.parametrize("d,dtype", [(16, torch.float32), (13, torch.float32),
                                     (32, torch.bfloat16), (100, torch.bfloat16)])
def test_gpu_tensor_ops(gpu_world, native, d, dtype):
    X, c = _blobs(20000, d, 7, d)
    x = torch.from_numpy(X).to(device="cuda", dtype=dtype)
    Xr = x.float().cpu().numpy().astype(np.float64)  # the values the kernel sees
    lab, d2 = ops.kmeans_assign(x, torch.from_numpy(c))
    assert lab.is_cuda and d2.is_cuda
    ref_lab, ref_d = vanilla.find_closest(Xr, c)
    assert np.array_equal(lab.cpu().numpy(), ref_lab)
    np.testing.assert_allclose(d2.cpu().numpy(), ref_d, rtol=1e-4, atol=1e-4)
    centers, cost, iters = ops.kmeans_fit(x, init_centers=c + 0.05, max_iter=5, tol=0.0)
    cpu = native.Context(-1)
    t = native.upload_dense(cpu, Xr, "f64", d)
    ref = native.kmeans_fit(cpu, native.LocalComm(False), t, c + 0.05, 7, 5, 0.0)
    assert np.array_equal(centers.numpy(), ref["centers"])
    if dtype == torch.float32:
        pc, ev = ops.pca(x, 3)
        w = np.linalg.eigvalsh(np.cov(Xr.T))[::-1]
        np.testing.assert_allclose(ev.numpy(), w[:3] / w.sum(), rtol=1e-4)


@pytest.mark.gpu
def test_gpu_sliced_view_padding_not_read(gpu_world, native):
    """A column-sliced view whose row stride equals the kernel's padded layout (52 floats for
    d = 50) must not be used in place: columns 50-51 hold real data, not zero padding."""
    X, c = _blobs(8000, 50, 5, 3)
    wide = torch.full((8000, 52), 1e3, dtype=torch.float32, device="cuda")
    wide[:, :50] = torch.from_numpy(X).cuda()
    x = wide[:, :50]
    assert x.stride(0) == native.kmeans_ld(50)
    lab, d2 = ops.kmeans_assign(x, torch.from_numpy(c))
    ref_lab, ref_d = vanilla.find_closest(X.astype(np.float64), c)
    assert np.array_equal(lab.cpu().numpy(), ref_lab)
    np.testing.assert_allclose(d2.cpu().numpy(), ref_d, rtol=1e-4, atol=1e-4)
