"""Test configuration.

* ``@pytest.mark.gpu`` tests need a visible MI355X and the native engine; they run on the GPU box
  (``python -m pytest tests -m gpu``).  Everything else runs on CPU (native CPU engine, vanilla
  numpy oracle, multi-process gloo worlds).
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a visible MI355X GPU and the native engine")
    config.addinivalue_line("markers", "slow: long-running test")


def _gpu_visible() -> bool:
    try:
        import torch

        return torch.cuda.device_count() > 0
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu_visible():
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def native():
    from oap_mllib_amd import _loader

    return _loader.load()


@pytest.fixture
def cpu_world():
    """Single-process world on the native CPU engine."""
    import oap_mllib_amd as O

    O.shutdown_world()
    w = O.init_world(O.get_config().replace(device="cpu"), rank=0, size=1, local_rank=0)
    yield w
    O.shutdown_world()


@pytest.fixture
def vanilla_world():
    import oap_mllib_amd as O

    O.shutdown_world()
    w = O.init_world(O.get_config().replace(device="vanilla"), rank=0, size=1, local_rank=0)
    yield w
    O.shutdown_world()


@pytest.fixture
def gpu_world():
    import oap_mllib_amd as O

    O.shutdown_world()
    w = O.init_world(O.get_config().replace(device="gpu", device_id=0), rank=0, size=1,
                     local_rank=0)
    yield w
    O.shutdown_world()


@pytest.fixture
def rccl1_world():
    """A world of one GPU rank with a REAL 1-rank RCCL communicator (force_device_comm): the
    multi-GPU drivers' device-collective branches run on the single GPU of the box."""
    import oap_mllib_amd as O

    O.shutdown_world()
    w = O.init_world(O.get_config().replace(device="gpu", device_id=0, force_device_comm=True),
                     rank=0, size=1, local_rank=0)
    assert w.comm.name == "rccl" and w.comm.size == 1 and not w.comm.trivial
    yield w
    O.shutdown_world()
