import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libptgpu.so on cuda:0)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


_LAST = ("test_gpu_fullsize.py",)


def pytest_runtest_setup(item):
    """GPU tests mix libptgpu.so (system HIP runtime) with torch (its own
    bundled HIP runtime): torch's must initialise first (see
    dsgpuraytracing_amd.native._init_torch_hip_first), whatever the test order."""
    if item.get_closest_marker("gpu") is not None:
        import torch
        if torch.cuda.device_count() > 0:
            torch.cuda.init()


def pytest_collection_modifyitems(config, items):
    """Cheap GPU parity cases first, full-size BASELINE configs last, so a
    `-x` run reports the small HIP-vs-oracle cases before the long ones."""
    items.sort(key=lambda it: os.path.basename(str(it.fspath)) in _LAST)


@pytest.fixture(scope="session")
def restate():
    from tests import oracle_helpers
    return oracle_helpers.Restatement()


@pytest.fixture(scope="session")
def gpu_ctx():
    from dsgpuraytracing_amd import pathtracer
    return pathtracer.Device(0)
