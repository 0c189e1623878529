import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: multi-second CPU oracle runs")


@pytest.fixture(scope="session")
def oracle():
    import psoracle

    psoracle.build()
    return psoracle


@pytest.fixture(scope="session")
def gpu_poly():
    """A device context; fails (never skips) when the HIP path is unavailable."""
    from parsip_amd import gpu

    gpu.load()
    assert gpu.device_count() > 0, "no HIP device visible: GPU tests must run on an MI355X"
    p = gpu.Polygonizer(0)
    yield p
    p.close()
