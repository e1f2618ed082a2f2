import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libvoxmap_hip.so on device 0)")
    config.addinivalue_line("markers", "slow: larger CPU oracle work")


@pytest.fixture(scope="session")
def built():
    """Both native pieces built in-tree (the HIP library and the C oracle)."""
    from voxmap_amd import build as vb
    import oracle
    vb.build(verbose=False)
    oracle.build()
    return True


@pytest.fixture(scope="session")
def noise(built):
    import voxmap_amd as vx
    return vx.noise_synth(0)
