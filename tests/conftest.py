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
    """The reference's own noise texture (res/noise.bin.gz, shipped in
    voxmap_amd/data), decoded through the product codec."""
    import numpy as np
    import voxmap_amd as vx
    from voxmap_amd import scenes
    raw = vx.decode(open(scenes.NOISE_PATH, "rb").read(), vx.FORMAT_BIN_GZ)
    return np.frombuffer(raw, np.uint8).reshape(1024, 1024, 4).copy()
