import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def C():
    import wave3d

    if wave3d._native.extension_path() is None:
        wave3d.build()
    return wave3d.load_native()


@pytest.fixture(scope="session")
def cpu_prog(C):
    import wave3d

    return wave3d.program("wave3d_cpu")


@pytest.fixture(scope="session")
def gpu_prog(C):
    import wave3d

    return wave3d.program("wave3d")
