import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libflipwalk.so)")
    config.addinivalue_line("markers", "slow: longer CPU statistical checks")


@pytest.fixture(scope="session")
def gpu_lib():
    from flipcomplexityempirical_amd import _lib

    L = _lib.load()
    if L.fw_device_count() <= 0:
        pytest.fail("no HIP device visible for a gpu-marked test")
    return L
