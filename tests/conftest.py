import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libsiddhi_hip on the device)")


def pytest_collection_modifyitems(config, items):
    pass


@pytest.fixture(scope="session")
def hip_available():
    from siddhi_amd import hip_engine
    lib = hip_engine.load_library()
    import ctypes
    n = ctypes.c_int()
    lib.shd_device_count(ctypes.byref(n))
    if n.value == 0:
        pytest.fail("gpu test selected but no HIP device is visible")
    return True
