import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built libpopbam_gpu.so")


@pytest.fixture(scope="session")
def gpu_lib():
    """The product library on a real device; GPU tests fail loudly (never skip to a CPU
    path) when it is missing."""
    from popbam_amd import _lib
    lib = _lib.load()
    if lib.pbg_device_count() < 1:
        pytest.fail("no HIP device visible to libpopbam_gpu.so")
    return lib
