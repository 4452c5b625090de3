import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def _has_gpu():
    try:
        from mav_trajectory_generation_cmake_amd import _native
        return _native.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu_ctx():
    from mav_trajectory_generation_cmake_amd import Context
    if not _has_gpu():
        pytest.fail("GPU test selected but no HIP device / libmav_trajectory_generation.so is available")
    ctx = Context(0)
    yield ctx
    ctx.close()
