import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libewal.so on the GPU)")


def gpu_available():
    try:
        from etcd_amd import _lib
        return _lib.lib.ewal_device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def ctx():
    if not gpu_available():
        pytest.fail("GPU test selected but no GPU / libewal.so is unusable (no CPU fallback exists)")
    from etcd_amd.wal import Context
    c = Context(0)
    yield c
    c.close()
