import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the oracle's FFT threads: the GPU box shows the whole machine's CPUs but gives a job a 16-CPU share
os.environ.setdefault("ORACLE_FFT_WORKERS", str(min(16, os.cpu_count() or 1)))
for p in (os.path.join(ROOT, "pdhg-optimal-control_amd"), os.path.join(ROOT, "oracle"), ROOT,
          os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests through the C ABI")


@pytest.fixture(scope="session")
def native():
    """The built HIP library; GPU tests fail loudly if it is missing (no CPU fallback)."""
    import __graft_entry__
    __graft_entry__.build()
    from pdhg_amd import _native
    if _native.device_count() < 1:
        pytest.fail("gpu test selected but no HIP device is visible")
    return _native
