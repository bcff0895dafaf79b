import json
import os
import sys
import time

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


@pytest.fixture(scope="session")
def parity_log():
    """Append one JSON line per measured parity case to $PDHG_PARITY_LOG (default gpurun_out/parity.jsonl):
    the achieved errors and the bounds they were held to, so the numbers outlive pytest's stdout
    (profiles/parity_r03.json is made from this file)."""
    path = os.environ.get("PDHG_PARITY_LOG", os.path.join(ROOT, "gpurun_out", "parity.jsonl"))
    os.makedirs(os.path.dirname(path), exist_ok=True)

    def record(test, case, measured, bounds, **extra):
        row = {"test": test, "case": case, "time": time.strftime("%Y-%m-%dT%H:%M:%S"),
               "measured": {k: float(v) for k, v in measured.items()},
               "bounds": {k: float(v) for k, v in bounds.items()}}
        row.update(extra)
        with open(path, "a") as fh:
            fh.write(json.dumps(row) + "\n")
    return record
