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
    config.addinivalue_line("markers", "extended: non-default kernel schedules and duplicate decompositions "
                                       "(tuning A/B coverage); skipped unless PDHG_TESTS=full")


# The GPU suite runs as ONE pytest call with -x inside the driver's time limit, so the parity-critical tests go first
# (stop rules, NaN stop, drop-ins, window marching, the driver, x-slab, the slab's oracle step, the golden fixtures,
# the per-call parity tests), then the rest in file order with the full-size windows last.  Unknown tests keep
# their collection order between the listed groups.
_FIRST = [
    "test_gpu_parity.py::test_nan_stop", "test_gpu_parity.py::test_solver_oneiter_converges_like_oracle",
    "test_gpu_parity.py::test_dropin_update_functions", "test_gpu_parity.py::test_divergence_matches_oracle",
    "test_gpu_parity.py::test_multi_step_window_marching", "test_gpu_parity.py::test_marching_window_counts_fp64",
    "test_run_example.py", "test_gpu_xslab.py", "test_gpu_slab64.py::test_fp64_slab_eps_one_step_vs_oracle",
    "test_golden.py", "test_gpu_parity.py",
]
_LAST = ["test_gpu_decomp.py", "test_gpu_fullsize.py"]


def _rank(item):
    nid = item.nodeid.split("/")[-1]
    for i, key in enumerate(_FIRST):
        if nid.startswith(key):
            return i
    for i, key in enumerate(_LAST):
        if nid.startswith(key):
            return len(_FIRST) + 1 + i
    return len(_FIRST)


def pytest_collection_modifyitems(config, items):
    items.sort(key=_rank)   # stable: collection order inside each group
    if os.environ.get("PDHG_TESTS", "") != "full":
        skip = pytest.mark.skip(reason="extended tier (non-default schedule / duplicate coverage; PDHG_TESTS=full)")
        for it in items:
            if "extended" in it.keywords:
                it.add_marker(skip)


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
