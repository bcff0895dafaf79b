"""bench.py --gpus N launches its own ranks (CPU, gloo): the driver's `bench.py --gpus N` without an
external torchrun must run N processes and report n_gpus = N (north_star: it/s at 1, 2, 4, 8 GPUs)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, extra_env=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env.update(extra_env or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_gpus2_launches_two_ranks():
    out = _run(["--gpus", "2", "--selftest"], {"PDHG_DIST_BACKEND": "gloo"})
    assert out == {"selftest": True, "n_gpus": 2, "ranks_seen": 2, "backend": "gloo"}


def test_gpus1_runs_in_process():
    out = _run(["--gpus", "1", "--selftest"])
    assert out["n_gpus"] == 1 and out["ranks_seen"] == 1


def test_gpus_mismatch_with_launcher_env_fails():
    env = {k: v for k, v in os.environ.items()}
    env.update({"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--selftest"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "WORLD_SIZE=1" in (p.stderr + p.stdout)


def test_dual_passes_of_the_chunked_loop():
    """The chunked dual (kernels_dual_multi.hpp) moves one sub-iteration's bytes per pass: ceil(inner / 5) chunk
    passes + the final re-run when the exit falls inside a chunk -- what bench.py prices the dual class with, so no
    record reports more bytes than crossed HBM (frac 2.01 from bytes x inner count)."""
    sys.path.insert(0, ROOT)
    import bench
    assert bench.dual_passes(10.0) == 2.0        # no early exit at k = 10: two chunks of 5
    assert bench.dual_passes(5.0) == 1.0
    assert bench.dual_passes(3.0) == 2.0         # exit inside the first chunk: chunk + final
    assert bench.dual_passes(7.0) == 3.0
    assert bench.dual_passes(1.0) == 2.0
