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


def _scale_worker(rank, world, port, out_path):
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:{}".format(port), rank=rank, world_size=world)
    try:
        iters = 4
        # synthetic per-rank numbers: rank r is 1 ms slower per step, its exposed rho halo 0.1 * r ms per step
        kern = {c: {"avg_ms": 2.0 + i, "launches": iters} for i, c in enumerate(bench.KERNEL_CLASSES)}
        exch = {"halo_rho": 1.0, "exposed_halo_rho": 0.1 * rank, "exposed_carry_planes": 0.05, "allreduce": 0.02}
        rep = bench.scale_report(dist, "gloo", (20.0 + rank) * iters * 1e-3, iters, kern, exch)
        if rank == 0:
            with open(out_path, "w") as fh:
                json.dump(rep, fh)
    finally:
        dist.destroy_process_group()


def test_scale_report_gloo_world4(tmp_path):
    """The N > 1 bench line's self-check keys: world size as the process group reports it, per-rank
    step times and their max, kernel / exchange / exposed-wait times per rank, and the unexplained remainder --
    gathered over gloo at world size 4 with synthetic per-rank numbers."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = str(tmp_path / "rep.json")
    mp.spawn(_scale_worker, args=(4, port, out), nprocs=4, join=True)
    with open(out) as fh:
        rep = json.load(fh)
    assert rep["world_size_reported"] == 4 and rep["backend"] == "gloo"
    assert rep["ms_per_step_by_rank"] == [20.0, 21.0, 22.0, 23.0]
    assert rep["ms_per_step_max"] == 23.0 and rep["slowest_rank"] == 3
    assert rep["kernel_ms_per_step_by_rank"]["dual"] == [5.0] * 4        # 2 + 3 ms per launch, one launch per step
    assert max(abs(a - 0.1 * r) for r, a in enumerate(rep["exchange_ms_per_step_by_rank"]["exposed_halo_rho"])) < 1e-12
    assert abs(rep["exposed_exchange_ms_by_rank"][2] - 0.25) < 1e-12
    assert abs(rep["unexplained_ms_by_rank"][3] - (23.0 - 14.0 - 0.35)) < 1e-9


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
