"""Benchmark: PDHG iterations/s on the north-star grid (BASELINE.json) on 1..N MI355X.

Workload (N = 1): configs[3] of BASELINE.json run on one GPU — egno 2, ndim 2, epsl 0.1,
nx = ny = 4096, nt = 201 as ONE PDHG window of T = nt - 1 = 200 unknown time rows
(time_step_per_PDHG = nt), rho_alp_iters = 1 (the fused-sweep headline),
fp32 state resident in HBM, reference initial state (phi = g, rho = 70, alp = 0;
utils_pdhg_solver.py:123-137).  One "step" = one outer PDHG iteration
(utils_pdhg_solver.py:51-88): primal (residual + H1 preconditioner + update), extrapolation,
dual (alpha/rho prox), err1/err2 and the device-side stop tests.

N > 1 (launched by torch.distributed.run): one process per GPU, the SAME window split into N t-slabs
of T/N rows (pdhg_amd/slab.py): rho / phi_bar halos point to point, the distributed
t-solve's two plane allgathers and the stop-test allreduces over RCCL.  Total work is fixed, so the
scaling is "strong"; value = iterations of the window / max-over-ranks time.

--decomp xslab (with --config c3w1: the reference's marching default, one T = 1 window of the 4096^2
grid): the window's x rows split into N x-slabs (pdhg_amd/xslab.py): halo-row
allgathers and two all-to-all transposes of the spectrum per iteration.  At N = 1 it runs one x-slab
through the same phases (LocalComm), so its line measures the decomposition's overhead.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "pdhg-optimal-control_amd"))

import numpy as np  # noqa: E402

METRIC = "PDHG iterations/sec and achieved HBM GB/s on nt×nx[×ny] grid, 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

CONFIGS = {
    # name: (egno, ndim, epsl, nx, ny, nt)
    "c3": (2, 2, 0.1, 4096, 4096, 201),
    "c4": (2, 2, 0.1, 8192, 8192, 401),   # 8-GPU point (t-slabs; >= 4 GPUs for memory)
    "c2": (1, 2, 0.0, 2048, 2048, 101),
    "c1": (1, 1, 0.0, 65536, 1, 401),
    "c0": (1, 1, 0.0, 160, 1, 41),
    "c3w1": (2, 2, 0.1, 4096, 4096, 2),   # one T = 1 window of C3's grid (time_step_per_PDHG = 2 default)
    "c3w4": (2, 2, 0.1, 4096, 4096, 5),   # short windows of C3's grid (kernel-policy crossover)
    "c3w8": (2, 2, 0.1, 4096, 4096, 9),
}


def grid(ndim, nx, ny):
    x1 = np.linspace(0.0, 2.0, num=nx, endpoint=False)
    if ndim == 1:
        return x1, None
    return x1, np.linspace(0.0, 2.0, num=ny, endpoint=False)


def cpu_baseline(cfg, T_sample, threads):
    """The float64 oracle (restatement of the reference, labelled 'port') on a bounded sample:
    the full nx x ny plane with T_sample unknown rows; extrapolated linearly to the full T."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ["ORACLE_FFT_WORKERS"] = str(threads)
    import pdhg_oracle as O
    egno, ndim, epsl, nx, ny, nt = cfg
    T = nt - 1
    x_arr = O.make_grid(ndim, nx, ny, egno)
    bc = O.default_bc(egno, ndim)
    fns = O.set_up_example_fns(egno, ndim, 0)
    g = O.set_up_J(egno, ndim, (2.0, 2.0))(x_arr)
    dt = 1.0 / (nt - 1)
    dsp = (2.0 / nx,) if ndim == 1 else (2.0 / nx, 2.0 / ny)
    nsp = (nx,) if ndim == 1 else (nx, ny)
    fv = O.compute_Dxx_fft_fv(ndim, nsp, dsp, bc)
    primal, dual = O.make_update_fns(ndim, bc, rho_alp_iters=1)
    phi = np.repeat(g, T_sample + 1, axis=0)
    rho = np.full((T_sample,) + nsp, 70.0)
    nctrl = ndim
    alp = tuple(np.zeros((T_sample,) + nsp + (nctrl,)) for _ in range(2 if ndim == 1 else 4))

    def one():
        nonlocal phi, rho, alp
        phi_n = primal(phi, rho, 70.0, alp, 0.1 / 1.5, dt, dsp, fns, fv, epsl, x_arr, None)
        rho_n, alp_n = dual(2 * phi_n - phi, rho, 70.0, alp, 0.15, dt, dsp, epsl, fns, x_arr, None, ndim, 1e-6)
        O.outer_errors(phi, phi_n, rho, rho_n, alp, alp_n)
        phi, rho, alp = phi_n, rho_n, alp_n

    one()                      # warm-up
    reps, t0 = 0, time.perf_counter()
    while True:
        one()
        reps += 1
        el = time.perf_counter() - t0
        if el > 8.0 or reps >= 5:
            break
    per_it = el / reps
    pts_per_s = T_sample * np.prod(nsp) / per_it
    full_pts = T * np.prod(nsp)
    return {"value": float(pts_per_s / full_pts), "unit": "it/s", "cores": threads, "kind": "port",
            "sample": "float64 NumPy/SciPy oracle (restatement of the JAX reference, which cannot run here), "
                      "{} x {} plane with T'={} of T={} rows, {} iterations in {:.1f}s, it/s extrapolated "
                      "linearly in T; scipy.fft workers={}, NumPy elementwise single-threaded".format(
                          nx, ny, T_sample, T, reps, el, threads)}


def pmc_traffic(args):
    """HBM bytes per launch of every kernel class from rocprofv3 PMC counters, collected in two
    separate child runs (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950) that are started
    BEFORE this process touches the GPU (a process that initialised HIP must not fork+exec).
    FETCH_SIZE is doubled per MI355X_MICROARCH.md §HBM (gfx950 reports half of a wide coalesced
    stream; uncalibrated for 4-B loads); WRITE_SIZE is exact for 16-B streaming stores.
    Returns ({class: {"bytes", "fetch_bytes_x2", "write_bytes"}}, None) or (None, reason)."""
    import csv
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if prof is None:
        return None, "rocprofv3 not found"
    vals = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="pdhg_pmc_", dir="/tmp")
        cmd = [prof, "--pmc", ctr, "--output-format", "csv", "-d", d, "-o", "run", "--",
               sys.executable, os.path.abspath(__file__), "--config", args.config, "--steps", "2", "--warmup", "1",
               "--rho-alp-iters", str(args.rho_alp_iters), "--no-cpu-baseline", "--no-pmc"]
        try:
            subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=600,
                           env=dict(os.environ, TMPDIR="/tmp"))
        except Exception as e:  # noqa: BLE001
            return None, "rocprofv3 {} pass failed: {}".format(ctr, e)
        for root, _, files in os.walk(d):
            for f in files:
                if f.endswith("counter_collection.csv"):
                    with open(os.path.join(root, f)) as fh:
                        for r in csv.DictReader(fh):
                            if r["Counter_Name"] != ctr:
                                continue
                            for cls, sym in KERNEL_SYMBOL.items():
                                if sym in r["Kernel_Name"]:
                                    vals.setdefault((cls, ctr), {}).setdefault(r["Kernel_Name"], []).append(
                                        float(r["Counter_Value"]) * 1024.0)
        shutil.rmtree(d, ignore_errors=True)
    # a class can hold two kernels (the first primal of a fused-residual context forms the residual
    # unfused): keep the one launched most, i.e. the steady-state kernel the timed region runs
    vals = {key: max(by_name.values(), key=len) for key, by_name in vals.items()}
    out = {}
    for cls in KERNEL_SYMBOL:
        f, w = vals.get((cls, "FETCH_SIZE")), vals.get((cls, "WRITE_SIZE"))
        if f and w:
            fb, wb = 2.0 * sum(f) / len(f), sum(w) / len(w)
            out[cls] = {"bytes": fb + wb, "fetch_bytes_x2": fb, "write_bytes": wb}
    return (out, None) if out else (None, "no PMC rows matched")


KERNEL_SYMBOL = {"dual": "k_dual_", "residual": "k_res_fwd", "precond": "k_precond_xt", "update": "k_inv"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--rho-alp-iters", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-T", type=int, default=2)
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 PMC traffic passes")
    ap.add_argument("--decomp", default="tslab", choices=["tslab", "xslab"],
                    help="multi-GPU decomposition of the window (xslab also at N = 1: one slab through its phases)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        # device = local rank (modulo the visible GPUs: PDHG_DIST_BACKEND=gloo rehearses the multi-rank
        # path with several ranks on one GPU; the driver's runs use one GPU per rank over RCCL)
        dev = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev)
        tdist.init_process_group(os.environ.get("PDHG_DIST_BACKEND", "nccl"))
        dist = tdist

    pmc, pmc_err = None, "disabled"
    if world == 1 and not args.no_pmc and args.decomp == "tslab":
        pmc, pmc_err = pmc_traffic(args)   # before this process initialises the GPU

    from pdhg_amd.context import PDHGContext

    egno, ndim, epsl, nx, ny, nt = CONFIGS[args.config]
    T = nt - 1
    k = args.rho_alp_iters
    xs, ys = grid(ndim, nx, ny)
    dt = 1.0 / (nt - 1)
    runner = None
    xslab = args.decomp == "xslab"
    if xslab:
        import torch
        from pdhg_amd.xslab import XSlabContext
        ctx = XSlabContext(rank, world, egno, nx, ny, T, 2.0 / nx, 2.0 / ny, dt, xs, ys, epsl=epsl,
                           rho_alp_iters=k, device=torch.cuda.current_device())
    elif world > 1:
        from pdhg_amd.slab import DistComm, SlabContext, SlabRunner
        ctx = SlabContext(rank, world, T, egno, nx, ny, 2.0 / nx, 2.0 / ny, dt, xs, ys, epsl=epsl,
                          rho_alp_iters=k, device=torch.cuda.current_device())
    else:
        ctx = PDHGContext(egno, ndim, nx, ny, T, 2.0 / nx, 2.0 / ny if ndim == 2 else 0.0, dt, xs, ys, epsl=epsl,
                          precision="fp32", rho_alp_iters=k, device=0)
    if ndim == 1:
        g = np.sin(np.pi * xs)
    else:
        g = np.sin(np.pi * xs)[:, None] + np.sin(np.pi * ys)[None, :]
    if xslab:
        ctx.init_global_state(g)
    else:
        ctx.init_state(g)
    # epsl = 0.1 on a 4096^2 grid is outside the reference algorithm's stability range (explicit
    # sigma*epsl*Lap in the dual; its fp64 restatement diverges already at 256^2): keep executing
    # exactly the requested iterations after the state goes non-finite, and report it.
    ctx.set_stop_rules(converge=True, nan=False)
    tau, sigma = 0.1 / 1.5, 0.1 * 1.5
    eps = 1e-6

    if xslab:
        from pdhg_amd.xslab import DistComm as XComm, LocalComm as XLocal, XSlabRunner
        xrunner = XSlabRunner([ctx], XComm() if world > 1 else XLocal(1))

        def run(n):
            s = xrunner.iterate(n, tau, sigma, eps, k)
            return {"iters_run": s["iters"], "status": s["status"], "nan_seen": s["nan_seen"]}

        def sync():
            torch.cuda.synchronize()
    elif world > 1:
        import torch
        runner = SlabRunner([ctx], DistComm(), exchange=os.environ.get("PDHG_SLAB_EXCHANGE", "neighbour"))

        def run(n):
            s = runner.iterate(n, tau, sigma, eps, k)
            return {"iters_run": s["iters"], "status": s["status"], "nan_seen": s["nan_seen"]}

        def sync():
            torch.cuda.synchronize()
    else:
        def run(n):
            return ctx.iterate(n, tau, sigma, eps, k)

        def sync():
            ctx.synchronize()

    if args.warmup > 0:
        run(args.warmup)
    sync()

    def barrier():
        if dist is not None:
            dist.barrier()

    ctx.profile_enable(True)
    barrier()
    sync()
    t0 = time.perf_counter()
    st = run(args.steps)
    sync()
    barrier()
    el = time.perf_counter() - t0
    iters = st["iters_run"]
    if dist is not None:
        import torch
        t = torch.tensor([el, float(iters)], dtype=torch.float64, device="cuda")
        tmax = t.clone()
        dist.all_reduce(tmax[0:1], op=dist.ReduceOp.MAX)
        el_max, iters_total = float(tmax[0]), iters          # one window: every rank ran the same iterations
    else:
        el_max, iters_total = el, iters

    # per-kernel live timing (HIP events on the context's stream)
    kern = {}
    for cls in ("residual", "precond", "update", "dual"):
        ms, n = ctx.profile_query(cls)
        if n:
            kern[cls] = {"avg_ms": ms / n, "launches": n, "bytes_per_launch": ctx.algorithmic_bytes(k, cls)}
    if world > 1 or xslab:   # slabs: sweeps and halo/interior row parts are separate launches -> per iteration
        for cls, d in kern.items():
            per = max(iters, 1) * (k if cls == "dual" else 1)
            d["avg_ms"] = d["avg_ms"] * d["launches"] / per
            d["launches"] = per
    ctx.profile_enable(False)
    dom = max(kern, key=lambda c: kern[c]["avg_ms"] * kern[c]["launches"])
    d = kern[dom]
    achieved = d["bytes_per_launch"] / (d["avg_ms"] * 1e-3) / 1e9
    it_bytes = ctx.algorithmic_bytes(k, "iteration") * world   # whole window (slabs are equal-ish)
    ms_per_step = el_max / max(iters, 1) * 1e3

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    out = {
        "metric": METRIC,
        "value": iters_total / el_max,
        "unit": "it/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if world > 1 else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (reference initial state phi=g, rho=70, alp=0)",
        "config": {"workload": "egno{} ndim{} epsl{} nx={} ny={} nt={}: one PDHG window of T={} rows, "
                               "rho_alp_iters={}".format(egno, ndim, epsl, nx, ny, nt, T, k),
                   "parallelism": ("x-slab x{} (halo-row allgathers, two all-to-all spectrum transposes per "
                                   "iteration)".format(world) if xslab else
                                   "t-slab x{} (RCCL point-to-point halos and carries, overlapped)".format(world))
                   if (world > 1 or xslab) else "single GPU",
                   "iters_executed": iters, "stop_status": st["status"], "state_nonfinite": bool(st["nan_seen"])},
        **({"slab_exchange": {"carries": runner.exchange, "long_range_modes": runner.n_long,
                              "halo_overlap": runner.side is not None}} if runner is not None else {}),
        "hbm_gbps_iteration": it_bytes / (ms_per_step * 1e-3) / 1e9,
        "iteration_bytes": it_bytes,
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS, "traffic": None},
        "kernels": kern,
    }
    if pmc and dom in pmc:
        out["roofline"]["traffic"] = pmc[dom]["bytes"]
        out["roofline"]["traffic_detail"] = pmc[dom]
        for cls in kern:
            if cls in pmc:
                kern[cls]["pmc_bytes_per_launch"] = pmc[cls]["bytes"]
    elif world == 1:
        out["roofline"]["traffic_note"] = pmc_err
    if world == 1 and not args.no_cpu_baseline:
        threads = min(16, os.cpu_count() or 1)
        sample_cfg = CONFIGS[args.config]
        out["cpu_baseline"] = cpu_baseline(sample_cfg, args.cpu_sample_T if ndim == 2 else 8, threads)
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
