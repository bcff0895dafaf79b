"""Benchmark: PDHG iterations/s on the north-star grid (BASELINE.json) on 1..N MI355X.

Workload (N = 1): configs[3] of BASELINE.json run on one GPU — egno 2, ndim 2, epsl 0.1,
nx = ny = 4096, nt = 201 as ONE PDHG window of T = nt - 1 = 200 unknown time rows
(time_step_per_PDHG = nt), rho_alp_iters = 1 (the fused-sweep headline),
fp64 state resident in HBM -- the reference's arithmetic (jaxsrc/update_fns_in_pdhg.py:10), the one that meets
north_star's 1e-5 at this config's epsl = 0.1 -- reference initial state (phi = g, rho = 70, alp = 0;
utils_pdhg_solver.py:123-137).  The same workload in fp32 is reported nested ("fp32_precision") as a throughput
reference: fp32 does not meet the 1e-5 bar at epsl = 0.1.  One "step" = one outer PDHG iteration
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
    "c2w1": (1, 2, 0.0, 2048, 2048, 2),   # one T = 1 window of C2's grid (the marching default's window)
    "c3w4": (2, 2, 0.1, 4096, 4096, 5),   # short windows of C3's grid (kernel-policy crossover)
    "c3w8": (2, 2, 0.1, 4096, 4096, 9),
    # one GPU's share of the 8-GPU t-slab runs as a window of its own (C3: 200 / 8 rows, C4: 400 / 8 rows; the
    # per-GPU compute term of the multi-GPU cost model)
    "c3w25": (2, 2, 0.1, 4096, 4096, 26),
    "c3w100": (2, 2, 0.1, 4096, 4096, 101),   # C3's per-GPU share at 2 GPUs
    "c4w50": (2, 2, 0.1, 8192, 8192, 51),
}


def progress(msg):
    """One progress line per phase on stderr (long runs: the PMC passes and the nested run are child processes)."""
    print("[bench {}] {}".format(time.strftime("%H:%M:%S"), msg), file=sys.stderr, flush=True)


def grid(ndim, nx, ny):
    x1 = np.linspace(0.0, 2.0, num=nx, endpoint=False)
    if ndim == 1:
        return x1, None
    return x1, np.linspace(0.0, 2.0, num=ny, endpoint=False)


def cpu_baseline(cfg, T_sample, threads, reps_min=3):
    """The float64 oracle (restatement of the reference, labelled 'port') on a bounded sample:
    the full nx x ny plane with T_sample unknown rows, one warm-up iteration then reps_min timed
    iterations (median); extrapolated linearly in T to the full window."""
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
    times = []
    t_all = time.perf_counter()
    while len(times) < reps_min or (time.perf_counter() - t_all < 8.0 and len(times) < 50):
        t0 = time.perf_counter()
        one()
        times.append(time.perf_counter() - t0)
    per_it = float(np.median(times))
    pts_per_s = T_sample * np.prod(nsp) / per_it
    full_pts = T * np.prod(nsp)
    return {"value": float(pts_per_s / full_pts), "unit": "it/s", "cores": threads, "kind": "port",
            "sample": "float64 NumPy/SciPy oracle (restatement of the JAX reference, which cannot run here), "
                      "{} x {} plane with T'={} of T={} rows: {} timed iterations after 1 warm-up, median "
                      "{:.2f} s (min {:.2f}, max {:.2f}), it/s extrapolated linearly in T; scipy.fft workers={}, "
                      "NumPy elementwise single-threaded".format(nx, ny, T_sample, T, len(times), per_it,
                                                                min(times), max(times), threads),
            "reps": len(times)}


PMC_ITERS = 3   # outer iterations of each PMC child run (1 warm-up + 2 steps, no probe)


def pmc_traffic(args):
    """HBM bytes per launch of every kernel class from rocprofv3 PMC counters, collected in two
    separate child runs (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950) that are started
    BEFORE this process touches the GPU (a process that initialised HIP must not fork+exec).
    FETCH_SIZE is doubled per MI355X_MICROARCH.md §HBM (gfx950 reports half of a coalesced stream);
    calibrated on this pool for 4-, 8- and 16-B loads per lane alike, and WRITE_SIZE exact for 4-, 8- and
    16-B stores (scripts/fetch_calib.hip, profiles/r04_fetch_calib.txt).
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
        progress("rocprofv3 {} pass".format(ctr))
        d = tempfile.mkdtemp(prefix="pdhg_pmc_", dir="/tmp")
        cmd = [prof, "--pmc", ctr, "--output-format", "csv", "-d", d, "-o", "run", "--",
               sys.executable, os.path.abspath(__file__), "--config", args.config, "--steps", str(PMC_ITERS - 1),
               "--warmup", "1",
               "--rho-alp-iters", str(args.rho_alp_iters), "--precision", args.precision, "--no-cpu-baseline",
               "--no-pmc", "--no-probe", "--no-reference-precision"]
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
                            for cls, syms in KERNEL_SYMBOL.items():
                                if any(sym in r["Kernel_Name"] for sym in syms):
                                    vals.setdefault((cls, ctr), {}).setdefault(r["Kernel_Name"], []).append(
                                        float(r["Counter_Value"]) * 1024.0)
        shutil.rmtree(d, ignore_errors=True)
    # by kernel name: a class's bytes per launch are the sum over its kernels of each kernel's average (C1's
    # 16 x 4096 transform runs two kernels per residual / update launch).  The first primal of a fused-residual
    # context forms its residual unfused (k_res_fwdy_fast_2d, from rho + 4 alp: ~3x the fused kernel's bytes);
    # with a fused kernel present that one is reported apart as "residual_first" and kept out of "residual".
    names = {}
    for (cls, ctr), by_name in vals.items():
        for name, v in by_name.items():
            names.setdefault(name, {})[ctr] = (sum(v) / len(v), len(v))
    split = {}
    for (cls, ctr), by_name in list(vals.items()):
        if cls == "residual" and any("fused" in n for n in by_name):
            # the first iteration's unfused kernels: not "fused" and launched fewer times than the fused ones (C1's
            # stage B, k_f16b_fwd_1d, follows either stage A form and stays in the class)
            nf = max(len(v) for n, v in by_name.items() if "fused" in n)
            first = {n for n, v in by_name.items() if "fused" not in n and len(v) < nf}
            split[("residual_first", ctr)] = {n: v for n, v in by_name.items() if n in first}
            vals[(cls, ctr)] = {n: v for n, v in by_name.items() if n not in first}
    vals.update(split)
    # per class launch: each kernel name's average per launch, summed over the class's names -- except the dual:
    # with rho_alp_iters > 1 one dual "launch" (outer iteration) runs several kernel launches (the chunked loop's
    # passes, kernels_dual_multi.hpp), so its bytes are all its kernels' bytes over the child's PMC_ITERS iterations
    vals = {key: (sum(sum(v) for v in by_name.values()) / PMC_ITERS if key[0] == "dual" else
                  sum(sum(v) / len(v) for v in by_name.values())) for key, by_name in vals.items() if by_name}
    out = {}
    for cls in list(KERNEL_SYMBOL) + ["residual_first"]:
        f, w = vals.get((cls, "FETCH_SIZE")), vals.get((cls, "WRITE_SIZE"))
        if f is not None and w is not None:
            fb, wb = 2.0 * f, w
            out[cls] = {"bytes": fb + wb, "fetch_bytes_x2": fb, "write_bytes": wb}
    if out:
        out["_by_kernel"] = {n: {"fetch_bytes_x2": 2.0 * c["FETCH_SIZE"][0] if "FETCH_SIZE" in c else None,
                                 "write_bytes": c["WRITE_SIZE"][0] if "WRITE_SIZE" in c else None,
                                 "launches": max(x[1] for x in c.values())} for n, c in names.items()}
    return (out, None) if out else (None, "no PMC rows matched")


# kernel-name substrings of the four classes (precond: k_precond_xt_* and the one-row k_precond_x_t1_2d,
# 1-D k_thomas_1d / k_thomas_chunk_1d; C1's 16 x 4096 transform: k_f16a/b_fwd_1d form the residual class,
# k_f16b/a_inv_1d the update class; the older four-step kernels k_fs1/k_fs2 (PDHG_FS16=0) are not attributed)
KERNEL_SYMBOL = {"dual": ("k_dual_",), "residual": ("k_res_fwd", "k_f16a_fwd", "k_f16b_fwd"),
                 "precond": ("k_precond_x", "k_thomas_1d", "k_thomas_chunk"),
                 "update": ("k_inv", "k_f16b_inv", "k_f16a_inv")}


def marching(args):
    """--marching: time to solution of the reference's default execution mode -- window marching with T = 1
    windows (time_step_per_PDHG = 2, run_example.py:431; PDHG_multi_step, utils_pdhg_solver.py:97-225), every
    window solved to eps = 1e-6 with the reference's dual loop (rho_alp_iters, default 10 with early exit,
    update_fns_in_pdhg.py:167-180), stepsz 0.1, through the drop-in driver (pdhg_amd.utils_pdhg_solver), on the
    config's grid with its nt - 1 windows.  CPU column: the float64 oracle timed for a few outer iterations of one
    window of the same grid on this host (cpu_baseline leg), extrapolated to the device run's total iterations
    (the same algorithm and stop rule: the oracle needs the same iterations up to rounding)."""
    from pdhg_amd import set_fns, utils_pdhg_solver as S, utils_precond
    egno, ndim, epsl, nx, ny, nt = CONFIGS[args.config]
    if ndim == 1:
        ny = 1
    k = args.rho_alp_iters
    n_ctrl, bc = (ndim, 0 if ndim == 1 else (0, 0)) if egno != 3 else (1, (1, 0))
    fns = set_fns.set_up_example_fns(egno, ndim, 0)
    xs, ys = grid(ndim, nx, ny)
    x_arr = xs[None, :, None] if ndim == 1 else np.stack(np.meshgrid(xs, ys, indexing="ij"), axis=-1)[None]
    dt = 1.0 / (nt - 1)
    dsp = (2.0 / nx,) if ndim == 1 else (2.0 / nx, 2.0 / ny)
    nsp = (nx,) if ndim == 1 else (nx, ny)
    g = set_fns.set_up_J(egno, ndim, (2.0, 2.0))(x_arr)
    fv = utils_precond.compute_Dxx_fft_fv(ndim, nsp, dsp, bc)
    fp, fd = S.make_update_fns(ndim, bc, rho_alp_iters=k, precision=args.precision)
    stats = []
    nt_run = nt if not args.windows else min(nt, args.windows + 1)   # the first W windows (same dt)
    # process setup outside the clock: loading libpdhg.so (and the torch HIP runtime it loads first, ~1.2 s on a
    # fresh box); contexts, their allocations and every state transfer stay inside
    from pdhg_amd import _native
    _native.load()
    t0 = time.perf_counter()
    results, errs = S.PDHG_multi_step(fp, fd, fns, g, x_arr, ndim, nt_run, nsp, dt, dsp, 70.0, time_step_per_PDHG=2,
                                      epsl=epsl, stepsz_param=0.1, fv=fv, n_ctrl=n_ctrl, N_maxiter=1000000,
                                      print_freq=10000, eps=1e-6, verbose=True, stats=stats)   # per-window progress lines
    wall = time.perf_counter() - t0
    per_window = [int(r["window_iters"]) for r in stats]
    total = int(sum(per_window))
    out = {"metric": "time to solution, window marching (T = 1 windows to eps 1e-6)", "value": wall, "unit": "s",
           "higher_is_better": False, "n_gpus": 1, "dtype": {"fp32": "f32", "fp64": "f64"}.get(args.precision),
           "config": {"workload": "egno{} ndim{} epsl{} nx={} ny={} nt={}: {} windows of T = 1, rho_alp_iters={}, "
                                  "stepsz 0.1, eps 1e-6".format(egno, ndim, epsl, nx, ny, nt, nt_run - 1, k),
                      "precision": args.precision},
           "windows": len(errs), "total_outer_iters": total, "max_iters_per_window": int(results[0][0]),
           "iters_per_window_first10": per_window[:10], "iters_per_window": per_window,
           "ms_per_outer_iter": wall / max(1, total) * 1e3,
           "stop_status_last_window": int(stats[-1]["status"]) if stats else None}
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_marching_baseline(args.config, k, total, min(16, os.cpu_count() or 1))
        out["cpu_baseline"]["speedup"] = out["cpu_baseline"]["extrapolated_s"] / wall
    print(json.dumps(out), flush=True)


def cpu_marching_baseline(config, k, total_iters, threads, reps=3):
    """The float64 oracle (restatement of the reference, 'port') for `reps` outer iterations of the first T = 1
    window of the config's grid (reference initial state), median per iteration, times the device run's iterations."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ["ORACLE_FFT_WORKERS"] = str(threads)
    import pdhg_oracle as O
    egno, ndim, epsl, nx, ny, nt = CONFIGS[config]
    x_arr = O.make_grid(ndim, nx, ny, egno)
    bc = O.default_bc(egno, ndim)
    fns = O.set_up_example_fns(egno, ndim, 0)
    g = O.set_up_J(egno, ndim, (2.0, 2.0))(x_arr)
    dt = 1.0 / (nt - 1)
    dsp = (2.0 / nx,) if ndim == 1 else (2.0 / nx, 2.0 / ny)
    nsp = (nx,) if ndim == 1 else (nx, ny)
    fv = O.compute_Dxx_fft_fv(ndim, nsp, dsp, bc)
    inner = []
    primal, dual = O.make_update_fns(ndim, bc, rho_alp_iters=k, dual_stats=inner)
    n_ctrl = 1 if egno == 3 else ndim
    phi = np.repeat(g, 2, axis=0)
    rho = np.full((1,) + nsp, 70.0)
    alp = tuple(np.zeros((1,) + nsp + (n_ctrl,)) for _ in range(2 if ndim == 1 else 4))
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        phi_n = primal(phi, rho, 70.0, alp, 0.1 / 1.5, dt, dsp, fns, fv, epsl, x_arr, None)
        rho, alp = dual(2 * phi_n - phi, rho, 70.0, alp, 0.15, dt, dsp, epsl, fns, x_arr, None, ndim, 1e-6)
        phi = phi_n
        times.append(time.perf_counter() - t0)
    per = float(np.median(times))
    return {"value": per, "unit": "s per outer iteration", "cores": threads, "kind": "port",
            "extrapolated_s": per * total_iters,
            "sample": "float64 NumPy/SciPy oracle, {} outer iterations of the first T = 1 window ({} dual "
                      "sub-iterations each: {}), median, times the device run's {} iterations".format(
                          reps, k, inner, total_iters)}


def other_precision_run(args, prec):
    """The same workload in the other arithmetic (fp64 = the reference's, jaxsrc/update_fns_in_pdhg.py:10; fp32),
    run as a child process BEFORE this process initialises the GPU (its own PMC passes are grandchildren started
    before it touches the GPU).  Returns the child's JSON line (nested as "reference_precision" / "fp32_precision")
    or an error note."""
    import subprocess
    progress("nested {} run (child process)".format(prec))
    cmd = [sys.executable, os.path.abspath(__file__), "--config", args.config, "--steps", str(args.steps),
           "--warmup", str(args.warmup), "--rho-alp-iters", str(args.rho_alp_iters), "--precision", prec,
           "--no-cpu-baseline", "--no-reference-precision"]
    if args.no_pmc:
        cmd.append("--no-pmc")
    try:
        r = subprocess.run(cmd, check=True, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, timeout=900,
                           env=dict(os.environ, TMPDIR="/tmp"))
    except Exception as e:  # noqa: BLE001
        return {"error": "fp64 child run failed: {}".format(e)}
    lines = [ln for ln in r.stdout.decode().splitlines() if ln.startswith("{")]
    if not lines:
        return {"error": "fp64 child printed no JSON line"}
    d = json.loads(lines[-1])
    d.pop("metric", None)
    d["parity"] = PARITY[prec]
    return d


PARITY = {
    "fp64": "fp64 device path (the reference's arithmetic) vs the float64 oracle: <= 1e-9 relative L2 on phi / rho "
            "at every config fixture incl. epsl 0.1 (tests/test_gpu_configs.py fp64 cases, tests/test_gpu_res64.py, "
            "tests/test_gpu_divergence.py pointwise), t-slabs vs the single fp64 context <= 1e-11 "
            "(tests/test_gpu_slab64.py, tests/test_gpu_decomp.py)",
    "fp32": "fp32 does NOT meet north_star's 1e-5 at epsl 0.1: one iteration from the seeded state phi 1.5-3.5e-5, "
            "from the reference state rho 4.9e-5 (C3) (profiles/parity_r04.json; DESIGN.md section 6: the explicit "
            "sigma*epsl*Lap(phi_bar) term amplifies phi_bar's float32 representation); a throughput reference only",
}


def dual_passes(inner_mean, nsub=5):
    """HBM passes of the chunked dual loop for a mean inner count (kernels_dual_multi.hpp): ceil(inner / nsub) chunk
    passes, plus the final re-run pass when the exit falls inside a chunk."""
    import math
    q = inner_mean / nsub
    chunks = math.ceil(q - 1e-9)
    return float(chunks + (0 if abs(q - round(q)) < 1e-9 else 1))


EXCH_KEYS = ("halo_rho", "halo_phibar", "carry_planes", "carry_long", "allreduce",
             "exposed_halo_rho", "exposed_halo_phibar", "exposed_carry_planes")
KERNEL_CLASSES = ("residual", "precond", "update", "dual")


def scale_report(dist, backend, el_s, iters, kern, exch):
    """The N > 1 line's self-check (a collective: every rank calls it).  Gathers each rank's wall time, kernel time
    per class and exchange / exposed-wait times (SlabRunner.exchange_times(), ms per iteration) to every rank, so the
    driver's first multi-GPU run can be read against the cost model of DESIGN.md section 7: per rank, step ms =
    kernel ms + exposed exchange ms + launch gaps.  Returns the report (identical on every rank)."""
    import torch
    world = dist.get_world_size()
    n = max(iters, 1)
    row = [el_s * 1e3 / n] + [kern.get(c, {}).get("avg_ms", 0.0) * kern.get(c, {}).get("launches", 0) / n
                              for c in KERNEL_CLASSES] + [float((exch or {}).get(c, 0.0)) for c in EXCH_KEYS]
    dev = "cuda" if backend == "nccl" else "cpu"
    mine = torch.tensor(row, dtype=torch.float64, device=dev)
    allr = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allr, mine)
    tab = np.array([t.cpu().numpy() for t in allr])
    step = tab[:, 0]
    kms = tab[:, 1:1 + len(KERNEL_CLASSES)]
    ex = tab[:, 1 + len(KERNEL_CLASSES):]
    exposed = ex[:, [EXCH_KEYS.index(c) for c in EXCH_KEYS if c.startswith("exposed_")]].sum(axis=1)
    return {"world_size_reported": world, "backend": backend,
            "ms_per_step_by_rank": step.tolist(), "ms_per_step_max": float(step.max()),
            "slowest_rank": int(step.argmax()),
            "kernel_ms_per_step_by_rank": {c: kms[:, i].tolist() for i, c in enumerate(KERNEL_CLASSES)},
            "exchange_ms_per_step_by_rank": {c: ex[:, i].tolist() for i, c in enumerate(EXCH_KEYS)},
            "exposed_exchange_ms_by_rank": exposed.tolist(),
            # what the kernels + exposed waits do not explain: launch / event gaps and host stalls
            "unexplained_ms_by_rank": (step - kms.sum(axis=1) - exposed).tolist()}


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n, argv):
    """--gpus N > 1 without a launcher: start N rank processes (torch.distributed.run, one per GPU) as a
    child process group before this process touches the GPU, and return their exit code."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node={}".format(n),
           "--master-addr", "127.0.0.1", "--master-port={}".format(_free_port()), os.path.abspath(__file__)] + argv
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC (RCCL on this host)
    env.setdefault("OMP_NUM_THREADS", "1")
    proc = subprocess.Popen(cmd, env=env, start_new_session=True)
    try:
        return proc.wait()
    except KeyboardInterrupt:
        os.killpg(proc.pid, 15)
        return proc.wait()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks); > 1 without WORLD_SIZE in the environment launches the ranks itself")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--rho-alp-iters", type=int, default=1)
    ap.add_argument("--precision", default=None, choices=["fp32", "fp64"],
                    help="fp64 (default: the reference's arithmetic, the one that meets the parity bar at epsl 0.1; "
                         "also the marching stop counts are only the reference's in it) or fp32")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-T", type=int, default=1)
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 PMC traffic passes")
    ap.add_argument("--no-probe", action="store_true", help="skip the non-finite probe and the finite segment")
    ap.add_argument("--no-reference-precision", action="store_true",
                    help="skip the nested line in the other precision (fp32 next to the fp64 single-GPU line, fp64 "
                         "next to an fp32 one)")
    ap.add_argument("--decomp", default="tslab", choices=["tslab", "xslab"],
                    help="multi-GPU decomposition of the window (xslab also at N = 1: one slab through its phases)")
    ap.add_argument("--marching", action="store_true",
                    help="time to solution of the T = 1 window-marching default on the config's grid (one GPU)")
    ap.add_argument("--windows", type=int, default=0,
                    help="--marching: only the first W windows (0: all nt - 1)")
    ap.add_argument("--selftest", action="store_true",
                    help="launcher / process-group check only: no GPU work, prints the world size")
    args = ap.parse_args()
    if args.precision is None:
        args.precision = "fp64"

    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        raise SystemExit("bench: --gpus {} but WORLD_SIZE={}".format(args.gpus, world))
    dist = None
    backend = os.environ.get("PDHG_DIST_BACKEND", "gloo" if args.selftest else "nccl")
    if world > 1:
        import torch
        import torch.distributed as tdist
        if not args.selftest:
            # device = local rank (modulo the visible GPUs: PDHG_DIST_BACKEND=gloo rehearses the multi-rank
            # path with several ranks on one GPU; the driver's runs use one GPU per rank over RCCL)
            dev = local_rank % max(1, torch.cuda.device_count())
            torch.cuda.set_device(dev)
        tdist.init_process_group(backend)
        dist = tdist
        if tdist.get_world_size() != world:
            raise SystemExit("bench: process group has {} ranks, WORLD_SIZE={}".format(tdist.get_world_size(), world))
    if args.selftest:
        if dist is not None:
            import torch
            t = torch.ones(1)
            dist.all_reduce(t)
            ranks_seen = int(t.item())
            dist.destroy_process_group()
        else:
            ranks_seen = 1
        if rank == 0:
            print(json.dumps({"selftest": True, "n_gpus": world, "ranks_seen": ranks_seen, "backend": backend}),
                  flush=True)
        return

    if args.marching:
        return marching(args)

    pmc, pmc_err = None, "disabled"
    if world == 1 and not args.no_pmc and args.decomp == "tslab":
        pmc, pmc_err = pmc_traffic(args)   # before this process initialises the GPU
    other_prec = None
    if world == 1 and args.decomp == "tslab" and not args.no_reference_precision:
        # likewise before this process initialises the GPU
        other_prec = other_precision_run(args, "fp32" if args.precision == "fp64" else "fp64")

    from pdhg_amd.context import PDHGContext

    progress("context ({}, {})".format(args.config, args.precision))
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
                           precision=args.precision, rho_alp_iters=k, device=torch.cuda.current_device())
    elif world > 1:
        from pdhg_amd.slab import DistComm, SlabContext, SlabRunner
        ctx = SlabContext(rank, world, T, egno, nx, ny, 2.0 / nx, 2.0 / ny, dt, xs, ys, epsl=epsl,
                          precision=args.precision, rho_alp_iters=k, device=torch.cuda.current_device())
    else:
        ctx = PDHGContext(egno, ndim, nx, ny, T, 2.0 / nx, 2.0 / ny if ndim == 2 else 0.0, dt, xs, ys, epsl=epsl,
                          precision=args.precision, rho_alp_iters=k, device=0)
    if ndim == 1:
        g = np.sin(np.pi * xs)
    else:
        g = np.sin(np.pi * xs)[:, None] + np.sin(np.pi * ys)[None, :]

    def init():
        """The reference initial state (phi = g, rho = 70, alp = 0; utils_pdhg_solver.py:123-137)."""
        if xslab:
            ctx.init_global_state(g)
        else:
            ctx.init_state(g)

    tau, sigma = 0.1 / 1.5, 0.1 * 1.5
    eps = 1e-6

    if xslab:
        from pdhg_amd.xslab import DistComm as XComm, LocalComm as XLocal, XSlabRunner
        xrunner = XSlabRunner([ctx], XComm() if world > 1 else XLocal(1))

        def run(n):
            s = xrunner.iterate(n, tau, sigma, eps, k)
            return {"iters_run": s["iters"], "status": s["status"], "nan_seen": s["nan_seen"],
                    "first_nan_iter": s.get("first_nan_iter", 0)}

        def sync():
            torch.cuda.synchronize()
    elif world > 1:
        import torch
        runner = SlabRunner([ctx], DistComm(), exchange=os.environ.get("PDHG_SLAB_EXCHANGE", "neighbour"))

        def run(n):
            s = runner.iterate(n, tau, sigma, eps, k)
            return {"iters_run": s["iters"], "status": s["status"], "nan_seen": s["nan_seen"],
                    "first_nan_iter": s.get("first_nan_iter", 0)}

        def sync():
            torch.cuda.synchronize()
    else:
        def run(n):
            return ctx.iterate(n, tau, sigma, eps, k)

        def sync():
            ctx.synchronize()

    def barrier():
        if dist is not None:
            dist.barrier()

    def max_over_ranks(x):
        if dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t[0])

    # epsl = 0.1 on a 4096^2 grid is outside the reference algorithm's stability range (explicit
    # sigma*epsl*Lap in the dual; its fp64 restatement diverges already at 256^2).  Probe: from the
    # reference initial state, the first iteration whose phi' or rho' holds a NaN (NaN stop on).
    first_nonfinite = None
    probe_n = 0
    progress("context ready")
    if not args.no_probe:
        init()
        ctx.set_stop_rules(converge=True, nan=True)
        probe_n = max(args.warmup + args.steps, 20)
        st = run(probe_n)
        sync()
        if st["status"] == 2 or st["nan_seen"]:
            first_nonfinite = int(st.get("first_nan_iter") or st["iters_run"])
    # the timed runs execute exactly the requested iterations (NaN stop off), each from the reference state
    ctx.set_stop_rules(converge=True, nan=False)

    def timed(n, fresh):
        """n iterations bracketed by barrier + synchronize; fresh: from the reference state, else continuing
        the current state (after the warm-up)."""
        if fresh:
            init()
        sync()
        ctx.profile_enable(True)
        barrier()
        sync()
        t0 = time.perf_counter()
        st = run(n)
        sync()
        barrier()
        el = time.perf_counter() - t0
        kern = {}
        # rho_alp_iters > 1 with the chunked dual (path_info dual_multi): one "dual" launch per outer iteration runs
        # the whole loop as passes of kMultiSub = 5 sub-iterations in registers (kernels_dual_multi.hpp), each pass
        # reading phi_bar, rho, alp and writing rho, alp ONCE -- so its HBM bytes are one sub-iteration's per pass,
        # not per sub-iteration: ceil(inner / 5) chunk passes + a final pass when the exit fell inside a chunk
        multi = k > 1 and ctx.path_info("dual_multi") == 1
        inner_mean = (st.get("inner_total", 0) / max(st["iters_run"], 1)) if multi else 1.0
        passes = dual_passes(inner_mean) if multi else 1.0
        for cls in ("residual", "precond", "update", "dual"):
            ms, nl = ctx.profile_query(cls)
            if nl:
                b = ctx.algorithmic_bytes(k, cls) * (passes if cls == "dual" else 1.0)
                kern[cls] = {"avg_ms": ms / nl, "launches": nl, "bytes_per_launch": b}
                if cls == "dual" and multi:
                    kern[cls]["passes"] = passes
                    kern[cls]["passes_note"] = ("chunk passes of 5 sub-iterations + final pass (kernels_dual_multi.hpp), "
                                                "inner mean {:.2f}: bytes = passes x one sub-iteration's".format(inner_mean))
        ctx.profile_enable(False)
        return st, el, kern, passes

    # finite segment: iterations 2..F from the reference state (the first, untimed, forms its residual from
    # scratch), all before the first non-finite one
    finite = None
    if not args.no_probe:
        F = 10 if first_nonfinite is None else min(10, first_nonfinite - 1)
        if F >= 2:
            init()
            run(1)
            st_f, el_f, kern_f, _ = timed(F - 1, fresh=False)
            el_f = max_over_ranks(el_f)
            finite = {"iters": "2..{}".format(F), "ms_per_step": el_f / (F - 1) * 1e3, "value": (F - 1) / el_f,
                      "nonfinite": bool(st_f["nan_seen"]),
                      "kernels_avg_ms": {c: d["avg_ms"] for c, d in kern_f.items()}}

    # the contract's run: W untimed warm-up iterations from the reference state, then exactly K timed
    # iterations continuing from there (so the first iteration's unfused residual is in the warm-up)
    progress("warm-up + timed run")
    init()
    if args.warmup > 0:
        run(args.warmup)
    sync()
    if runner is not None:
        runner.timing = True
    st, el, kern, dual_pass = timed(args.steps, fresh=args.warmup == 0)
    exch = runner.exchange_times() if runner is not None else None
    if runner is not None:
        runner.timing = False
    el_max = max_over_ranks(el)
    iters = st["iters_run"]
    iters_total = iters          # one window: every rank ran the same iterations

    if world > 1 or xslab:   # slabs: sweeps and halo/interior row parts are separate launches -> per iteration
        for cls, d in kern.items():
            per = max(iters, 1) * (k if cls == "dual" else 1)
            d["avg_ms"] = d["avg_ms"] * d["launches"] / per
            d["launches"] = per
    dom = max(kern, key=lambda c: kern[c]["avg_ms"] * kern[c]["launches"])
    d = kern[dom]
    achieved = d["bytes_per_launch"] / (d["avg_ms"] * 1e-3) / 1e9
    # per-rank dominant-kernel time (slabs differ by one row at most): the slowest rank bounds the step
    dom_ms_max = max_over_ranks(d["avg_ms"])
    it_bytes = ctx.algorithmic_bytes(k, "iteration") * world   # whole window (slabs are equal-ish): SURVEY 8(d)
    # the chunked dual moves one sub-iteration's bytes per pass (timed()): the iteration's HBM bytes are 8(d)'s with
    # the k sub-iterations' dual bytes replaced by the passes' (else the rate would exceed what crossed HBM)
    it_bytes_hbm = it_bytes + ctx.algorithmic_bytes(k, "dual") * world * (dual_pass - k) if (k > 1 and "passes" in
                                                                                           kern.get("dual", {})) else it_bytes
    ms_per_step = el_max / max(iters, 1) * 1e3
    report = None
    if dist is not None:   # every rank: collective
        report = scale_report(dist, backend, el, iters, kern,
                              {c: v / max(iters, 1) for c, v in (exch or {}).items()})
    if exch is not None:
        exch = {c: max_over_ranks(v) / max(iters, 1) for c, v in sorted(exch.items())}

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
        "dtype": {"fp32": "f32", "fp64": "f64"}[args.precision],
        "data": "synthetic: the reference initial state (phi=g, rho=70, alp=0), W warm-up iterations from it, "
                "then the K timed iterations continuing from there",
        "config": {"workload": "egno{} ndim{} epsl{} nx={} ny={} nt={}: one PDHG window of T={} rows, "
                               "rho_alp_iters={}".format(egno, ndim, epsl, nx, ny, nt, T, k),
                   "parallelism": ("x-slab x{} (halo-row allgathers, two all-to-all spectrum transposes per "
                                   "iteration)".format(world) if xslab else
                                   "t-slab x{} (RCCL point-to-point halos and carries, overlapped)".format(world))
                   if (world > 1 or xslab) else "single GPU",
                   "precision": args.precision,
                   "contig_fail": ctx.path_info("contig_fail") if hasattr(ctx, "path_info") else None,
                   "iters_executed": iters, "stop_status": st["status"], "state_nonfinite": bool(st["nan_seen"]),
                   "dual_subiters_mean": (st.get("inner_total", 0) / max(iters, 1)) if k > 1 else 1,
                   "first_nonfinite_iter": first_nonfinite,
                   "nonfinite_probe_iters": probe_n},
        "hbm_gbps_iteration": it_bytes_hbm / (ms_per_step * 1e-3) / 1e9,
        "iteration_bytes": it_bytes_hbm,
        "iteration_bytes_s8d": it_bytes,
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS, "traffic": None},
        "kernels": kern,
    }
    if finite is not None:
        out["finite_segment"] = finite
    if world > 1:
        out["world"] = {"world_size": dist.get_world_size(), "backend": dist.get_backend(),
                        "dominant_kernel_ms_max_over_ranks": dom_ms_max}
        out["scale_check"] = report
    if runner is not None:
        from pdhg_amd.slab import slab_bounds
        out["slab"] = {"rows_per_slab": [j1 - j0 for j0, j1 in slab_bounds(T, world)],
                       "carries": runner.exchange, "carry_parts": runner.parts, "long_range_modes": runner.n_long,
                       "halo_overlap": runner.side is not None,
                       "exchange_ms_per_iter_max_over_ranks": exch}
    if pmc and dom in pmc:
        out["roofline"]["traffic"] = pmc[dom]["bytes"]
        out["roofline"]["traffic_detail"] = pmc[dom]
        for cls in kern:
            if cls in pmc:
                kern[cls]["pmc_bytes_per_launch"] = pmc[cls]["bytes"]
        if "residual_first" in pmc:   # the unfused residual of a run's first iteration (in the warm-up here)
            out["kernels_first_iteration"] = {"residual_unfused": {"pmc_bytes_per_launch": pmc["residual_first"]["bytes"]}}
        out["pmc_by_kernel"] = pmc.get("_by_kernel")
    elif world == 1:
        out["roofline"]["traffic_note"] = pmc_err
    out["parity"] = PARITY[args.precision]
    if other_prec is not None:
        out["reference_precision" if args.precision == "fp32" else "fp32_precision"] = other_prec
    if world == 1 and not args.no_cpu_baseline:
        threads = min(16, os.cpu_count() or 1)
        sample_cfg = CONFIGS[args.config]
        progress("cpu baseline (float64 oracle, bounded sample)")
        out["cpu_baseline"] = cpu_baseline(sample_cfg, args.cpu_sample_T if ndim == 2 else 8, threads)
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
