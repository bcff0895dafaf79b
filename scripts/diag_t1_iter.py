"""Per-iteration wall time of iterate() on C2's T = 1 window (fp64, rho_alp_iters = 10, eps 1e-6) in the steady phase
of a marching window (the dual loop exits after sub-iteration 0), for environment variants, interleaved (run via
gpurun).  usage: python scripts/diag_t1_iter.py [iters=2000] [rounds=3] "PDHG_SPEC=0" "PDHG_SPEC=1" ..."""
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(ROOT, "pdhg-optimal-control_amd"), ROOT]

import numpy as np  # noqa: E402

import bench  # noqa: E402
from pdhg_amd.context import PDHGContext  # noqa: E402


def run(variant, iters):
    ov = dict(kv.split("=", 1) for kv in variant.split())
    saved = {n: os.environ.get(n) for n in ov}
    os.environ.update(ov)
    try:
        egno, ndim, epsl, nx, ny, nt = bench.CONFIGS["c2"]
        xs, ys = bench.grid(ndim, nx, ny)
        ctx = PDHGContext(egno, ndim, nx, ny, 1, 2.0 / nx, 2.0 / ny, 1.0 / (nt - 1), xs, ys, epsl=epsl,
                          rho_alp_iters=10, device=0, precision="fp64")
    finally:
        for n, v in saved.items():
            if v is None:
                os.environ.pop(n, None)
            else:
                os.environ[n] = v
    g = np.sin(np.pi * xs)[:, None] + np.sin(np.pi * ys)[None, :]
    ctx.init_state(g)
    ctx.set_stop_rules(converge=False, nan=True)
    tau, sigma = 0.1 / 1.5, 0.1 * 1.5
    ctx.iterate(200, tau, sigma, 1e-6, 10)          # past the window's multi-sub-iteration start
    ctx.synchronize()
    t0 = time.perf_counter()
    st = ctx.iterate(iters, tau, sigma, 1e-6, 10)
    ctx.synchronize()
    el = time.perf_counter() - t0
    out = {"variant": variant, "ms_per_iter": el / max(st["iters_run"], 1) * 1e3, "iters": st["iters_run"],
           "inner_total": st["inner_total"], "spec_iters": ctx.path_info("spec_iters"),
           "spec_halts": ctx.path_info("spec_halts")}
    ctx.close()
    return out


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    variants = sys.argv[3:] or ["PDHG_SPEC=0", "PDHG_SPEC=1"]
    res = {v: [] for v in variants}
    for _ in range(rounds):
        for v in variants:
            o = run(v, iters)
            res[v].append(o["ms_per_iter"])
            print(json.dumps(o), flush=True)
    for v in variants:
        print("MEDIAN", repr(v), round(float(np.median(res[v])), 4), "ms per iteration", flush=True)


if __name__ == "__main__":
    main()
