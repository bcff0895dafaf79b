"""Interleaved same-process A/B of tuning environment variables (run via gpurun).

Each variant is a set of NAME=value overrides read by the context at creation (pdhg_api.hip setup()); the
variants are created, timed and destroyed in turn, ROUNDS times interleaved, so box drift hits all of them
alike.  Per kernel class: the median over rounds of the HIP-event average (pdhg_profile_query).

usage: python scripts/ab_env.py <config> <rounds> <steps> "A=1 B=2" "A=2" ...   ("" = no overrides)
AB_PREC=fp64: the contexts' precision (default fp32).
AB_REPS=n: n timed segments per context (re-initialised state each), to separate per-context from per-run spread.
"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(ROOT, "pdhg-optimal-control_amd"), ROOT]

import numpy as np  # noqa: E402

import bench  # noqa: E402
from pdhg_amd.context import PDHGContext  # noqa: E402

CLASSES = ("residual", "precond", "update", "dual")


def run_variant(cfg, steps, overrides, k=1):
    saved = {n: os.environ.get(n) for n in overrides}
    os.environ.update(overrides)
    try:
        egno, ndim, epsl, nx, ny, nt = bench.CONFIGS[cfg]
        T = nt - 1
        xs, ys = bench.grid(ndim, nx, ny)
        ctx = PDHGContext(egno, ndim, nx, ny, T, 2.0 / nx, 2.0 / ny if ndim == 2 else 0.0, 1.0 / T, xs, ys,
                          epsl=epsl, rho_alp_iters=k, device=0, precision=os.environ.get("AB_PREC", "fp32"))
    finally:
        for n, v in saved.items():
            if v is None:
                os.environ.pop(n, None)
            else:
                os.environ[n] = v
    g = np.sin(np.pi * xs)[:, None] + np.sin(np.pi * ys)[None, :] if ndim == 2 else np.sin(np.pi * xs)
    ctx.init_state(g)
    ctx.set_stop_rules(converge=True, nan=False)
    tau, sigma = 0.1 / 1.5, 0.1 * 1.5
    outs = []
    for _ in range(int(os.environ.get("AB_REPS", "1"))):   # repeated segments in the same context
        ctx.init_state(g)
        ctx.iterate(3, tau, sigma, 1e-6, k)
        ctx.synchronize()
        ctx.profile_enable(True)
        t0 = time.perf_counter()
        ctx.iterate(steps, tau, sigma, 1e-6, k)
        ctx.synchronize()
        el = (time.perf_counter() - t0) / steps * 1e3
        out = {"step_ms": el, "contig_fail": ctx.path_info("contig_fail")}
        for cls in CLASSES:
            ms, nl = ctx.profile_query(cls)
            if nl:
                out[cls] = ms / nl
        ctx.profile_enable(False)
        outs.append(out)
    ctx.close()
    return outs


def main():
    cfg, rounds, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    variants = [dict(kv.split("=", 1) for kv in v.replace("+", " ").split()) for v in sys.argv[4:]] or [{}]
    res = [[] for _ in variants]
    for r in range(rounds):
        for i, ov in enumerate(variants):
            for rep, o in enumerate(run_variant(cfg, steps, ov)):
                res[i].append(o)
                print(json.dumps({"round": r, "rep": rep, "variant": sys.argv[4 + i] if len(sys.argv) > 4 else "",
                                  **{k: round(v, 3) for k, v in o.items()}}), flush=True)
    for i, rs in enumerate(res):
        med = {k: round(statistics.median(x[k] for x in rs), 3) for k in rs[0]}
        print("MEDIAN", repr(sys.argv[4 + i] if len(sys.argv) > 4 else ""), json.dumps(med), flush=True)


if __name__ == "__main__":
    main()
