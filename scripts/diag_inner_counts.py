"""Dual sub-iterations per outer iteration along C2's marching windows (fp64, T = 1, rho_alp_iters = 10, eps 1e-6):
the histogram that decides whether the speculative single-sub-iteration schedule pays (run via gpurun).

usage: python scripts/diag_inner_counts.py [windows=2] [max_iters=4000]
Window w starts from window w-1's final state (as PDHG_multi_step marches: phi row 0 = the previous phi row 1)."""
import collections
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(ROOT, "pdhg-optimal-control_amd"), ROOT]

import numpy as np  # noqa: E402

import bench  # noqa: E402
from pdhg_amd.context import PDHGContext  # noqa: E402


def main():
    windows = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    max_iters = int(sys.argv[2]) if len(sys.argv) > 2 else 4000
    egno, ndim, epsl, nx, ny, nt = bench.CONFIGS["c2"]
    xs, ys = bench.grid(ndim, nx, ny)
    dt = 1.0 / (nt - 1)
    k = 10
    ctx = PDHGContext(egno, ndim, nx, ny, 1, 2.0 / nx, 2.0 / ny, dt, xs, ys, epsl=epsl, rho_alp_iters=k, device=0,
                      precision="fp64")
    print(json.dumps({"dual_head": ctx.path_info("dual_head"), "dual_multi": ctx.path_info("dual_multi")}), flush=True)
    g = np.sin(np.pi * xs)[:, None] + np.sin(np.pi * ys)[None, :]
    phi0 = np.stack([g, g])
    rho0 = np.full((1, nx, ny), 70.0)
    alp0 = tuple(np.zeros((1, nx, ny, 2)) for _ in range(4))
    tau, sigma = 0.1 / 1.5, 0.1 * 1.5
    for w in range(windows):
        ctx.set_state(phi0, rho0, alp0)
        hist = collections.Counter()
        runs = []          # lengths of runs of consecutive one-sub-iteration iterations
        cur = 0
        status = 0
        for i in range(max_iters):
            st = ctx.iterate(1, tau, sigma, 1e-6, k)
            c = st["inner_total"]
            hist[c] += 1
            if c == 1:
                cur += 1
            else:
                runs.append(cur)
                cur = 0
            if st["status"] != 0:
                status = st["status"]
                break
        runs.append(cur)
        print(json.dumps({"window": w, "iters": i + 1, "status": status, "hist": dict(sorted(hist.items())),
                          "runs_of_ones": {"count": len(runs), "mean": float(np.mean(runs)),
                                           "median": float(np.median(runs)), "first20": runs[:20]}}), flush=True)
        phi, rho, alp = ctx.get_state()
        phi0 = np.stack([phi[1], phi[1]])
        rho0, alp0 = rho, alp
    ctx.close()


if __name__ == "__main__":
    main()
