"""Diagnostic (round 5): run-to-run determinism of the fp64 single context's kernels at C4's slab shape
(nx = 8192 half-real fp64 x transform, generic row kernels at ny = 256, the LDS dual), one phase at a time from
a seeded state: update_primal (residual + x transform + update), then update_dual.  Bitwise equality expected."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pdhg-optimal-control_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
from _problems import device_ctx, make_problem  # noqa: E402

TAU, SIGMA = 0.1 / 1.5, 0.1 * 1.5
nx, ny, T = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (8192, 256, 128)))
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 12
P = make_problem(2, 2, nx, ny, T, 0.1, seeded=True)
ref = None
for rep in range(reps):
    ctx = device_ctx(P, "fp64")
    ctx.set_state(P["phi"], P["rho"], P["alp"])
    ctx.update_primal(TAU)
    phi1 = ctx.get_state(rho=False, alp=False)[0]
    ctx.update_dual(SIGMA, -1.0, 1)
    _, rho1, alp1 = ctx.get_state(phi=False)
    info = {k: ctx.path_info(k) for k in ("f64_xt", "half_real", "res64", "fast_dual", "fused_residual")}
    ctx.close()
    if ref is None:
        ref = (phi1, rho1, alp1)
        print("paths", info, flush=True)
        continue
    dphi = np.flatnonzero(phi1 != ref[0])
    drho = np.flatnonzero(rho1 != ref[1])
    print("rep", rep, "phi diffs", dphi.size, "rho diffs", drho.size,
          "first phi idx (t,x,y)", np.unravel_index(dphi[:3], phi1.shape) if dphi.size else "-", flush=True)
