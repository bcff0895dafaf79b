"""Diagnostic (round 5): where the fp64 device's late pointwise distance to the float64 oracle on C3's plane comes
from (test_gpu_divergence.py::test_c3_plane_pointwise_fp64: 2.6e-5 at iterations 7-10, where the same oracle on
numpy.fft instead of scipy.fft stays within 5e-7): the same comparison with kernel variants switched by env."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VARIANTS = {"default": {}, "unfused": {"PDHG_FUSE_RES": "0"}, "generic_res": {"PDHG_FUSE_RES": "0", "PDHG_RES64": "0"},
            "generic_dual": {"PDHG_FUSE_RES": "0", "PDHG_DUAL64": "0"}}


def one():
    sys.path[:0] = [os.path.join(ROOT, "pdhg-optimal-control_amd"), os.path.join(ROOT, "oracle"),
                    os.path.join(ROOT, "tests")]
    from _problems import device_ctx, make_problem
    from pdhg_amd import _native as N
    F = np.load(os.path.join(ROOT, "tests", "golden", "divergence_c3_plane_T4_points.npz"))
    egno, ndim, nx, ny, T = (int(v) for v in F["meta"])
    phi_idx, rho_idx = tuple(F["phi_idx"]), tuple(F["rho_idx"])
    G = make_problem(egno, ndim, nx, ny, 1, float(F["epsl"]), seeded=False)
    G.update(T=T, dt=float(F["dt"]))
    ctx = device_ctx(G, "fp64")
    ctx.init_state(G["g"][0])
    ctx.set_stop_rules(converge=False, nan=False)
    phi, rho = np.empty((T + 1, nx, ny)), np.empty((T, nx, ny))
    out = []
    for it in range(F["phi_pts"].shape[0]):
        ctx.iterate(1, 0.1 / 1.5, 0.15, -1.0, 1)
        N.check(ctx._lib.pdhg_get_state(ctx._h, N.dptr(phi), N.dptr(rho), None))
        out.append("%.1e/%.1e" % (np.linalg.norm(phi[phi_idx] - F["phi_pts"][it]) / np.linalg.norm(F["phi_pts"][it]),
                                  np.linalg.norm(rho[rho_idx] - F["rho_pts"][it]) / np.linalg.norm(F["rho_pts"][it])))
    print(os.environ.get("VARIANT"), {k: ctx.path_info(k) for k in ("fused_residual", "res64", "dual64")}, out,
          flush=True)
    ctx.close()


if __name__ == "__main__":
    if len(sys.argv) > 1:
        one()
    else:
        for name, env in VARIANTS.items():   # one process per variant (contexts read the env at creation)
            subprocess.run([sys.executable, os.path.abspath(__file__), "one"], env=dict(os.environ, VARIANT=name, **env),
                           check=True, timeout=400)
