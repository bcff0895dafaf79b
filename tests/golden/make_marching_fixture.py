"""Per-window stop iterations of the window-marching default (PDHG_multi_step, utils_pdhg_solver.py:97-225: T = 1
windows, rho_alp_iters = 10 with early exit, stepsz 0.1 with the NaN back-off, eps 1e-6) from the float64 oracle, at
C2's time step (dt = 0.01, egno 1, 2-D, epsl 0) on a 64^2 grid for the first 4 windows -- window 1 backs off to
stepsz 0.09 there, as C2's window 1 does on the device.  tests/test_gpu_parity.py::test_marching_window_counts_fp64
runs the fp64 device driver on the same problem and compares the counts, the step sizes and the final state.
Run: python tests/golden/make_marching_fixture.py   (~70 s)"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import pdhg_oracle as O  # noqa: E402

CASE = {"egno": 1, "ndim": 2, "nx": 64, "ny": 64, "windows": 4, "dt": 0.01, "epsl": 0.0, "rho_alp_iters": 10,
        "stepsz": 0.1, "eps": 1e-6}


def main():
    c = CASE
    nx, ny, ndim, egno = c["nx"], c["ny"], c["ndim"], c["egno"]
    x_arr = O.make_grid(ndim, nx, ny, egno)
    bc = O.default_bc(egno, ndim)
    fns = O.set_up_example_fns(egno, ndim, 0)
    g = O.set_up_J(egno, ndim, (2.0, 2.0))(x_arr)
    dsp = (2.0 / nx, 2.0 / ny)
    fv = O.compute_Dxx_fft_fv(ndim, (nx, ny), dsp, bc)
    primal, dual = O.make_update_fns(ndim, bc, rho_alp_iters=c["rho_alp_iters"])
    stats = []
    with np.errstate(all="ignore"):   # the backed-off attempt overflows before its NaN
        res, errs = O.PDHG_multi_step(primal, dual, fns, g, x_arr, ndim, c["windows"] + 1, (nx, ny), c["dt"], dsp, 70.0,
                                      time_step_per_PDHG=2, epsl=c["epsl"], stepsz_param=c["stepsz"], fv=fv,
                                      n_ctrl=ndim, N_maxiter=1000000, print_freq=1000000, eps=c["eps"], stats=stats)
    _, phi, rho, alp = res[0]
    out = dict(CASE, window_iters=[int(s["window_iters"]) for s in stats], window_stepsz=[s["stepsz"] for s in stats],
               phi_norm=float(np.linalg.norm(phi)), rho_norm=float(np.linalg.norm(rho)),
               phi_sample=phi.reshape(-1)[::997].tolist(), rho_sample=rho.reshape(-1)[::997].tolist())
    path = os.path.join(HERE, "marching_c2dt_64.json")
    json.dump(out, open(path, "w"), indent=1)
    print("wrote", path, out["window_iters"], out["window_stepsz"])


if __name__ == "__main__":
    main()
