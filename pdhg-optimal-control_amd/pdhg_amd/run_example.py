"""Command-line driver mirroring jaxsrc/run_example.py (flags :403-440, main :212-330, solve_HJ :157-210).

    python -m pdhg_amd.run_example --egno 1 --ndim 2 --nx 256 --ny 256 --nt 41 --time_step_per_PDHG 41

Same flags, grid (egno 3: centred grid, bc (1, 0), n_ctrl 1), initial value J(x), symbol fv, window
marching (PDHG_multi_step with the NaN step-size back-off) and result layout
(results = [(iters, phi, rho, alp)], errs_all).  The PDHG iterations of every window run on the GPU
through libpdhg.so (make_update_fns tags the callables for the device loop).  Results are saved as an
npz tree (pdhg_amd.solver) instead of a pickle.  --plot writes the reference's figures (phi, each alp
component, their sum; matplotlib, PNG) under plots/<stamp>/eg<egno>_<ndim>d, and with --plot_traj_num_1d > 0
simulates the controlled trajectories from the solved alp (pdhg_amd.trajectories, run_example.py:342-393)
and saves them as traj_<prefix>.npz (+ figures).  --tfboard is accepted and ignored (no TensorBoard).
Extra flags: --precision {fp32,fp64}, --rho_alp_iters (the reference fixes 10), --out (root dir),
--load_middle / --load_middle_timestamp (resume from middle results, run_example.py:246-248).
"""
import argparse
import os
import time

import numpy as np

from . import set_fns, solver, trajectories, utils_pdhg_solver, utils_precond


def build_parser():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    A = ap.add_argument
    # problem parameters (run_example.py:405-409)
    A("--egno", type=int, default=1)
    A("--ndim", type=int, default=1)
    A("--epsl", type=float, default=0.0)
    A("--x_period", type=float, default=2.0)
    A("--y_period", type=float, default=2.0)
    # grid sizes (:411-413)
    A("--nt", type=int, default=11)
    A("--nx", type=int, default=20)
    A("--ny", type=int, default=20)
    A("--stepsz_param", type=float, default=0.1)
    # saving / loading (:417-421)
    A("--save", type=int, default=1)
    A("--save_middle", type=int, default=0)
    A("--load", type=int, default=0)
    A("--load_timestamp", default="")
    A("--load_middle", type=int, default=0)
    A("--load_middle_timestamp", default="")
    # plotting (:423-425)
    A("--tfboard", type=int, default=0)
    A("--plot", type=int, default=0)
    A("--plot_traj_num_1d", type=int, default=0)
    # hyper-parameters (:428-440)
    A("--T", type=float, default=1.0)
    A("--c_on_rho", type=float, default=70.0)
    A("--time_step_per_PDHG", type=int, default=2)
    A("--N_maxiter", type=int, default=1000000)
    A("--print_freq", type=int, default=10000)
    A("--eps", type=float, default=1e-6)
    A("--C", type=float, default=1.0)
    A("--pow", type=float, default=1.0)
    A("--Ct", type=float, default=1.0)
    A("--numerical_L_ind", type=int, default=0)
    # this build
    A("--precision", choices=("fp32", "fp64"), default="fp64",
      help="device arithmetic (the reference runs float64)")
    A("--rho_alp_iters", type=int, default=10)
    A("--out", default=".")
    return ap


def make_grid(ndim, egno, nx, ny, nt, x_period, y_period, T):
    """x_arr [1, nx, 1] or [1, nx, ny, 2] and t_arr as run_example.py:268-285 (egno 3 centred)."""
    centred = egno == 3
    x1 = np.linspace(0.0, x_period, nx, endpoint=False) - (x_period / 2 if centred else 0.0)
    if ndim == 1:
        return x1[None, :, None], np.linspace(0.0, T, nt)[:, None]
    x2 = np.linspace(0.0, y_period, ny, endpoint=False) - (y_period / 2 if centred else 0.0)
    xm, ym = np.meshgrid(x1, x2, indexing="ij")
    return np.stack([xm, ym], axis=-1)[None], np.linspace(0.0, T, nt)[:, None, None]


def solve_HJ(ndim, n_ctrl, egno, epsl, fns_dict, nx, ny, nt, x_period, y_period, T, x_arr, c_on_rho,
             time_step_per_PDHG, stepsz_param, N_maxiter, print_freq, eps, bc, C=1.0, pow=1.0, Ct=1.0,
             rho_alp_iters=10, precision="fp64", save_middle_dir=None, save_middle_prefix=None, load_middle_dir=None,
             load_middle_prefix=None, verbose=True):
    """run_example.py:157-210 with the device-resident update functions."""
    dt = T / (nt - 1)
    dx, dy = x_period / nx, y_period / ny
    if ndim == 1:
        period, dspatial, nspatial = (x_period,), (dx,), (nx,)
    else:
        period, dspatial, nspatial = (x_period, y_period), (dx, dy), (nx, ny)
    g = set_fns.set_up_J(egno, ndim, period)(x_arr)
    fv = utils_precond.compute_Dxx_fft_fv(ndim, nspatial, dspatial, bc)
    fp, fd = utils_pdhg_solver.make_update_fns(ndim, bc, C=C, pow=pow, Ct=Ct, rho_alp_iters=rho_alp_iters,
                                               precision=precision)
    return utils_pdhg_solver.PDHG_multi_step(fp, fd, fns_dict, g, x_arr, ndim, nt, nspatial, dt, dspatial, c_on_rho,
                                             time_step_per_PDHG=time_step_per_PDHG, epsl=epsl,
                                             stepsz_param=stepsz_param, fv=fv, n_ctrl=n_ctrl, N_maxiter=N_maxiter,
                                             print_freq=print_freq, eps=eps, save_middle_dir=save_middle_dir,
                                             save_middle_prefix=save_middle_prefix, load_middle_dir=load_middle_dir,
                                             load_middle_prefix=load_middle_prefix, verbose=verbose)


def main(argv=None):
    F = build_parser().parse_args(argv)
    for k, v in sorted(vars(F).items()):
        print(k, ": ", v, flush=True)
    if F.egno == 3:          # Newton: n_ctrl 1, ndim 2, bc (1, 0), centred grid (run_example.py:227-233)
        if F.ndim != 2:
            raise SystemExit("egno 3 requires --ndim 2")
        n_ctrl, bc = 1, (1, 0)
    else:
        n_ctrl, bc = F.ndim, (0 if F.ndim == 1 else (0, 0))
    prefix = "nt{}_nx{}".format(F.nt, F.nx) if F.ndim == 1 else "nt{}_nx{}_ny{}".format(F.nt, F.nx, F.ny)
    if F.load:
        stamp = F.load_timestamp
    elif F.load_middle:
        stamp = F.load_middle_timestamp
    else:
        stamp = time.strftime("%Y%m%d-%H%M%S")
    if (F.load or F.load_middle) and not stamp:
        raise SystemExit("--load / --load_middle need --load_timestamp / --load_middle_timestamp")
    save_dir = os.path.join(F.out, "check_points", stamp, "eg{}_{}d".format(F.egno, F.ndim))
    plot_dir = os.path.join(F.out, "plots", stamp, "eg{}_{}d".format(F.egno, F.ndim))
    os.makedirs(save_dir, exist_ok=True)
    fns = set_fns.set_up_example_fns(F.egno, F.ndim, F.numerical_L_ind)
    x_arr, t_arr = make_grid(F.ndim, F.egno, F.nx, F.ny, F.nt, F.x_period, F.y_period, F.T)
    if F.load:
        results, errs_all = solver.load_solution(save_dir, prefix)
    else:
        results, errs_all = solve_HJ(F.ndim, n_ctrl, F.egno, F.epsl, fns, F.nx, F.ny, F.nt, F.x_period, F.y_period,
                                     F.T, x_arr, F.c_on_rho, F.time_step_per_PDHG, F.stepsz_param, F.N_maxiter,
                                     F.print_freq, F.eps, bc, C=F.C, pow=F.pow, Ct=F.Ct,
                                     rho_alp_iters=F.rho_alp_iters, precision=F.precision,
                                     save_middle_dir=save_dir if F.save_middle else None,
                                     save_middle_prefix=prefix if F.save_middle else None,
                                     load_middle_dir=save_dir if F.load_middle else None,
                                     load_middle_prefix=prefix if F.load_middle else None)
        if F.save:
            solver.save(save_dir, prefix, (results, errs_all))
    iters, phi = results[-1][0], results[-1][1]
    if F.plot:
        plot_results(F, results, x_arr, t_arr, fns, bc, n_ctrl, plot_dir, prefix)
    print("windows: {}  last window iterations: {}  phi shape: {}  saved: {}".format(
        len(results), iters, np.shape(phi), save_dir if F.save else "-"), flush=True)
    return results, errs_all


def plot_results(F, results, x_arr, t_arr, fns, bc, n_ctrl, plot_dir, prefix):
    """The plot block of run_example.main (:296-393): figures of phi and alp, and the trajectories."""
    os.makedirs(plot_dir, exist_ok=True)
    phi, alp = np.asarray(results[-1][1]), np.asarray(results[-1][3])
    try:
        from . import plotting
    except ImportError:            # matplotlib absent: trajectories are still computed and saved
        plotting = None
    if plotting is not None:
        plotting.plot_solution_figs(phi, alp, x_arr, t_arr, F.ndim, F.egno, n_ctrl, plot_dir)
    if F.plot_traj_num_1d > 0:
        traj_alp, traj_x = trajectories.run_trajectories(F.egno, F.ndim, alp, fns, F.nt, x_arr, t_arr, F.x_period,
                                                         F.y_period, F.T, bc, F.epsl, F.plot_traj_num_1d)
        np.savez(os.path.join(plot_dir, "traj_{}.npz".format(prefix)), traj_x=traj_x, traj_alp=traj_alp,
                 t=np.asarray(t_arr).reshape(-1))
        if plotting is not None:
            plotting.plot_traj_figs(traj_x, traj_alp, np.asarray(t_arr).reshape(-1), F.ndim, F.egno, n_ctrl,
                                    plot_dir)


if __name__ == "__main__":
    main()
