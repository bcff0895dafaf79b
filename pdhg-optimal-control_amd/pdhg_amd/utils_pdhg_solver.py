"""PDHG drivers with the reference signatures (jaxsrc/utils/utils_pdhg_solver.py).

``PDHG_solver_oneiter`` and ``PDHG_multi_step`` accept the same arguments and
return the same structures as the reference.  When the update callables come
from ``make_update_fns`` (the analogue of the lambdas solve_HJ builds,
run_example.py:192-203) the whole outer loop runs on the device through
``pdhg_iterate``: state stays in HBM, convergence / NaN stops are decided on
the device, and the host only synchronises at print points
(``i % print_freq == 0``) to take the reference's snapshots.  Other callables
are driven by the reference's Python loop, one call per iteration.
"""
import numpy as np

from . import update_fns_in_pdhg as U
from .solver import save


def make_update_fns(ndim, bc, C=1.0, pow=1.0, Ct=1.0, rho_alp_iters=10, precision=None):
    """fn_update_primal / fn_update_dual as bound in solve_HJ (run_example.py:192-203), tagged for the device loop."""
    upd_primal = U.update_primal_1d if ndim == 1 else U.update_primal_2d

    def fn_update_primal(phi_prev, rho_prev, c_on_rho, alp_prev, tau, dt, dspatial, fns_dict, fv, epsl, x_arr, t_arr):
        return upd_primal(phi_prev, rho_prev, c_on_rho, alp_prev, tau, dt, dspatial, fns_dict, fv, epsl, x_arr, t_arr,
                          bc, C=C, pow=pow, Ct=Ct)

    def fn_update_dual(phi_bar, rho_prev, c_on_rho, alp_prev, sigma, dt, dspatial, epsl, fns_dict, x_arr, t_arr, nd,
                       eps):
        return U.update_dual_alternative(phi_bar, rho_prev, c_on_rho, alp_prev, sigma, dt, dspatial, epsl, fns_dict,
                                         x_arr, t_arr, nd, bc, rho_alp_iters=rho_alp_iters, eps=eps)

    tag = {"bc": bc, "C": C, "pow": pow, "Ct": Ct, "rho_alp_iters": rho_alp_iters, "precision": precision}
    fn_update_primal._pdhg_native = tag
    fn_update_dual._pdhg_native = tag
    return fn_update_primal, fn_update_dual


def _native_tag(fp, fd):
    tp, td = getattr(fp, "_pdhg_native", None), getattr(fd, "_pdhg_native", None)
    return tp if (tp is not None and tp is td) else None


def _device_oneiter(tag, fns_dict, phi0, rho0, alp0, x_arr, ndim, dt, dspatial, c_on_rho, epsl, stepsz_param,
                    N_maxiter, print_freq, eps, verbose, stats, last_only=False):
    """last_only (PDHG_multi_step, which reads results_all[-1] only, utils_pdhg_solver.py:187): the print-point
    records keep no state copies (they would be discarded)."""
    spec = U._spec(fns_dict)
    phi0 = np.asarray(phi0, dtype=np.float64)
    T = phi0.shape[0] - 1
    ctx = U.get_context(spec, T, phi0.shape[1:], dt, dspatial, epsl, x_arr, tag["bc"], tag["C"], tag["pow"],
                        tag["Ct"], c_on_rho, tag["rho_alp_iters"], tag["precision"])
    if ctx.is_resident(rho0, alp0):   # the previous window's result, still on the device: re-seed phi alone
        ctx.set_state(phi0, None, None)
    else:
        ctx.set_state(phi0, rho0, alp0)
    scale = 1.5                                           # utils_pdhg_solver.py:44-46
    tau, sigma = stepsz_param / scale, stepsz_param * scale
    k = tag["rho_alp_iters"]
    results_all, error_all = [], []
    i = 0
    last = None
    while i < N_maxiter:
        if print_freq > 0 and i % print_freq == 0:
            if last_only:
                pass
            elif i == 0:   # the state just set: the caller's arrays (as the reference records them), no device copy
                phi_prev = phi0.copy()
                rho_prev = np.array(rho0, dtype=np.float64).reshape((T,) + phi0.shape[1:])
            else:
                phi_prev, rho_prev, _ = ctx.get_state(alp=False)
            st = ctx.iterate(1, tau, sigma, eps, k)
            last = st
            if st["status"] != 0:
                break
            error = np.array([st["err1"], st["err2"]])
            if not last_only:
                _, _, alp_next = ctx.get_state(phi=False, rho=False)
                results_all.append((i, phi_prev, rho_prev, alp_next))
            error_all.append(error)
            if verbose:
                print("iteration {}, primal error {:.2E}, dual error {:.2E}".format(i, error[0], error[1]), flush=True)
            i += 1
            continue
        n = N_maxiter - i
        if print_freq > 0:
            n = min(n, print_freq - i % print_freq)
        st = ctx.iterate(n, tau, sigma, eps, k)
        last = st
        i += st["iters_run"]
        if st["status"] != 0:
            i -= 1            # index of the stopping iteration
            break
    else:
        i -= 1
    if last is None:
        raise ValueError("N_maxiter must be >= 1")
    if verbose and last["status"] == 1:
        print("PDHG converges at iter {}".format(i), flush=True)
    if verbose and last["status"] == 2:
        print("Nan error at iter {}".format(i))
    if stats is not None:
        stats.append(dict(last, window_iters=i + 1))   # + the iterations this window ran
    phi, rho, alp = ctx.get_state()
    # rho / alp as the device holds them: read-only (the reference returns immutable jax arrays), so the next window's
    # set_state can keep them on the device when they come back unchanged (PDHG_multi_step: rho0, alp0 = rho_c, alp_c)
    for a in (rho,) + tuple(alp):
        a.flags.writeable = False
    ctx.mark_resident(rho, alp)
    error = np.array([last["err1"], last["err2"]])
    results_all.append((i + 1, phi, rho, alp))
    error_all.append(error)
    return results_all, np.array(error_all)


def PDHG_solver_oneiter(fn_update_primal, fn_update_dual, fns_dict, phi0, rho0, alp0, x_arr, t_arr, ndim, dt, dspatial,
                        c_on_rho, epsl=0.0, stepsz_param=0.9, fv=None, N_maxiter=1000000, print_freq=1000, eps=1e-6,
                        tfboard=False, tfrecord_ind=0, verbose=True, stats=None, _last_only=False):
    """Outer PDHG loop (utils_pdhg_solver.py:9-94).  Returns (results_all, error_all).  _last_only (internal, used by
    PDHG_multi_step): the print-point entries of results_all carry no state (only results_all[-1] is read there)."""
    tag = _native_tag(fn_update_primal, fn_update_dual)
    if tag is not None:
        U.check_fv(fv, ndim, np.shape(phi0)[1:], dspatial, tag["bc"])
        return _device_oneiter(tag, fns_dict, phi0, rho0, alp0, x_arr, ndim, dt, dspatial, c_on_rho, epsl,
                               stepsz_param, N_maxiter, print_freq, eps, verbose, stats, last_only=_last_only)
    # generic callables: the reference's host loop, one device call per update
    phi_prev, rho_prev, alp_prev = phi0, rho0, alp0
    tau, sigma = stepsz_param / 1.5, stepsz_param * 1.5
    error_all, results_all = [], []
    for i in range(N_maxiter):
        phi_next = fn_update_primal(phi_prev, rho_prev, c_on_rho, alp_prev, tau, dt, dspatial, fns_dict, fv, epsl,
                                    x_arr, t_arr)
        phi_bar = 2 * phi_next - phi_prev
        rho_next, alp_next = fn_update_dual(phi_bar, rho_prev, c_on_rho, alp_prev, sigma, dt, dspatial, epsl, fns_dict,
                                            x_arr, t_arr, ndim, eps)
        with np.errstate(divide="ignore", invalid="ignore"):
            err1 = np.linalg.norm(phi_next - phi_prev) / np.linalg.norm(phi_prev)
            err2 = np.linalg.norm(rho_next - rho_prev) / np.linalg.norm(rho_prev)
            for a_p, a_n in zip(alp_prev, alp_next):
                na, ne = np.linalg.norm(a_p), np.linalg.norm(a_p - a_n)
                if na < 1e-6 and ne > 1e-6:
                    err2 += ne
                elif na >= 1e-6:
                    err2 += ne / na
        error = np.array([err1, err2])
        if error[0] < eps and error[1] < eps:
            break
        if np.any(np.isnan(phi_next)) or np.any(np.isnan(rho_next)):
            break
        if print_freq > 0 and i % print_freq == 0:
            results_all.append((i, phi_prev, rho_prev, alp_next))
            error_all.append(error)
        phi_prev, rho_prev, alp_prev = phi_next, rho_next, alp_next
    results_all.append((i + 1, phi_next, rho_next, alp_next))
    error_all.append(error)
    return results_all, np.array(error_all)


def _stacked(alp):
    """np.stack(alp, axis=0) without the copy when the arrays are views of one such block (get_state's result)."""
    b = getattr(alp[0], "base", None) if len(alp) else None
    if isinstance(b, np.ndarray) and b.shape == (len(alp),) + alp[0].shape and b.flags.c_contiguous and \
            all(a.base is b and np.shares_memory(a, b[i]) and a.__array_interface__["data"][0] ==
                b[i].__array_interface__["data"][0] for i, a in enumerate(alp)):
        return b
    return np.stack(alp, axis=0)


def PDHG_multi_step(fn_update_primal, fn_update_dual, fns_dict, g, x_arr, ndim, nt, nspatial, dt, dspatial, c_on_rho,
                    time_step_per_PDHG=2, epsl=0.0, stepsz_param=0.9, n_ctrl=None, fv=None, N_maxiter=1000000,
                    print_freq=1000, eps=1e-6, tfboard=False, save_middle_dir=None, save_middle_prefix=None,
                    load_middle_dir=None, load_middle_prefix=None, verbose=True, stats=None):
    """Time-window marching with NaN step-size back-off (utils_pdhg_solver.py:97-225)."""
    from .solver import load_middle_solution
    if n_ctrl is None:
        n_ctrl = ndim
    assert (nt - 1) % (time_step_per_PDHG - 1) == 0
    nt_PDHG = (nt - 1) // (time_step_per_PDHG - 1)
    T = time_step_per_PDHG - 1
    g = np.asarray(g, dtype=np.float64)
    phi0 = np.repeat(g, time_step_per_PDHG, axis=0)
    space = tuple(nspatial)
    n_alp = 2 if ndim == 1 else 4
    rho0 = np.full((T,) + space, float(c_on_rho))
    alp0 = tuple(np.zeros((T,) + space + (n_ctrl,)) for _ in range(n_alp))
    max_iters = 0
    phi_all, rho_all, alp_all, errs_all = [], [], [], []
    init_t = 0
    phi_end = None
    # back-off schedule from the CALLER's step size (utils_pdhg_solver.py:160-161), fixed before a middle file
    # restores a reduced one, so a resumed run steps down exactly as the uninterrupted run does
    s_delta = stepsz_param / 10
    s_min = stepsz_param / 10
    if load_middle_dir is not None and load_middle_prefix is not None:
        # middle results: [max_iters, phi_all, rho_all, alp_all, errs_all, phi0_next, stepsz_param]; phi_all keeps
        # phi_c[:-1] for every window but the last (utils_pdhg_solver.py:192-195), so the warm start the next
        # window begins from (phi0 + (phi_c[-1:] - phi0[0:1]), :201-203) is saved whole (phi0_next) and restored
        # bit for bit, with the step size the run had reached (after any back-off).  Files of round 2 hold only
        # the end row there (shape [1, ...]): it is repeated.
        # The reference's own 5-entry list (:211-212) holds no end row; it restarts from phi_all[-1:] (:145-147),
        # the last saved window's entries.  Here that window is solved again: every window's phi0 repeats one row
        # (:123, and the warm start adds the same row to every row, :201-203), and that row is phi_all[-1][0]
        # (row 0 never changes, utils_precond.py:139/177), so its start state is known exactly -- rho / alp from
        # the window before it (or the initial ones).  The 5-entry list holds no step size: the re-solved window
        # and those after it start from the CALLER's stepsz_param, so the run matches the uninterrupted one only
        # when no earlier window backed off (after a NaN back-off the uninterrupted run had continued at the
        # reduced step; tests/test_host.py::test_resume_5_entry_list_after_backoff).
        middle = load_middle_solution(load_middle_dir, load_middle_prefix)
        max_iters, phi_all, rho_all, alp_all, errs_all = [middle[0]] + [list(m) for m in middle[1:5]]
        init_t = len(phi_all)
        assert init_t == len(rho_all) == len(alp_all) == len(errs_all)
        if 0 < init_t < nt_PDHG:
            if len(middle) >= 7:
                phi_end, stepsz_param = np.asarray(middle[5], dtype=np.float64), float(middle[6])
                if phi_end.shape == phi0.shape:
                    phi0 = phi_end.copy()
                else:
                    phi0 = np.repeat(phi_end.reshape((1,) + phi0.shape[1:]), time_step_per_PDHG, axis=0)
                rho0 = rho_all[-1]
                alp0 = tuple(alp_all[-1][i] for i in range(n_alp))
            else:
                row = np.asarray(phi_all[-1], dtype=np.float64)[0:1]
                phi0 = np.repeat(row, time_step_per_PDHG, axis=0)
                for lst in (phi_all, rho_all, alp_all, errs_all):
                    lst.pop()
                init_t -= 1
                if init_t > 0:
                    rho0 = rho_all[-1]
                    alp0 = tuple(alp_all[-1][i] for i in range(n_alp))
    sol_nan = False
    for i in range(init_t, nt_PDHG):
        t_arr = np.linspace(i * dt * T, (i + 1) * dt * T, num=time_step_per_PDHG)[1:]
        t_arr = t_arr[:, None] if ndim == 1 else t_arr[:, None, None]
        while True:
            results_all, errs = PDHG_solver_oneiter(fn_update_primal, fn_update_dual, fns_dict, phi0, rho0, alp0,
                                                    x_arr, t_arr, ndim, dt, dspatial, c_on_rho, epsl=epsl,
                                                    stepsz_param=stepsz_param, fv=fv, N_maxiter=N_maxiter,
                                                    print_freq=print_freq, eps=eps, verbose=verbose, stats=stats,
                                                    _last_only=True)
            if np.any(np.isnan(errs)):
                if stepsz_param > s_min + s_delta:            # back-off, utils_pdhg_solver.py:180-183
                    stepsz_param -= s_delta
                    if verbose:
                        print("pdhg does not conv at t_ind = {}, decrease step size to {}".format(i, stepsz_param),
                              flush=True)
                else:
                    sol_nan = True
                    break
            else:
                iters, phi_c, rho_c, alp_c = results_all[-1]
                max_iters = max(max_iters, iters)
                phi_all.append(phi_c[:-1] if i < nt_PDHG - 1 else phi_c)
                rho_all.append(rho_c)
                alp_all.append(_stacked(alp_c))
                errs_all.append(errs)
                phi0 = phi0 + (phi_c[-1:] - phi0[0:1])        # warm start, :201-203
                rho0, alp0 = rho_c, alp_c
                phi_end = phi0               # the next window's warm start, saved whole (a new array, never written)
                break
        if save_middle_dir is not None and save_middle_prefix is not None and phi_end is not None:
            save(save_middle_dir, save_middle_prefix,
                 [max_iters, phi_all, rho_all, alp_all, errs_all, phi_end, stepsz_param])
        if sol_nan:
            break
    phi_out = np.concatenate(phi_all, axis=0)
    rho_out = np.concatenate(rho_all, axis=0)
    alp_out = np.concatenate(alp_all, axis=1)
    if verbose:
        if sol_nan:
            print("pdhg does not conv, please decrease stepsize to be less than {}".format(stepsz_param), flush=True)
        else:
            print("pdhg conv. Max err is {:.2E}. Max iters is {}".format(
                max(float(np.max(e)) for e in errs_all), max_iters), flush=True)
    return [(max_iters, phi_out, rho_out, alp_out)], errs_all
