"""Host-side logic on CPU: persistence, the problem plugin, and the drivers' control flow.

The driver tests pass the oracle's update callables into the product's PDHG_solver_oneiter /
PDHG_multi_step (their generic "callables" loop), so the window marching, warm start, result
assembly and NaN step back-off logic of the product is checked against the oracle's driver on the
same arithmetic (utils_pdhg_solver.py:9-225)."""
import numpy as np
import pytest

import pdhg_oracle as O
from pdhg_amd import set_fns, solver, utils_pdhg_solver as S, utils_precond

rng = np.random.default_rng(1)


def test_save_load_roundtrip(tmp_path):
    res = [(12, rng.standard_normal((3, 4)), rng.standard_normal((2, 4)), rng.standard_normal((2, 2, 4, 1)))]
    errs = [np.array([[1e-3, 2e-3], [1e-7, 3e-7]])]
    solver.save(str(tmp_path), "sol", (res, errs))
    r2, e2 = solver.load_solution(str(tmp_path), "sol")
    assert r2[0][0] == 12 and isinstance(r2[0], tuple)
    for a, b in zip(res[0][1:], r2[0][1:]):
        assert np.array_equal(a, b)
    assert np.array_equal(errs[0], e2[0])
    mid = [7, [rng.standard_normal((2, 4))], [rng.standard_normal((1, 4))], [rng.standard_normal((2, 1, 4, 1))], []]
    solver.save(str(tmp_path), "mid", mid)
    m2 = solver.load_middle_solution(str(tmp_path), "mid")
    assert m2[0] == 7 and np.array_equal(m2[1][0], mid[1][0]) and m2[4] == []


@pytest.mark.parametrize("egno,ndim", [(1, 1), (2, 1), (1, 2), (2, 2), (3, 2)])
def test_plugin_matches_oracle(egno, ndim):
    nx, ny, T = 6, 5, 3
    x = O.make_grid(ndim, nx, ny, egno)
    po, pp = O.set_up_example_fns(egno, ndim, 0), set_fns.set_up_example_fns(egno, ndim, 0)
    assert pp.spec["egno"] == egno and "alp_update_fn" in pp._fields
    nc = 1 if (ndim == 1 or egno == 3) else 2
    sp = (T, nx) if ndim == 1 else (T, nx, ny)
    alp = tuple(rng.standard_normal(sp + (nc,)) for _ in range(2 if ndim == 1 else 4))
    if ndim == 2 and egno != 3:                      # dead components are zero in the examples
        alp[0][..., 1] = alp[1][..., 1] = alp[2][..., 0] = alp[3][..., 0] = 0
    if egno == 3:
        alp = alp[:2] + (np.zeros_like(alp[0]), np.zeros_like(alp[0]))
    rho = rng.uniform(1, 2, sp)
    assert np.allclose(po.f_fn(alp[0], x, None), pp.f_fn(alp[0], x, None))
    assert np.allclose(po.numerical_L_fn(alp, x, None), pp.numerical_L_fn(alp, x, None))
    if ndim == 1:
        D = rng.standard_normal(sp), rng.standard_normal(sp)
        for a, b in zip(po.alp_update_fn(alp, *D, rho, 0.15, x, None), pp.alp_update_fn(alp, *D, rho, 0.15, x, None)):
            assert np.allclose(a, b)
    else:
        D = tuple(rng.standard_normal(sp) for _ in range(4))
        for a, b in zip(po.alp_update_fn(alp, D, rho, 0.15, x, None), pp.alp_update_fn(alp, D, rho, 0.15, x, None)):
            assert np.allclose(a, b)
    po_J = O.set_up_J(egno, ndim, (2.0, 2.0))(x)
    assert np.allclose(po_J, set_fns.set_up_J(egno, ndim, (2.0, 2.0))(x))


def test_symbol_matches_oracle():
    assert np.allclose(utils_precond.compute_Dxx_fft_fv(1, (12,), (0.2,), 0), O.compute_Dxx_fft_fv(1, (12,), (0.2,), 0))
    for bc in ((0, 0), (1, 0)):
        assert np.allclose(utils_precond.compute_Dxx_fft_fv(2, (8, 6), (0.2, 0.3), bc),
                           O.compute_Dxx_fft_fv(2, (8, 6), (0.2, 0.3), bc), rtol=1e-12, atol=1e-9)


def _setup(nx=12, nt=5):
    x = O.make_grid(1, nx, 1, 1)
    fns = O.set_up_example_fns(1, 1, 0)
    g = O.set_up_J(1, 1, (2.0,))(x)
    fv = O.compute_Dxx_fft_fv(1, (nx,), (2.0 / nx,), 0)
    return x, fns, g, fv


def test_multi_step_driver_matches_oracle_driver():
    nx, nt = 12, 5
    x, fns, g, fv = _setup(nx, nt)
    primal, dual = O.make_update_fns(1, 0, rho_alp_iters=10)
    kw = dict(time_step_per_PDHG=3, stepsz_param=0.1, n_ctrl=1, fv=fv, N_maxiter=3000, print_freq=400, eps=1e-6)
    res_o, errs_o = O.PDHG_multi_step(primal, dual, fns, g, x, 1, nt, (nx,), 0.25, (2.0 / nx,), 70.0, **kw)
    res_p, errs_p = S.PDHG_multi_step(primal, dual, fns, g, x, 1, nt, (nx,), 0.25, (2.0 / nx,), 70.0, verbose=False,
                                      **kw)
    assert res_p[0][0] == res_o[0][0]
    for a, b in zip(res_p[0][1:], res_o[0][1:]):
        assert a.shape == b.shape and np.allclose(a, b, rtol=0, atol=0)
    assert len(errs_p) == len(errs_o)
    for a, b in zip(errs_p, errs_o):
        assert np.array_equal(a, b)


def test_nan_backoff_sequence_matches_oracle():
    """A primal that blows up for step sizes above 0.055 triggers the back-off of utils_pdhg_solver.py:174-187."""
    nx, nt = 8, 3
    x, fns, g, fv = _setup(nx, nt)
    primal, dual = O.make_update_fns(1, 0, rho_alp_iters=1)
    tried = {"o": [], "p": []}

    def mk(key):
        def p2(phi, rho, c, alp, tau, dt, ds, f, fv_, epsl, xa, t):
            tried[key].append(round(tau * 1.5, 12))
            out = primal(phi, rho, c, alp, tau, dt, ds, f, fv_, epsl, xa, t)
            return out * np.nan if tau * 1.5 > 0.055 else out
        return p2
    kw = dict(time_step_per_PDHG=2, stepsz_param=0.1, n_ctrl=1, fv=fv, N_maxiter=50, print_freq=10, eps=1e-6)
    res_o, _ = O.PDHG_multi_step(mk("o"), dual, fns, g, x, 1, nt, (nx,), 0.5, (2.0 / nx,), 70.0, **kw)
    res_p, _ = S.PDHG_multi_step(mk("p"), dual, fns, g, x, 1, nt, (nx,), 0.5, (2.0 / nx,), 70.0, verbose=False, **kw)
    assert sorted(set(tried["p"])) == sorted(set(tried["o"]))
    assert res_p[0][0] == res_o[0][0]
    assert np.allclose(res_p[0][1], res_o[0][1])


def test_update_fns_tagged_for_device_loop():
    fp, fd = S.make_update_fns(2, (0, 0), rho_alp_iters=10)
    assert fp._pdhg_native is fd._pdhg_native and fp._pdhg_native["rho_alp_iters"] == 10
    assert S._native_tag(fp, fd) is not None
    assert S._native_tag(fp, lambda *a: None) is None


def test_resume_from_middle_matches_straight_run(tmp_path, monkeypatch):
    """Resuming PDHG_multi_step from the middle results after 2 of 4 windows gives the straight run's result
    (the end row of the last finished window is saved for the next window's phi0)."""
    nx, nt = 12, 5
    x, fns, g, fv = _setup(nx, nt)
    primal, dual = O.make_update_fns(1, 0, rho_alp_iters=10)
    kw = dict(time_step_per_PDHG=2, stepsz_param=0.1, n_ctrl=1, fv=fv, N_maxiter=3000, print_freq=400, eps=1e-6,
              verbose=False)
    real_save = S.save

    def save_and_snapshot(d, prefix, results):
        real_save(d, prefix, results)
        if len(results[1]) == 2:
            real_save(d, "after2", results)
    monkeypatch.setattr(S, "save", save_and_snapshot)
    res_s, errs_s = S.PDHG_multi_step(primal, dual, fns, g, x, 1, nt, (nx,), 0.25, (2.0 / nx,), 70.0,
                                      save_middle_dir=str(tmp_path), save_middle_prefix="mid", **kw)
    res_r, errs_r = S.PDHG_multi_step(primal, dual, fns, g, x, 1, nt, (nx,), 0.25, (2.0 / nx,), 70.0,
                                      load_middle_dir=str(tmp_path), load_middle_prefix="after2", **kw)
    assert res_r[0][0] == res_s[0][0]
    for a, b in zip(res_r[0][1:], res_s[0][1:]):
        assert a.shape == b.shape and np.array_equal(a, b)
    assert len(errs_r) == len(errs_s)


def test_resume_from_reference_middle_list(tmp_path, monkeypatch):
    """The reference's own middle file is the 5-entry list [max_iters, phi_all, rho_all, alp_all, errs_all]
    (utils_pdhg_solver.py:211-212) with no end row; resuming from it (:139-147) solves the last saved window
    again from its known start state and then matches the uninterrupted run."""
    nx, nt = 12, 5
    x, fns, g, fv = _setup(nx, nt)
    primal, dual = O.make_update_fns(1, 0, rho_alp_iters=10)
    kw = dict(time_step_per_PDHG=2, stepsz_param=0.1, n_ctrl=1, fv=fv, N_maxiter=3000, print_freq=400, eps=1e-6,
              verbose=False)
    real_save = S.save

    def save_and_snapshot(d, prefix, results):
        real_save(d, prefix, results)
        if len(results[1]) == 2:
            real_save(d, "ref5", list(results[:5]))        # the reference's layout
    monkeypatch.setattr(S, "save", save_and_snapshot)
    res_s, errs_s = S.PDHG_multi_step(primal, dual, fns, g, x, 1, nt, (nx,), 0.25, (2.0 / nx,), 70.0,
                                      save_middle_dir=str(tmp_path), save_middle_prefix="mid", **kw)
    assert len(solver.load_middle_solution(str(tmp_path), "ref5")) == 5
    res_r, errs_r = S.PDHG_multi_step(primal, dual, fns, g, x, 1, nt, (nx,), 0.25, (2.0 / nx,), 70.0,
                                      load_middle_dir=str(tmp_path), load_middle_prefix="ref5", **kw)
    assert res_r[0][0] == res_s[0][0]
    for a, b in zip(res_r[0][1:], res_s[0][1:]):
        assert a.shape == b.shape and np.array_equal(a, b)
    assert len(errs_r) == len(errs_s)
    for a, b in zip(errs_r, errs_s):
        assert np.array_equal(a, b)


def test_resume_after_backoff_keeps_the_schedule(tmp_path, monkeypatch):
    """A run that backed off its step size before the middle file was written steps down on the SAME schedule
    after a resume: s_delta / s_min come from the caller's step size (utils_pdhg_solver.py:160-161), not from
    the reduced one the file restores.  Window 0 blows up above 0.095 (0.1 -> 0.09), window 2 above 0.075
    (0.09 -> 0.08 -> 0.07); resuming after window 1 with a schedule derived from 0.09 would try 0.081, 0.072."""
    nx, nt = 8, 5
    x, fns, g, fv = _setup(nx, nt)
    primal, dual = O.make_update_fns(1, 0, rho_alp_iters=1)
    tried = {"s": [], "r": []}

    def mk(key):
        def p2(phi, rho, c, alp, tau, dt, ds, f, fv_, epsl, xa, t):
            step = round(tau * 1.5, 12)
            w = int(round(float(np.asarray(t).ravel()[0]) / dt)) - 1       # window index (T = 1 rows)
            if not tried[key] or tried[key][-1] != (w, step):
                tried[key].append((w, step))
            out = primal(phi, rho, c, alp, tau, dt, ds, f, fv_, epsl, xa, t)
            thr = {0: 0.095, 2: 0.075}.get(w, 1.0)
            return out * np.nan if step > thr else out
        return p2
    kw = dict(time_step_per_PDHG=2, stepsz_param=0.1, n_ctrl=1, fv=fv, N_maxiter=40, print_freq=10, eps=1e-6,
              verbose=False)
    real_save = S.save

    def save_and_snapshot(d, prefix, results):
        real_save(d, prefix, results)
        if len(results[1]) == 2:
            real_save(d, "after2", results)
    monkeypatch.setattr(S, "save", save_and_snapshot)
    res_s, errs_s = S.PDHG_multi_step(mk("s"), dual, fns, g, x, 1, nt, (nx,), 0.25, (2.0 / nx,), 70.0,
                                      save_middle_dir=str(tmp_path), save_middle_prefix="mid", **kw)
    assert [s for w, s in tried["s"] if w == 2] == [0.09, 0.08, 0.07]
    res_r, errs_r = S.PDHG_multi_step(mk("r"), dual, fns, g, x, 1, nt, (nx,), 0.25, (2.0 / nx,), 70.0,
                                      load_middle_dir=str(tmp_path), load_middle_prefix="after2", **kw)
    assert [e for e in tried["r"] if e[0] >= 2] == [e for e in tried["s"] if e[0] >= 2]
    assert res_r[0][0] == res_s[0][0]
    for a, b in zip(res_r[0][1:], res_s[0][1:]):
        assert a.shape == b.shape and np.array_equal(a, b)


def test_resume_5_entry_list_after_backoff(tmp_path, monkeypatch):
    """The reference's 5-entry middle list holds no step size (utils_pdhg_solver.py:211-212).  Resuming from it after
    a NaN back-off (window 0: 0.1 -> 0.09) re-solves the last saved window (1) and continues at the CALLER's step
    size, 0.1, where the uninterrupted run had continued at 0.09: window 0 comes back from the file bit for bit,
    window 1 is re-solved at 0.1 (so its state is not the uninterrupted run's), window 2 backs off 0.1 -> 0.07."""
    nx, nt = 8, 5
    x, fns, g, fv = _setup(nx, nt)
    primal, dual = O.make_update_fns(1, 0, rho_alp_iters=1)
    tried = {"s": [], "r": []}

    def mk(key):
        def p2(phi, rho, c, alp, tau, dt, ds, f, fv_, epsl, xa, t):
            step = round(tau * 1.5, 12)
            w = int(round(float(np.asarray(t).ravel()[0]) / dt)) - 1
            if not tried[key] or tried[key][-1] != (w, step):
                tried[key].append((w, step))
            out = primal(phi, rho, c, alp, tau, dt, ds, f, fv_, epsl, xa, t)
            thr = {0: 0.095, 2: 0.075}.get(w, 1.0)
            return out * np.nan if step > thr else out
        return p2
    kw = dict(time_step_per_PDHG=2, stepsz_param=0.1, n_ctrl=1, fv=fv, N_maxiter=40, print_freq=10, eps=1e-6,
              verbose=False)
    real_save = S.save

    def save_and_snapshot(d, prefix, results):
        real_save(d, prefix, results)
        if len(results[1]) == 2:
            real_save(d, "ref5", list(results[:5]))
    monkeypatch.setattr(S, "save", save_and_snapshot)
    res_s, _ = S.PDHG_multi_step(mk("s"), dual, fns, g, x, 1, nt, (nx,), 0.25, (2.0 / nx,), 70.0,
                                 save_middle_dir=str(tmp_path), save_middle_prefix="mid", **kw)
    assert [s for w, s in tried["s"] if w == 1] == [0.09]
    res_r, _ = S.PDHG_multi_step(mk("r"), dual, fns, g, x, 1, nt, (nx,), 0.25, (2.0 / nx,), 70.0,
                                 load_middle_dir=str(tmp_path), load_middle_prefix="ref5", **kw)
    assert [s for w, s in tried["r"] if w == 1] == [0.1]
    assert [s for w, s in tried["r"] if w == 2] == [0.1, 0.09, 0.08, 0.07]
    assert not any(w == 0 for w, _ in tried["r"])                       # window 0 restored, not re-solved
    phi_s, phi_r = res_s[0][1], res_r[0][1]
    assert np.array_equal(phi_r[0], phi_s[0])                          # window 0's rows from the file
    assert not np.array_equal(res_r[0][2][1], res_s[0][2][1])          # window 1 re-solved at another step


def test_dropin_default_precision_is_fp64():
    """The drop-ins compute in float64 unless asked otherwise, as the reference (update_fns_in_pdhg.py:10)."""
    from pdhg_amd import update_fns_in_pdhg as U
    assert U.get_precision() == "fp64"
    fp, fd = S.make_update_fns(1, 0)
    assert fp._pdhg_native["precision"] is None   # resolved to the module default when the context is made


@pytest.mark.parametrize("ndim,bc", [(1, 0), (2, (0, 0)), (2, (1, 0))])
def test_dropin_refuses_a_foreign_fv(ndim, bc):
    """The drop-ins' preconditioner is the reference stencil's symbol (utils_precond.py:42-71): the oracle's fv
    (the reference's FFT of the stencil) is accepted, any other fv raises NotImplementedError before any device
    work instead of being silently replaced (update_fns_in_pdhg.py:139, 146 would use it)."""
    from pdhg_amd import update_fns_in_pdhg as U
    space, dsp = ((16,), (0.125,)) if ndim == 1 else ((8, 6), (0.25, 1 / 3))
    fv = O.compute_Dxx_fft_fv(ndim, space, dsp, bc)
    U.check_fv(fv, ndim, space, dsp, bc)
    U.check_fv(None, ndim, space, dsp, bc)
    with pytest.raises(NotImplementedError, match="symbol"):
        U.check_fv(fv * 1.01, ndim, space, dsp, bc)
    T = 2
    phi = np.zeros((T + 1,) + space)
    rho = np.full((T,) + space, 70.0)
    alp = tuple(np.zeros((T,) + space + (ndim,)) for _ in range(2 if ndim == 1 else 4))
    fns = set_fns.set_up_example_fns(1, ndim, 0)
    upd = U.update_primal_1d if ndim == 1 else U.update_primal_2d
    with pytest.raises(NotImplementedError, match="symbol"):
        upd(phi, rho, 70.0, alp, 0.1, 0.5, dsp, fns, fv + 3.0, 0.0, O.make_grid(ndim, *(space + (1,))[:2], 1), None,
            bc)
