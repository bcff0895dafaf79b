"""HIP kernels vs the float64 oracle, through the C ABI (pytest -m gpu).

Tolerances (stated per SURVEY.md Appendix B.8):
  * fp64 device path: relative L2 <= 1e-10 on every state array after 1 and 10 iterations
    (same algorithm up to FFT/Hartley/closed-form-pivot roundoff); x10 for lines of >= 16384 points
    (C1's 65536: FFT roundoff grows with log n and the stencil's 1/dx^2 reaches 1e9);
  * fp32 device path from the reference's own initial state (phi = g, rho = c, alp = 0;
    utils_pdhg_solver.py:123-137): relative L2 of the primal update U = (phi' - phi)/tau <= 2e-6,
    of phi after 10 iterations <= 1e-5 (the north-star "phi within 1e-5 rel-L2"), rho <= 1e-5;
  * fp32 from the seeded rough state (uniform-noise rho, used to drive every mask/clip branch):
    the residual is dominated by eps*Lap(noise) ~ 1e4, so fp32 input rounding alone gives
    ~kappa*6e-8 ~ 1e-5 relative error in U; bounds there are 1e-4 (U, alp) and 2e-4 (rho).
"""
import os

import numpy as np
import pytest

import pdhg_oracle as O
from _problems import device_ctx, make_problem, oracle_fns, rel

HERE = os.path.dirname(os.path.abspath(__file__))

pytestmark = pytest.mark.gpu

TAU, SIGMA = 0.1 / 1.5, 0.1 * 1.5

CASES = [
    # egno, ndim, nx, ny, T, epsl
    (1, 1, 16, 1, 4, 0.0),
    (2, 1, 160, 1, 5, 0.0),
    (1, 1, 17, 1, 3, 0.1),      # odd nx
    (2, 1, 32, 1, 1, 0.0),      # T = 1 (the window-marching default)
    (1, 1, 256, 1, 8, 0.0),     # fixed-size FFT path in fp32
    (1, 2, 16, 12, 4, 0.0),
    (2, 2, 16, 16, 5, 0.1),
    (1, 2, 20, 18, 3, 0.1),     # non power-of-two (mixed radix 5 / 3)
    (2, 2, 15, 17, 2, 0.0),     # odd nx (zero-paired row) and odd ny (padded column block)
    (1, 2, 32, 32, 1, 0.0),     # T = 1
    (2, 2, 64, 48, 8, 0.1),
    (1, 2, 256, 256, 3, 0.0),   # fixed-size FFT paths (rows 256, x-slab 256 x 8 lines) in fp32
    (2, 2, 512, 256, 2, 0.0),   # fp32 fast row kernels (8-row groups, in-place 4-line FFT)
    (3, 2, 16, 12, 4, 0.0),     # egno 3: bc (1,0), DCT-II along x (utils_precond.py:159-174)
    (3, 2, 20, 18, 3, 0.1),     # egno 3, mixed radix, eps > 0
    (3, 2, 64, 48, 6, 0.0),
    (3, 2, 256, 128, 3, 0.0),   # egno 3 in fp32 through the generic x kernel
    (1, 1, 16384, 1, 5, 0.0),   # 1-D lines beyond LDS: Stockham passes over global scratch
    (2, 1, 65536, 1, 3, 0.0),   # C1's line length (BASELINE configs[1])
]
IDS = ["e{}d{}_{}x{}_T{}_eps{}".format(*c) for c in CASES]


def _big(P):
    """fp64 tolerance factor for long lines (see the module docstring)."""
    return 10.0 if max(P["nx"], P["ny"]) >= 16384 else 1.0


def _oracle_primal(P, phi, rho, alp):
    primal, _ = oracle_fns(P)
    return primal(phi, rho, 70.0, alp, TAU, P["dt"], P["dsp"], P["fns"], P["fv"], P["epsl"], P["x_arr"], None)


def _oracle_dual(P, phi_bar, rho, alp, k=1, eps=-1.0, stats=None):
    _, dual = oracle_fns(P, rho_alp_iters=k, stats=stats)
    return dual(phi_bar, rho, 70.0, alp, SIGMA, P["dt"], P["dsp"], P["epsl"], P["fns"], P["x_arr"], None, P["ndim"],
                eps)


@pytest.mark.parametrize("case", CASES, ids=IDS)
@pytest.mark.parametrize("prec", ["fp64", "fp32"])
def test_primal(native, case, prec):
    P = make_problem(*case)
    ctx = device_ctx(P, prec)
    ctx.set_state(P["phi"], P["rho"], P["alp"])
    ctx.update_primal(TAU)
    phi_d = ctx.get_state()[0]
    pbar_d = ctx.get_phi_bar()
    phi_o = _oracle_primal(P, P["phi"], P["rho"], P["alp"])
    U_o = (phi_o - P["phi"]) / TAU
    U_d = (phi_d - P["phi"]) / TAU
    if prec == "fp64":
        assert rel(U_d, U_o) < 1e-10 * _big(P)
        assert rel(pbar_d, 2 * phi_o - P["phi"]) < 1e-12 * _big(P)
    else:
        # U recovered from fp32 phi' carries phi's rounding / tau; phi' itself is the checked quantity
        assert rel(U_d, U_o) < 5e-4
        assert rel(phi_d, phi_o) < 1e-6
        assert rel(pbar_d, 2 * phi_o - P["phi"]) < 1e-5
    assert np.array_equal(phi_d[0], P["phi"][0].astype(np.float32 if prec == "fp32" else np.float64))
    ctx.close()


@pytest.mark.parametrize("case", CASES, ids=IDS)
@pytest.mark.parametrize("prec", ["fp64", "fp32"])
def test_dual_oneiter(native, case, prec):
    P = make_problem(*case)
    rng = np.random.default_rng(7)
    phi_bar = P["phi"] + 0.05 * rng.standard_normal(P["phi"].shape)
    ctx = device_ctx(P, prec)
    ctx.set_state(P["phi"], P["rho"], P["alp"])
    ctx.set_phi_bar(phi_bar)
    ctx.update_dual(SIGMA, -np.inf, 1)
    err_d = ctx.inner_error()
    _, rho_d, alp_d = ctx.get_state()
    rho_o, alp_o, err_o = O.update_dual_oneiter(phi_bar, P["rho"], 70.0, P["alp"], SIGMA, P["dt"], P["dsp"], P["epsl"],
                                                P["x_arr"], None, P["bc"], P["fns"], P["ndim"])
    tol = 1e-11 if prec == "fp64" else 1e-4
    assert rel(rho_d, rho_o) < tol
    for a_d, a_o in zip(alp_d, alp_o):
        assert rel(a_d, a_o) < tol
    if np.isnan(err_o):      # egno 3: 0/0 over the dead y-controls (update_fns_in_pdhg.py:162-164)
        assert np.isnan(err_d)
    else:
        assert abs(err_d - err_o) <= (1e-9 if prec == "fp64" else 1e-4) * abs(err_o)
    ctx.close()


@pytest.mark.parametrize("case", [c for c in CASES if c[4] > 1][:6], ids=[i for c, i in zip(CASES, IDS) if c[4] > 1][:6])
def test_dual_alternative_early_exit(native, case):
    """<= 10 sub-iterations with the err < eps early exit (update_fns_in_pdhg.py:167-180)."""
    P = make_problem(*case)
    phi_bar = P["phi"]
    for eps in (1e-3, 1e-6):
        stats = []
        rho_o, alp_o = _oracle_dual(P, phi_bar, P["rho"], P["alp"], k=10, eps=eps, stats=stats)
        ctx = device_ctx(P, "fp64", rho_alp_iters=10)
        ctx.set_state(P["phi"], P["rho"], P["alp"])
        ctx.set_phi_bar(phi_bar)
        used = ctx.update_dual(SIGMA, eps, 10)
        _, rho_d, alp_d = ctx.get_state()
        assert used == stats[0]
        assert rel(rho_d, rho_o) < 1e-10
        for a_d, a_o in zip(alp_d, alp_o):
            assert rel(a_d, a_o) < 1e-10
        ctx.close()


def _oracle_iterate(P, n, k=1):
    primal, dual = oracle_fns(P, rho_alp_iters=k)
    phi, rho, alp = P["phi"], P["rho"], P["alp"]
    for _ in range(n):
        phi_n = primal(phi, rho, 70.0, alp, TAU, P["dt"], P["dsp"], P["fns"], P["fv"], P["epsl"], P["x_arr"], None)
        rho_n, alp_n = dual(2 * phi_n - phi, rho, 70.0, alp, SIGMA, P["dt"], P["dsp"], P["epsl"], P["fns"],
                            P["x_arr"], None, P["ndim"], 1e-6 if k > 1 else -1.0)
        e1, e2 = O.outer_errors(phi, phi_n, rho, rho_n, alp, alp_n)
        phi, rho, alp = phi_n, rho_n, alp_n
    return phi, rho, alp, e1, e2


@pytest.mark.parametrize("case", CASES, ids=IDS)
@pytest.mark.parametrize("prec", ["fp64", "fp32"])
def test_iterate_10(native, case, prec):
    P = make_problem(*case)
    phi_o, rho_o, alp_o, e1_o, e2_o = _oracle_iterate(P, 10)
    ctx = device_ctx(P, prec)
    ctx.set_state(P["phi"], P["rho"], P["alp"])
    st = ctx.iterate(10, TAU, SIGMA, -1.0, 1)
    assert st["iters_run"] == 10 and st["status"] == 0
    phi_d, rho_d, alp_d = ctx.get_state()
    if prec == "fp64":
        assert rel(phi_d, phi_o) < 1e-11 * _big(P) and rel(rho_d, rho_o) < 1e-10 * _big(P)
        assert abs(st["err1"] - e1_o) <= 1e-8 * e1_o and abs(st["err2"] - e2_o) <= 1e-8 * e2_o
    else:
        assert rel(phi_d, phi_o) < 1e-5
        assert rel(rho_d, rho_o) < 2e-4
        assert abs(st["err1"] - e1_o) <= 1e-2 * e1_o
    ctx.close()


SMOOTH = [c for c in CASES if c[2] >= 32] + [(2, 1, 160, 1, 5, 0.1), (2, 2, 128, 128, 20, 0.1),
                                            (1, 1, 1024, 1, 40, 0.0), (1, 2, 1024, 512, 2, 0.0),
                                            (2, 2, 256, 1024, 3, 0.0)]
SMOOTH_IDS = ["e{}d{}_{}x{}_T{}_eps{}".format(*c) for c in SMOOTH]


@pytest.mark.parametrize("case", SMOOTH, ids=SMOOTH_IDS)
def test_fp32_from_reference_init(native, case):
    """fp32 vs the fp64 oracle from the reference's initial state: the north-star phi tolerance.

    With epsl > 0 the reference's dual step holds an explicit sigma*epsl*Lap(phi_bar) term; for
    sigma*epsl/dx^2 >> 1 its high-frequency modes are unstable, so fp32 rounding noise (1e-7) is
    amplified a few-fold per iteration while fp64 noise stays invisible (and the fp64 oracle itself
    diverges later, e.g. 256^2, epsl 0.1).  The multi-iteration fp32 bound is therefore checked over
    10 iterations for epsl = 0 and over 2 iterations for epsl > 0."""
    P = make_problem(*case, seeded=False)
    phi_o = _oracle_primal(P, P["phi"], P["rho"], P["alp"])
    ctx = device_ctx(P, "fp32")
    ctx.set_state(P["phi"], P["rho"], P["alp"])
    ctx.update_primal(TAU)
    phi_d = ctx.get_state()[0]
    assert rel(phi_d, phi_o) < 1e-6
    n = 10 if P["epsl"] == 0 else 2
    phi_o, rho_o, alp_o, e1_o, e2_o = _oracle_iterate(P, n)
    ctx.set_state(P["phi"], P["rho"], P["alp"])
    st = ctx.iterate(n, TAU, SIGMA, -1.0, 1)
    phi_d, rho_d, alp_d = ctx.get_state()
    assert rel(phi_d, phi_o) < 1e-5
    assert rel(rho_d, rho_o) < 1e-5
    assert abs(st["err1"] - e1_o) <= 1e-3 * e1_o
    ctx.close()


@pytest.mark.parametrize("case", [CASES[1], CASES[6], CASES[7]], ids=[IDS[1], IDS[6], IDS[7]])
def test_iterate_k10(native, case):
    """Reference default rho_alp_iters = 10 with early exit inside every outer iteration."""
    P = make_problem(*case)
    phi_o, rho_o, alp_o, e1_o, e2_o = _oracle_iterate(P, 4, k=10)
    ctx = device_ctx(P, "fp64", rho_alp_iters=10)
    ctx.set_state(P["phi"], P["rho"], P["alp"])
    st = ctx.iterate(4, TAU, SIGMA, 1e-6, 10)
    phi_d, rho_d, alp_d = ctx.get_state()
    assert st["iters_run"] == 4
    assert rel(phi_d, phi_o) < 1e-10 and rel(rho_d, rho_o) < 1e-9
    assert abs(st["err2"] - e2_o) <= 1e-7 * e2_o
    ctx.close()


def test_divergence_matches_oracle(native):
    """A rough state with eps*sigma/dx^2 >> 1 blows up; the device stops (status 2) at the oracle's NaN iteration."""
    P = make_problem(1, 2, 256, 256, 3, 0.1)
    primal, dual = oracle_fns(P)
    phi, rho, alp = P["phi"], P["rho"], P["alp"]
    nan_at = None
    with np.errstate(all="ignore"):
        for i in range(20):
            phi_n = primal(phi, rho, 70.0, alp, TAU, P["dt"], P["dsp"], P["fns"], P["fv"], P["epsl"], P["x_arr"], None)
            rho_n, alp_n = dual(2 * phi_n - phi, rho, 70.0, alp, SIGMA, P["dt"], P["dsp"], P["epsl"], P["fns"],
                                P["x_arr"], None, 2, -1.0)
            if np.isnan(phi_n).any() or np.isnan(rho_n).any():
                nan_at = i
                break
            phi, rho, alp = phi_n, rho_n, alp_n
    assert nan_at is not None
    ctx = device_ctx(P, "fp64")
    ctx.set_state(P["phi"], P["rho"], P["alp"])
    st = ctx.iterate(20, TAU, SIGMA, -1.0, 1)
    assert st["status"] == 2 and st["iters_run"] == nan_at + 1
    ctx.close()


def test_nan_stop(native):
    """A NaN in rho stops the loop at that iteration with status 2 (utils_pdhg_solver.py:78-80)."""
    P = make_problem(1, 2, 16, 16, 3, 0.0)
    rho = P["rho"].copy()
    rho[1, 3, 4] = np.nan
    ctx = device_ctx(P, "fp32")
    ctx.set_state(P["phi"], rho, P["alp"])
    st = ctx.iterate(50, TAU, SIGMA, 1e-6, 1)
    assert st["status"] == 2 and st["iters_run"] == 1
    ctx.close()


def test_solver_oneiter_converges_like_oracle(native):
    """PDHG_solver_oneiter device loop vs the oracle loop: same stop iteration and state (fp64)."""
    from pdhg_amd import set_fns, update_fns_in_pdhg as U, utils_pdhg_solver as S
    P = make_problem(1, 1, 32, 1, 1, 0.0, seeded=False)
    primal_o, dual_o = oracle_fns(P, rho_alp_iters=10)
    res_o, err_o = O.PDHG_solver_oneiter(primal_o, dual_o, P["fns"], P["phi"], P["rho"], P["alp"], P["x_arr"], None,
                                         1, P["dt"], P["dsp"], 70.0, stepsz_param=0.1, fv=P["fv"], N_maxiter=20000,
                                         print_freq=1000, eps=1e-6)
    fns = set_fns.set_up_example_fns(1, 1, 0)
    fp, fd = S.make_update_fns(1, 0, rho_alp_iters=10, precision="fp64")
    res_d, err_d = S.PDHG_solver_oneiter(fp, fd, fns, P["phi"], P["rho"], P["alp"], P["x_arr"], None, 1, P["dt"],
                                         P["dsp"], 70.0, stepsz_param=0.1, fv=P["fv"], N_maxiter=20000,
                                         print_freq=1000, eps=1e-6, verbose=False)
    assert len(res_d) == len(res_o)
    assert abs(res_d[-1][0] - res_o[-1][0]) <= 1
    assert rel(res_d[-1][1], res_o[-1][1]) < 1e-8
    assert np.allclose(err_d[:-1], err_o[:-1], rtol=1e-7)
    U.clear_cache()


def test_multi_step_window_marching(native):
    """PDHG_multi_step with the reference default time_step_per_PDHG = 2 (T = 1 windows), small C0."""
    from pdhg_amd import set_fns, update_fns_in_pdhg as U, utils_pdhg_solver as S
    nx, nt = 32, 6
    res_o, errs_o = O.solve_HJ(1, 1, 0.0, nx, 1, nt, N_maxiter=20000, print_freq=10000)
    fns = set_fns.set_up_example_fns(1, 1, 0)
    x_arr = O.make_grid(1, nx, 1, 1)
    g = set_fns.set_up_J(1, 1, (2.0,))(x_arr)
    fp, fd = S.make_update_fns(1, 0, rho_alp_iters=10, precision="fp64")
    res_d, errs_d = S.PDHG_multi_step(fp, fd, fns, g, x_arr, 1, nt, (nx,), 1.0 / (nt - 1), (2.0 / nx,), 70.0,
                                      time_step_per_PDHG=2, stepsz_param=0.1, n_ctrl=1, N_maxiter=20000,
                                      print_freq=10000, eps=1e-6, verbose=False)
    it_o, phi_o, rho_o, alp_o = res_o[0]
    it_d, phi_d, rho_d, alp_d = res_d[0]
    assert abs(it_d - it_o) <= 1
    assert phi_d.shape == phi_o.shape and alp_d.shape == alp_o.shape
    assert rel(phi_d, phi_o) < 1e-8 and rel(rho_d, rho_o) < 1e-6
    U.clear_cache()


def test_dropin_update_functions(native):
    """update_fns_in_pdhg drop-ins (reference signatures) in fp64 vs the oracle."""
    from pdhg_amd import set_fns, update_fns_in_pdhg as U
    prev = U.get_precision()
    U.set_precision("fp64")
    try:
        P = make_problem(2, 2, 16, 12, 3, 0.1)
        fns = set_fns.set_up_example_fns(2, 2, 0)
        phi_d = U.update_primal_2d(P["phi"], P["rho"], 70.0, P["alp"], TAU, P["dt"], P["dsp"], fns, P["fv"],
                                   P["epsl"], P["x_arr"], None, P["bc"])
        phi_o = _oracle_primal(P, P["phi"], P["rho"], P["alp"])
        assert rel((phi_d - P["phi"]) / TAU, (phi_o - P["phi"]) / TAU) < 1e-10
        pb = 2 * phi_o - P["phi"]
        r_d, a_d, e_d = U.update_dual_oneiter(pb, P["rho"], 70.0, P["alp"], SIGMA, P["dt"], P["dsp"], P["epsl"],
                                              P["x_arr"], None, P["bc"], fns, 2)
        r_o, a_o, e_o = O.update_dual_oneiter(pb, P["rho"], 70.0, P["alp"], SIGMA, P["dt"], P["dsp"], P["epsl"],
                                              P["x_arr"], None, P["bc"], P["fns"], 2)
        assert rel(r_d, r_o) < 1e-11 and abs(e_d - e_o) <= 1e-9 * e_o
        r_d, a_d = U.update_dual_alternative(pb, P["rho"], 70.0, P["alp"], SIGMA, P["dt"], P["dsp"], P["epsl"], fns,
                                             P["x_arr"], None, 2, P["bc"], rho_alp_iters=10, eps=1e-6)
        r_o, a_o = O.update_dual_alternative(pb, P["rho"], 70.0, P["alp"], SIGMA, P["dt"], P["dsp"], P["epsl"],
                                             P["fns"], P["x_arr"], None, 2, P["bc"], rho_alp_iters=10, eps=1e-6)
        assert rel(r_d, r_o) < 1e-10
    finally:
        U.set_precision(prev)
        U.clear_cache()


HALF_REAL = [(1, 2, 8192, 256, 3, 0.0), (2, 2, 8192, 256, 4, 0.0)]   # C4's nx: one real column per x block


# extended tier: C4's fp32 half-real x transform is pinned to the oracle by test_gpu_configs.py (the
# c4_halfreal_x8192 fixture and the one-step epsl = 0.1 case, both the DMA kernel the config runs)
@pytest.mark.extended
@pytest.mark.parametrize("case", HALF_REAL, ids=["e{}d{}_{}x{}_T{}_eps{}".format(*c) for c in HALF_REAL])
def test_half_real_x_transform_fp32(native, case):
    """nx = 8192 (BASELINE configs[4]) in fp32: the x-DHT of one real 8192-point column per block via a
    packed 4096-point FFT and the real split; same bounds as the other fp32 cases."""
    P = make_problem(*case)
    ctx = device_ctx(P, "fp32")
    ctx.set_state(P["phi"], P["rho"], P["alp"])
    ctx.update_primal(TAU)
    phi_o = _oracle_primal(P, P["phi"], P["rho"], P["alp"])
    assert rel(ctx.get_state()[0], phi_o) < 1e-6
    ctx.set_state(P["phi"], P["rho"], P["alp"])
    phi_o, rho_o, alp_o, e1_o, e2_o = _oracle_iterate(P, 5)
    st = ctx.iterate(5, TAU, SIGMA, -1.0, 1)
    phi_d, rho_d, _ = ctx.get_state()
    assert st["iters_run"] == 5
    assert rel(phi_d, phi_o) < 1e-5
    assert rel(rho_d, rho_o) < 2e-4
    ctx.close()


@pytest.mark.parametrize("prec", ["fp32"])
def test_glb_lines_1d_fp32(native, prec, monkeypatch):
    """C1's line length in fp32 through the one-workgroup-per-row-pair global-scratch lines (PDHG_FOURSTEP=0;
    the default fp32 path at nx = 65536 is the four-step DHT, covered by the CASES above) vs the oracle."""
    monkeypatch.setenv("PDHG_FOURSTEP", "0")
    P = make_problem(2, 1, 65536, 1, 3, 0.0)
    ctx = device_ctx(P, prec)
    ctx.set_state(P["phi"], P["rho"], P["alp"])
    ctx.update_primal(TAU)
    phi_o = _oracle_primal(P, P["phi"], P["rho"], P["alp"])
    assert rel(ctx.get_state()[0], phi_o) < 1e-6
    phi_o, rho_o, _, e1_o, _ = _oracle_iterate(P, 10)
    ctx.set_state(P["phi"], P["rho"], P["alp"])
    st = ctx.iterate(10, TAU, SIGMA, -1.0, 1)
    phi_d, rho_d, _ = ctx.get_state()
    assert rel(phi_d, phi_o) < 1e-5 and rel(rho_d, rho_o) < 2e-4
    assert abs(st["err1"] - e1_o) <= 1e-2 * e1_o
    ctx.close()


T1_FAST = [(1, 2, 4096, 256, 1, 0.0), (2, 2, 2048, 256, 1, 0.0), (2, 2, 1024, 512, 1, 0.0), (1, 2, 512, 256, 1, 0.0)]


@pytest.mark.parametrize("case", T1_FAST, ids=["e{}d{}_{}x{}_T{}_eps{}".format(*c) for c in T1_FAST])
def test_t1_x_transform_fp32(native, case):
    """One-row windows (the marching default) through the carry-free x transform k_precond_x_t1_2d vs the
    oracle: primal U and 10 iterations, fp32 bounds of test_fp32_from_reference_init."""
    P = make_problem(*case, seeded=False)
    phi_o = _oracle_primal(P, P["phi"], P["rho"], P["alp"])
    ctx = device_ctx(P, "fp32")
    assert ctx.path_info("fast_xt") == 1
    ctx.set_state(P["phi"], P["rho"], P["alp"])
    ctx.update_primal(TAU)
    assert rel(ctx.get_state()[0], phi_o) < 1e-6
    phi_o, rho_o, _, e1_o, _ = _oracle_iterate(P, 10)
    ctx.set_state(P["phi"], P["rho"], P["alp"])
    st = ctx.iterate(10, TAU, SIGMA, -1.0, 1)
    phi_d, rho_d, _ = ctx.get_state()
    assert rel(phi_d, phi_o) < 1e-5 and rel(rho_d, rho_o) < 1e-5
    assert abs(st["err1"] - e1_o) <= 1e-3 * e1_o
    ctx.close()


@pytest.mark.parametrize("case", T1_FAST, ids=["e{}d{}_{}x{}_T{}_eps{}".format(*c) for c in T1_FAST])
def test_t1_x_transform_fp64(native, monkeypatch, case):
    """The same one-row windows in the reference's precision: k_precond_x_t1_2d<..., double> vs the oracle (primal
    U <= 1e-12, 10 iterations <= 1e-10) and vs the generic runtime-radix x kernel (PDHG_T1_XT=0) to rounding; at nx =
    2048 / 4096 the default G16 form (later passes' twiddle seeds from global memory) bitwise against the all-LDS
    seed table (PDHG_T1_G16=0)."""
    P = make_problem(*case, seeded=False)
    phi_o = _oracle_primal(P, P["phi"], P["rho"], P["alp"])
    out = []
    g16 = case[2] in (2048, 4096)
    for t1, g in (("1", "1"), ("0", "1"), ("1", "0")):
        monkeypatch.setenv("PDHG_T1_XT", t1)
        monkeypatch.setenv("PDHG_T1_G16", g)
        ctx = device_ctx(P, "fp64")
        try:
            assert ctx.path_info("t1_xt64") == int(t1)
            assert ctx.path_info("t1_g16") == int(t1 == "1" and g == "1" and g16)
            ctx.set_state(P["phi"], P["rho"], P["alp"])
            ctx.update_primal(TAU)
            out.append(ctx.get_state()[0])
        finally:
            ctx.close()
    monkeypatch.setenv("PDHG_T1_G16", "1")
    assert rel(out[0], phi_o) < 1e-12 and rel(out[0], out[1]) < 1e-13
    assert np.array_equal(out[0], out[2])
    phi_o, rho_o, _, e1_o, _ = _oracle_iterate(P, 10)
    monkeypatch.setenv("PDHG_T1_XT", "1")
    ctx = device_ctx(P, "fp64")
    try:
        ctx.set_state(P["phi"], P["rho"], P["alp"])
        st = ctx.iterate(10, TAU, SIGMA, -1.0, 1)
        phi_d, rho_d, _ = ctx.get_state()
    finally:
        ctx.close()
    assert rel(phi_d, phi_o) < 1e-10 and rel(rho_d, rho_o) < 1e-10
    assert abs(st["err1"] - e1_o) <= 1e-8 * e1_o


PRECOND_1D = [   # (C, pow, Ct): utils_precond.py:125-134, run_example.py:436-438 flags
    (2.0, 1.0, 1.0), (1.0, 2.0, 1.0), (1.0, 1.0, 0.0), (1.0, 1.0, 2.0), (0.5, 2.0, 0.0), (3.0, 2.0, 2.0)]


@pytest.mark.parametrize("cpc", PRECOND_1D, ids=["C{}_pow{}_Ct{}".format(*c) for c in PRECOND_1D])
@pytest.mark.parametrize("prec", ["fp64", "fp32"])
@pytest.mark.parametrize("case", [(1, 1, 256, 1, 8, 0.0), (2, 1, 65536, 1, 6, 0.0)], ids=["e1_256_T8", "e2_65536_T6"])
def test_precond_1d_parameters(native, case, prec, cpc, parity_log):
    """H1_precond_1d with non-default C, pow and Ct (diagonal (C - fv)^pow + Ct * Lap_t, off-diagonals
    -Ct/dt^2; Ct = 0 decouples the time rows): the primal update and 3 iterations vs the oracle.  fp64
    <= 1e-10 (x10 at 65536 points, see _big); fp32 from the seeded state: phi' <= max(1e-6, 4 e32) and
    U <= max(5e-4, 4 e32), e32 = distance of the oracle run in float32 from the float64 one (with Ct = 0 at
    65536 points U = R/(C - lam)^pow recovers the low modes of a residual dominated by high ones: the
    float32 oracle itself is 1e-5 off in phi' there); the 3 iterations likewise against the float32
    oracle's distance from the float64 one."""
    C, pw, Ct = cpc
    P = make_problem(*case)
    primal, dual = oracle_fns(P, C=C, pow=pw, Ct=Ct)
    phi_o = primal(P["phi"], P["rho"], 70.0, P["alp"], TAU, P["dt"], P["dsp"], P["fns"], P["fv"], P["epsl"],
                   P["x_arr"], None)
    ctx = device_ctx(P, prec, C=C, pow=pw, Ct=Ct)
    try:
        ctx.set_state(P["phi"], P["rho"], P["alp"])
        ctx.update_primal(TAU)
        phi_d = ctx.get_state()[0]
        U_o, U_d = (phi_o - P["phi"]) / TAU, (phi_d - P["phi"]) / TAU
        if prec == "fp64":
            assert rel(U_d, U_o) < 1e-10 * _big(P)
        else:
            f = np.float32
            phi0 = P["phi"].astype(f)
            phi_32 = primal(phi0, P["rho"].astype(f), 70.0, tuple(a.astype(f) for a in P["alp"]), TAU, P["dt"],
                            P["dsp"], P["fns"], P["fv"], P["epsl"], P["x_arr"].astype(f), None)
            assert phi_32.dtype == f
            e32_phi, e32_U = rel(phi_32, phi_o), rel((phi_32 - phi0) / TAU, U_o)
            parity_log("test_precond_1d_parameters/first_update", "{}_{}_C{}_pow{}_Ct{}".format(case[2], case[4], *cpc),
                       {"phi1": rel(phi_d, phi_o), "U1": rel(U_d, U_o)},
                       {"phi1": max(1e-6, 4 * e32_phi), "U1": max(5e-4, 4 * e32_U)},
                       e32={"phi1": e32_phi, "U1": e32_U})
            assert rel(phi_d, phi_o) < max(1e-6, 4 * e32_phi), (rel(phi_d, phi_o), e32_phi)
            assert rel(U_d, U_o) < max(5e-4, 4 * e32_U), (rel(U_d, U_o), e32_U)
        phi, rho, alp = P["phi"], P["rho"], P["alp"]
        for _ in range(3):
            phi_n = primal(phi, rho, 70.0, alp, TAU, P["dt"], P["dsp"], P["fns"], P["fv"], P["epsl"], P["x_arr"], None)
            rho, alp = dual(2 * phi_n - phi, rho, 70.0, alp, SIGMA, P["dt"], P["dsp"], P["epsl"], P["fns"],
                            P["x_arr"], None, 1, -1.0)
            phi = phi_n
        ctx.set_state(P["phi"], P["rho"], P["alp"])
        st = ctx.iterate(3, TAU, SIGMA, -1.0, 1)
        assert st["iters_run"] == 3
        phi_d, rho_d, _ = ctx.get_state()
        if prec == "fp64":
            tol = 1e-10 * _big(P)
            assert rel(phi_d, phi) < tol and rel(rho_d, rho) < tol
        else:   # the same 3 iterations of the oracle in float32 calibrate the fp32 bound
            f = np.float32
            p32, r32, a32 = P["phi"].astype(f), P["rho"].astype(f), tuple(a.astype(f) for a in P["alp"])
            for _ in range(3):
                pn = primal(p32, r32, 70.0, a32, TAU, P["dt"], P["dsp"], P["fns"], P["fv"], P["epsl"],
                            P["x_arr"].astype(f), None)
                r32, a32 = dual(2 * pn - p32, r32, 70.0, a32, SIGMA, P["dt"], P["dsp"], P["epsl"], P["fns"],
                                P["x_arr"].astype(f), None, 1, -1.0)
                p32 = pn
            e_phi, e_rho = rel(p32, phi), rel(r32, rho)
            parity_log("test_precond_1d_parameters", "{}_{}_C{}_pow{}_Ct{}".format(case[2], case[4], *cpc),
                       {"phi": rel(phi_d, phi), "rho": rel(rho_d, rho)}, {"phi": max(1e-5, 8 * e_phi),
                                                                          "rho": max(2e-4, 8 * e_rho)},
                       e32={"phi": e_phi, "rho": e_rho})
            # x8: with Ct = 0 at 65536 points the device's 65536-point four-step DHT (twiddled fp32 passes)
            # rounds deeper than the oracle's float32 FFT and the decoupled low modes amplify it (measured 3.6-4.4x)
            assert rel(phi_d, phi) < max(1e-5, 8 * e_phi), (rel(phi_d, phi), e_phi)
            assert rel(rho_d, rho) < max(2e-4, 8 * e_rho), (rel(rho_d, rho), e_rho)
    finally:
        ctx.close()


@pytest.mark.parametrize("case", [(1, 1, 160, 1, 1, 0.0), (2, 2, 64, 48, 1, 0.1), (1, 2, 256, 256, 6, 0.0)],
                         ids=["c0_1d_T1", "e2_2d_T1", "e1_2d_fused_T6"])
def test_graph_replay_matches_eager(native, monkeypatch, case):
    """iterate() replays windows of 8 iterations from a captured HIP graph (PDHG_GRAPH, default on): the
    same kernels with the same arguments as the eager loop, so the state is bit-identical, and the device
    stop flags end a converging run at the same iteration even inside a replayed window (the converge test
    of utils_pdhg_solver.py:74-76 with eps = 1e-3: wherever it fires, both loops must stop there)."""
    egno, ndim, nx, ny, T, epsl = case
    P = make_problem(egno, ndim, nx, ny, T, epsl, seeded=False)
    out = []
    for g in ("0", "1"):
        monkeypatch.setenv("PDHG_GRAPH", g)
        ctx = device_ctx(P, "fp32")
        try:
            ctx.set_state(P["phi"], P["rho"], P["alp"])
            a = ctx.iterate(37, TAU, SIGMA, -1.0, 1)        # no stop: 37 = 4 windows + 5 eager
            b = ctx.iterate(400, TAU, SIGMA, 1e-3, 1)       # stops on convergence (or runs out)
            assert ctx.path_info("graph") == int(g)
            if g == "1":
                assert ctx.path_info("graph_window") == 8
            s_b = ctx.get_state()
            # window marching re-seeds the same context (PDHG_multi_step's warm start, a new phi row 0) and
            # iterates with unchanged (tau, sigma, eps, k): the replayed graph must use the new row 0 in err1
            phi2 = P["phi"] * 1.7 + 0.3
            ctx.set_state(phi2, P["rho"], P["alp"])
            c1 = ctx.iterate(1, TAU, SIGMA, -1.0, 1)
            c = ctx.iterate(16, TAU, SIGMA, -1.0, 1)
            out.append((a, b, s_b, c1, c, ctx.get_state()))
        finally:
            ctx.close()
    (a0, b0, s0, c10, c0, t0), (a1, b1, s1, c11, c1, t1) = out
    assert a0["iters_run"] == a1["iters_run"] == 37
    assert b0["iters_run"] == b1["iters_run"] and b0["status"] == b1["status"], (b0, b1)
    assert b0["err1"] == b1["err1"] and b0["err2"] == b1["err2"]
    assert np.array_equal(s0[0], s1[0]) and np.array_equal(s0[1], s1[1])
    assert c10["err1"] == c11["err1"] and c0["iters_run"] == c1["iters_run"] == 16
    assert c0["err1"] == c1["err1"] and c0["err2"] == c1["err2"], (c0, c1)
    assert np.array_equal(t0[0], t1[0]) and np.array_equal(t0[1], t1[1])


@pytest.mark.parametrize("case", [(2, 2, 4096, 16, 6, 0.0), (1, 2, 4096, 32, 3, 0.0), (2, 2, 4096, 8, 1, 0.0)],
                         ids=["e2_4096x16_T6", "e1_4096x32_T3", "e2_4096x8_T1"])
def test_fp64_nx4096_x_transform(native, case):
    """The reference's precision on C3's x extent: fp64 at nx = 4096 runs k_precond_xt_f64_2d (in-place LDS
    line, Thomas carries in registers; the generic fp64 kernel stops at nx = 2048), 10 iterations from the
    seeded rough state against the fp64 oracle at the fp64 bars of test_iterate_10."""
    P = make_problem(*case)
    phi_o, rho_o, alp_o, e1_o, e2_o = _oracle_iterate(P, 10)
    ctx = device_ctx(P, "fp64")
    try:
        assert ctx.path_info("f64_xt") == 1
        ctx.set_state(P["phi"], P["rho"], P["alp"])
        st = ctx.iterate(10, TAU, SIGMA, -1.0, 1)
        assert st["iters_run"] == 10 and st["status"] == 0
        phi_d, rho_d, alp_d = ctx.get_state()
    finally:
        ctx.close()
    assert rel(phi_d, phi_o) < 1e-11 and rel(rho_d, rho_o) < 1e-10, (rel(phi_d, phi_o), rel(rho_d, rho_o))
    assert abs(st["err1"] - e1_o) <= 1e-8 * e1_o and abs(st["err2"] - e2_o) <= 1e-8 * e2_o


def _march(monkeypatch, env, n=None, windows=None):
    """The marching fixture's run (tests/golden/marching_c2dt_64.json: C2's dt, T = 1 windows, k = 10, eps 1e-6) through
    the drop-in driver with `env`, on an n x n grid (default the fixture's 64^2) and the first `windows` windows;
    returns (per-window stop counts, final state, {spec, spec_iters, spec_halts} summed over the driver's contexts)."""
    import json
    from pdhg_amd import set_fns, utils_pdhg_solver as S
    from pdhg_amd import update_fns_in_pdhg as U
    for key, v in env.items():
        monkeypatch.setenv(key, v)
    U.clear_cache()
    F = json.load(open(os.path.join(HERE, "golden", "marching_c2dt_64.json")))
    nx = ny = n or F["nx"]
    ndim, egno = F["ndim"], F["egno"]
    fns = set_fns.set_up_example_fns(egno, ndim, 0)
    x_arr = O.make_grid(ndim, nx, ny, egno)
    g = set_fns.set_up_J(egno, ndim, (2.0, 2.0))(x_arr)
    dsp = (2.0 / nx, 2.0 / ny)
    fv = O.compute_Dxx_fft_fv(ndim, (nx, ny), dsp, (0, 0))
    fp, fd = S.make_update_fns(ndim, (0, 0), rho_alp_iters=F["rho_alp_iters"], precision="fp64")
    stats = []
    res, _ = S.PDHG_multi_step(fp, fd, fns, g, x_arr, ndim, (windows or F["windows"]) + 1, (nx, ny), F["dt"], dsp,
                               70.0, time_step_per_PDHG=2, epsl=F["epsl"], stepsz_param=F["stepsz"], fv=fv,
                               n_ctrl=ndim, N_maxiter=1000000, print_freq=1000000, eps=F["eps"], verbose=False,
                               stats=stats)
    spec = {key: sum(c.path_info(key) for c in U._CACHE.values())
            for key in ("spec", "spec_iters", "spec_halts", "dual_one")}
    U.clear_cache()
    return [int(st["window_iters"]) for st in stats], res[0], spec


def test_speculative_schedule_bitwise(native, monkeypatch, parity_log):
    """iterate()'s speculative one-sub-iteration schedule (the marching default's T = 1 windows; pdhg_api.hip
    iterate / finish_halted) against the full schedule (PDHG_SPEC=0) on the marching fixture: the same per-window stop
    counts, NaN back-offs and final state bit for bit -- it leaves out only launches that return at once, and an
    iteration whose loop does not exit after sub-iteration 0 halts and is finished by the host with the full
    schedule's launches.  The default policy must have speculated; PDHG_SPEC_FORCE=1 speculates from every window's
    first iteration and right after every halt, so the halt / finish path runs many times (asserted).  256^2 (the
    head form needs ny % 256 == 0), the fixture's dt / k / eps / step size, its first 3 windows."""
    it1, r1, sp1 = _march(monkeypatch, {"PDHG_SPEC": "1", "PDHG_SPEC_FORCE": "0"}, 256, 3)
    itf, rf, spf = _march(monkeypatch, {"PDHG_SPEC": "1", "PDHG_SPEC_FORCE": "1"}, 256, 3)
    it0, r0, sp0 = _march(monkeypatch, {"PDHG_SPEC": "0", "PDHG_SPEC_FORCE": "0"}, 256, 3)
    parity_log("test_speculative_schedule_bitwise", "marching_c2dt_256_w3",
               {"halts": sp1["spec_halts"], "spec_iters": sp1["spec_iters"], "forced_halts": spf["spec_halts"],
                "forced_spec_iters": spf["spec_iters"]}, {}, iters=it1)
    assert sp1["spec"] > 0 and sp1["spec_iters"] > 0 and sp0["spec_iters"] == 0, (sp1, sp0)
    assert spf["spec_halts"] > 0, spf
    assert it1 == it0 == itf
    assert r1[0] == r0[0] == rf[0]
    for a, b, c in zip(r1[1:], r0[1:], rf[1:]):
        assert np.array_equal(a, b) and np.array_equal(c, b)


def test_dual_one_row_bitwise(native, monkeypatch, parity_log):
    """The row-per-thread dual's one-row form (k_dual_fast_2d<.., ONE>: every workgroup one time row, as in the T = 1
    marching windows; loaded once, no prefetch registers) against its marching form (PDHG_DUAL_ONE=0) and the
    4-waves-per-SIMD build (=2) on the marching fixture at 256^2 (the row-per-thread dual needs ny % 256 == 0), its
    first 3 windows: the same stop counts, back-offs and final state bit for bit (same arithmetic per point)."""
    it1, r1, sp1 = _march(monkeypatch, {"PDHG_DUAL_ONE": "1"}, 256, 3)
    it2, r2, sp2 = _march(monkeypatch, {"PDHG_DUAL_ONE": "2"}, 256, 3)
    it0, r0, sp0 = _march(monkeypatch, {"PDHG_DUAL_ONE": "0"}, 256, 3)
    parity_log("test_dual_one_row_bitwise", "marching_c2dt_256_w3", {"dual_one": sp1["dual_one"]}, {}, iters=it1)
    assert sp1["dual_one"] > 0 and sp2["dual_one"] > 0 and sp0["dual_one"] == 0, (sp1, sp2, sp0)
    assert it1 == it0 == it2
    assert r1[0] == r0[0] == r2[0]
    for a, b, c in zip(r1[1:], r0[1:], r2[1:]):
        assert np.array_equal(a, b) and np.array_equal(c, b)


@pytest.mark.parametrize("head,k1", [("1", "1"), ("0", "1"), ("1", "0"), ("0", "0")],
                         ids=["default", "head0", "k1outer0", "head0_k1outer0"])
def test_marching_window_counts_fp64(native, monkeypatch, parity_log, head, k1):
    """The marching default's per-window stop iterations (PDHG_multi_step, utils_pdhg_solver.py:97-225; T = 1
    windows, rho_alp_iters = 10, eps 1e-6, NaN back-off) in the reference's arithmetic: the fp64 device driver
    against the float64 oracle's counts at C2's dt on 64^2 (tests/golden/marching_c2dt_64.json, window 1 backs
    off to stepsz 0.09).  Counts within one iteration, the same step size per window, the final state to 1e-8.
    With the dual loop's head form and the outer-sum skip after a one-sub-iteration loop on (the defaults) and off
    (PDHG_DUAL_HEAD=0: every sub-iteration per-sub-iteration; PDHG_K1_OUTER=0: always the outer-sum pass), the
    counts are logged per variant (parity_log) -- both shortcuts change sums by rounding only.
    (fp32 stops elsewhere: err1 < 1e-6 is within a few float32 ulps of relative change)"""
    import json
    from pdhg_amd import set_fns, utils_pdhg_solver as S
    from pdhg_amd import update_fns_in_pdhg as U
    monkeypatch.setenv("PDHG_DUAL_HEAD", head)
    monkeypatch.setenv("PDHG_K1_OUTER", k1)
    U.clear_cache()
    F = json.load(open(os.path.join(HERE, "golden", "marching_c2dt_64.json")))
    nx, ny, ndim, egno = F["nx"], F["ny"], F["ndim"], F["egno"]
    fns = set_fns.set_up_example_fns(egno, ndim, 0)
    x_arr = O.make_grid(ndim, nx, ny, egno)
    g = set_fns.set_up_J(egno, ndim, (2.0, 2.0))(x_arr)
    dsp = (2.0 / nx, 2.0 / ny)
    fv = O.compute_Dxx_fft_fv(ndim, (nx, ny), dsp, (0, 0))
    fp, fd = S.make_update_fns(ndim, (0, 0), rho_alp_iters=F["rho_alp_iters"], precision="fp64")
    stats = []
    res, _ = S.PDHG_multi_step(fp, fd, fns, g, x_arr, ndim, F["windows"] + 1, (nx, ny), F["dt"], dsp, 70.0,
                               time_step_per_PDHG=2, epsl=F["epsl"], stepsz_param=F["stepsz"], fv=fv, n_ctrl=ndim,
                               N_maxiter=1000000, print_freq=1000000, eps=F["eps"], verbose=False, stats=stats)
    iters, stepsz, s, nan_attempts = [], [], F["stepsz"], 0
    for st in stats:
        if st["status"] == 2:
            nan_attempts += 1
            continue
        iters.append(int(st["window_iters"]))
        stepsz.append(s - 0.01 * nan_attempts)
    assert len(iters) == F["windows"], stats
    parity_log("test_marching_window_counts_fp64", "head{}_k1outer{}".format(head, k1),
               {"max_count_diff": max(abs(a - b) for a, b in zip(iters, F["window_iters"]))}, {"max_count_diff": 1},
               iters=iters, oracle_iters=F["window_iters"])
    assert all(abs(a - b) <= 1 for a, b in zip(iters, F["window_iters"])), (iters, F["window_iters"])
    assert np.allclose(stepsz, F["window_stepsz"], rtol=0, atol=1e-12), (stepsz, F["window_stepsz"])
    _, phi, rho, _ = res[0]
    assert abs(np.linalg.norm(phi) - F["phi_norm"]) <= 1e-8 * F["phi_norm"]
    assert rel(phi.reshape(-1)[::997], np.array(F["phi_sample"])) < 1e-8
    assert rel(rho.reshape(-1)[::997], np.array(F["rho_sample"])) < 1e-6
    from pdhg_amd import update_fns_in_pdhg as U
    U.clear_cache()


@pytest.mark.parametrize("prec", ["fp64", "fp32"])
@pytest.mark.parametrize("egno,T,epsl", [(1, 100, 0.0), (2, 13, 1e-9), (1, 1, 0.0)], ids=["c1_T100", "e2_T13_eps", "T1"])
def test_fused_1d_residual(native, monkeypatch, parity_log, prec, egno, T, epsl):
    """C1's fused residual (k_dual_1d_fr forms the next residual rows in the dual sweep, k_f16a_fwd_fused_1d reads them
    with the wave-edge terms and the chunk-boundary time differences; nx = 65536, 8 time chunks) against the unfused
    stage A (PDHG_FUSE_RES1D=0), 5 iterations from the seeded state (fp64; fp32 10 from the reference initial
    state): the same arithmetic up to the order the chunk
    boundary rows add their time difference and the association of the residual's terms, whose 1/dx^2 ~ 1e9 scale
    cancels (fp64 1e-10, measured 3e-12 at C1; fp32 1e-5 relative), and against the float64 oracle (C1's fp64 bar)."""
    # fp32 from the seeded rough state at dx = 2/65536 leaves float32's range within a few iterations (both forms):
    # fp32 runs from the reference initial state.  epsl > 0 at this dx is the reference's unstable regime
    # (sigma*epsl/dx^2 >> 1, test_fp32_from_reference_init): the eps case takes epsl = 1e-9
    P = make_problem(egno, 1, 65536, 1, T, epsl, seeded=prec == "fp64")
    n = 5 if prec == "fp64" else 10
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("PDHG_FUSE_RES1D", flag)
        ctx = device_ctx(P, prec)
        try:
            assert ctx.path_info("fused_residual") == int(flag) and ctx.path_info("fs16") == 1
            ctx.set_state(P["phi"], P["rho"], P["alp"])
            st = ctx.iterate(n, TAU, SIGMA, -1.0, 1)
            out[flag] = (ctx.get_state(), st)
        finally:
            ctx.close()
    (s1, st1), (s0, st0) = out["1"], out["0"]
    assert all(np.isfinite(a).all() for a in (s1[0], s1[1], s0[0], s0[1])), \
        ("non-finite", [bool(np.isfinite(a).all()) for a in (s1[0], s1[1], s0[0], s0[1])])
    tol = 1e-10 if prec == "fp64" else 1e-5
    m = {"phi": rel(s1[0], s0[0]), "rho": rel(s1[1], s0[1]), "alp": rel(np.stack(s1[2]), np.stack(s0[2])),
         "err1": abs(st1["err1"] - st0["err1"]) / st0["err1"]}
    if prec == "fp64":
        phi_o, rho_o, _, _, _ = _oracle_iterate(P, n)
        m["phi_vs_oracle"] = rel(s1[0], phi_o)
        m["rho_vs_oracle"] = rel(s1[1], rho_o)
    b = {k: (1e-9 * _big(P) if k.endswith("oracle") else tol) for k in m}
    if prec == "fp32":   # the controls follow phi_bar's float32 one-sided differences at dx = 2/65536 (the float32
        b["alp"] = 2e-3  # oracle itself: 9.4e-4 from the float64 one): rounding-level changes
    parity_log("test_fused_1d_residual", "e{}_65536_T{}_eps{}@{}".format(egno, T, epsl, prec), m, b)
    assert all(m[k] <= b[k] for k in m), (m, b)
