"""fp64 residual and update through the fast row kernels (k_res_fwdy_fast_2d / k_invy_update_fast_2d <..., double>,
4-row groups) at the row lengths
that select it (ny = 2048, 4096; the reference's arithmetic at C2's / C3's ny): the primal update against the fp64
oracle (update_fns_in_pdhg.py:72-96, 135-147), the generic row-pair kernels (PDHG_RES64=0) on the same state, and
two full iterations.  Small nx keeps the oracle fast (column blocks of B = 16); one case at nx = 2048 has C3's
B = 2 blocked layout."""
import numpy as np
import pytest

from _problems import device_ctx, make_problem, oracle_fns, rel

pytestmark = pytest.mark.gpu

TAU, SIGMA = 0.1 / 1.5, 0.1 * 1.5
CASES = [
    # egno, ndim, nx, ny, T, epsl
    (1, 2, 8, 2048, 3, 0.0),
    (2, 2, 8, 4096, 3, 0.1),
    (2, 2, 12, 2048, 2, 0.0),
    (3, 2, 8, 2048, 2, 0.1),    # bc (1, 0): Neumann rows in x
    (2, 2, 2048, 2048, 2, 0.1),  # nx >= 2048: column blocks of B = 2 (C3's layout, the paired-read unpack)
]
IDS = ["e{}_{}x{}_T{}_eps{}".format(c[0], c[2], c[3], c[4], c[5]) for c in CASES]


def _primal(P):
    primal, _ = oracle_fns(P)
    return primal(P["phi"], P["rho"], 70.0, P["alp"], TAU, P["dt"], P["dsp"], P["fns"], P["fv"], P["epsl"],
                  P["x_arr"], None)


@pytest.mark.parametrize("case", CASES, ids=IDS)
def test_res64_primal_matches_oracle_and_generic(native, case, monkeypatch, parity_log):
    P = make_problem(*case)
    ctx = device_ctx(P, "fp64")
    try:
        assert ctx.path_info("res64") == 1
        ctx.set_state(P["phi"], P["rho"], P["alp"])
        ctx.update_primal(TAU)
        phi_d = ctx.get_state()[0]
        pbar_d = ctx.get_phi_bar()
    finally:
        ctx.close()
    monkeypatch.setenv("PDHG_RES64", "0")
    gen = device_ctx(P, "fp64")
    try:
        assert gen.path_info("res64") == 0
        gen.set_state(P["phi"], P["rho"], P["alp"])
        gen.update_primal(TAU)
        phi_g = gen.get_state()[0]
    finally:
        gen.close()
    phi_o = _primal(P)
    U_o, U_d, U_g = ((x - P["phi"]) / TAU for x in (phi_o, phi_d, phi_g))
    parity_log("test_res64_primal", "_".join(map(str, case)), {"U_vs_oracle": rel(U_d, U_o), "U_vs_generic": rel(U_d, U_g)},
               {"U_vs_oracle": 1e-10, "U_vs_generic": 1e-12})
    assert rel(U_d, U_o) < 1e-10
    assert rel(U_d, U_g) < 1e-12
    assert rel(pbar_d, 2 * phi_o - P["phi"]) < 1e-12


@pytest.mark.parametrize("case", CASES[:2], ids=IDS[:2])
def test_res64_iterations_match_oracle(native, case):
    P = make_problem(*case)
    primal, dual = oracle_fns(P)
    phi, rho, alp = P["phi"], P["rho"], P["alp"]
    for _ in range(2):
        phi_n = primal(phi, rho, 70.0, alp, TAU, P["dt"], P["dsp"], P["fns"], P["fv"], P["epsl"], P["x_arr"], None)
        rho, alp = dual(2 * phi_n - phi, rho, 70.0, alp, SIGMA, P["dt"], P["dsp"], P["epsl"], P["fns"], P["x_arr"],
                        None, 2, -1.0)
        phi = phi_n
    ctx = device_ctx(P, "fp64")
    try:
        ctx.set_state(P["phi"], P["rho"], P["alp"])
        ctx.set_stop_rules(converge=False, nan=False)
        st = ctx.iterate(2, TAU, SIGMA, -1.0, 1)
        assert st["iters_run"] == 2
        phi_d, rho_d, alp_d = ctx.get_state()
    finally:
        ctx.close()
    assert rel(phi_d, phi) < 1e-10
    assert rel(rho_d, rho) < 1e-10


DUAL_CASES = [
    # egno, ndim, nx, ny, T, epsl
    (1, 2, 6, 256, 3, 0.0),
    (2, 2, 5, 512, 3, 0.1),
    (3, 2, 4, 256, 2, 0.1),
    # nx % 8 == 0: with rho_alp_iters = 1 the x rows go through LDS (k_dual_lds_2d<EGNO, 8, false, double>)
    (1, 2, 16, 256, 3, 0.0),
    (2, 2, 24, 512, 4, 0.1),
    (3, 2, 16, 256, 2, 0.1),
]


@pytest.mark.parametrize("k", [1, 3])
@pytest.mark.parametrize("case", DUAL_CASES, ids=["e{}_{}x{}_T{}_eps{}".format(c[0], c[2], c[3], c[4], c[5])
                                                  for c in DUAL_CASES])
def test_dual64_matches_oracle(native, case, k, monkeypatch):
    """fp64 dual through the time-marching kernels (ny % 256 == 0): x rows through LDS (k_dual_lds_2d<EGNO, 8, false,
    double>, k = 1 and nx % 8 == 0) or row-per-thread (k_dual_fast_2d<EGNO, double>), against the fp64 oracle
    (update_fns_in_pdhg.py:150-180) and the generic per-point kernel (PDHG_DUAL64=0)."""
    P = make_problem(*case)
    rng = np.random.default_rng(11)
    phi_bar = P["phi"] + 0.05 * rng.standard_normal(P["phi"].shape)
    _, dual = oracle_fns(P, rho_alp_iters=k)
    rho_o, alp_o = dual(phi_bar, P["rho"], 70.0, P["alp"], SIGMA, P["dt"], P["dsp"], P["epsl"], P["fns"], P["x_arr"],
                        None, 2, -1.0)
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("PDHG_DUAL64", flag)
        ctx = device_ctx(P, "fp64", rho_alp_iters=k)
        try:
            assert ctx.path_info("dual64") == int(flag)
            if flag == "1":   # LDS x rows (8 per workgroup) for k = 1 and nx % 8 == 0, else row-per-thread
                # (windows shorter than 3 rows keep the row-per-thread kernel: short_t_dual in pdhg_api.hip)
                lds = k == 1 and case[2] % 8 == 0 and case[4] >= 3
                assert ctx.path_info("fast_dual") == (8 if lds else 0)
            ctx.set_state(P["phi"], P["rho"], P["alp"])
            ctx.set_phi_bar(phi_bar)
            ctx.update_dual(SIGMA, -1.0, k)
            _, rho_d, alp_d = ctx.get_state()
        finally:
            ctx.close()
        out[flag] = (rho_d, alp_d)
    rho_d, alp_d = out["1"]
    assert rel(rho_d, rho_o) < 1e-10
    for a_d, a_o in zip(alp_d, alp_o):
        if np.linalg.norm(a_o) > 0:
            assert rel(a_d, a_o) < 1e-10
    assert rel(rho_d, out["0"][0]) < 1e-12


@pytest.mark.parametrize("case", [c for c in CASES if c[3] == 2048], ids=[i for c, i in zip(CASES, IDS) if c[3] == 2048])
def test_res64_threads(native, case, monkeypatch, parity_log):
    """ny = 2048: the residual's 256-thread workgroups (two per CU, each thread two y groups; the default on one-row
    windows) against the 512-thread form (PDHG_RES64_NT2048): the same per-point expressions and transform, compiled
    for a different thread mapping; phi' agrees to rounding (measured: not bit for bit; the difference is logged)."""
    P = make_problem(*case)
    out = []
    for nt in ("256", "512"):
        monkeypatch.setenv("PDHG_RES64_NT2048", nt)
        ctx = device_ctx(P, "fp64")
        try:
            assert ctx.path_info("res64_nt") == int(nt)
            ctx.set_state(P["phi"], P["rho"], P["alp"])
            ctx.update_primal(TAU)
            out.append(ctx.get_state()[0])
        finally:
            ctx.close()
    parity_log("test_res64_threads", "_".join(map(str, case)), {"phi_256_vs_512": rel(out[0], out[1])},
               {"phi_256_vs_512": 1e-13})
    assert rel(out[0], out[1]) < 1e-13


T1_CASES = [(1, 2, 8, 2048, 1, 0.0), (2, 2, 2048, 2048, 1, 0.1)]


@pytest.mark.parametrize("case", T1_CASES, ids=["e{}_{}x{}_T1_eps{}".format(c[0], c[2], c[3], c[5]) for c in T1_CASES])
def test_update_t1_shapes(native, case, monkeypatch, parity_log):
    """One-row windows at ny = 2048: the update's 256-thread workgroups with the G16 seed table (two per CU; prefetch
    depth 2 = default, 4) against the 512-thread form (PDHG_UPD_T1=0) -- phi' and phi_bar to rounding (the difference
    is logged) -- and the primal against the fp64 oracle."""
    P = make_problem(*case)
    out = []
    for v in ("1", "2", "0"):
        monkeypatch.setenv("PDHG_UPD_T1", v)
        ctx = device_ctx(P, "fp64")
        try:
            assert ctx.path_info("upd_t1") == int(v)
            ctx.set_state(P["phi"], P["rho"], P["alp"])
            ctx.update_primal(TAU)
            out.append((ctx.get_state()[0], ctx.get_phi_bar()))
        finally:
            ctx.close()
    phi_o = _primal(P)
    d = {"v1_vs_512": rel(out[0][0], out[2][0]), "v2_vs_512": rel(out[1][0], out[2][0]),
         "U_vs_oracle": rel((out[0][0] - P["phi"]) / TAU, (phi_o - P["phi"]) / TAU)}
    parity_log("test_update_t1_shapes", "_".join(map(str, case)), d,
               {"v1_vs_512": 1e-13, "v2_vs_512": 1e-13, "U_vs_oracle": 1e-10})
    assert d["v1_vs_512"] < 1e-13 and d["v2_vs_512"] < 1e-13 and d["U_vs_oracle"] < 1e-10
    assert rel(out[0][1], out[2][1]) < 1e-13
