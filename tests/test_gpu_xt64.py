"""The fp64 x transform + t-solve kernel (kernels_xt_f64.hpp) at every nx it runs -- 512, 1024 (one column pair per
block, b' in registers) and 2048 (C2's, BPR) -- against the generic runtime-radix kernel it replaced (PDHG_XT64=0: 2 / 4 / 8 columns per block, carries in global memory) and against the float64 oracle
(H1_precond_2d, jaxsrc/utils/utils_precond.py:142-178, through update_primal_2d).  Same float64 arithmetic up to
the transform's association: states within 1e-12 of each other, 1e-9 of the oracle.  (nx = 4096 has no generic
fp64 kernel to compare with -- 5 M reals of LDS -- and is pinned by the C3 fixtures of test_gpu_configs.py.)"""
import numpy as np
import pytest

from _problems import device_ctx, make_problem, oracle_fns, rel

pytestmark = pytest.mark.gpu

TAU, SIGMA = 0.1 / 1.5, 0.1 * 1.5


@pytest.mark.parametrize("egno,nx,ny,T", [(1, 512, 256, 12), (2, 1024, 256, 9), (2, 2048, 128, 7)],
                         ids=["e1_512", "e2_1024", "e2_2048"])
def test_fp64_x_kernel(native, monkeypatch, parity_log, egno, nx, ny, T):
    P = make_problem(egno, 2, nx, ny, T, 0.0, seeded=True)
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("PDHG_XT64", flag)
        ctx = device_ctx(P, "fp64")
        try:
            assert ctx.path_info("f64_xt") == int(flag), (flag, ctx.path_info("f64_xt"))
            ctx.set_state(P["phi"], P["rho"], P["alp"])
            ctx.update_primal(TAU)
            phi1 = ctx.get_state(rho=False, alp=False)[0]
            st = ctx.iterate(3, TAU, SIGMA, -1.0, 1)
            out[flag] = (phi1, ctx.get_state(), st)
        finally:
            ctx.close()
    primal, _ = oracle_fns(P)
    phi_o = primal(P["phi"], P["rho"], 70.0, P["alp"], TAU, P["dt"], P["dsp"], P["fns"], P["fv"], 0.0, P["x_arr"], None)
    (p1, s1, st1), (p0, s0, st0) = out["1"], out["0"]
    m = {"primal_vs_oracle": rel(p1, phi_o), "primal_vs_generic": rel(p1, p0), "phi": rel(s1[0], s0[0]),
         "rho": rel(s1[1], s0[1]), "err1": abs(st1["err1"] - st0["err1"]) / st0["err1"]}
    b = {"primal_vs_oracle": 1e-9, "primal_vs_generic": 1e-12, "phi": 1e-12, "rho": 1e-12, "err1": 1e-10}
    parity_log("test_fp64_x_kernel", "e{}_{}x{}_T{}".format(egno, nx, ny, T), m, b)
    assert all(m[k] <= b[k] for k in m), m


@pytest.mark.parametrize("fuse", ["1", pytest.param("0", marks=pytest.mark.extended)], ids=["fused", "unfused"])
def test_fp64_task_order_spectrum(native, monkeypatch, parity_log, fuse):
    """fp64 at C3's extents (4096^2): the residual spectrum handed to the x transform in task order (PDHG_TC_SPEC,
    one contiguous run per 4-row task; the x kernel's forward sweep reads 64-B groups) against the blocked layout --
    the same arithmetic on the same values, so the states agree to the last bit up to the compiler's contraction of
    the two x-kernel instantiations (bound 1e-13; measured values to parity_log)."""
    monkeypatch.setenv("PDHG_FUSE_RES", fuse)
    P = make_problem(2, 2, 4096, 4096, 6, 0.0, seeded=True)
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("PDHG_TC_SPEC", flag)
        ctx = device_ctx(P, "fp64")
        try:
            assert ctx.path_info("tc_spec") == int(flag) and ctx.path_info("fused_residual") == int(fuse)
            ctx.set_state(P["phi"], P["rho"], P["alp"])
            st = ctx.iterate(4, TAU, SIGMA, -1.0, 1)
            out[flag] = (ctx.get_state(), st)
        finally:
            ctx.close()
    (s1, st1), (s0, st0) = out["1"], out["0"]
    m = {"phi": rel(s1[0], s0[0]), "rho": rel(s1[1], s0[1]),
         "alp": max(rel(a, b) for a, b in zip(s1[2], s0[2])),
         "err1": abs(st1["err1"] - st0["err1"]) / st0["err1"],
         "bitwise": float(np.array_equal(s1[0], s0[0]) and np.array_equal(s1[1], s0[1]))}
    parity_log("test_fp64_task_order_spectrum", "c3_4096x4096_T6_fuse" + fuse, m, {k: 1e-13 for k in m if k != "bitwise"})
    assert all(m[k] <= 1e-13 for k in m if k != "bitwise"), m


def test_fp64_task_order_spectrum_primal_twice(native, monkeypatch, parity_log):
    """Drop-in pairing the loop never makes: two update_primal calls in a row after a fused dual sweep.  With the
    task-order spectrum stored over the R plane (tc_spec + fused residual) the first primal consumes R, so the
    second must re-form the residual from (rho, alp) instead of reading the spectrum as R; against the
    blocked layout, whose R survives the first call, on the same sequence (1e-12: fused vs unfused residual)."""
    monkeypatch.setenv("PDHG_FUSE_RES", "1")
    P = make_problem(2, 2, 4096, 4096, 4, 0.0, seeded=True)
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("PDHG_TC_SPEC", flag)
        ctx = device_ctx(P, "fp64")
        try:
            assert ctx.path_info("tc_spec") == int(flag) and ctx.path_info("fused_residual") == 1
            ctx.set_state(P["phi"], P["rho"], P["alp"])
            ctx.iterate(1, TAU, SIGMA, -1.0, 1)          # the dual sweep leaves R formed
            ctx.update_primal(TAU)
            p1 = ctx.get_state(rho=False, alp=False)[0]
            ctx.update_primal(TAU)
            out[flag] = (p1, ctx.get_state(rho=False, alp=False)[0])
        finally:
            ctx.close()
    m = {"first": rel(out["1"][0], out["0"][0]), "second": rel(out["1"][1], out["0"][1])}
    parity_log("test_fp64_task_order_spectrum_primal_twice", "c3_4096x4096_T4", m, {k: 1e-12 for k in m})
    assert all(v <= 1e-12 for v in m.values()), m
