"""The dual loop of rho_alp_iters > 1 in probe + final passes (kernels_dual_multi.hpp) against the per-sub-iteration
kernels and the float64 oracle (pytest -m gpu).

update_dual_alternative (update_fns_in_pdhg.py:167-180) runs <= rho_alp_iters sub-iterations of
update_dual_oneiter (:150-165) with phi_bar fixed and stops after the first whose err < eps.  The multi-pass form
runs the sub-iterations in registers (they are pointwise in rho, alpha), finds the exit sub-iteration from the err
sums of a probe pass, and stores the state once.  It keeps the per-sub-iteration kernels' arithmetic and their
grid (PDHG_DUAL_MULTI=0 selects those kernels); the compiler contracts a few products into FMAs differently once
the phi_bar terms are hoisted out of the sub-iteration loop, so the states agree to rounding (measured: 1 ulp in
~30 % of the alpha entries after one dual call), with the same inner counts.  The head form (the default below
2^25 points per window; PDHG_DUAL_HEAD) runs sub-iteration 0 through the per-sub-iteration kernel and the rest in
chunks, so a loop that exits after sub-iteration 0 is bitwise the per-sub-iteration one.
"""
import numpy as np
import pytest

import pdhg_oracle as O
from _problems import device_ctx, make_problem, rel

pytestmark = pytest.mark.gpu

TAU, SIGMA = 0.1 / 1.5, 0.1 * 1.5

CASES = [
    # egno, ndim, nx, ny, T, epsl   (ny % 256 == 0: the row-per-thread dual grid the multi-pass form runs on)
    (1, 2, 32, 256, 3, 0.0),
    (2, 2, 16, 512, 4, 1e-3),
    (3, 2, 24, 256, 2, 0.0),
    (2, 2, 64, 256, 1, 0.1),
    (2, 2, 512, 256, 8, 1e-3),   # time chunks of 2 rows (jchunk_d = 2 < T, gzd = 4) on a 512-row grid
]
IDS = ["e{}_{}x{}_T{}_eps{}".format(c[0], c[2], c[3], c[4], c[5]) for c in CASES]


def _ctx(P, prec, k, multi, monkeypatch, head=False):
    """multi: every sub-iteration in chunks; head: sub-iteration 0 per-sub-iteration, the rest in chunks; neither:
    the per-sub-iteration kernels throughout."""
    monkeypatch.setenv("PDHG_DUAL_MULTI", "1" if multi else "0")
    monkeypatch.setenv("PDHG_DUAL_HEAD", "1" if head else "0")
    ctx = device_ctx(P, prec, rho_alp_iters=k)
    assert ctx.path_info("dual_multi") == (1 if multi else 0)
    assert ctx.path_info("dual_head") == (1 if head else 0)
    return ctx


@pytest.mark.parametrize("case", CASES, ids=IDS)
@pytest.mark.parametrize("prec", ["fp32", "fp64"])
@pytest.mark.parametrize("k,eps", [(3, 1e-6), (10, 1e-6), (10, 1e-2), (7, -1.0)], ids=["k3", "k10", "k10_exit", "k7"])
@pytest.mark.parametrize("form", ["multi", "head"])
def test_multi_pass_matches_per_sub_iteration(native, monkeypatch, case, prec, k, eps, form):
    """4 outer iterations: the multi-pass dual loop (all chunks, or the head form) against the per-sub-iteration
    kernels -- the same outer and inner iteration counts, states and err1 / err2 to rounding (fp32 1e-5, fp64 1e-12
    relative)."""
    P = make_problem(*case)
    out = []
    for multi in (False, True):
        ctx = _ctx(P, prec, k, multi and form == "multi", monkeypatch, head=multi and form == "head")
        try:
            ctx.set_state(P["phi"], P["rho"], P["alp"])
            st = ctx.iterate(4, TAU, SIGMA, eps, k)
            out.append((ctx.get_state(), st))
        finally:
            ctx.close()
    (s0, st0), (s1, st1) = out
    assert st1["iters_run"] == st0["iters_run"] and st1["inner_total"] == st0["inner_total"], (st0, st1)
    tol = 1e-5 if prec == "fp32" else 1e-12
    for a, b in zip((s1[0], s1[1]) + tuple(s1[2]), (s0[0], s0[1]) + tuple(s0[2])):
        assert rel(a, b) < tol
    for key in ("err1", "err2"):
        assert abs(st1[key] - st0[key]) <= 1e3 * tol * abs(st0[key]) or (np.isnan(st1[key]) and np.isnan(st0[key])), \
            (key, st0[key], st1[key])


@pytest.mark.parametrize("form", ["multi", "head"])
@pytest.mark.parametrize("case", CASES[:3], ids=IDS[:3])
def test_multi_pass_vs_oracle(native, monkeypatch, case, form):
    """update_dual with rho_alp_iters = 10 and eps = 1e-3 / 1e-6 (the exit at different sub-iterations) against the
    float64 oracle's update_dual_alternative: the same sub-iteration count, states to 1e-10."""
    P = make_problem(*case)
    rng = np.random.default_rng(5)
    phi_bar = P["phi"] + 0.02 * rng.standard_normal(P["phi"].shape)
    for eps in (1e-3, 1e-6):
        stats = []
        rho_o, alp_o = O.update_dual_alternative(phi_bar, P["rho"], 70.0, P["alp"], SIGMA, P["dt"], P["dsp"],
                                                 P["epsl"], P["fns"], P["x_arr"], None, P["ndim"], P["bc"],
                                                 rho_alp_iters=10, eps=eps, stats=stats)
        ctx = _ctx(P, "fp64", 10, form == "multi", monkeypatch, head=form == "head")
        try:
            ctx.set_state(P["phi"], P["rho"], P["alp"])
            ctx.set_phi_bar(phi_bar)
            used = ctx.update_dual(SIGMA, eps, 10)
            _, rho_d, alp_d = ctx.get_state()
        finally:
            ctx.close()
        assert used == stats[0], (used, stats)
        assert rel(rho_d, rho_o) < 1e-10
        for a_d, a_o in zip(alp_d, alp_o):
            assert rel(a_d, a_o) < 1e-10


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
def test_fold_finalize_and_one_sub_iteration_outer_sums(native, monkeypatch, prec):
    """The head form's launch savings (a table long enough to fold): the fold and
    finalize in one launch (k_fold_finalize_dual) is bitwise the two-launch form; skipping the outer-sum pass after a
    one-sub-iteration loop (its sub-iteration-0 sums are the outer sums) keeps the iteration counts and err2 to
    summation-order rounding.  4096 x 256 (4096 partial rows: folded); eps = 0.5 makes loops exit after one
    sub-iteration."""
    P = make_problem(2, 2, 4096, 256, 1, 1e-3)
    out = {}
    for fold_fin, k1 in (("0", "0"), ("1", "0"), ("1", "1")):
        monkeypatch.setenv("PDHG_FOLD_FIN", fold_fin)
        monkeypatch.setenv("PDHG_K1_OUTER", k1)
        ctx = _ctx(P, prec, 10, False, monkeypatch, head=True)
        try:
            ctx.set_state(P["phi"], P["rho"], P["alp"])
            sts = [ctx.iterate(1, TAU, SIGMA, 0.5, 10) for _ in range(6)]
            out[fold_fin + k1] = (ctx.get_state(), sts)
        finally:
            ctx.close()
    (s0, st0), (s1, st1), (s2, st2) = out["00"], out["10"], out["11"]
    assert [s["inner_total"] for s in st0] == [s["inner_total"] for s in st1] == [s["inner_total"] for s in st2]
    assert any(s["inner_total"] == 1 for s in st0), [s["inner_total"] for s in st0]
    for a, b in zip((s1[0], s1[1]) + tuple(s1[2]), (s0[0], s0[1]) + tuple(s0[2])):
        assert np.array_equal(a, b)
    assert [s["err2"] for s in st1] == [s["err2"] for s in st0]
    tol = 1e-5 if prec == "fp32" else 1e-12
    for a, b in zip((s2[0], s2[1]) + tuple(s2[2]), (s0[0], s0[1]) + tuple(s0[2])):
        assert rel(a, b) < tol
    for x, y in zip(st2, st0):
        assert abs(x["err2"] - y["err2"]) <= 1e2 * tol * abs(y["err2"]), (x["err2"], y["err2"])
