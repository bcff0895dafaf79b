"""C3's divergence on the FULL 4096^2 plane, against the oracle's fixtures (tests/golden/divergence_c3_plane_T4.npz
in float64, divergence_c3_plane_T4_f32.npz in float32; made by tests/golden/make_divergence_fixture.py).

The bench (C3: egno 2, epsl 0.1, 4096^2, dt = 1/200) reports the first iteration whose phi' or rho' is non-finite
(bench.py "first_nonfinite_iter").  That is the reference algorithm's own instability (the explicit
sigma*epsl*Lap(phi_bar) term of its dual step, update_fns_in_pdhg.py:58-70), not a device defect: on the same
window (T rows of the bench's dt on the whole plane, from the reference initial state) the oracle's |rho'| grows
geometrically (x ~3000 per iteration once the unstable modes dominate), in either precision.  The device must
follow the oracle of its own arithmetic:
  * fp64 (the reference's arithmetic; k_precond_xt_f64_2d at nx = 4096): |rho'|, |phi'| and err2 per iteration
    within FP64_TOL of the float64 oracle over every fixture iteration, and no NaN within them;
  * fp32 (the bench's arithmetic): fp32 rounding (1e-7 relative) seeds the unstable modes, so the float32
    trajectory leaves the float64 one after ~2 iterations (|rho'| 1e9 at iteration 3 against 6e5) -- the device
    must match the float32 oracle (same norms within FP32_TOL per iteration while finite: once the unstable
    modes dominate, a relative difference stays put while both grow) and turn non-finite (phi' or rho' NaN, the
    reference's test, utils_pdhg_solver.py:78-80) within one iteration of it.  That is where the bench's
    first_nonfinite_iter comes from.  Achieved values go to parity_log.
Pointwise (test_c3_plane_pointwise_fp64): the fp64 device's phi' and rho' at 4096 fixed sample points of the plane
after each of the first 10 iterations against the float64 oracle's values there (divergence_c3_plane_T4_points.npz),
relative L2 over the sample <= 1e-5 (the north-star bound, fixed) through iteration 6 of the geometric growth and
<= 1e-4 after it (PTS_TOL_LATE: the spread of an equally exact float64 reformulation, see below)."""
import glob
import os

import numpy as np
import pytest

from _problems import device_ctx, make_problem

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
TAU, SIGMA = 0.1 / 1.5, 0.1 * 1.5
F32_MAX = float(np.finfo(np.float32).max)
FP64_TOL = 1e-6      # relative, per iteration
FP32_TOL = 1e-5      # relative, per finite iteration, against the float32 oracle (measured 7.3e-7, round 3)
# relative L2 over the sample points, per iteration (fp64 device vs float64 oracle): the north-star 1e-5 through
# iteration PTS_TIGHT; after it 1e-4.  The reference's explicit sigma*epsl*Lap(phi_bar) term amplifies any
# difference of one rounding by ~2e3-5e3 per iteration until the unstable modes dominate both runs (measured: 9e-17,
# 2e-13, 1e-9, 8e-7 at iterations 2-5).  The float64 oracle started from phi_0 perturbed by +-1 ulp per entry drifts
# from itself further still (phi 4e-13, 2e-9, 1e-5, 8e-3 and rho 5e-9, 2e-5, 7e-3, 4e-2 at iterations 2-5; 0.16 / 0.42
# at 10: tests/golden/divergence_c3_plane_T4_points_ulp.npz).  Like-for-like yardsticks (round
# 5, the same points): the oracle on numpy.fft instead of scipy.fft spreads only 5e-7 / 2e-6 (phi / rho) at iteration
# 10 -- both are pocketfft, nearly the same rounding -- while the oracle with ONE step reformulated the way the device
# does it, exactly in exact arithmetic (its Thomas solve in the device's pivot algebra: _points_devthomas.npz),
# spreads phi 1.3e-5, 5.1e-5, 3.4e-4, 2.5e-4 and rho 5.6e-6 ... 2.4e-5 at iterations 7-10 (<= 1.6e-6 through 6).
# The device reformulates the t-solve AND the transforms (Hartley) and measures phi 0.8-3.1e-5, rho 1.1-5.2e-5 at 7-10
# (round 5, every kernel variant).  So 1e-5 holds through iteration 6 for every formulation, and the late bound is no
# looser than what one exact reformulation of one step moves: test_pointwise_bounds_vs_reformulation_spread (CPU)
# pins both bounds against the committed yardstick fixtures.
PTS_TOL, PTS_TIGHT, PTS_TOL_LATE = 1e-5, 6, 1e-4
# err2 (utils_pdhg_solver.py:60-68) of the fp32 run: a sum of ratios ||d alp|| / ||alp|| whose numerators are
# differences of float32 states in the growth phase (measured 2.5e-4, round 3); the norms themselves keep FP32_TOL
FP32_ERR2_TOL = 1e-3


def _fixture(prec):
    suffix = "_f32" if prec == "fp32" else ""
    paths = sorted(glob.glob(os.path.join(HERE, "golden", "divergence_c3_plane_T*{}.npz".format(suffix))))
    paths = [q for q in paths if q.endswith(suffix + ".npz") and (suffix or not (q.endswith("_f32.npz") or "_points" in q))]
    if not paths:
        pytest.fail("missing fixture (python tests/golden/make_divergence_fixture.py 4 24 {})".format(
            "f32" if suffix else ""))
    return np.load(paths[0])


def _norms(ctx):
    from pdhg_amd import _native as N
    phi = np.empty((ctx.T + 1,) + ctx._space)
    rho = np.empty((ctx.T,) + ctx._space)
    N.check(ctx._lib.pdhg_get_state(ctx._h, N.dptr(phi), N.dptr(rho), None))
    fp, fr = np.isfinite(phi), np.isfinite(rho)
    return (float(np.linalg.norm(phi[fp])), float(np.linalg.norm(rho[fr])),
            float(np.max(np.abs(np.where(fr, rho, 0.0)))), bool(fp.all() and fr.all()))


@pytest.mark.parametrize("prec", ["fp64", "fp32"])
def test_c3_plane_divergence_matches_oracle(native, prec, parity_log):
    F = _fixture(prec)
    rows = F["rows"]             # iter, |phi|, |rho|, |alp|, err1, err2, finite, max|phi|, max|rho|
    egno, ndim, nx, ny, T = (int(v) for v in F["meta"])
    n = rows.shape[0]
    first_o = int(F["first_nonfinite"])     # the oracle's first NaN iteration (0: none within the fixture)
    G = make_problem(egno, ndim, nx, ny, 1, float(F["epsl"]), seeded=False)
    G.update(T=T, dt=float(F["dt"]))
    ctx = device_ctx(G, prec)
    dev, first_d = [], 0
    try:
        if prec == "fp64":
            assert ctx.path_info("f64_xt") == 1
        ctx.init_state(G["g"][0])
        ctx.set_stop_rules(converge=True, nan=True)
        last = n if not first_o else first_o + 1
        for it in range(1, last + 1):
            st = ctx.iterate(1, TAU, SIGMA, -1.0, 1)
            if st["nan_seen"] or st["status"] == 2:
                first_d = it
                break
            nphi, nrho, mrho, fin = _norms(ctx)
            dev.append((it, nphi, nrho, st["err2"], fin))
    finally:
        ctx.close()
    checked = [d for d in dev if d[4] and d[0] <= n and rows[d[0] - 1, 6] > 0]
    e = {"phi_norm": max(abs(p - rows[i - 1, 1]) / rows[i - 1, 1] for i, p, _, _, _ in checked),
         "rho_norm": max(abs(r - rows[i - 1, 2]) / rows[i - 1, 2] for i, _, r, _, _ in checked),
         # err2 where the oracle's own float32 sums stayed finite (the device sums in fp64)
         "err2": max(abs(e2 - rows[i - 1, 5]) / rows[i - 1, 5] for i, _, _, e2, _ in checked
                     if np.isfinite(rows[i - 1, 5]))}
    tol = {k: FP64_TOL if prec == "fp64" else FP32_TOL for k in e}
    if prec == "fp32":
        tol["err2"] = FP32_ERR2_TOL
    parity_log("test_c3_plane_divergence_matches_oracle", prec, e, tol,
               iterations_checked=len(checked), first_nonfinite_device=first_d, first_nonfinite_oracle=first_o,
               rho_norm_device=[d[2] for d in dev], rho_norm_oracle=[float(v) for v in rows[:, 2]])
    assert len(checked) >= min(n, 5), (len(checked), dev)
    assert all(v <= tol[k] for k, v in e.items()), (e, tol, dev)
    if first_o:
        assert abs(first_d - first_o) <= 1, (first_d, first_o)
    else:
        assert first_d == 0 or first_d > n, (first_d, n)   # no NaN within the fixture's iterations


def test_c3_plane_pointwise_fp64(native, parity_log):
    """phi' and rho' themselves (not only their norms) on C3's full plane through 10 iterations of the divergence:
    the fp64 device against the float64 oracle at the fixture's sample points, relative L2 <= PTS_TOL per
    iteration (update_fns_in_pdhg.py:83-96, 115-119 feed every point's value)."""
    path = os.path.join(HERE, "golden", "divergence_c3_plane_T4_points.npz")
    if not os.path.exists(path):
        pytest.fail("missing fixture (python tests/golden/make_divergence_fixture.py 4 10 points)")
    F = np.load(path)
    egno, ndim, nx, ny, T = (int(v) for v in F["meta"])
    phi_idx, rho_idx = tuple(F["phi_idx"]), tuple(F["rho_idx"])
    phi_o, rho_o = F["phi_pts"], F["rho_pts"]
    n = phi_o.shape[0]
    G = make_problem(egno, ndim, nx, ny, 1, float(F["epsl"]), seeded=False)
    G.update(T=T, dt=float(F["dt"]))
    ctx = device_ctx(G, "fp64")
    from pdhg_amd import _native as N
    e_phi, e_rho = [], []
    try:
        ctx.init_state(G["g"][0])
        ctx.set_stop_rules(converge=False, nan=False)
        phi = np.empty((T + 1, nx, ny))
        rho = np.empty((T, nx, ny))
        for it in range(n):
            ctx.iterate(1, TAU, SIGMA, -1.0, 1)
            N.check(ctx._lib.pdhg_get_state(ctx._h, N.dptr(phi), N.dptr(rho), None))
            e_phi.append(float(np.linalg.norm(phi[phi_idx] - phi_o[it]) / np.linalg.norm(phi_o[it])))
            e_rho.append(float(np.linalg.norm(rho[rho_idx] - rho_o[it]) / np.linalg.norm(rho_o[it])))
    finally:
        ctx.close()
    tight = {"phi": max(e_phi[:PTS_TIGHT]), "rho": max(e_rho[:PTS_TIGHT])}
    late = {"phi_late": max(e_phi[PTS_TIGHT:] or [0.0]), "rho_late": max(e_rho[PTS_TIGHT:] or [0.0])}
    parity_log("test_c3_plane_pointwise_fp64", "T{}_{}it".format(T, n), dict(tight, **late),
               {"phi": PTS_TOL, "rho": PTS_TOL, "phi_late": PTS_TOL_LATE, "rho_late": PTS_TOL_LATE},
               phi_per_iter=e_phi, rho_per_iter=e_rho, rho_norm_oracle_pts=[float(np.linalg.norm(r)) for r in rho_o])
    assert all(v <= PTS_TOL for v in tight.values()) and all(v <= PTS_TOL_LATE for v in late.values()), (e_phi, e_rho)
