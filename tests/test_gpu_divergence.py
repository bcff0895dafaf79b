"""C3's divergence on the FULL 4096^2 plane, against the fp64 oracle's fixture (tests/golden/divergence_c3_plane_T*.npz,
made by tests/golden/make_divergence_fixture.py).

The bench (C3: egno 2, epsl 0.1, 4096^2, dt = 1/200) reports the first iteration whose phi' or rho' is non-finite
(bench.py "first_nonfinite_iter").  That is the reference algorithm's own instability (the explicit
sigma*epsl*Lap(phi_bar) term of its dual step, update_fns_in_pdhg.py:58-70, amplifies ~5e5-fold per iteration at
dx = 2/4096), so the device must reproduce it where the fp64 oracle shows it: the same window (T rows of the
bench's dt on the whole plane) from the reference initial state, one outer iteration at a time, with the
reference's NaN stop (utils_pdhg_solver.py:78-80) on.  Checked per iteration: |rho'| (Frobenius) and err2 against
the oracle's, and the first non-finite iteration -- exactly in fp64 (the reference's arithmetic; the nx = 4096 x
transform k_precond_xt_f64_2d), within one iteration in fp32 (the bench's arithmetic, whose rounding the same
instability amplifies).  Achieved values go to parity_log."""
import ctypes
import glob
import os

import numpy as np
import pytest

from _problems import device_ctx, make_problem

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
TAU, SIGMA = 0.1 / 1.5, 0.1 * 1.5


def _fixture():
    paths = sorted(glob.glob(os.path.join(HERE, "golden", "divergence_c3_plane_T*.npz")))
    if not paths:
        pytest.fail("missing fixture (python tests/golden/make_divergence_fixture.py)")
    return np.load(paths[0])


def _rho_norm(ctx):
    from pdhg_amd import _native as N
    rho = np.empty((ctx.T,) + ctx._space)
    N.check(ctx._lib.pdhg_get_state(ctx._h, None, N.dptr(rho), None))
    return float(np.linalg.norm(rho[np.isfinite(rho)]))


@pytest.mark.parametrize("prec", ["fp64", "fp32"])
def test_c3_plane_divergence_matches_oracle(native, prec, parity_log):
    F = _fixture()
    rows, first_o = F["rows"], int(F["first_nonfinite"])
    egno, ndim, nx, ny, T = (int(v) for v in F["meta"])
    assert first_o > 0, "the fixture's oracle run did not diverge"
    G = make_problem(egno, ndim, nx, ny, 1, float(F["epsl"]), seeded=False)
    G.update(T=T, dt=float(F["dt"]))
    ctx = device_ctx(G, prec)
    try:
        if prec == "fp64":
            assert ctx.path_info("f64_xt") == 1
        ctx.init_state(G["g"][0])
        ctx.set_stop_rules(converge=True, nan=True)
        first_d, dev = 0, []
        for it in range(1, first_o + 3):
            st = ctx.iterate(1, TAU, SIGMA, -1.0, 1)
            if st["nan_seen"] or st["status"] == 2:
                first_d = it
                break
            dev.append((it, _rho_norm(ctx), st["err2"]))
    finally:
        ctx.close()
    # per finite iteration, relative distance of |rho'| and err2 from the oracle's
    e_rho = max(abs(r - rows[i - 1, 2]) / rows[i - 1, 2] for i, r, _ in dev)
    e_err2 = max(abs(e - rows[i - 1, 5]) / rows[i - 1, 5] for i, _, e in dev)
    tol = {"fp64": 1e-8, "fp32": 1e-2}[prec]
    parity_log("test_c3_plane_divergence_matches_oracle", prec,
               {"rho_norm": e_rho, "err2": e_err2, "first_nonfinite_delta": abs(first_d - first_o)},
               {"rho_norm": tol, "err2": tol, "first_nonfinite_delta": 0 if prec == "fp64" else 1},
               first_nonfinite_device=first_d, first_nonfinite_oracle=first_o)
    if prec == "fp64":
        assert first_d == first_o, (first_d, first_o)
    else:
        assert abs(first_d - first_o) <= 1, (first_d, first_o)
    assert e_rho <= tol and e_err2 <= tol, (e_rho, e_err2, dev)
