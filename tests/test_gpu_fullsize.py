"""The bench windows at their FULL size (3.36e9 points per array: past 2^31 elements, past 2^32 / 2^34 bytes) --
C3's 4096^2 x T = 200 and C4's per-GPU 8192^2 x T = 50 (bench.py --config c3 / c4w50), fp32 and fp64 -- checked
at sampled rows either side of every 2^31-element and 2^32-byte offset against host predictions that need no
window-sized array (tests/_fullsize.py, pinned against the oracle by tests/test_fullsize_host.py):

* iteration 1 from the reference initial state: phi' = g on every row, exactly; rho' / alp' one plane repeated on
  every row (bitwise the same rows) and equal to the oracle's one-row dual step;
* iteration 2: phi'' at the sampled rows against the closed-form per-mode two-right-hand-side t-solve
  (utils_precond.py:164-171) + one inverse FFT per row, from the device's own iteration-1 plane; rho'' / alp'' at
  sampled rows against the oracle's dual step of that row (update_fns_in_pdhg.py:150-165).

The other parity tests run reduced grids; this one is what catches an index or offset that overflows at the
bench's size.  Bounds: fp64 (the reference's arithmetic) 1e-10 relative L2 (phi, phi'' - g), 1e-9 (rho, alp);
fp32 phi 1e-6, rho / alp at epsl = 0.1 within the float32 representation bound of phi_bar (DESIGN.md section 6:
sigma*epsl*Lap(phi_bar) turns phi_bar's float32 rounding into ~5e-5 of rho at C3, ~2e-4 at C4)."""
import numpy as np
import pytest

from _fullsize import Iteration2, dual_row, grid_problem, iteration1_plane

pytestmark = pytest.mark.gpu

TAU, SIGMA = 0.1 / 1.5, 0.1 * 1.5

CASES = {
    # name: (egno, nx, ny, T, epsl)
    "c3": (2, 4096, 4096, 200, 0.1),
    "c4w50": (2, 8192, 8192, 50, 0.1),
}
BOUNDS = {
    "fp64": {"phi": 1e-10, "dphi": 1e-8, "rho": 1e-9, "alp": 1e-9},
    "fp32": {"phi": 1e-6, "dphi": 1e-2, "rho": 1e-3, "alp": 5e-2},
}


def _rel(a, b):
    nb = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / (nb if nb > 0 else 1.0))


def _rows(nx, ny, T, es):
    """phi rows (1..T) at the element offsets 2^31 and the byte offsets 2^32, 2^33, 2^34 (+ neighbours)."""
    plane = nx * ny
    marks = {(1 << 31) // plane} | {(1 << b) // (plane * es) for b in (32, 33, 34)}
    rows = {1, 2, T - 1, T}
    for m in marks:
        rows |= {m - 1, m, m + 1}
    return sorted(r for r in rows if 1 <= r <= T)


@pytest.mark.parametrize("prec", ["fp64", "fp32"])
@pytest.mark.parametrize("name", list(CASES))
def test_full_window_first_two_iterations(native, parity_log, name, prec):
    from pdhg_amd.context import PDHGContext
    egno, nx, ny, T, epsl = CASES[name]
    P = grid_problem(egno, nx, ny, T, epsl)
    es = 8 if prec == "fp64" else 4
    rows = _rows(nx, ny, T, es)
    b = BOUNDS[prec]
    ctx = PDHGContext(egno, 2, nx, ny, T, P["dsp"][0], P["dsp"][1], P["dt"], P["xs"], P["ys"], epsl=epsl,
                      precision=prec)
    m = {}
    try:
        ctx.init_state(P["g"])
        ctx.set_stop_rules(converge=False, nan=False)
        st = ctx.iterate(1, TAU, SIGMA, -1.0, 1)
        assert st["iters_run"] == 1
        # ---- iteration 1 ----
        g_dev = P["g"].astype(np.float32).astype(np.float64) if prec == "fp32" else P["g"]
        r, a = iteration1_plane(P, SIGMA)
        r_dev = a_dev = None
        for k in rows:
            ph, pb, _, _ = ctx.get_rows(k, 1, phi=True, phi_bar=True, rho=False, alp=False)
            assert np.array_equal(ph[0], g_dev) and np.array_equal(pb[0], g_dev), ("phi' != g", k)
        for j in sorted({0} | {k - 1 for k in rows}):
            _, _, rh, _ = ctx.get_rows(j, 1, phi=False, rho=True, alp=False)
            if r_dev is None:
                r_dev = rh[0]
            assert np.array_equal(rh[0], r_dev), ("rho' rows differ", j)
        for j in (0, rows[len(rows) // 2] - 1, T - 1):   # alp rows: 4 n_ctrl planes each
            _, _, _, al = ctx.get_rows(j, 1, phi=False, rho=False, alp=True)
            al = tuple(x[0] for x in al)
            if a_dev is None:
                a_dev = al
            assert all(np.array_equal(x, y) for x, y in zip(al, a_dev)), ("alp' rows differ", j)
        m["it1_rho"] = _rel(r_dev, r)
        m["it1_alp"] = max(_rel(x, y) for x, y in zip(a_dev, a) if np.linalg.norm(y) > 0)
        del r, a
        # ---- iteration 2 (from the device's own iteration-1 plane) ----
        st = ctx.iterate(1, TAU, SIGMA, -1.0, 1)
        assert st["iters_run"] == 1
        it2 = Iteration2(P, r_dev, a_dev)
        m["it2_phi"] = m["it2_dphi"] = 0.0
        for k in rows:
            ph, _, _, _ = ctx.get_rows(k, 1, phi=True, rho=False, alp=False)
            want = it2.phi(k, TAU)
            m["it2_phi"] = max(m["it2_phi"], _rel(ph[0], want))
            m["it2_dphi"] = max(m["it2_dphi"], _rel(ph[0] - P["g"], want - P["g"]))
        m["it2_rho"] = m["it2_alp"] = 0.0
        for j in (rows[0] - 1, rows[len(rows) // 2] - 1, T - 1):
            _, _, rh, al = ctx.get_rows(j, 1, phi=False, rho=True, alp=True)
            rn, an = dual_row(P, it2.phi_bar(j, TAU), it2.phi_bar(j + 1, TAU), r_dev, a_dev, SIGMA)
            m["it2_rho"] = max(m["it2_rho"], _rel(rh[0], rn))
            m["it2_alp"] = max([m["it2_alp"]] + [_rel(x[0], y) for x, y in zip(al, an) if np.linalg.norm(y) > 0])
    finally:
        ctx.close()
    bounds = {"it1_rho": b["rho"], "it1_alp": b["alp"], "it2_phi": b["phi"], "it2_dphi": b["dphi"],
              "it2_rho": b["rho"], "it2_alp": b["alp"]}
    parity_log("test_full_window_first_two_iterations", "{}@{}".format(name, prec), m, bounds, rows=rows)
    assert all(m[k] <= bounds[k] for k in m), (m, bounds)
