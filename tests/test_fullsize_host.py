"""Pins the host predictor of tests/_fullsize.py (the checker of the full-size window test) against the oracle's
own two PDHG iterations from the reference initial state on small windows (CPU)."""
import numpy as np
import pytest

import pdhg_oracle as O
from _fullsize import Iteration2, band, dual_row, grid_problem, iteration1_plane, mode_weights

TAU, SIGMA = 0.1 / 1.5, 0.1 * 1.5


def _oracle_two(P):
    T = P["T"]
    g = P["g"]
    phi = np.repeat(g[None], T + 1, axis=0)
    rho = np.full((T,) + g.shape, 70.0)
    alp = tuple(np.zeros((T,) + g.shape + (2,)) for _ in range(4))
    primal, dual = O.make_update_fns(2, P["bc"], rho_alp_iters=1)
    out = []
    for _ in range(2):
        phi_n = primal(phi, rho, 70.0, alp, TAU, P["dt"], P["dsp"], P["fns"], P["fv"], P["epsl"], P["x_arr"], None)
        pb = 2 * phi_n - phi
        rho, alp = dual(pb, rho, 70.0, alp, SIGMA, P["dt"], P["dsp"], P["epsl"], P["fns"], P["x_arr"], None, 2, -1.0)
        phi = phi_n
        out.append((phi, pb, rho, alp))
    return out


def _rel(a, b):
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


@pytest.mark.parametrize("egno,nx,ny,T,epsl", [(2, 32, 48, 24, 0.1), (1, 64, 32, 40, 0.0), (2, 48, 48, 200, 0.1)])
def test_predictor_matches_oracle(egno, nx, ny, T, epsl):
    P = grid_problem(egno, nx, ny, T, epsl)
    (phi1, pb1, rho1, alp1), (phi2, pb2, rho2, alp2) = _oracle_two(P)
    r, a = iteration1_plane(P, SIGMA)
    # iteration 1: phi' = g exactly, rho' / alp' the one plane on every row
    assert np.array_equal(phi1, np.repeat(P["g"][None], T + 1, axis=0))
    for j in range(T):
        assert np.array_equal(rho1[j], r)
        for k in range(4):
            assert np.array_equal(alp1[k][j], a[k])
    # iteration 2 at every row
    it2 = Iteration2(P, r, a)
    for k in range(T + 1):
        assert _rel(it2.phi(k, TAU), phi2[k]) < 1e-13, k
        assert _rel(it2.phi_bar(k, TAU), pb2[k]) < 1e-13, k
    for j in (0, 1, T // 2, T - 1):
        rn, an = dual_row(P, it2.phi_bar(j, TAU), it2.phi_bar(j + 1, TAU), r, a, SIGMA)
        assert _rel(rn, rho2[j]) < 1e-12, j
        for k in range(4):
            if np.linalg.norm(alp2[k][j]) > 0:
                assert _rel(an[k], alp2[k][j]) < 1e-12, (j, k)
    # the band forms (x rows [x0, x0 + w), margins wrapping periodically) equal the full-plane values there
    for x0, w in ((0, 5), (nx - 4, 4), (nx // 2, 3)):
        idx = band(nx, x0, w)
        rows_ = np.arange(x0, x0 + w) % nx
        rb, ab = iteration1_plane(P, SIGMA, idx=idx)
        assert np.array_equal(rb, r[rows_]) and all(np.array_equal(x, y[rows_]) for x, y in zip(ab, a))
        j = T // 2
        rn, an = dual_row(P, it2.phi_bar(j, TAU), it2.phi_bar(j + 1, TAU), r, a, SIGMA)
        rnb, anb = dual_row(P, it2.phi_bar(j, TAU), it2.phi_bar(j + 1, TAU), r, a, SIGMA, idx=idx)
        assert np.array_equal(rnb, rn[rows_]) and all(np.array_equal(x, y[rows_]) for x, y in zip(anb, an))


def test_mode_weights_solve_the_tridiagonal_systems():
    """u1, u2 solve tridiag(-1, dd + 2, -1) (last diagonal dd + 1) against 1 and e_T, for small to huge th T."""
    T = 50
    for dd in (1e-8, 2.5e-5, 0.3, 4.0, 839.0, 1e6):
        M = np.diag(np.full(T, dd + 2.0)) - np.diag(np.ones(T - 1), 1) - np.diag(np.ones(T - 1), -1)
        M[-1, -1] = dd + 1.0
        ones, eT = np.ones(T), np.zeros(T)
        eT[-1] = 1.0
        x1, x2 = np.linalg.solve(M, ones), np.linalg.solve(M, eT)
        ks = np.arange(1, T + 1)
        u1, u2 = mode_weights(np.float64(dd), T, ks)
        assert _rel(u1, x1) < 1e-9, dd
        assert np.allclose(u2, x2, rtol=1e-9, atol=1e-300), dd
