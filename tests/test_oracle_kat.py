"""Known-answer tests that pin the float64 oracle without the (unrunnable) JAX reference.

* adjoint identities of the finite-difference operators (utils_diff_op.py:9-298): the continuity
  residual is the negative adjoint of the HJ operator, which is what makes PDHG's K / K^T pair;
* the defining equation of the H1 preconditioner (utils_precond.py:105-178) applied back to its
  output with independent stencils;
* the Thomas recurrence (utils_precond.py:10-35) against a dense solve;
* the Fourier symbol (utils_precond.py:42-71) against the analytic eigenvalues.
"""
import numpy as np
import pytest

import pdhg_oracle as O

rng = np.random.default_rng(0)


def ip(a, b):
    return float(np.sum(a * b))


@pytest.mark.parametrize("shape", [(5, 12), (4, 8, 6)])
def test_adjoint_identities_periodic(shape):
    T1 = shape[0]
    phi = rng.standard_normal(shape)
    m = rng.standard_normal((T1 - 1,) + shape[1:])
    dx, dy, dt = 0.3, 0.7, 0.1
    assert np.isclose(ip(O.Dx_right_decreasedim(phi, dx, 0), m), -ip(phi, O.Dx_left_increasedim(m, dx, 0)))
    assert np.isclose(ip(O.Dx_left_decreasedim(phi, dx, 0), m), -ip(phi, O.Dx_right_increasedim(m, dx, 0)))
    assert np.isclose(ip(O.Dt_decreasedim(phi, dt), m), -ip(phi, O.Dt_increasedim(m, dt)))
    assert np.isclose(ip(O.Dxx_decreasedim(phi, dx, 0), m), ip(phi, O.Dxx_increasedim(m, dx, 0)))
    if len(shape) == 3:
        assert np.isclose(ip(O.Dy_right_decreasedim(phi, dy, 0), m), -ip(phi, O.Dy_left_increasedim(m, dy, 0)))
        assert np.isclose(ip(O.Dy_left_decreasedim(phi, dy, 0), m), -ip(phi, O.Dy_right_increasedim(m, dy, 0)))
        assert np.isclose(ip(O.Dyy_decreasedim(phi, dy, 0), m), ip(phi, O.Dyy_increasedim(m, dy, 0)))


def test_neumann_dirichlet_boundary_values():
    phi = rng.standard_normal((3, 7))
    dx = 0.5
    # Neumann: one-sided difference vanishes at the closed end (utils_diff_op.py:19-20, :61-62)
    assert np.all(O.Dx_right_decreasedim(phi, dx, 1)[:, -1] == 0)
    assert np.all(O.Dx_left_decreasedim(phi, dx, 1)[:, 0] == 0)
    # Dirichlet: zero outside (:21-22, :63-64)
    assert np.allclose(O.Dx_right_decreasedim(phi, dx, 2)[:, -1], -phi[1:, -1] / dx)
    assert np.allclose(O.Dx_left_decreasedim(phi, dx, 2)[:, 0], phi[1:, 0] / dx)
    assert np.allclose(O.Dxx_decreasedim(phi, dx, 1)[:, 0], (phi[1:, 1] - phi[1:, 0]) / dx ** 2)


def test_thomas_vs_dense():
    T, n = 9, 5
    dl = np.r_[0.0, -rng.uniform(1, 2, T - 1)]
    du = np.r_[-rng.uniform(1, 2, T - 1), 0.0]
    d = rng.uniform(5, 6, (T, n)) + 0j
    b = rng.standard_normal((T, n)) + 1j * rng.standard_normal((T, n))
    x = O.tridiagonal_solve(dl + 0j, d, du + 0j, b)
    for i in range(n):
        A = np.diag(d[:, i]) + np.diag(dl[1:], -1) + np.diag(du[:-1], 1)
        assert np.allclose(A @ x[:, i], b[:, i])


def _lap_periodic(u, d, axis):
    return (np.roll(u, -1, axis) + np.roll(u, 1, axis) - 2 * u) / d ** 2


def _dtt_dirichlet_neumann(u, dt):
    """rows 1..T of D_tt with u_0 = 0 pinned and u_{T+1} = u_T (Neumann)."""
    up = np.concatenate([u[2:], u[-1:]], axis=0)
    return (up + u[:-1] - 2 * u[1:]) / dt ** 2


@pytest.mark.parametrize("C,pw,Ct", [(1.0, 1, 1.0), (0.5, 1, 2.0), (1.0, 1, 0.0)])
def test_h1_precond_1d_defining_equation(C, pw, Ct):
    nt, nx = 7, 16
    dx, dt = 2 / nx, 0.05
    src = rng.standard_normal((nt, nx))
    fv = O.compute_Dxx_fft_fv(1, (nx,), (dx,), 0)
    u = O.H1_precond_1d(src, fv, dt, 0, C=C, pow=pw, Ct=Ct)
    assert np.all(u[0] == 0)
    lhs = C * u[1:] - _lap_periodic(u, dx, 1)[1:] - Ct * _dtt_dirichlet_neumann(u, dt)
    assert np.allclose(lhs, src[1:], atol=1e-9 * np.abs(src).max())


def test_h1_precond_2d_defining_equation():
    nt, nx, ny = 6, 12, 10
    dx, dy, dt = 2 / nx, 2 / ny, 0.1
    src = rng.standard_normal((nt, nx, ny))
    fv = O.compute_Dxx_fft_fv(2, (nx, ny), (dx, dy), (0, 0))
    u = O.H1_precond_2d(src, fv, dt, (0, 0), C=1.0)
    lhs = u[1:] - _lap_periodic(u, dx, 1)[1:] - _lap_periodic(u, dy, 2)[1:] - _dtt_dirichlet_neumann(u, dt)
    assert np.allclose(lhs, src[1:], atol=1e-9 * np.abs(src).max())


def test_fourier_symbol_analytic():
    nx, ny, dx, dy = 10, 14, 0.2, 0.15
    fv = O.compute_Dxx_fft_fv(2, (nx, ny), (dx, dy), (0, 0))
    lx = -2 * (1 - np.cos(2 * np.pi * np.arange(nx) / nx)) / dx ** 2
    ly = -2 * (1 - np.cos(2 * np.pi * np.arange(ny) / ny)) / dy ** 2
    assert np.allclose(fv, lx[:, None] + ly[None, :])
    assert np.abs(fv.imag).max() < 1e-9 * np.abs(fv).max()


def test_example_plugins_masks_and_bounds():
    """alpha prox branches (set_fns.py:63-95, 132-138, 157-159)."""
    x = O.make_grid(1, 8, 1, 1)
    fns = O.set_up_example_fns(1, 1, 0)
    a = rng.standard_normal((3, 8, 1))
    D = rng.standard_normal((3, 8)) * 10
    rho = rng.uniform(1, 2, (3, 8))
    n1, n2 = fns.alp_update_fn((a, a), D, D, rho, 0.15, x, None)
    assert np.all(n1 <= 0) and np.all(n2 >= 0)        # f = -a(x) alp: alp1 keeps f >= 0, alp2 keeps f < 0
    fns2 = O.set_up_example_fns(2, 1, 0)
    m1, m2 = fns2.alp_update_fn((a, a), D, D, rho, 0.15, x, None)
    assert np.all(np.abs(m1) <= 1) and np.all(np.abs(m2) <= 1)
    assert np.all(fns2.numerical_L_fn((m1, m2), x, None) == 0)


def test_terminal_costs():
    x2 = O.make_grid(2, 4, 4, 1)
    assert np.allclose(O.set_up_J(1, 2, (2.0, 2.0))(x2), np.sin(np.pi * x2[..., 0]) + np.sin(np.pi * x2[..., 1]))
    x3 = O.make_grid(2, 4, 4, 3)
    assert np.allclose(O.set_up_J(3, 2, (2.0, 2.0))(x3), np.sin(np.pi * x3[..., 1]) * np.exp(-x3[..., 0] ** 2 / 2))
