"""Host predictions of the first two PDHG iterations from the reference initial state at ANY window size
(test infrastructure; the checker for tests/test_gpu_fullsize.py, pinned against the oracle by
tests/test_fullsize_host.py).

From the reference initial state (utils_pdhg_solver.py:123-137: phi rows = g, rho = c_on_rho, alp = 0):

* iteration 1: alp = 0 makes every flux zero and rho is constant, so the continuity residual
  (update_fns_in_pdhg.py:83-96) is (rho_{j+1} - rho_j)/dt = 0 on rows 1..T-1 and (0 - c)/dt + c/dt = 0 on row T:
  phi' = phi = g exactly, phi_bar' = g, and the dual step (:150-165) sees the same phi_bar rows j, j+1 = g, g and
  the same rho, alp on every row -- rho' and alp' are ONE plane (r, a) repeated on every row, the oracle's dual
  step of a one-row window;
* iteration 2: with rho = r and alp = a on every row the residual is Q = epsl Lap(r) - div((r + 1e-4) f(a)) on rows
  1..T-1 and Q + (c - r)/dt on row T.  Per Fourier mode the preconditioner solves M u = dt^2 R with
  M = tridiag(-1, dd + 2, -1), last diagonal dd + 1 (Neumann), dd = (C - fv) dt^2 (utils_precond.py:164-169), so
  U = dt^2 (Q^ u1 + W^ u2) with the closed forms (cosh th = 1 + dd/2, rows k = 1..T, u_0 = 0):
      M u1 = 1:    u1_k = (1 - cosh(th (T + 1/2 - k)) / cosh(th (T + 1/2))) / dd
      M u2 = e_T:  u2_k = sinh(th k) / (2 cosh(th (T + 1/2)) sinh(th / 2))
  and phi''_k = g + tau U_k, phi_bar''_k = g + 2 tau U_k -- one inverse FFT per sampled row, no window-sized array.

The dual steps are local in x (one-sided differences and the Laplacian reach x +- 1), so they are evaluated on
BANDS of x rows (the oracle on the band with one margin row either side, periodic wrap only reaching the margins):
at C4's 67 M-point plane a full-plane oracle dual step takes minutes on the host.
"""
import os

import numpy as np
import scipy.fft as sfft

import pdhg_oracle as O

_W = int(os.environ.get("ORACLE_FFT_WORKERS", "1"))   # the box gives a job a 16-CPU share (conftest)


def grid_problem(egno, nx, ny, T, epsl, period=2.0):
    """The bench's grid (bench.py grid(): x_i = i dx, no centring for egno 1/2), dt = 1/T (nt = T + 1)."""
    x_arr = O.make_grid(2, nx, ny, egno, period, period)
    dt = 1.0 / T
    dsp = (period / nx, period / ny)
    bc = O.default_bc(egno, 2)
    return dict(egno=egno, nx=nx, ny=ny, T=T, epsl=epsl, x_arr=x_arr, dt=dt, dsp=dsp, bc=bc,
                fns=O.set_up_example_fns(egno, 2, 0), g=O.set_up_J(egno, 2, (period, period))(x_arr)[0],
                fv=O.compute_Dxx_fft_fv(2, (nx, ny), dsp, bc), xs=x_arr[0, :, 0, 0], ys=x_arr[0, 0, :, 1])


def band(nx, x0, w):
    """x rows of a band [x0, x0 + w) with one margin row either side (periodic indices); interior = [1:-1]."""
    return np.arange(x0 - 1, x0 + w + 1) % nx


def _xa(P, idx):
    return P["x_arr"] if idx is None else P["x_arr"][:, idx]


def _cut(a, idx):
    return a if idx is None else a[idx]


def _inner(a, idx):
    return a if idx is None else a[1:-1]


def iteration1_plane(P, sigma, c_on_rho=70.0, idx=None):
    """(r, a): the dual step of iteration 1 (one plane; every row of rho', alp' equals it); idx: on a band only."""
    g = _cut(P["g"], idx)
    n_ctrl = 1 if P["egno"] == 3 else 2
    phibar = np.stack([g, g])
    rho = np.full((1,) + g.shape, c_on_rho)
    alp = tuple(np.zeros((1,) + g.shape + (n_ctrl,)) for _ in range(4))
    r, a, _ = O.update_dual_oneiter(phibar, rho, c_on_rho, alp, sigma, P["dt"], P["dsp"], P["epsl"], _xa(P, idx), None,
                                    P["bc"], P["fns"], 2)
    return _inner(r[0], idx), tuple(_inner(x[0], idx) for x in a)


def _theta(dd):
    dl = 0.5 * dd
    return np.log1p(dl + np.sqrt(dl * (dl + 2.0)))


def mode_weights(dd, T, k):
    """(u1_k, u2_k) per mode for row k (1..T), numerically stable for any th T."""
    th = _theta(dd)
    b = th * (T + 0.5)
    den = 1.0 + np.exp(-2.0 * b)
    # 1 - cosh(a)/cosh(b) = (1 - e^{-th k}) (1 - e^{-2 th (T + 1/2 - k/2)}) / (1 + e^{-2b})
    u1 = (-np.expm1(-th * k)) * (-np.expm1(-2.0 * th * (T + 0.5 - 0.5 * k))) / (den * dd)
    # sinh(th k) / (2 cosh(b) sinh(th/2)) = e^{th k - b} (1 - e^{-2 th k}) / (2 sinh(th/2) (1 + e^{-2b}))
    u2 = np.exp(th * k - b) * (-np.expm1(-2.0 * th * k)) / (2.0 * np.sinh(0.5 * th) * den)
    return u1, u2


class Iteration2:
    """phi'' / phi_bar'' rows of iteration 2 from the state (r, a) after iteration 1 (any rows, no window array)."""

    def __init__(self, P, r, a, c_on_rho=70.0, C=1.0):
        if P["bc"] != (0, 0):
            raise NotImplementedError("periodic bc only (FFT2 modes)")
        dt = P["dt"]
        # the oracle's residual of a one-row window is the last row's, Q + (c - r)/dt (update_fns_in_pdhg.py:95)
        R1 = O.compute_cont_residual_2d(r[None], tuple(x[None] for x in a), dt, P["dsp"], P["fns"], c_on_rho,
                                        P["epsl"], P["x_arr"], None, P["bc"])
        W = (c_on_rho - r) / dt           # the last row's extra term
        Q = R1[-1] - W                    # an interior row (rho_{j+1} = rho_j)
        del R1
        # Q, W real and the symbol even in both axes: the half spectrum (rfft2 / irfft2) carries every mode
        self.Qh = sfft.rfft2(Q, workers=_W)
        self.Wh = sfft.rfft2(W, workers=_W)
        self.shape = Q.shape
        self.dd = ((C - np.asarray(P["fv"]).real) * dt * dt)[:, :Q.shape[1] // 2 + 1]
        self.dt, self.T, self.g = dt, P["T"], P["g"]
        self._cache = {}   # the last few rows' U (phi'' and phi_bar'' of a row share it)

    def U(self, k):
        if k == 0:
            return np.zeros_like(self.g)
        if k not in self._cache:
            u1, u2 = mode_weights(self.dd, self.T, k)
            if len(self._cache) >= 3:
                self._cache.pop(next(iter(self._cache)))
            self._cache[k] = sfft.irfft2(self.Qh * u1 + self.Wh * u2, s=self.shape, workers=_W) * (self.dt * self.dt)
        return self._cache[k]

    def phi(self, k, tau):
        return self.g + tau * self.U(k)

    def phi_bar(self, k, tau):
        return self.g + 2.0 * tau * self.U(k)


def dual_row(P, pb_j, pb_j1, r, a, sigma, c_on_rho=70.0, idx=None):
    """rho'' / alp'' of row j from phi_bar rows j, j+1 and the row's (r, a) (the oracle's dual on a one-row window);
    idx: on a band of x rows (inputs are full planes, the result the band's interior)."""
    c = lambda v: _cut(v, idx)  # noqa: E731
    rn, an, _ = O.update_dual_oneiter(np.stack([c(pb_j), c(pb_j1)]), c(r)[None], c_on_rho,
                                      tuple(c(x)[None] for x in a), sigma, P["dt"], P["dsp"], P["epsl"], _xa(P, idx),
                                      None, P["bc"], P["fns"], 2)
    return _inner(rn[0], idx), tuple(_inner(x[0], idx) for x in an)
