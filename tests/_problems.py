"""Shared problem construction for the parity tests (oracle side + device side)."""
import numpy as np

import pdhg_oracle as O

SEED = 20250117   # SURVEY.md §8(d) seeded state


def make_problem(egno, ndim, nx, ny, T, epsl, seeded=True, seed=SEED, period=2.0):
    ny = ny if ndim == 2 else 1
    x_arr = O.make_grid(ndim, nx, ny, egno, period, period)
    dt = 1.0 / max(T, 40)                 # C0 time step (T_hor = 1, nt = 41) unless the window is longer
    dx, dy = period / nx, period / ny
    bc = O.default_bc(egno, ndim)
    fns = O.set_up_example_fns(egno, ndim, 0)
    g = O.set_up_J(egno, ndim, (period, period))(x_arr)
    if ndim == 1:
        xs, ys, dsp, nsp = x_arr[0, :, 0], None, (dx,), (nx,)
    else:
        xs, ys, dsp, nsp = x_arr[0, :, 0, 0], x_arr[0, 0, :, 1], (dx, dy), (nx, ny)
    fv = O.compute_Dxx_fft_fv(ndim, nsp, dsp, bc)
    n_ctrl = 1 if (ndim == 1 or egno == 3) else 2
    n_alp = 2 if ndim == 1 else 4
    phi = np.repeat(g, T + 1, axis=0)
    rho = np.full((T,) + nsp, 70.0)
    alp = [np.zeros((T,) + nsp + (n_ctrl,)) for _ in range(n_alp)]
    if seeded:
        rng = np.random.default_rng(seed)
        phi = phi + 0.01 * rng.standard_normal(phi.shape)
        rho = 70.0 * rng.uniform(0.5, 1.5, rho.shape)
        for a in range(n_alp):
            if ndim == 1 or egno == 3:
                comp = 0 if a < 2 else None            # egno 3: y controls stay zero
            else:
                comp = 0 if a < 2 else 1               # live component of each 2-D array
            if comp is not None:
                alp[a][..., comp] = 0.1 * rng.standard_normal(alp[a].shape[:-1])
    return dict(egno=egno, ndim=ndim, nx=nx, ny=ny, T=T, epsl=epsl, x_arr=x_arr, dt=dt, dx=dx, dy=dy, dsp=dsp,
                nsp=nsp, bc=bc, fns=fns, fv=fv, g=g, xs=xs, ys=ys, phi=phi, rho=rho, alp=tuple(alp),
                n_ctrl=n_ctrl, n_alp=n_alp)


def device_ctx(P, precision="fp64", rho_alp_iters=1, C=1.0, pow=1.0, Ct=1.0):
    from pdhg_amd.context import PDHGContext
    return PDHGContext(P["egno"], P["ndim"], P["nx"], P["ny"], P["T"], P["dx"], P["dy"], P["dt"], P["xs"], P["ys"],
                       epsl=P["epsl"], bc=P["bc"], C=C, pow=pow, Ct=Ct, precision=precision,
                       rho_alp_iters=rho_alp_iters)


def oracle_fns(P, rho_alp_iters=1, C=1.0, pow=1.0, Ct=1.0, stats=None):
    return O.make_update_fns(P["ndim"], P["bc"], C=C, pow=pow, Ct=Ct, rho_alp_iters=rho_alp_iters, dual_stats=stats)


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (nb if nb > 0 else 1.0)
