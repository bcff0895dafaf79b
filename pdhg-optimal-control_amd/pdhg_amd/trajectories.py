"""Trajectory consumers of the computed controls (jaxsrc/run_example.py:18-155, used at :342-393).

After the solve, run_example simulates the controlled dynamics dx = f(alp(x, t), x, t) dt + sqrt(2 epsl) dW
forward in control time from sample starting points, interpolating the feedback control alp on the grid.
Host NumPy / SciPy: a few thousand samples x nt steps of interpolation, off the device hot path.

Time direction: the PDE runs backward from the terminal cost, so callers pass alp reversed in time
(``alp[:, ::-1]``, run_example.py:347) and f is evaluated at PDE time T - t (:41, :146).
The SDE noise draws from ``rng.normal`` (default: NumPy's global generator, as the reference's
``np.random.normal``); with epsl = 0 the trajectories are deterministic.
"""
import numpy as np
from scipy import interpolate

from .update_fns_in_pdhg import get_f_vals_1d, get_f_vals_2d


def _normal(rng, shape):
    return (rng or np.random).normal(size=shape)


def compute_traj_1d(x_init, alp, f_fn, nt, x_arr, t_arr, x_period, T, epsl=0.0, interp_method="linear", rng=None):
    """run_example.py:18-52.  x_arr [nx], t_arr [nt], alp [2, nt-1, nx], x_init [n_sample]
    -> traj_alp [nt-1, n_sample, 1], traj_x [nt, n_sample]."""
    x_arr = np.asarray(x_arr, dtype=np.float64)
    alp = np.asarray(alp, dtype=np.float64)
    t_arr = np.asarray(t_arr, dtype=np.float64)
    x_curr = np.asarray(x_init, dtype=np.float64)
    traj_alp, traj_x = [], [x_curr]
    for ind in range(nt - 1):
        dt = t_arr[ind + 1] - t_arr[ind]
        if interp_method == "linear":        # jnp.interp(..., period=x_period) == np.interp with period
            a1 = np.interp(x_curr, x_arr, alp[0, ind], period=x_period)[:, None]
            a2 = np.interp(x_curr, x_arr, alp[1, ind], period=x_period)[:, None]
        elif interp_method == "nearest":
            idx = np.abs(x_arr - (x_curr % x_period)[..., None]).argmin(axis=-1)
            a1, a2 = alp[0, ind, idx][:, None], alp[1, ind, idx][:, None]
        else:
            raise ValueError("interp_method must be 'linear' or 'nearest'")
        traj_alp.append(a1 + a2)
        f1, f2 = get_f_vals_1d(f_fn, (a1, a2), x_curr[:, None] % x_period, T - t_arr[ind])
        x_curr = x_curr + (f1 + f2) * dt + np.sqrt(2 * epsl * dt) * _normal(rng, x_curr.shape)
        traj_x.append(x_curr)
    return np.stack(traj_alp, axis=0), np.stack(traj_x, axis=0)


def extend_bdry_2d(x_arr, x_min, x_max, val_arr, period, axis, bc, center=False):
    """run_example.py:54-114: copies of the grid (periodic) or constant / zero padding (Neumann / Dirichlet)
    covering [x_min, x_max] along `axis` (1 or 2) of val_arr [:, n1, n2, val_dim], plus the closing point.
    Returns (x_arr_new [n_ext + 1], val_arr_new)."""
    if axis not in (1, 2):
        raise NotImplementedError("axis must be 1 or 2")
    x_arr = np.asarray(x_arr, dtype=np.float64)
    shift = 0.5 if center else 0.0
    lb = min(int(np.floor(x_min / period + shift)), 0)
    ub = max(int(np.floor(x_max / period + shift)), 0)
    n_period = ub - lb + 1
    edge = [slice(None)] * val_arr.ndim
    if bc == 0:
        val_arr = np.concatenate([val_arr] * n_period, axis=axis)
        edge[axis] = slice(0, 1)
        val_arr = np.concatenate([val_arr, val_arr[tuple(edge)]], axis=axis)
    else:
        n_per = val_arr.shape[axis]
        edge[axis] = slice(0, 1)
        left = val_arr[tuple(edge)]
        edge[axis] = slice(-1, None)
        right = val_arr[tuple(edge)]
        if bc == 2:
            left, right = np.zeros_like(left), np.zeros_like(right)
        parts = [np.repeat(left, -lb * n_per, axis=axis)] if lb < 0 else []
        parts.append(val_arr)
        if ub > 0:
            parts.append(np.repeat(right, ub * n_per, axis=axis))
        parts.append(right)
        val_arr = np.concatenate(parts, axis=axis)
    x_new = (x_arr[None, :] + np.arange(lb, ub + 1)[:, None] * period).reshape(-1)
    x_new = np.concatenate([x_new, x_new[0:1] + period * n_period])
    return x_new, val_arr


def compute_traj_2d(x_init, alp, f_fn, nt, x1_arr, x2_arr, t_arr, x_period, y_period, T, bc, center, epsl=0.0,
                    interp_method="linear", rng=None):
    """run_example.py:117-155.  alp [4, nt-1, nx, ny, n_ctrl], x_init [n_sample, 2]
    -> traj_alp [nt-1, n_sample, n_ctrl], traj_x [nt, n_sample, 2]."""
    alp = np.asarray(alp, dtype=np.float64)
    x1_arr, x2_arr = np.asarray(x1_arr, dtype=np.float64), np.asarray(x2_arr, dtype=np.float64)
    t_arr = np.asarray(t_arr, dtype=np.float64)
    x_curr = np.array(x_init, dtype=np.float64)
    bc_x, bc_y = bc
    cx, cy = center
    traj_alp, traj_x = [], [x_curr]
    for ind in range(nt - 1):
        dt = t_arr[ind + 1] - t_arr[ind]
        lo, hi = x_curr.min(axis=0), x_curr.max(axis=0)
        g1, a = extend_bdry_2d(x1_arr, lo[0], hi[0], alp[:, ind], x_period, axis=1, bc=bc_x, center=cx)
        g2, a = extend_bdry_2d(x2_arr, lo[1], hi[1], a, y_period, axis=2, bc=bc_y, center=cy)
        comps = tuple(interpolate.interpn((g1, g2), a[k], x_curr, method=interp_method) for k in range(4))
        traj_alp.append(comps[0] + comps[1] + comps[2] + comps[3])
        if bc_x == 0 and bc_y == 0:
            x_in = x_curr % np.array([x_period, y_period])
        elif bc_x == 1 and bc_y == 0:
            x_in = np.stack([x_curr[:, 0], x_curr[:, 1] % y_period], axis=-1)
        else:
            raise NotImplementedError("bc {} not supported by the reference trajectories".format(bc))
        f1x, f2x, f1y, f2y = get_f_vals_2d(f_fn, comps, x_in, T - t_arr[ind])
        vel = np.stack([f1x + f2x, f1y + f2y], axis=-1)
        x_curr = x_curr + vel * dt + np.sqrt(2 * epsl * dt) * _normal(rng, x_curr.shape)
        traj_x.append(x_curr)
    return np.stack(traj_alp, axis=0), np.stack(traj_x, axis=0)


def trajectory_samples(egno, ndim, n, x_period, y_period, epsl):
    """Sample starting points of run_example.py:350-378 (n = --plot_traj_num_1d)."""
    if egno == 3:     # Newton: (velocity 0.5, positions spread in y); epsl > 0 starts all at 0
        ys = np.linspace(-y_period / 2 + 0.1, y_period / 2 - 0.1, n)[:, None]
        if epsl > 0:
            ys = 0 * ys
        return np.pad(ys, ((0, 0), (1, 0)), mode="constant", constant_values=0.5)
    xs = np.linspace(0.0, x_period, n)
    if ndim == 1:
        return xs
    xm, ym = np.meshgrid(xs, np.linspace(0.0, y_period, n), indexing="ij")
    return np.stack([xm.reshape(-1), ym.reshape(-1)], axis=-1)


def run_trajectories(egno, ndim, alp, fns_dict, nt, x_arr, t_arr, x_period, y_period, T, bc, epsl, n, rng=None):
    """The trajectory block of run_example.main (:342-393): alp [2|4, nt-1, ...] from the solve (PDE time),
    reversed in time, interpolated linearly (nearest for egno 2's bang-bang control)."""
    alp_c = np.asarray(alp)[:, ::-1]
    t1 = np.asarray(t_arr).reshape(-1)
    x0 = trajectory_samples(egno, ndim, n, x_period, y_period, epsl)
    method = "nearest" if egno == 2 else "linear"
    if ndim == 1:
        return compute_traj_1d(x0, alp_c[..., 0], fns_dict.f_fn, nt, np.asarray(x_arr)[0, :, 0], t1, x_period, T,
                               epsl, method, rng=rng)
    x1, x2 = np.asarray(x_arr)[0, :, 0, 0], np.asarray(x_arr)[0, 0, :, 1]
    center = (egno == 3, egno == 3)
    if egno == 3:   # the reference passes no interp_method here (default linear)
        method = "linear"
    return compute_traj_2d(x0, alp_c, fns_dict.f_fn, nt, x1, x2, t1, x_period, y_period, T, bc, center, epsl,
                           method, rng=rng)
