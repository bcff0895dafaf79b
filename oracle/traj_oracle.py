"""CPU ORACLE — test infrastructure only, never the product path.

Per-sample, pure-Python restatement of the reference's trajectory consumers of the controls
(jaxsrc/run_example.py:18-155): compute_traj_1d (:18-52), extend_bdry_2d (:54-114), compute_traj_2d
(:117-155).  It checks pdhg_amd.trajectories (vectorised NumPy / scipy.interpolate) with an independent
formulation: explicit cell search and linear / bilinear weights, and the boundary extension evaluated
as a virtual grid instead of concatenated copies.  Small sample counts only.  Parity unpinned as for
pdhg_oracle (the JAX reference cannot run here and ships no trajectory fixtures).
"""
import math

import numpy as np


def _f_split(fval, positive):
    """f * (f >= 0) or f * (f < 0) (update_fns_in_pdhg.py:23-26, :41-46)."""
    if positive:
        return fval if fval >= 0.0 else 0.0
    return fval if fval < 0.0 else 0.0


def interp_periodic(x, xp, fp, period):
    """jnp.interp(x, xp, fp, period=period) for one point (run_example.py:35-36): xp ascending in [0, period)."""
    xm = x % period
    n = len(xp)
    base = [v % period for v in xp]
    order = sorted(range(n), key=lambda i: base[i])
    xs = [base[i] for i in order]
    fs = [fp[i] for i in order]
    # wrap-around neighbours
    xs = [xs[-1] - period] + xs + [xs[0] + period]
    fs = [fs[-1]] + fs + [fs[0]]
    for i in range(len(xs) - 1):
        if xs[i] <= xm <= xs[i + 1]:
            w = (xm - xs[i]) / (xs[i + 1] - xs[i]) if xs[i + 1] > xs[i] else 0.0
            return fs[i] + w * (fs[i + 1] - fs[i])
    raise AssertionError("unreachable")


def nearest_index(x, xp, period):
    """argmin |xp - x % period| with the first index on ties (run_example.py:38-40)."""
    xm = x % period
    best, bi = None, 0
    for i, v in enumerate(xp):
        d = abs(v - xm)
        if best is None or d < best:
            best, bi = d, i
    return bi


def compute_traj_1d(x_init, alp, f_fn, nt, x_arr, t_arr, x_period, T, epsl=0.0, interp_method="linear", rng=None):
    """run_example.py:18-52, one sample at a time.  The noise is drawn once per step for all samples, in
    the reference's order (np.random.normal(size=x_curr.shape))."""
    xs = [float(v) for v in np.asarray(x_init)]
    n = len(xs)
    traj_x = [list(xs)]
    traj_alp = []
    for ind in range(nt - 1):
        dt = float(t_arr[ind + 1] - t_arr[ind])
        noise = (rng or np.random).normal(size=(n,))
        row_alp, new = [], []
        for s, x in enumerate(xs):
            if interp_method == "linear":
                a1 = interp_periodic(x, x_arr, alp[0][ind], x_period)
                a2 = interp_periodic(x, x_arr, alp[1][ind], x_period)
            else:
                j = nearest_index(x, x_arr, x_period)
                a1, a2 = float(alp[0][ind][j]), float(alp[1][ind][j])
            row_alp.append([a1 + a2])
            xm = np.array([[x % x_period]])
            f1 = float(f_fn(np.array([[a1]]), xm, T - t_arr[ind])[0, 0])
            f2 = float(f_fn(np.array([[a2]]), xm, T - t_arr[ind])[0, 0])
            vel = _f_split(f1, True) + _f_split(f2, False)
            new.append(x + vel * dt + math.sqrt(2 * epsl * dt) * noise[s])
        xs = new
        traj_alp.append(row_alp)
        traj_x.append(list(xs))
    return np.array(traj_alp), np.array(traj_x)


class VirtualExtension:
    """extend_bdry_2d (run_example.py:54-114) along one axis, evaluated point-wise: extended index i ->
    (coordinate, which original index or boundary value)."""

    def __init__(self, x_arr, x_min, x_max, period, bc, center):
        shift = 0.5 if center else 0.0
        self.lb = min(int(math.floor(x_min / period + shift)), 0)
        self.ub = max(int(math.floor(x_max / period + shift)), 0)
        self.n = len(x_arr)
        self.x = [float(v) for v in x_arr]
        self.P, self.bc = period, bc
        self.size = (self.ub - self.lb + 1) * self.n + 1

    def coord(self, i):
        if i == self.size - 1:
            return self.x[0] + self.lb * self.P + self.P * (self.ub - self.lb + 1)
        return self.x[i % self.n] + (self.lb + i // self.n) * self.P

    def source(self, i):
        """('idx', j) for original index j, or ('zero',) for Dirichlet padding."""
        if self.bc == 0:
            return ("idx", i % self.n) if i < self.size - 1 else ("idx", 0)
        if i == self.size - 1:
            return ("zero",) if self.bc == 2 else ("idx", self.n - 1)
        k = self.lb + i // self.n
        if k == 0:
            return ("idx", i % self.n)
        if self.bc == 2:
            return ("zero",)
        return ("idx", 0) if k < 0 else ("idx", self.n - 1)


def _value(field, e1, e2, i1, i2):
    s1, s2 = e1.source(i1), e2.source(i2)
    if s1[0] == "zero" or s2[0] == "zero":
        return np.zeros(field.shape[-1])
    return field[s1[1], s2[1]]


def _locate(e, x):
    for i in range(e.size - 1):
        if e.coord(i) <= x <= e.coord(i + 1):
            return i, (x - e.coord(i)) / (e.coord(i + 1) - e.coord(i))
    raise ValueError("point {} outside the extended grid".format(x))


def interp2(field, e1, e2, x, y, method):
    """scipy interpn on the extended grid, restated: bilinear weights, or the nearest node per axis with
    ties to the lower node (RegularGridInterpolator 'nearest')."""
    i, u = _locate(e1, x)
    j, v = _locate(e2, y)
    if method == "nearest":
        return _value(field, e1, e2, i + (1 if u > 0.5 else 0), j + (1 if v > 0.5 else 0))
    return ((1 - u) * (1 - v) * _value(field, e1, e2, i, j) + u * (1 - v) * _value(field, e1, e2, i + 1, j)
            + (1 - u) * v * _value(field, e1, e2, i, j + 1) + u * v * _value(field, e1, e2, i + 1, j + 1))


def compute_traj_2d(x_init, alp, f_fn, nt, x1_arr, x2_arr, t_arr, x_period, y_period, T, bc, center, epsl=0.0,
                    interp_method="linear", rng=None):
    """run_example.py:117-155, one sample at a time."""
    alp = np.asarray(alp, dtype=np.float64)
    pts = [list(map(float, p)) for p in np.asarray(x_init)]
    n = len(pts)
    traj_x, traj_alp = [[list(p) for p in pts]], []
    for ind in range(nt - 1):
        dt = float(t_arr[ind + 1] - t_arr[ind])
        xmin = [min(p[d] for p in pts) for d in range(2)]
        xmax = [max(p[d] for p in pts) for d in range(2)]
        e1 = VirtualExtension(x1_arr, xmin[0], xmax[0], x_period, bc[0], center[0])
        e2 = VirtualExtension(x2_arr, xmin[1], xmax[1], y_period, bc[1], center[1])
        noise = (rng or np.random).normal(size=(n, 2))
        row_alp, new = [], []
        for s, (x, y) in enumerate(pts):
            comps = [interp2(alp[k, ind], e1, e2, x, y, interp_method) for k in range(4)]
            row_alp.append(list(comps[0] + comps[1] + comps[2] + comps[3]))
            if bc[0] == 0 and bc[1] == 0:
                xin = np.array([[x % x_period, y % y_period]])
            else:
                xin = np.array([[x, y % y_period]])
            fx = [float(f_fn(c[None, :], xin, T - t_arr[ind])[0, 0]) for c in comps[:2]]
            fy = [float(f_fn(c[None, :], xin, T - t_arr[ind])[0, 1]) for c in comps[2:]]
            vx = _f_split(fx[0], True) + _f_split(fx[1], False)
            vy = _f_split(fy[0], True) + _f_split(fy[1], False)
            sq = math.sqrt(2 * epsl * dt)
            new.append([x + vx * dt + sq * noise[s, 0], y + vy * dt + sq * noise[s, 1]])
        pts = new
        traj_alp.append(row_alp)
        traj_x.append([list(p) for p in pts])
    return np.array(traj_alp), np.array(traj_x)
