"""Problem plugin with the reference's entry points (jaxsrc/set_fns.py:10-166).

``set_up_example_fns`` returns the same ``Functions(f_fn, numerical_L_fn,
alp_update_fn)`` tuple, plus a ``spec`` field naming the built-in example.
The solver never calls these Python callables: the device kernels dispatch on
``spec`` (egno, ndim) and compute f, L and the alpha prox in registers
(csrc/params.hpp).  The callables stay for callers that evaluate the dynamics
themselves, e.g. trajectory simulation (run_example.py:18-155 uses f_fn).
"""
from collections import namedtuple

import numpy as np

Functions = namedtuple("Functions", ["f_fn", "numerical_L_fn", "alp_update_fn", "spec"], defaults=(None,))


def set_up_J(egno, ndim, period_spatial):
    """Terminal cost g = J(x) (set_fns.py:10-24)."""
    if egno == 3:
        y_period = period_spatial[1]
        return lambda x: np.sin(2 * np.pi / y_period * x[..., 1]) * np.exp(-x[..., 0] ** 2 / 2)
    if ndim not in (1, 2):
        raise ValueError("ndim {} not implemented".format(ndim))
    freq = 2 * np.pi / np.asarray(period_spatial[:ndim], dtype=np.float64)
    return lambda x: np.sin(freq * x).sum(axis=-1)


def set_up_numerical_L(egno, n_ctrl, ind, fn_coeff_H):
    """L(alp) summed over the 2 (n_ctrl=1) or 4 (n_ctrl=2) control arrays (set_fns.py:26-49)."""
    if ind != 0:
        raise ValueError("ind {} not implemented".format(ind))
    if n_ctrl not in (1, 2):
        raise ValueError("n_ctrl {} not implemented".format(n_ctrl))
    n_arr = 2 if n_ctrl == 1 else 4

    def L_fn(alp, x_arr, t_arr):
        out = 0.0
        for a in alp[:n_arr]:
            a = np.asarray(a)
            if egno == 2:
                term = 0.0 * a[..., 0]                       # indicator of |alp| <= c_H
            elif n_ctrl == 1:
                term = a[..., 0] ** 2 / fn_coeff_H(x_arr, t_arr)[..., 0] / 2
            else:
                term = np.sum(a ** 2 / fn_coeff_H(x_arr, t_arr), axis=-1) / 2
            out = out + term
        return out
    return L_fn


def _coeff(x):                      # a(x) = (x - 1)^2 + 0.1   (set_fns.py:117-118, :145)
    return (x - 1.0) ** 2 + 0.1


def set_up_example_fns(egno, ndim, numerical_L_ind):
    """Examples 1/2/3 of the paper (set_fns.py:52-166) as a Functions tuple with ``spec``."""
    if egno not in (1, 2, 3):
        raise ValueError("egno {} not implemented".format(egno))
    if egno == 3 and ndim != 2:
        raise ValueError("egno 3 is the 2-D Newton example")
    if ndim not in (1, 2):
        raise ValueError("ndim {} not implemented".format(ndim))
    n_ctrl = 1 if egno == 3 else ndim
    spec = {"egno": egno, "ndim": ndim, "n_ctrl": n_ctrl, "numerical_L_ind": numerical_L_ind}
    cH = lambda x_arr, t_arr: np.ones_like(x_arr[..., :n_ctrl]) if egno != 3 else np.ones_like(x_arr[..., 0:1])

    def prox(alp, D, p, a):
        # argmin_a p|a - alp|^2/2 - a*D*coef + L(a)  with the example's L (set_fns.py:63-95)
        if egno == 2:
            return np.clip(D * a / p + alp, -1.0, 1.0)
        return (D * a + p * alp) / (1.0 + p)

    if egno == 3:
        def f_fn(alp, x_arr, t_arr):                       # f = (alp, x_1)  (set_fns.py:98)
            xb = np.broadcast_to(x_arr[..., 0:1], np.shape(alp)[:-1] + (1,))
            return np.concatenate([alp, xb], axis=-1)

        def alp_update_fn(alp_prev, Dphi, rho, sigma, x_arr, t_arr):
            p = (rho[..., None] + 1e-4) / sigma
            n1 = (-Dphi[0][..., None] + p * alp_prev[0]) / (1.0 + p)
            n2 = (-Dphi[1][..., None] + p * alp_prev[1]) / (1.0 + p)
            return (n1 * (n1 >= 0.0), n2 * (n2 < 0.0), alp_prev[2], alp_prev[3])
    elif ndim == 2:
        def f_fn(alp, x_arr, t_arr):                       # f_d = -a(x_d) alp_d
            return -_coeff(x_arr) * alp

        def alp_update_fn(alp_prev, Dphi, rho, sigma, x_arr, t_arr):
            p = (rho[..., None] + 1e-4) / sigma
            ax, ay = _coeff(x_arr[..., 0:1]), _coeff(x_arr[..., 1:2])
            out = []
            for i, (D, a, comp, right) in enumerate(((Dphi[0], ax, 0, True), (Dphi[1], ax, 0, False),
                                                     (Dphi[2], ay, 1, True), (Dphi[3], ay, 1, False))):
                coef = np.concatenate([a, 0 * a] if comp == 0 else [0 * a, a], axis=-1)
                n = prox(alp_prev[i], D[..., None], p, coef)
                f = -np.sum(coef * n, axis=-1, keepdims=True)
                out.append(n * ((f >= 0.0) if right else (f < 0.0)))
            return tuple(out)
    else:
        def f_fn(alp, x_arr, t_arr):
            return -alp * _coeff(x_arr)

        def alp_update_fn(alp_prev, Dx_right_phi, Dx_left_phi, rho, sigma, x_arr, t_arr):
            p = ((rho + 1e-4) / sigma)[..., None]
            a = _coeff(x_arr)
            n1 = prox(alp_prev[0], Dx_right_phi[..., None], p, a)
            n2 = prox(alp_prev[1], Dx_left_phi[..., None], p, a)
            return (n1 * (-a * n1 >= 0.0), n2 * (-a * n2 < 0.0))

    L_fn = set_up_numerical_L(egno, n_ctrl, numerical_L_ind, cH)
    return Functions(f_fn=f_fn, numerical_L_fn=L_fn, alp_update_fn=alp_update_fn, spec=spec)
