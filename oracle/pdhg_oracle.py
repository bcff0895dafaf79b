"""CPU ORACLE — test infrastructure only, never the product path.

Float64 NumPy/SciPy restatement of the reference's PDHG hot path
(TingweiMeng/PDHG-optimal-control @ 2025-01-17, ``jaxsrc/``).  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker / CPU timing column.

PARITY UNPINNED: the reference cannot run in this container (jax, jaxlib,
einshape, tensorflow and absl are not installed; plain ModuleNotFoundError, no
command was refused) and it ships no tests, fixtures or golden vectors
(SURVEY.md §4, §8c).  This restatement is therefore pinned only by the
known-answer tests in ``tests/test_oracle_kat.py`` (adjoint identities of the
stencils, the defining equation of the H1 preconditioner, Thomas vs dense
solve) and by the committed fixtures it generated itself.

It follows the reference's algorithm literally — complex FFTs, the complex
Thomas recurrence of ``utils_precond.py:10-35`` — so that the product's
different formulation (real Hartley transforms, closed-form Thomas factors)
is checked against an independent computation.  Quirks of the reference that
the product must reproduce are kept; every function
cites the reference lines it restates.
"""
from collections import namedtuple
import os

import numpy as np
import scipy.fft as sfft

_WORKERS = int(os.environ.get("ORACLE_FFT_WORKERS", os.cpu_count() or 1))

# ---------------------------------------------------------------------------
# finite-difference operators  (jaxsrc/utils/utils_diff_op.py)
# bc: 0 periodic, 1 Neumann, 2 Dirichlet  (utils_diff_op.py:5-7)
# ---------------------------------------------------------------------------


def _zeros_like_slice(a, axis):
    shape = list(a.shape)
    shape[axis] = 1
    return np.zeros(shape, dtype=a.dtype)


def _take(a, sl, axis):
    idx = [slice(None)] * a.ndim
    idx[axis] = sl
    return a[tuple(idx)]


def _right_base(phi, d, bc, axis):
    """utils_diff_op.py:9-23 (x, axis 1) and :93-107 (y, axis 2)."""
    if bc == 0:
        out = np.roll(phi, -1, axis=axis) - phi
    elif bc == 1:
        out = np.concatenate([_take(phi, slice(1, None), axis) - _take(phi, slice(None, -1), axis),
                              _zeros_like_slice(phi, axis)], axis=axis)
    elif bc == 2:
        out = np.concatenate([_take(phi, slice(1, None), axis), _zeros_like_slice(phi, axis)], axis=axis) - phi
    else:
        raise NotImplementedError(bc)
    return out / d


def _left_base(phi, d, bc, axis):
    """utils_diff_op.py:51-65 (x) and :135-149 (y)."""
    if bc == 0:
        out = phi - np.roll(phi, 1, axis=axis)
    elif bc == 1:
        out = np.concatenate([_zeros_like_slice(phi, axis),
                              _take(phi, slice(1, None), axis) - _take(phi, slice(None, -1), axis)], axis=axis)
    elif bc == 2:
        out = phi - np.concatenate([_zeros_like_slice(phi, axis), _take(phi, slice(None, -1), axis)], axis=axis)
    else:
        raise NotImplementedError(bc)
    return out / d


def _second_base(phi, d, bc, axis):
    """utils_diff_op.py:208-226 (Dxx) and :255-273 (Dyy)."""
    if bc == 0:
        p_ip1 = np.roll(phi, -1, axis=axis)
        p_im1 = np.roll(phi, 1, axis=axis)
    elif bc == 1:
        p_ip1 = np.concatenate([_take(phi, slice(1, None), axis), _take(phi, slice(-1, None), axis)], axis=axis)
        p_im1 = np.concatenate([_take(phi, slice(0, 1), axis), _take(phi, slice(None, -1), axis)], axis=axis)
    elif bc == 2:
        p_ip1 = np.concatenate([_take(phi, slice(1, None), axis), _zeros_like_slice(phi, axis)], axis=axis)
        p_im1 = np.concatenate([_zeros_like_slice(phi, axis), _take(phi, slice(None, -1), axis)], axis=axis)
    else:
        raise NotImplementedError(bc)
    return (p_ip1 + p_im1 - 2 * phi) / d ** 2


def _prepend_zero_row(out):
    return np.concatenate([np.zeros_like(out[0:1]), out], axis=0)


def Dx_right_decreasedim(phi, dx, bc):   # utils_diff_op.py:25-35
    return _right_base(phi, dx, bc, 1)[1:]


def Dx_right_increasedim(m, dx, bc):     # utils_diff_op.py:37-49
    return _prepend_zero_row(_right_base(m, dx, bc, 1))


def Dx_left_decreasedim(phi, dx, bc):    # utils_diff_op.py:67-77
    return _left_base(phi, dx, bc, 1)[1:]


def Dx_left_increasedim(m, dx, bc):      # utils_diff_op.py:79-91
    return _prepend_zero_row(_left_base(m, dx, bc, 1))


def Dy_right_decreasedim(phi, dy, bc):   # utils_diff_op.py:109-119
    return _right_base(phi, dy, bc, 2)[1:]


def Dy_right_increasedim(m, dy, bc):     # utils_diff_op.py:121-133
    return _prepend_zero_row(_right_base(m, dy, bc, 2))


def Dy_left_decreasedim(phi, dy, bc):    # utils_diff_op.py:151-162
    return _left_base(phi, dy, bc, 2)[1:]


def Dy_left_increasedim(m, dy, bc):      # utils_diff_op.py:164-176
    return _prepend_zero_row(_left_base(m, dy, bc, 2))


def Dt_decreasedim(phi, dt):             # utils_diff_op.py:179-191
    return (phi[1:] - phi[:-1]) / dt


def Dt_increasedim(rho, dt):             # utils_diff_op.py:193-206
    rho_km1 = np.concatenate([np.zeros_like(rho[0:1]), rho], axis=0)
    rho_k = np.concatenate([rho, np.zeros_like(rho[0:1])], axis=0)
    return (rho_k - rho_km1) / dt


def Dxx_decreasedim(phi, dx, bc):        # utils_diff_op.py:228-238
    return _second_base(phi, dx, bc, 1)[1:]


def Dxx_increasedim(rho, dx, bc):        # utils_diff_op.py:241-253
    return _prepend_zero_row(_second_base(rho, dx, bc, 1))


def Dyy_decreasedim(phi, dy, bc):        # utils_diff_op.py:275-285
    return _second_base(phi, dy, bc, 2)[1:]


def Dyy_increasedim(rho, dy, bc):        # utils_diff_op.py:287-299
    return _prepend_zero_row(_second_base(rho, dy, bc, 2))


# ---------------------------------------------------------------------------
# preconditioner  (jaxsrc/utils/utils_precond.py)
# ---------------------------------------------------------------------------


def tridiagonal_solve(dl, d, du, b):
    """Thomas algorithm exactly as the lax.scan version, utils_precond.py:10-35.

    dl, du: [T] (shared); d, b: [T, ...] batched over trailing axes."""
    T = d.shape[0]
    tu = np.empty_like(d)
    carry = du[0] / d[0]
    for j in range(T):                       # fwd1, :13, :19-22
        carry = du[j] / (d[j] - dl[j] * carry)
        tu[j] = carry
    tu_prev = np.concatenate([np.zeros_like(tu[0:1]), tu[:-1]], axis=0)   # prepend_zero, :12
    bb = np.empty(np.broadcast(d, b).shape, dtype=np.result_type(d, b))
    carry = b[0] / d[0]
    for j in range(T):                       # fwd2, :14, :24-27
        carry = (b[j] - dl[j] * carry) / (d[j] - dl[j] * tu_prev[j])
        bb[j] = carry
    x = np.empty_like(bb)
    carry = bb[-1]
    for j in range(T - 1, -1, -1):           # bwd1, :15, :30-33
        carry = bb[j] - tu[j] * carry
        x[j] = carry
    return x


def compute_Dxx_fft_fv(ndim, nspatial, dspatial, bc):
    """Fourier/cosine symbol of the discrete Laplacian, utils_precond.py:42-71."""
    if ndim == 1:
        dx = dspatial[0]
        nx = nspatial[0]
        lap = np.array([-2 / (dx * dx), 1 / (dx * dx)] + [0.0] * (nx - 3) + [1 / (dx * dx)])
        if bc == 0:
            return np.fft.fft(lap)
        if bc == 1:
            return sfft.dct(lap).astype(np.complex128)
        raise NotImplementedError
    if ndim == 2:
        dx, dy = dspatial
        nx, ny = nspatial
        bc_x, bc_y = bc
        lap = np.zeros((nx, ny))
        lap[0, 0] = -2 / (dx * dx) - 2 / (dy * dy)
        lap[0, 1] = 1 / (dy * dy)
        lap[0, -1] += 1 / (dy * dy)
        lap[1, 0] += 1 / (dx * dx)
        lap[-1, 0] += 1 / (dx * dx)
        if bc_x == 0 and bc_y == 0:
            return np.fft.fft2(lap)
        if bc_x == 1 and bc_y == 0:
            return np.fft.fft(sfft.dct(lap, axis=0), axis=-1)
        raise NotImplementedError
    raise NotImplementedError


def _lap_t(T, dt, cdtype=np.complex128):
    """dl, du, Lap_t_diag of utils_precond.py:128-130 / :164-166 (Ct factor applied by caller).
    cdtype: complex128 as the reference; complex64 when the oracle is run in float32 (test calibration)."""
    dl = -np.pad(1 / (dt * dt) * np.ones((T - 1,)), (1, 0))
    du = -np.pad(1 / (dt * dt) * np.ones((T - 1,)), (0, 1))
    diag = -np.array([-2 / (dt * dt)] * (T - 1) + [-1 / (dt * dt)])
    return dl.astype(cdtype), du.astype(cdtype), diag.astype(np.finfo(cdtype).dtype)


def _dtypes(a):
    """(real, complex) dtypes the preconditioner computes in: float64 / complex128 as the reference, or
    float32 / complex64 for a float32 input (the float32 run of this oracle calibrates fp32 test bounds)."""
    return (np.float32, np.complex64) if a.dtype == np.float32 else (np.float64, np.complex128)


def H1_precond_1d(source_term, fv, dt, bc, C=1.0, pow=1, Ct=1):
    """(C - Dxx)^pow u - Ct Dtt u = source, u_0 = 0; utils_precond.py:105-140."""
    nt, nx = source_term.shape
    if bc != 0:
        raise NotImplementedError
    rdt, cdt = _dtypes(source_term)
    fv = np.asarray(fv).astype(cdt)
    v = sfft.fft(source_term[1:, :], axis=1, workers=_WORKERS)
    thomas_b = (np.broadcast_to(-fv, (nt - 1, nx)) + C) ** pow
    if Ct != 0:
        dl, du, diag = _lap_t(nt - 1, dt, cdt)
        dl, du = dl * Ct, du * Ct
        part = tridiagonal_solve(dl, thomas_b + diag[:, None] * Ct, du, v)
    else:
        part = v / thomas_b
    upd = sfft.ifft(part, axis=1, workers=_WORKERS).real
    return np.concatenate([np.zeros((1, nx), dtype=rdt), upd], axis=0)


def H1_precond_2d(source_term, fv, dt, bc, C=1.0):
    """C u - (Dtt + Dxx + Dyy) u = source, u_0 = 0; utils_precond.py:142-178."""
    nt, nx, ny = source_term.shape
    bc_x, bc_y = bc
    rdt, cdt = _dtypes(source_term)
    fv = np.asarray(fv).astype(cdt)
    if bc_x == 0 and bc_y == 0:
        v = sfft.fft2(source_term[1:], axes=(1, 2), workers=_WORKERS)
    elif bc_x == 1 and bc_y == 0:
        v = sfft.dct(source_term[1:], axis=1, workers=_WORKERS)
        v = sfft.fft(v, axis=2, workers=_WORKERS)
    else:
        raise NotImplementedError
    dl, du, diag = _lap_t(nt - 1, dt, cdt)
    thomas_b = np.broadcast_to(-fv, (nt - 1, nx, ny)) + diag[:, None, None] + C
    part = tridiagonal_solve(dl, thomas_b, du, v)
    if bc_x == 0 and bc_y == 0:
        upd = sfft.ifft2(part, axes=(1, 2), workers=_WORKERS).real
    else:
        upd = sfft.ifft(part, axis=2, workers=_WORKERS).real
        upd = sfft.idct(upd, axis=1, workers=_WORKERS)
    return np.concatenate([np.zeros((1, nx, ny), dtype=rdt), upd], axis=0)


# ---------------------------------------------------------------------------
# problem plugin  (jaxsrc/set_fns.py)
# ---------------------------------------------------------------------------

Functions = namedtuple("Functions", ["f_fn", "numerical_L_fn", "alp_update_fn"])


def set_up_J(egno, ndim, period_spatial):
    """Terminal cost J, set_fns.py:10-24."""
    if egno != 3:
        if ndim == 1:
            alpha = 2 * np.pi / period_spatial[0]
        elif ndim == 2:
            alpha = np.array([2 * np.pi / period_spatial[0], 2 * np.pi / period_spatial[1]])
        else:
            raise ValueError("ndim {} not implemented".format(ndim))
        return lambda x: np.sum(np.sin(alpha * x), axis=-1)
    _, y_period = period_spatial
    return lambda x: np.sin(2 * np.pi / y_period * x[..., 1]) * np.exp(-x[..., 0] ** 2 / 2)


def set_up_numerical_L(egno, n_ctrl, ind, fn_coeff_H):
    """set_fns.py:26-49."""
    if egno != 2:
        L1 = lambda alp, x, t: alp[..., 0] ** 2 / fn_coeff_H(x, t)[..., 0] / 2
        L2 = lambda alp, x, t: np.sum(alp ** 2 / fn_coeff_H(x, t), axis=-1) / 2
    else:
        L1 = lambda alp, x, t: 0.0 * alp[..., 0]
        L2 = lambda alp, x, t: 0.0 * alp[..., 0]
    if ind != 0:
        raise ValueError("ind {} not implemented".format(ind))
    if n_ctrl == 1:
        return lambda alp, x, t: L1(alp[0], x, t) + L1(alp[1], x, t)
    if n_ctrl == 2:
        return lambda alp, x, t: L2(alp[0], x, t) + L2(alp[1], x, t) + L2(alp[2], x, t) + L2(alp[3], x, t)
    raise ValueError("n_ctrl {} not implemented".format(n_ctrl))


def set_up_example_fns(egno, ndim, numerical_L_ind):
    """Examples egno 1/2/3, set_fns.py:52-166."""
    if egno == 1:
        def base(alp_prev, Dphi, p, cf, cH):        # set_fns.py:63-77
            return (Dphi[..., None] * cf + p * alp_prev) / (1 / cH + p)
    elif egno == 2:
        def base(alp_prev, Dphi, p, cf, cH):        # set_fns.py:79-95
            a = Dphi[..., None] * cf / p + alp_prev
            return np.minimum(cH, np.maximum(-cH, a))
    if egno == 3:                                    # set_fns.py:96-111
        n_ctrl = 1

        def f_fn(alp, x, t):
            xb = np.broadcast_to(x[..., 0:1], alp.shape[:-1] + (1,))
            return np.concatenate([alp, xb], axis=-1)
        cH_fn = lambda x, t: np.ones_like(x[..., 0:1])
        L_fn = set_up_numerical_L(egno, n_ctrl, numerical_L_ind, cH_fn)

        def alp_update_fn(alp_prev, Dphi, rho, sigma, x, t):
            a1x, a2x, a1y, a2y = alp_prev
            DxR, DxL, _, _ = Dphi
            p = (rho[..., None] + 1e-4) / sigma
            cL = 1 / cH_fn(x, t)
            n1 = (-DxR[..., None] + p * a1x) / (cL + p)
            n1 = n1 * (f_fn(n1, x, t)[..., 0:1] >= 0.0)
            n2 = (-DxL[..., None] + p * a2x) / (cL + p)
            n2 = n2 * (f_fn(n2, x, t)[..., 0:1] < 0.0)
            return (n1, n2, a1y, a2y)
    elif ndim == 2:                                  # set_fns.py:112-139
        n_ctrl = ndim
        cf1_fn = lambda x, t: np.concatenate([(x[..., 0:1] - 1.0) ** 2 + 0.1, np.zeros_like(x[..., 0:1])], axis=-1)
        cf2_fn = lambda x, t: np.concatenate([np.zeros_like(x[..., 0:1]), (x[..., 1:2] - 1.0) ** 2 + 0.1], axis=-1)
        cH_fn = lambda x, t: np.ones_like(x)

        def f_fn(alp, x, t):
            return -np.concatenate([np.sum(cf1_fn(x, t) * alp, axis=-1, keepdims=True),
                                    np.sum(cf2_fn(x, t) * alp, axis=-1, keepdims=True)], axis=-1)
        L_fn = set_up_numerical_L(egno, n_ctrl, numerical_L_ind, cH_fn)

        def alp_update_fn(alp_prev, Dphi, rho, sigma, x, t):
            a1x, a2x, a1y, a2y = alp_prev
            DxR, DxL, DyR, DyL = Dphi
            p = (rho[..., None] + 1e-4) / sigma
            cf1, cf2, cH = cf1_fn(x, t), cf2_fn(x, t), cH_fn(x, t)
            n1x = base(a1x, DxR, p, cf1, cH)
            n1x = n1x * (f_fn(n1x, x, t)[..., 0:1] >= 0.0)
            n2x = base(a2x, DxL, p, cf1, cH)
            n2x = n2x * (f_fn(n2x, x, t)[..., 0:1] < 0.0)
            n1y = base(a1y, DyR, p, cf2, cH)
            n1y = n1y * (f_fn(n1y, x, t)[..., 1:2] >= 0.0)
            n2y = base(a2y, DyL, p, cf2, cH)
            n2y = n2y * (f_fn(n2y, x, t)[..., 1:2] < 0.0)
            return (n1x, n2x, n1y, n2y)
    elif ndim == 1:                                  # set_fns.py:140-160
        n_ctrl = ndim
        cf_fn = lambda x, t: (x - 1.0) ** 2 + 0.1
        cH_fn = lambda x, t: np.ones_like(x)
        f_fn = lambda alp, x, t: -alp * cf_fn(x, t)
        L_fn = set_up_numerical_L(egno, n_ctrl, numerical_L_ind, cH_fn)

        def alp_update_fn(alp_prev, DxR, DxL, rho, sigma, x, t):
            a1, a2 = alp_prev
            p = ((rho + 1e-4) / sigma)[..., None]
            cf, cH = cf_fn(x, t), cH_fn(x, t)
            n1 = base(a1, DxR, p, cf, cH)
            n1 = n1 * (f_fn(n1, x, t) >= 0.0)
            n2 = base(a2, DxL, p, cf, cH)
            n2 = n2 * (f_fn(n2, x, t) < 0.0)
            return (n1, n2)
    else:
        raise ValueError("egno {} not implemented".format(egno))
    return Functions(f_fn=f_fn, numerical_L_fn=L_fn, alp_update_fn=alp_update_fn)


# ---------------------------------------------------------------------------
# PDHG updates  (jaxsrc/update_fns_in_pdhg.py)
# ---------------------------------------------------------------------------


def get_f_vals_1d(f_fn, alp, x_arr, t_arr):          # update_fns_in_pdhg.py:13-27
    a1, a2 = alp
    f1 = f_fn(a1, x_arr, t_arr)[..., 0]
    f1 = f1 * (f1 >= 0.0)
    f2 = f_fn(a2, x_arr, t_arr)[..., 0]
    f2 = f2 * (f2 < 0.0)
    return f1, f2


def get_f_vals_2d(f_fn, alp, x_arr, t_arr):          # update_fns_in_pdhg.py:29-47
    a1x, a2x, a1y, a2y = alp
    f1x = f_fn(a1x, x_arr, t_arr)[..., 0]
    f1x = f1x * (f1x >= 0.0)
    f2x = f_fn(a2x, x_arr, t_arr)[..., 0]
    f2x = f2x * (f2x < 0.0)
    f1y = f_fn(a1y, x_arr, t_arr)[..., 1]
    f1y = f1y * (f1y >= 0.0)
    f2y = f_fn(a2y, x_arr, t_arr)[..., 1]
    f2y = f2y * (f2y < 0.0)
    return f1x, f2x, f1y, f2y


def compute_HJ_residual_1d(phi, alp, dt, dspatial, fns_dict, epsl, x_arr, t_arr, bc):   # :49-56
    dx = dspatial[0]
    L = fns_dict.numerical_L_fn(alp, x_arr, t_arr)
    f1, f2 = get_f_vals_1d(fns_dict.f_fn, alp, x_arr, t_arr)
    vec = Dt_decreasedim(phi, dt) - epsl * Dxx_decreasedim(phi, dx, bc)
    vec = vec - (Dx_right_decreasedim(phi, dx, bc) * f1 + Dx_left_decreasedim(phi, dx, bc) * f2)
    return vec - L


def compute_HJ_residual_2d(phi, alp, dt, dspatial, fns_dict, epsl, x_arr, t_arr, bc):   # :58-70
    dx, dy = dspatial
    bcx, bcy = bc
    L = fns_dict.numerical_L_fn(alp, x_arr, t_arr)
    DxR = Dx_right_decreasedim(phi, dx, bcx)
    DxL = Dx_left_decreasedim(phi, dx, bcx)
    DyR = Dy_right_decreasedim(phi, dy, bcy)
    DyL = Dy_left_decreasedim(phi, dy, bcy)
    f1x, f2x, f1y, f2y = get_f_vals_2d(fns_dict.f_fn, alp, x_arr, t_arr)
    vec = Dt_decreasedim(phi, dt) - epsl * Dxx_decreasedim(phi, dx, bcx) - epsl * Dyy_decreasedim(phi, dy, bcy)
    vec = vec - (DxR * f1x + DxL * f2x + DyR * f1y + DyL * f2y)
    return vec - L


def compute_cont_residual_1d(rho, alp, dt, dspatial, fns_dict, c_on_rho, epsl, x_arr, t_arr, bc):   # :72-81
    dx = dspatial[0]
    f1, f2 = get_f_vals_1d(fns_dict.f_fn, alp, x_arr, t_arr)
    m1 = (rho + 1e-4) * f1
    m2 = (rho + 1e-4) * f2
    res = Dt_increasedim(rho, dt) + epsl * Dxx_increasedim(rho, dx, bc)
    res = res - (Dx_left_increasedim(m1, dx, bc) + Dx_right_increasedim(m2, dx, bc))
    res[-1] = res[-1] + c_on_rho / dt
    return res


def compute_cont_residual_2d(rho, alp, dt, dspatial, fns_dict, c_on_rho, epsl, x_arr, t_arr, bc):   # :83-96
    dx, dy = dspatial
    bcx, bcy = bc
    f1x, f2x, f1y, f2y = get_f_vals_2d(fns_dict.f_fn, alp, x_arr, t_arr)
    m1x, m2x = (rho + 1e-4) * f1x, (rho + 1e-4) * f2x
    m1y, m2y = (rho + 1e-4) * f1y, (rho + 1e-4) * f2y
    res = Dt_increasedim(rho, dt) + epsl * Dxx_increasedim(rho, dx, bcx) + epsl * Dyy_increasedim(rho, dy, bcy)
    res = res - (Dx_left_increasedim(m1x, dx, bcx) + Dx_right_increasedim(m2x, dx, bcx)
                 + Dy_left_increasedim(m1y, dy, bcy) + Dy_right_increasedim(m2y, dy, bcy))
    res[-1] = res[-1] + c_on_rho / dt
    return res


def update_rho_1d(rho_prev, phi, alp, sigma, dt, dspatial, epsl, fns_dict, x_arr, t_arr, bc):   # :99-103
    vec = compute_HJ_residual_1d(phi, alp, dt, dspatial, fns_dict, epsl, x_arr, t_arr, bc)
    return np.maximum(rho_prev + sigma * vec, 0.0)


def update_alp_1d(alp_prev, phi, rho, sigma, dspatial, fns_dict, x_arr, t_arr, bc):   # :105-113
    dx = dspatial[0]
    return fns_dict.alp_update_fn(alp_prev, Dx_right_decreasedim(phi, dx, bc), Dx_left_decreasedim(phi, dx, bc),
                                  rho, sigma, x_arr, t_arr)


def update_rho_2d(rho_prev, phi, alp, sigma, dt, dspatial, epsl, fns_dict, x_arr, t_arr, bc):   # :115-119
    vec = compute_HJ_residual_2d(phi, alp, dt, dspatial, fns_dict, epsl, x_arr, t_arr, bc)
    return np.maximum(rho_prev + sigma * vec, 0.0)


def update_alp_2d(alp_prev, phi, rho, sigma, dspatial, fns_dict, x_arr, t_arr, bc):   # :121-133
    dx, dy = dspatial
    bcx, bcy = bc
    Dphi = (Dx_right_decreasedim(phi, dx, bcx), Dx_left_decreasedim(phi, dx, bcx),
            Dy_right_decreasedim(phi, dy, bcy), Dy_left_decreasedim(phi, dy, bcy))
    return fns_dict.alp_update_fn(alp_prev, Dphi, rho, sigma, x_arr, t_arr)


def update_primal_1d(phi_prev, rho_prev, c_on_rho, alp_prev, tau, dt, dspatial, fns_dict, fv, epsl, x_arr, t_arr, bc,
                     C=1.0, pow=1, Ct=1):        # update_fns_in_pdhg.py:135-140
    delta = compute_cont_residual_1d(rho_prev, alp_prev, dt, dspatial, fns_dict, c_on_rho, epsl, x_arr, t_arr, bc)
    return phi_prev + tau * H1_precond_1d(delta, fv, dt, bc, C=C, pow=pow, Ct=Ct)


def update_primal_2d(phi_prev, rho_prev, c_on_rho, alp_prev, tau, dt, dspatial, fns_dict, fv, epsl, x_arr, t_arr, bc,
                     C=1.0, pow=1, Ct=1):        # update_fns_in_pdhg.py:142-147 (pow, Ct ignored)
    delta = compute_cont_residual_2d(rho_prev, alp_prev, dt, dspatial, fns_dict, c_on_rho, epsl, x_arr, t_arr, bc)
    return phi_prev + tau * H1_precond_2d(delta, fv, dt, bc, C=C)


def update_dual_oneiter(phi_bar, rho_prev, c_on_rho, alp_prev, sigma, dt, dspatial, epsl, x_arr, t_arr, bc,
                        fns_dict, ndim):          # update_fns_in_pdhg.py:150-165
    if ndim == 1:
        ua, ur = update_alp_1d, update_rho_1d
    elif ndim == 2:
        ua, ur = update_alp_2d, update_rho_2d
    else:
        raise NotImplementedError
    alp_next = ua(alp_prev, phi_bar, rho_prev, sigma, dspatial, fns_dict, x_arr, t_arr, bc)
    rho_next = ur(rho_prev, phi_bar, alp_next, sigma, dt, dspatial, epsl, fns_dict, x_arr, t_arr, bc)
    with np.errstate(divide="ignore", invalid="ignore"):
        err = np.sum((rho_next - rho_prev) ** 2) / np.sum(rho_next ** 2)
        for a_p, a_n in zip(alp_prev, alp_next):
            err += np.sum((a_n - a_p) ** 2) / np.sum(a_n ** 2)
    return rho_next, alp_next, err


def update_dual_alternative(phi_bar, rho_prev, c_on_rho, alp_prev, sigma, dt, dspatial, epsl, fns_dict, x_arr, t_arr,
                            ndim, bc, rho_alp_iters=10, eps=1e-7, stats=None):   # update_fns_in_pdhg.py:167-180
    for j in range(rho_alp_iters):
        rho_next, alp_next, err = update_dual_oneiter(phi_bar, rho_prev, c_on_rho, alp_prev, sigma, dt, dspatial,
                                                      epsl, x_arr, t_arr, bc, fns_dict, ndim)
        if err < eps:
            break
        rho_prev, alp_prev = rho_next, alp_next
    if stats is not None:
        stats.append(j + 1)
    return rho_next, alp_next


# ---------------------------------------------------------------------------
# drivers  (jaxsrc/utils/utils_pdhg_solver.py)
# ---------------------------------------------------------------------------


def outer_errors(phi_prev, phi_next, rho_prev, rho_next, alp_prev, alp_next):
    """err1, err2 of utils_pdhg_solver.py:58-68."""
    with np.errstate(divide="ignore", invalid="ignore"):
        err1 = np.linalg.norm(phi_next - phi_prev) / np.linalg.norm(phi_prev)
        err2 = np.linalg.norm(rho_next - rho_prev) / np.linalg.norm(rho_prev)
        for a_p, a_n in zip(alp_prev, alp_next):
            na = np.linalg.norm(a_p)
            ne = np.linalg.norm(a_p - a_n)
            if na < 1e-6 and ne > 1e-6:
                err2 += ne
            elif na >= 1e-6:
                err2 += ne / na
    return err1, err2


def PDHG_solver_oneiter(fn_update_primal, fn_update_dual, fns_dict, phi0, rho0, alp0, x_arr, t_arr, ndim, dt,
                        dspatial, c_on_rho, epsl=0.0, stepsz_param=0.9, fv=None, N_maxiter=1000000, print_freq=1000,
                        eps=1e-6, verbose=False):
    """Outer PDHG loop, utils_pdhg_solver.py:9-94 (tensorboard branch dropped)."""
    phi_prev, rho_prev, alp_prev = phi0, rho0, alp0
    scale = 1.5
    tau_phi = stepsz_param / scale
    tau_rho = stepsz_param * scale
    error_all, results_all = [], []
    for i in range(N_maxiter):
        phi_next = fn_update_primal(phi_prev, rho_prev, c_on_rho, alp_prev, tau_phi, dt, dspatial, fns_dict, fv,
                                    epsl, x_arr, t_arr)
        phi_bar = 2 * phi_next - phi_prev
        rho_next, alp_next = fn_update_dual(phi_bar, rho_prev, c_on_rho, alp_prev, tau_rho, dt, dspatial, epsl,
                                            fns_dict, x_arr, t_arr, ndim, eps=eps)
        err1, err2 = outer_errors(phi_prev, phi_next, rho_prev, rho_next, alp_prev, alp_next)
        error = np.array([err1, err2])
        if error[0] < eps and error[1] < eps:
            if verbose:
                print("PDHG converges at iter {}".format(i), flush=True)
            break
        if np.any(np.isnan(phi_next)) or np.any(np.isnan(rho_next)):
            if verbose:
                print("Nan error at iter {}".format(i))
            break
        if print_freq > 0 and i % print_freq == 0:
            results_all.append((i, phi_prev, rho_prev, alp_next))
            error_all.append(error)
            if verbose:
                print("iteration {}, primal error {:.2E}, dual error {:.2E}, min rho {:.2f}, max rho {:.2f}".format(
                    i, error[0], error[1], np.min(rho_next), np.max(rho_next)), flush=True)
        phi_prev, rho_prev, alp_prev = phi_next, rho_next, alp_next
    results_all.append((i + 1, phi_next, rho_next, alp_next))
    error_all.append(error)
    return results_all, np.array(error_all)


def PDHG_multi_step(fn_update_primal, fn_update_dual, fns_dict, g, x_arr, ndim, nt, nspatial, dt, dspatial, c_on_rho,
                    time_step_per_PDHG=2, epsl=0.0, stepsz_param=0.9, n_ctrl=None, fv=None, N_maxiter=1000000,
                    print_freq=1000, eps=1e-6, verbose=False, stats=None):
    """Time-window marching with NaN step back-off, utils_pdhg_solver.py:97-225 (no checkpoint resume).
    stats (test bookkeeping, not in the reference): a list that receives {"window", "window_iters", "stepsz"}
    per solved window, as the device driver's."""
    if n_ctrl is None:
        n_ctrl = ndim
    assert (nt - 1) % (time_step_per_PDHG - 1) == 0
    nt_PDHG = (nt - 1) // (time_step_per_PDHG - 1)
    phi0 = np.concatenate([g] * time_step_per_PDHG, axis=0)
    T = time_step_per_PDHG - 1
    if ndim == 1:
        nx = nspatial[0]
        rho0 = np.zeros([T, nx]) + c_on_rho
        alp0 = tuple(np.zeros([T, nx, n_ctrl]) for _ in range(2))
    else:
        nx, ny = nspatial
        rho0 = np.zeros([T, nx, ny]) + c_on_rho
        alp0 = tuple(np.zeros([T, nx, ny, n_ctrl]) for _ in range(4))
    max_iters = 0
    phi_all, rho_all, alp_all, errs_all = [], [], [], []
    s_min = stepsz_param / 10
    s_delta = stepsz_param / 10
    sol_nan = False
    for i in range(nt_PDHG):
        t_arr = np.linspace(i * dt * T, (i + 1) * dt * T, num=time_step_per_PDHG)[1:]
        t_arr = t_arr[:, None] if ndim == 1 else t_arr[:, None, None]
        while True:
            results_all, errs = PDHG_solver_oneiter(fn_update_primal, fn_update_dual, fns_dict, phi0, rho0, alp0,
                                                    x_arr, t_arr, ndim, dt, dspatial, c_on_rho, epsl=epsl,
                                                    stepsz_param=stepsz_param, fv=fv, N_maxiter=N_maxiter,
                                                    print_freq=print_freq, eps=eps, verbose=verbose)
            if np.any(np.isnan(errs)):
                if stepsz_param > s_min + s_delta:
                    stepsz_param -= s_delta
                else:
                    sol_nan = True
                    break
            else:
                iters, phi_c, rho_c, alp_c = results_all[-1]
                max_iters = max(max_iters, iters)
                if stats is not None:
                    stats.append({"window": i, "window_iters": iters, "stepsz": stepsz_param})
                phi_all.append(phi_c[:-1] if i < nt_PDHG - 1 else phi_c)
                rho_all.append(rho_c)
                alp_all.append(np.stack(alp_c, axis=0))
                errs_all.append(errs)
                g_diff = phi_c[-1:] - phi0[0:1]
                phi0 = phi0 + g_diff
                rho0, alp0 = rho_c, alp_c
                break
        if sol_nan:
            break
    phi_out = np.concatenate(phi_all, axis=0)
    rho_out = np.concatenate(rho_all, axis=0)
    alp_out = np.concatenate(alp_all, axis=1)
    return [(max_iters, phi_out, rho_out, alp_out)], errs_all


# ---------------------------------------------------------------------------
# solve_HJ wiring  (jaxsrc/run_example.py:157-210, grid :273-287)
# ---------------------------------------------------------------------------


def make_grid(ndim, nx, ny, egno, x_period=2.0, y_period=2.0):
    """x_arr as run_example.py:273-287 ([1,nx,1] or [1,nx,ny,2])."""
    centered = egno == 3
    if ndim == 1:
        x = np.linspace(0.0, x_period, num=nx, endpoint=False)
        if centered:
            x = x - x_period / 2
        return x[None, :, None]
    x1 = np.linspace(0.0, x_period, num=nx, endpoint=False)
    x2 = np.linspace(0.0, y_period, num=ny, endpoint=False)
    if centered:
        x1, x2 = x1 - x_period / 2, x2 - y_period / 2
    xm, ym = np.meshgrid(x1, x2, indexing="ij")
    return np.stack([xm, ym], axis=-1)[None]


def default_bc(egno, ndim):
    """run_example.py:229-240."""
    if egno == 3:
        return (1, 0)
    return 0 if ndim == 1 else (0, 0)


def make_update_fns(ndim, bc, C=1.0, pow=1.0, Ct=1.0, rho_alp_iters=10, dual_stats=None):
    """The fn_update_primal / fn_update_dual lambdas of run_example.py:192-203."""
    if ndim == 1:
        def primal(phi, rho, c, alp, tau, dt, ds, fns, fv, epsl, x, t):
            return update_primal_1d(phi, rho, c, alp, tau, dt, ds, fns, fv, epsl, x, t, bc, C=C, pow=pow, Ct=Ct)
    else:
        def primal(phi, rho, c, alp, tau, dt, ds, fns, fv, epsl, x, t):
            return update_primal_2d(phi, rho, c, alp, tau, dt, ds, fns, fv, epsl, x, t, bc, C=C, pow=pow, Ct=Ct)

    def dual(phi_bar, rho, c, alp, sigma, dt, ds, epsl, fns, x, t, nd, eps):
        return update_dual_alternative(phi_bar, rho, c, alp, sigma, dt, ds, epsl, fns, x, t, nd, bc,
                                       rho_alp_iters=rho_alp_iters, eps=eps, stats=dual_stats)
    return primal, dual


def solve_HJ(ndim, egno, epsl, nx, ny, nt, time_step_per_PDHG=2, stepsz_param=0.1, N_maxiter=1000000,
             print_freq=10000, eps=1e-6, c_on_rho=70.0, x_period=2.0, y_period=2.0, T=1.0, C=1.0, pow=1.0, Ct=1.0,
             verbose=False):
    """run_example.py:157-210 with the defaults of :403-440."""
    dt = T / (nt - 1)
    dx = x_period / nx
    dy = y_period / ny
    bc = default_bc(egno, ndim)
    n_ctrl = 1 if egno == 3 else ndim
    if ndim == 1:
        period, dspatial, nspatial = (x_period,), (dx,), (nx,)
    else:
        period, dspatial, nspatial = (x_period, y_period), (dx, dy), (nx, ny)
    fns = set_up_example_fns(egno, ndim, 0)
    x_arr = make_grid(ndim, nx, ny, egno, x_period, y_period)
    g = set_up_J(egno, ndim, period)(x_arr)
    fv = compute_Dxx_fft_fv(ndim, nspatial, dspatial, bc)
    primal, dual = make_update_fns(ndim, bc, C, pow, Ct)
    return PDHG_multi_step(primal, dual, fns, g, x_arr, ndim, nt, nspatial, dt, dspatial, c_on_rho,
                           time_step_per_PDHG=time_step_per_PDHG, epsl=epsl, stepsz_param=stepsz_param, n_ctrl=n_ctrl,
                           fv=fv, N_maxiter=N_maxiter, print_freq=print_freq, eps=eps, verbose=verbose)
