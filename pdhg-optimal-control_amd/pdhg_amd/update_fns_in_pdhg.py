"""Drop-in PDHG update functions with the reference signatures (jaxsrc/update_fns_in_pdhg.py).

Each call uploads its arguments to a cached device context, runs the HIP
kernels (no CPU fallback) and returns NumPy arrays, so code written against
the reference's jitted functions runs unchanged.  For speed use the
device-resident loop in ``utils_pdhg_solver`` instead: per-call use moves the
whole state over PCIe twice.

Precision: float64 by default, as the reference (jax_enable_x64, update_fns_in_pdhg.py:10), so a caller
swapping these in for the reference's functions gets its arithmetic; ``set_precision("fp32")`` (or
``make_update_fns(..., precision="fp32")``) selects the fp32 fast kernels the benchmark runs.
"""
import numpy as np

from .context import PDHGContext

_PRECISION = ["fp64"]
_CACHE = {}
_CACHE_MAX = 4


def set_precision(p):
    assert p in ("fp32", "fp64")
    _PRECISION[0] = p


def get_precision():
    return _PRECISION[0]


def _spec(fns_dict):
    spec = getattr(fns_dict, "spec", None)
    if not spec:
        raise NotImplementedError("fns_dict is not a built-in example from pdhg_amd.set_fns.set_up_example_fns; "
                                  "the device kernels implement egno 1/2/3 only")
    return spec


def grid_coords(x_arr, ndim):
    """x and y coordinate vectors from the reference's x_arr ([1,nx,1] or [1,nx,ny,2])."""
    x_arr = np.asarray(x_arr, dtype=np.float64)
    if ndim == 1:
        return x_arr.reshape(-1), None
    return x_arr[0, :, 0, 0].copy(), x_arr[0, 0, :, 1].copy()


def get_context(spec, T, space, dt, dspatial, epsl, x_arr, bc, C=1.0, pow=1.0, Ct=1.0, c_on_rho=70.0,
                rho_alp_iters=1, precision=None):
    precision = precision or _PRECISION[0]
    ndim = spec["ndim"]
    xs, ys = grid_coords(x_arr, ndim)
    bc_key = bc if ndim == 1 else tuple(bc)
    key = (spec["egno"], ndim, T, tuple(space), float(dt), tuple(float(d) for d in dspatial), float(epsl),
           bc_key, float(C), float(pow), float(Ct), float(c_on_rho), rho_alp_iters > 1, precision,
           xs.tobytes(), None if ys is None else ys.tobytes())
    ctx = _CACHE.get(key)
    if ctx is None:
        if len(_CACHE) >= _CACHE_MAX:
            _CACHE.pop(next(iter(_CACHE))).close()
        nx = space[0]
        ny = space[1] if ndim == 2 else 1
        dx = dspatial[0]
        dy = dspatial[1] if ndim == 2 else 0.0
        ctx = PDHGContext(spec["egno"], ndim, nx, ny, T, dx, dy, dt, xs, ys, epsl=epsl, c_on_rho=c_on_rho, bc=bc,
                          C=C, pow=pow, Ct=Ct, precision=precision, rho_alp_iters=max(1, rho_alp_iters))
        _CACHE[key] = ctx
    return ctx


def clear_cache():
    while _CACHE:
        _CACHE.popitem()[1].close()


# ---- f values (used by trajectory post-processing, run_example.py:10) ----
def get_f_vals_1d(f_fn, alp, x_arr, t_arr):               # update_fns_in_pdhg.py:13-27
    f1 = f_fn(alp[0], x_arr, t_arr)[..., 0]
    f2 = f_fn(alp[1], x_arr, t_arr)[..., 0]
    return f1 * (f1 >= 0.0), f2 * (f2 < 0.0)


def get_f_vals_2d(f_fn, alp, x_arr, t_arr):               # update_fns_in_pdhg.py:29-47
    out = []
    for a, comp, pos in ((alp[0], 0, True), (alp[1], 0, False), (alp[2], 1, True), (alp[3], 1, False)):
        f = f_fn(a, x_arr, t_arr)[..., comp]
        out.append(f * ((f >= 0.0) if pos else (f < 0.0)))
    return tuple(out)


# ---- the preconditioner's symbol ----
_FV_OK = [None]


def check_fv(fv, ndim, space, dspatial, bc):
    """The device kernels use the analytic Laplacian symbol of the reference's stencil (utils_precond.py:42-71;
    pdhg_amd.utils_precond.compute_Dxx_fft_fv).  A caller's fv that is not that symbol (up to the FFT's roundoff)
    would be silently replaced, where the reference would use it (update_fns_in_pdhg.py:139, 146): refuse it with
    PDHGUnsupported (NotImplementedError).  fv = None selects the analytic symbol."""
    if fv is None or _FV_OK[0] is fv:
        return
    from ._native import PDHGUnsupported
    from .utils_precond import compute_Dxx_fft_fv
    ref = compute_Dxx_fft_fv(ndim, tuple(space), tuple(dspatial), bc if ndim == 2 else 0)
    f = np.asarray(fv)
    if f.shape != ref.shape:
        f = np.broadcast_to(f, ref.shape) if f.size == 1 else f
    if f.shape != ref.shape or not np.all(np.abs(f - ref) <= 1e-9 * np.max(np.abs(ref)) + 1e-9):
        raise PDHGUnsupported(-2, "fv differs from the Laplacian symbol of the reference stencil "
                                  "(compute_Dxx_fft_fv, utils_precond.py:42-71); the device preconditioner "
                                  "implements that symbol only")
    _FV_OK[0] = fv


# ---- primal ----
def _primal(phi_prev, rho_prev, c_on_rho, alp_prev, tau, dt, dspatial, fns_dict, epsl, x_arr, bc, C, pow, Ct):
    spec = _spec(fns_dict)
    phi_prev = np.asarray(phi_prev, dtype=np.float64)
    T = phi_prev.shape[0] - 1
    ctx = get_context(spec, T, phi_prev.shape[1:], dt, dspatial, epsl, x_arr, bc, C, pow, Ct, c_on_rho)
    ctx.set_state(phi_prev, rho_prev, alp_prev)
    ctx.update_primal(tau)
    return ctx.get_state()[0]


def update_primal_1d(phi_prev, rho_prev, c_on_rho, alp_prev, tau, dt, dspatial, fns_dict, fv, epsl, x_arr, t_arr, bc,
                     C=1.0, pow=1, Ct=1):
    """phi + tau * H1^{-1} cont_residual (update_fns_in_pdhg.py:135-140); fv must be the stencil's symbol
    (check_fv), which the kernels form analytically."""
    check_fv(fv, 1, np.shape(phi_prev)[1:], dspatial, bc)
    return _primal(phi_prev, rho_prev, c_on_rho, alp_prev, tau, dt, dspatial, fns_dict, epsl, x_arr, bc, C, pow, Ct)


def update_primal_2d(phi_prev, rho_prev, c_on_rho, alp_prev, tau, dt, dspatial, fns_dict, fv, epsl, x_arr, t_arr, bc,
                     C=1.0, pow=1, Ct=1):
    """update_fns_in_pdhg.py:142-147 (pow and Ct are ignored in 2-D, as in the reference); fv as update_primal_1d."""
    check_fv(fv, 2, np.shape(phi_prev)[1:], dspatial, bc)
    return _primal(phi_prev, rho_prev, c_on_rho, alp_prev, tau, dt, dspatial, fns_dict, epsl, x_arr, bc, C, 1.0, 1.0)


# ---- dual ----
def _dual(phi_bar, rho_prev, c_on_rho, alp_prev, sigma, dt, dspatial, epsl, fns_dict, x_arr, bc, iters, eps):
    spec = _spec(fns_dict)
    phi_bar = np.asarray(phi_bar, dtype=np.float64)
    T = phi_bar.shape[0] - 1
    ctx = get_context(spec, T, phi_bar.shape[1:], dt, dspatial, epsl, x_arr, bc, c_on_rho=c_on_rho,
                      rho_alp_iters=iters)
    ctx.set_state(None, rho_prev, alp_prev)
    ctx.set_phi_bar(phi_bar)
    used = ctx.update_dual(sigma, eps, iters)
    _, rho, alp = ctx.get_state()
    return rho, alp, used, ctx


def update_dual_oneiter(phi_bar, rho_prev, c_on_rho, alp_prev, sigma, dt, dspatial, epsl, x_arr, t_arr, bc, fns_dict,
                        ndim):
    """One alpha/rho prox step and its error (update_fns_in_pdhg.py:150-165)."""
    rho, alp, _, ctx = _dual(phi_bar, rho_prev, c_on_rho, alp_prev, sigma, dt, dspatial, epsl, fns_dict, x_arr, bc,
                             1, -np.inf)
    return rho, alp, ctx.inner_error()


def update_dual_alternative(phi_bar, rho_prev, c_on_rho, alp_prev, sigma, dt, dspatial, epsl, fns_dict, x_arr, t_arr,
                            ndim, bc, rho_alp_iters=10, eps=1e-7):
    """<= rho_alp_iters sub-iterations with early exit at err < eps (update_fns_in_pdhg.py:167-180)."""
    rho, alp, _, _ = _dual(phi_bar, rho_prev, c_on_rho, alp_prev, sigma, dt, dspatial, epsl, fns_dict, x_arr, bc,
                           rho_alp_iters, eps)
    return rho, alp
