"""PDHGContext: one PDHG time window resident in HBM, driven through the C ABI.

This is the object behind the reference-shaped functions in
``update_fns_in_pdhg`` and ``utils_pdhg_solver``.  All arrays crossing this
boundary are float64 NumPy arrays in the reference's layouts
(``utils_pdhg_solver.py:18-24``):

* phi  ``[T+1, nx]``            or ``[T+1, nx, ny]``
* rho  ``[T, nx]``              or ``[T, nx, ny]``
* alp  tuple of 2 ``[T, nx, 1]`` or 4 ``[T, nx, ny, n_ctrl]`` arrays
"""
import ctypes

import numpy as np

from . import _native as N


class PDHGContext:
    def __init__(self, egno, ndim, nx, ny, T, dx, dy, dt, xs, ys=None, epsl=0.0, c_on_rho=70.0, bc=None,
                 C=1.0, pow=1.0, Ct=1.0, precision="fp32", rho_alp_iters=1, device=0):
        self._lib = N.load()
        if bc is None:
            bc = 0 if ndim == 1 else ((1, 0) if egno == 3 else (0, 0))
        bcx, bcy = (bc, 0) if ndim == 1 else tuple(bc)
        self.egno, self.ndim, self.nx, self.ny, self.T = int(egno), int(ndim), int(nx), int(ny if ndim == 2 else 1), int(T)
        self.n_ctrl = 1 if (ndim == 1 or egno == 3) else 2
        self.n_alp = 2 if ndim == 1 else 4
        self.precision = precision
        self._xs = np.ascontiguousarray(xs, dtype=np.float64).reshape(-1)
        self._ys = None if ndim == 1 else np.ascontiguousarray(ys, dtype=np.float64).reshape(-1)
        prob = N.pdhg_problem()
        prob.egno, prob.ndim, prob.bc_x, prob.bc_y = self.egno, self.ndim, int(bcx), int(bcy)
        prob.nx, prob.ny, prob.T = self.nx, self.ny, self.T
        prob.precision = {"fp32": 4, "fp64": 8, 4: 4, 8: 8}[precision]
        prob.rho_alp_iters = int(rho_alp_iters)
        prob.dx, prob.dy, prob.dt = float(dx), float(dy if ndim == 2 else 0.0), float(dt)
        prob.epsl, prob.c_on_rho = float(epsl), float(c_on_rho)
        prob.C, prob.pow_, prob.Ct = float(C), float(pow), float(Ct)
        prob.xs = N.dptr(self._xs)
        prob.ys = N.dptr(self._ys) if self._ys is not None else None
        self.rho_alp_iters = int(rho_alp_iters)
        self._prob = prob
        self._h = self._create(prob, int(device))
        self._version = 0         # bumped by every call that changes the device state
        self._resident = None     # (version, rho, alp): host arrays known to equal the device's rho / alp

    def _create(self, prob, device):
        h = ctypes.c_void_p()
        N.check(self._lib.pdhg_create(ctypes.byref(prob), device, ctypes.byref(h)))
        return h

    # ---- shapes ----
    @property
    def _space(self):
        return (self.nx,) if self.ndim == 1 else (self.nx, self.ny)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.pdhg_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- state ----
    def alp_block(self, alp):
        """The contiguous [n_alp, T, ...space, n_ctrl] block a tuple of control arrays views (get_state returns such
        views), or None: lets set_state / the marching driver skip a stacking copy."""
        b = getattr(alp[0], "base", None) if len(alp) else None
        shape = (self.n_alp, self.T) + self._space + (self.n_ctrl,)
        if not (isinstance(b, np.ndarray) and b.dtype == np.float64 and b.flags.c_contiguous and b.shape == shape
                and len(alp) == self.n_alp):
            return None
        p0 = b.__array_interface__["data"][0]
        for i, a in enumerate(alp):
            if a.base is not b or a.shape != shape[1:] or a.__array_interface__["data"][0] != p0 + i * b.strides[0]:
                return None
        return b

    def set_state(self, phi=None, rho=None, alp=None):
        """Upload the given parts of the state (reference layouts); a part passed as None keeps the device's values."""
        phi = None if phi is None else np.ascontiguousarray(phi, dtype=np.float64).reshape((self.T + 1,) + self._space)
        rho = None if rho is None else np.ascontiguousarray(rho, dtype=np.float64).reshape((self.T,) + self._space)
        if alp is not None:
            blk = self.alp_block(alp)
            if blk is None:
                blk = np.ascontiguousarray(np.stack([np.asarray(a, dtype=np.float64) for a in alp], axis=0))
            alp = blk.reshape((self.n_alp, self.T) + self._space + (self.n_ctrl,))
        self._version += 1
        N.check(self._lib.pdhg_set_state(self._h, N.dptr(phi), N.dptr(rho), N.dptr(alp)))

    def mark_resident(self, rho, alp):
        """rho / alp (host arrays the caller will not modify) equal the device's state now."""
        self._resident = (self._version, rho, tuple(alp))

    def is_resident(self, rho, alp):
        """True if rho / alp are the very arrays mark_resident recorded and the device state has not changed since."""
        r = self._resident
        return (r is not None and r[0] == self._version and rho is r[1] and alp is not None and
                len(alp) == len(r[2]) and all(a is b for a, b in zip(alp, r[2])))

    def get_state(self, phi=True, rho=True, alp=True):
        """(phi, rho, alp) from the device; a part passed as False is not copied and comes back as None."""
        phi = np.empty((self.T + 1,) + self._space) if phi else None
        rho = np.empty((self.T,) + self._space) if rho else None
        alp = np.empty((self.n_alp, self.T) + self._space + (self.n_ctrl,)) if alp else None
        N.check(self._lib.pdhg_get_state(self._h, N.dptr(phi), N.dptr(rho), N.dptr(alp)))
        return phi, rho, (None if alp is None else tuple(alp[i] for i in range(self.n_alp)))

    def get_rows(self, row0, nrows, phi=True, phi_bar=False, rho=True, alp=True):
        """Rows [row0, row0 + nrows) of (phi, phi_bar, rho, alp) in the reference layouts (pdhg_get_rows): for
        windows too large for a host copy of the whole state.  A part passed as False comes back as None."""
        sp = self._space
        f = lambda on: np.empty((nrows,) + sp) if on else None  # noqa: E731
        a = np.empty((self.n_alp, nrows) + sp + (self.n_ctrl,)) if alp else None
        ph, pb, rh = f(phi), f(phi_bar), f(rho)
        N.check(self._lib.pdhg_get_rows(self._h, int(row0), int(nrows), N.dptr(ph), N.dptr(pb), N.dptr(rh),
                                        N.dptr(a)))
        return ph, pb, rh, (None if a is None else tuple(a[i] for i in range(self.n_alp)))

    def get_phi_bar(self):
        pb = np.empty((self.T + 1,) + self._space)
        N.check(self._lib.pdhg_get_phi_bar(self._h, N.dptr(pb)))
        return pb

    def set_phi_bar(self, phi_bar):
        self._version += 1
        pb = np.ascontiguousarray(phi_bar, dtype=np.float64).reshape((self.T + 1,) + self._space)
        N.check(self._lib.pdhg_set_phi_bar(self._h, N.dptr(pb)))

    def init_state(self, g):
        g = np.ascontiguousarray(g, dtype=np.float64).reshape(self._space)
        self._version += 1
        N.check(self._lib.pdhg_init_state(self._h, N.dptr(g)))

    # ---- updates ----
    def update_primal(self, tau):
        self._version += 1
        N.check(self._lib.pdhg_update_primal(self._h, float(tau)))

    def update_dual(self, sigma, eps, rho_alp_iters):
        used = ctypes.c_int(0)
        self._version += 1
        N.check(self._lib.pdhg_update_dual(self._h, float(sigma), float(eps), int(rho_alp_iters), ctypes.byref(used)))
        return used.value

    def errors(self):
        e1, e2 = ctypes.c_double(), ctypes.c_double()
        N.check(self._lib.pdhg_errors(self._h, ctypes.byref(e1), ctypes.byref(e2)))
        return e1.value, e2.value

    def inner_error(self):
        e = ctypes.c_double()
        N.check(self._lib.pdhg_inner_error(self._h, ctypes.byref(e)))
        return e.value

    def iterate(self, n_iters, tau, sigma, eps, rho_alp_iters):
        st = N.pdhg_stats()
        self._version += 1
        N.check(self._lib.pdhg_iterate(self._h, int(n_iters), float(tau), float(sigma), float(eps),
                                       int(rho_alp_iters), ctypes.byref(st)))
        return {"iters_run": st.iters_run, "status": st.status, "inner_last": st.inner_last,
                "inner_total": st.inner_total, "err1": st.err1, "err2": st.err2, "err_inner": st.err_inner,
                "nan_seen": st.nan_seen, "first_nan_iter": st.first_nan_iter}

    def set_stop_rules(self, converge=True, nan=True):
        N.check(self._lib.pdhg_set_stop_rules(self._h, 1 if converge else 0, 1 if nan else 0))

    def synchronize(self):
        N.check(self._lib.pdhg_synchronize(self._h))

    # ---- measurement ----
    def device_bytes(self):
        b = ctypes.c_ulonglong()
        N.check(self._lib.pdhg_device_bytes(self._h, ctypes.byref(b)))
        return b.value

    def path_info(self, key):
        """Kernel variant selected for this context (pdhg_path_info): "fused_residual", "fast_rows",
        "fast_dual", "fast_xt"."""
        v = ctypes.c_int()
        N.check(self._lib.pdhg_path_info(self._h, key.encode(), ctypes.byref(v)))
        return v.value

    def profile_enable(self, on=True):
        N.check(self._lib.pdhg_profile_enable(self._h, 1 if on else 0))

    def profile_query(self, cls):
        ms, n = ctypes.c_double(), ctypes.c_int()
        N.check(self._lib.pdhg_profile_query(self._h, cls.encode(), ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def algorithmic_bytes(self, k, cls="iteration"):
        b = ctypes.c_double()
        N.check(self._lib.pdhg_algorithmic_bytes(self._h, int(k), cls.encode(), ctypes.byref(b)))
        return b.value
