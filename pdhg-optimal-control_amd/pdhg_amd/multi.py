"""MultiContext: one PDHG window over a list of devices, driven by the library's own host thread.

The C ABI's multi-device context (include/pdhg.h, ``pdhg_create_multi``; SURVEY.md 8(b)'s
``pdhg_create(prob, devices, ndev)``) splits the window's T rows into one t-slab per listed device and
runs the slab choreography natively (``csrc/pdhg_multi.hpp``: device-to-device plane copies over xGMI,
fixed-order sum folds), so a caller needs no communicator.  ``pdhg_amd.slab`` is the one-process-per-GPU
form of the same algorithm (RCCL through torch.distributed), used by ``bench.py --gpus N``.
Arrays are the whole window in the reference layouts, as for PDHGContext.
"""
import ctypes

import numpy as np

from . import _native as N
from .context import PDHGContext


class MultiContext(PDHGContext):
    def __init__(self, egno, nx, ny, T, dx, dy, dt, xs, ys, devices=(0, 0), **kw):
        self._devices = (ctypes.c_int * len(devices))(*[int(d) for d in devices])
        self._ndev = len(devices)
        kw.setdefault("precision", "fp32")
        super().__init__(egno, 2, nx, ny, T, dx, dy, dt, xs, ys, **kw)

    def _create(self, prob, device):
        h = ctypes.c_void_p()
        N.check(self._lib.pdhg_create_multi(ctypes.byref(prob), self._devices, self._ndev, ctypes.byref(h)))
        return h

    def close(self):
        if getattr(self, "_h", None):
            self._lib.pdhg_multi_destroy(self._h)
            self._h = None

    def set_state(self, phi=None, rho=None, alp=None):
        phi = None if phi is None else np.ascontiguousarray(phi, dtype=np.float64).reshape((self.T + 1,) + self._space)
        rho = None if rho is None else np.ascontiguousarray(rho, dtype=np.float64).reshape((self.T,) + self._space)
        if alp is not None:
            alp = np.ascontiguousarray(np.stack([np.asarray(a, dtype=np.float64) for a in alp], axis=0))
            alp = alp.reshape((self.n_alp, self.T) + self._space + (self.n_ctrl,))
        N.check(self._lib.pdhg_multi_set_state(self._h, N.dptr(phi), N.dptr(rho), N.dptr(alp)))

    def get_state(self):
        phi = np.empty((self.T + 1,) + self._space)
        rho = np.empty((self.T,) + self._space)
        alp = np.empty((self.n_alp, self.T) + self._space + (self.n_ctrl,))
        N.check(self._lib.pdhg_multi_get_state(self._h, N.dptr(phi), N.dptr(rho), N.dptr(alp)))
        return phi, rho, tuple(alp[i] for i in range(self.n_alp))

    def iterate(self, n_iters, tau, sigma, eps, rho_alp_iters):
        st = N.pdhg_stats()
        N.check(self._lib.pdhg_multi_iterate(self._h, int(n_iters), float(tau), float(sigma), float(eps),
                                             int(rho_alp_iters), ctypes.byref(st)))
        return {"iters_run": st.iters_run, "status": st.status, "inner_last": st.inner_last,
                "inner_total": st.inner_total, "err1": st.err1, "err2": st.err2, "err_inner": st.err_inner,
                "nan_seen": st.nan_seen, "first_nan_iter": st.first_nan_iter}

    def set_stop_rules(self, converge=True, nan=True):
        N.check(self._lib.pdhg_multi_set_stop_rules(self._h, 1 if converge else 0, 1 if nan else 0))

    def synchronize(self):
        N.check(self._lib.pdhg_multi_synchronize(self._h))

    def info(self, key):
        v = ctypes.c_int()
        N.check(self._lib.pdhg_multi_info(self._h, key.encode(), ctypes.byref(v)))
        return v.value
