"""MultiContext: one PDHG window over a list of devices, driven by the library's own host thread.

The C ABI's multi-device context (include/pdhg.h, ``pdhg_create_multi``; SURVEY.md 8(b)'s
``pdhg_create(prob, devices, ndev)``) splits the window's T rows into one t-slab per listed device and
runs the slab choreography natively (``csrc/pdhg_multi.hpp``: device-to-device plane copies over xGMI on
per-slab side streams, per-neighbour events, fixed-order sum folds), so a caller needs no communicator.
``pdhg_amd.slab`` is the one-process-per-GPU form of the same algorithm (RCCL through torch.distributed),
used by ``bench.py --gpus N``.  Arrays are the whole window in the reference layouts, as for PDHGContext.

The handle is a ``pdhg_multi*``, not a ``pdhg_ctx*``: this class therefore does not derive from
PDHGContext, and offers only the whole-window calls the multi-device ABI has (state, iterate, stop rules,
synchronize, info).  The library also rejects a foreign handle passed to a ``pdhg_ctx`` entry point.
"""
import ctypes

import numpy as np

from . import _native as N


class MultiContext:
    def __init__(self, egno, nx, ny, T, dx, dy, dt, xs, ys, devices=(0, 0), epsl=0.0, c_on_rho=70.0,
                 precision="fp32", rho_alp_iters=1):
        if precision not in ("fp32", "fp64", 4, 8):
            raise ValueError("precision must be fp32 or fp64")
        self._lib = N.load()
        self.egno, self.ndim, self.nx, self.ny, self.T = int(egno), 2, int(nx), int(ny), int(T)
        self.n_ctrl = 1 if egno == 3 else 2
        self.n_alp = 4
        self.rho_alp_iters = int(rho_alp_iters)
        self._xs = np.ascontiguousarray(xs, dtype=np.float64).reshape(-1)
        self._ys = np.ascontiguousarray(ys, dtype=np.float64).reshape(-1)
        bcx = 1 if egno == 3 else 0
        prob = N.pdhg_problem()
        prob.egno, prob.ndim, prob.bc_x, prob.bc_y = self.egno, 2, bcx, 0
        prob.nx, prob.ny, prob.T = self.nx, self.ny, self.T
        prob.precision = {"fp32": 4, "fp64": 8, 4: 4, 8: 8}[precision]   # fp64: the reference's arithmetic
        self.precision = precision
        prob.rho_alp_iters = self.rho_alp_iters
        prob.dx, prob.dy, prob.dt = float(dx), float(dy), float(dt)
        prob.epsl, prob.c_on_rho = float(epsl), float(c_on_rho)
        prob.C, prob.pow_, prob.Ct = 1.0, 1.0, 1.0
        prob.xs, prob.ys = N.dptr(self._xs), N.dptr(self._ys)
        self._prob = prob
        self._devices = (ctypes.c_int * len(devices))(*[int(d) for d in devices])
        self._ndev = len(devices)
        h = ctypes.c_void_p()
        N.check(self._lib.pdhg_create_multi(ctypes.byref(prob), self._devices, self._ndev, ctypes.byref(h)))
        self._h = h

    @property
    def _space(self):
        return (self.nx, self.ny)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.pdhg_multi_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_state(self, phi=None, rho=None, alp=None):
        phi = None if phi is None else np.ascontiguousarray(phi, dtype=np.float64).reshape((self.T + 1,) + self._space)
        rho = None if rho is None else np.ascontiguousarray(rho, dtype=np.float64).reshape((self.T,) + self._space)
        if alp is not None:
            alp = np.ascontiguousarray(np.stack([np.asarray(a, dtype=np.float64) for a in alp], axis=0))
            alp = alp.reshape((self.n_alp, self.T) + self._space + (self.n_ctrl,))
        N.check(self._lib.pdhg_multi_set_state(self._h, N.dptr(phi), N.dptr(rho), N.dptr(alp)))

    def init_state(self, g):
        """The reference initial state (phi = g on every row, rho = c_on_rho, alp = 0) on every slab."""
        g = np.ascontiguousarray(g, dtype=np.float64).reshape(self._space)
        N.check(self._lib.pdhg_multi_init_state(self._h, N.dptr(g)))

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

    def phase_ms(self, reset=True):
        """{phase: total ms} recorded on slab 0's streams since profiling was switched on
        (pdhg_multi_profile): per-phase cost of the slab choreography."""
        out = {}
        for key in ("residual", "forward", "backward", "allreduce", "dual", "outer", "step"):
            ms = ctypes.c_double()
            n = ctypes.c_int()
            N.check(self._lib.pdhg_multi_phase_ms(self._h, key.encode(), ctypes.byref(ms), ctypes.byref(n)))
            if n.value:
                out[key] = ms.value
        if reset:
            N.check(self._lib.pdhg_multi_profile(self._h, 1))
        return out

    def profile(self, on=True):
        N.check(self._lib.pdhg_multi_profile(self._h, 1 if on else 0))
