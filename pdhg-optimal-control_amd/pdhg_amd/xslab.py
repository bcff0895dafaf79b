"""x-slab decomposition of a PDHG window over P GPUs.

The reference's default marches windows of T = time_step_per_PDHG - 1 = 1 unknown rows
(run_example.py:425, utils_pdhg_solver.py:121-206): a t-slab (slab.py) cannot split those.  Here the
GLOBAL grid's nx rows are split into P contiguous slabs of nloc = nx / P rows, one XSlabContext (one GPU,
one process) each.  Every stencil of the residual and the dual reaches +-1 row in x, so a slab keeps one
ghost row on each side; the x transform of the H1 preconditioner (utils_precond.py:142-178) needs whole x
lines, so the y-transformed spectrum is transposed over the slabs (all-to-all), transformed and solved in
t per column block, and transposed back.  Per outer iteration (utils_pdhg_solver.py:51-88), over RCCL:

* allgather of the halo rows of rho and the controls (the continuity residual's x neighbours,
  update_fns_in_pdhg.py:83-96): 2 rows x (1 + 4) arrays x T x ny floats per slab;
* two all-to-alls of the spectrum (T x nloc x ny floats per slab each way);
* allgather of the phi_bar halo rows (the dual's x differences, update_fns_in_pdhg.py:150-165);
* allreduces of the 16-double sum vectors behind every stop test, exactly as the t-slab runner.

Local arrays (the context's set_state / get_state shapes) hold nx_local = nloc + 16 rows: row i is global
row (x0 - xl0 + i) mod nx, the live rows are [xl0, xl0 + nloc).  ``local_rows`` / ``live_rows`` convert.
"""
import ctypes

import numpy as np

from . import _native as N
from .context import PDHGContext
from .slab import DistComm, LocalComm, PhaseOps, _ptr  # noqa: F401  (communicators re-exported)

HALO_STATE, HALO_PHIBAR = 0, 1                     # pdhg_xslab_halo_out / _in
ROWS_OUT, COLS_IN, COLS_OUT, ROWS_IN = 0, 1, 2, 3   # pdhg_xslab_wire stages


class XSlabContext(PhaseOps, PDHGContext):
    """Slab `rank` of `nranks` of the global nx rows (2-D, bc (0,0) or egno 3's (1,0); precision "fp32", or "fp64" =
    the reference's arithmetic, jaxsrc/update_fns_in_pdhg.py:10, at ny = 2048 / 4096).  nx / xs describe the global
    grid.  Halo and wire buffers are in the slab's precision (plane_dtype)."""

    def __init__(self, rank, nranks, egno, nx, ny, T, dx, dy, dt, xs, ys, device=0, **kw):
        self.rank, self.nranks, self.nx_global = int(rank), int(nranks), int(nx)
        bc = kw.get("bc")
        self.bc_x = int((bc if bc is not None else ((1, 0) if egno == 3 else (0, 0)))[0])
        kw.setdefault("precision", "fp32")
        super().__init__(egno, 2, nx, ny, T, dx, dy, dt, xs, ys, device=device, **kw)
        x0, nloc, nxl, xl0 = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        N.check(self._lib.pdhg_xslab_layout(self._h, ctypes.byref(x0), ctypes.byref(nloc), ctypes.byref(nxl),
                                            ctypes.byref(xl0)))
        self.x0, self.nloc, self.xl0 = x0.value, nloc.value, xl0.value
        self.nx = nxl.value          # local arrays (set_state / get_state / init_state shapes)
        w, hs, hp = ctypes.c_ulonglong(), ctypes.c_ulonglong(), ctypes.c_ulonglong()
        N.check(self._lib.pdhg_xslab_sizes(self._h, ctypes.byref(w), ctypes.byref(hs), ctypes.byref(hp)))
        self.wire_size, self.halo_sizes = w.value, (hs.value, hp.value)

    def _create(self, prob, device):
        h = ctypes.c_void_p()
        N.check(self._lib.pdhg_create_xslab(ctypes.byref(prob), self.rank, self.nranks, device, ctypes.byref(h)))
        return h

    # ---- local <-> global rows (x is axis 1 of every state array) ----
    def row_index(self):
        """Global row of every local row (ghost and padding rows wrap periodically; Neumann x edges: clamped)."""
        g = self.x0 - self.xl0 + np.arange(self.nx)
        return np.clip(g, 0, self.nx_global - 1) if self.bc_x == 1 else g % self.nx_global

    def local_rows(self, a):
        return np.take(np.asarray(a), self.row_index(), axis=1)

    def live_rows(self, a):
        return np.asarray(a)[:, self.xl0:self.xl0 + self.nloc]

    def set_global_state(self, phi, rho, alp):
        self.set_state(self.local_rows(phi), self.local_rows(rho), tuple(self.local_rows(a) for a in alp))

    def init_global_state(self, g):
        self.init_state(np.asarray(g).reshape(self.nx_global, self.ny)[self.row_index()])

    # ---- phases ----
    def halo_out(self, which, dst):
        N.check(self._lib.pdhg_xslab_halo_out(self._h, int(which), _ptr(dst)))

    def halo_in(self, which, from_left, from_right):
        N.check(self._lib.pdhg_xslab_halo_in(self._h, int(which), _ptr(from_left), _ptr(from_right)))

    def residual(self):
        N.check(self._lib.pdhg_xslab_residual(self._h))

    def wire(self, stage, buf):
        N.check(self._lib.pdhg_xslab_wire(self._h, int(stage), _ptr(buf)))

    def precond(self):
        N.check(self._lib.pdhg_xslab_precond(self._h))

    def update(self, tau, sums):
        N.check(self._lib.pdhg_xslab_update(self._h, float(tau), _ptr(sums)))


class XSlabRunner:
    """Drives the x-slabs of this process through outer iterations (pdhg_iterate's loop, split at every
    exchange).  comm: LocalComm (P slabs in one process) or DistComm (one slab per rank)."""

    def __init__(self, slabs, comm):
        import torch
        self.torch = torch
        self.slabs, self.comm = list(slabs), comm
        dev = torch.device("cuda", torch.cuda.current_device())
        handle = torch.cuda.current_stream().cuda_stream
        f32 = self.slabs[0].plane_dtype   # halos and wires in the slabs' precision; sums fp64
        if any(s.plane_dtype != f32 for s in self.slabs):
            raise ValueError("slabs of one runner must share a precision")
        self.b = []
        for s in self.slabs:
            s.set_stream(handle)
            hs, hp = s.halo_sizes
            self.b.append({"send": torch.zeros(s.wire_size, dtype=f32, device=dev),
                           "recv": torch.zeros(s.wire_size, dtype=f32, device=dev),
                           "hs": torch.zeros(hs, dtype=f32, device=dev),
                           "hp": torch.zeros(hp, dtype=f32, device=dev),
                           "sums": torch.zeros(16, dtype=torch.float64, device=dev)})

    def _each(self, name, *args):
        for s in self.slabs:
            getattr(s, name)(*args)

    def _halo(self, which, key):
        S, B, C = self.slabs, self.b, self.comm
        for s, b in zip(S, B):
            s.halo_out(which, b[key])
        allh = C.allgather([b[key] for b in B])   # [P, n] per local slab
        return allh

    def _halo_in(self, which, allh):
        for i, s in enumerate(self.slabs):
            P, r = s.nranks, s.rank
            s.halo_in(which, allh[i][(r - 1) % P], allh[i][(r + 1) % P])

    def step(self, tau, sigma, eps, k):
        S, B, C = self.slabs, self.b, self.comm
        # rho / control halo rows -> residual + y-DHT of the local rows -> transpose -> x-DHT, t-solve,
        # inverse x-DHT per column block -> transpose back -> inverse y-DHT + update
        self._halo_in(HALO_STATE, self._halo(HALO_STATE, "hs"))
        for s, b in zip(S, B):
            s.residual()
            s.wire(ROWS_OUT, b["send"])
        C.alltoall([b["send"] for b in B], [b["recv"] for b in B])
        for s, b in zip(S, B):
            s.wire(COLS_IN, b["recv"])
            s.precond()
            s.wire(COLS_OUT, b["send"])
        C.alltoall([b["send"] for b in B], [b["recv"] for b in B])
        for s, b in zip(S, B):
            s.wire(ROWS_IN, b["recv"])
            s.update(tau, b["sums"])
        allp = self._halo(HALO_PHIBAR, "hp")
        C.allreduce([b["sums"] for b in B])
        for s, b in zip(S, B):
            s.primal_finalize(b["sums"])
        self._halo_in(HALO_PHIBAR, allp)
        # dual sub-iterations (device-side early exit once the global inner error is below eps)
        for sub in range(k):
            for s, b in zip(S, B):
                s.dual(sigma, k, sub, b["sums"], 3)
            C.allreduce([b["sums"] for b in B])
            for s, b in zip(S, B):
                s.dual_finalize(eps, sub, b["sums"])
        for s, b in zip(S, B):
            s.outer(k, b["sums"])
        if k > 1:
            C.allreduce([b["sums"] for b in B])
        for s, b in zip(S, B):
            s.outer_finalize(eps, k, b["sums"])

    def iterate(self, n, tau, sigma, eps, k, check_every=8):
        """Up to n outer iterations; stops when the device control block says done (checked every
        check_every iterations, like pdhg_iterate).  Returns the first slab's status dict."""
        self._each("begin")
        for it in range(n):
            self.step(tau, sigma, eps, k)
            if (it + 1) % check_every == 0 and it + 1 < n and self.slabs[0].status()["status"]:
                break
        return self.slabs[0].status()


def join_rows(slabs, parts):
    """Global arrays from the live rows of every slab's local arrays (slabs in rank order)."""
    return np.concatenate([s.live_rows(p) for s, p in zip(slabs, parts)], axis=1)


def multi_step_xslab(runner, g, nt, c_on_rho, time_step_per_PDHG=2, stepsz_param=0.1, N_maxiter=1000000, eps=1e-6,
                     rho_alp_iters=1, verbose=False):
    """PDHG_multi_step's window marching (utils_pdhg_solver.py:97-225) over x-slabs: warm starts
    (:193-206) and the NaN step-size back-off (:174-187), applied by every slab to its own rows (the
    hand-off is pointwise in x).  Returns, per local slab, (max_iters, phi [nt, nloc, ny], rho [nt-1, nloc, ny],
    alp [4, nt-1, nloc, ny, 2]) -- the live rows of the reference's result tuple -- and the per-window errors."""
    S = runner.slabs
    T = time_step_per_PDHG - 1
    assert (nt - 1) % T == 0
    nt_PDHG = (nt - 1) // T
    g = np.asarray(g, dtype=np.float64)
    loc = []
    for s in S:
        gl = g.reshape(s.nx_global, s.ny)[s.row_index()]
        phi0 = np.repeat(gl[None], time_step_per_PDHG, axis=0)
        rho0 = np.full((T, s.nx, s.ny), float(c_on_rho))
        alp0 = tuple(np.zeros((T, s.nx, s.ny, s.n_ctrl)) for _ in range(4))
        loc.append([phi0, rho0, alp0])
    out = [([], [], []) for _ in S]
    errs_all, max_iters = [], 0
    s_delta = s_min = stepsz_param / 10
    sol_nan = False
    for i in range(nt_PDHG):
        while True:
            for s, (phi0, rho0, alp0) in zip(S, loc):
                s.set_state(phi0, rho0, alp0)
            st = runner.iterate(N_maxiter, stepsz_param / 1.5, stepsz_param * 1.5, eps, rho_alp_iters)
            if st["status"] == 2:                          # NaN: back-off, utils_pdhg_solver.py:180-187
                if stepsz_param > s_min + s_delta:
                    stepsz_param -= s_delta
                    if verbose:
                        print("pdhg does not conv at t_ind = {}, decrease step size to {}".format(i, stepsz_param))
                    continue
                sol_nan = True
            break
        if sol_nan:
            if verbose:
                print("pdhg does not conv, please decrease stepsize to be less than {}".format(stepsz_param))
            break
        iters = st["iters"]
        max_iters = max(max_iters, iters)
        errs_all.append(np.array([[st["err1"], st["err2"]]]))
        for q, s in enumerate(S):
            phi_c, rho_c, alp_c = s.get_state()
            phi0, _, _ = loc[q]
            out[q][0].append(s.live_rows(phi_c[:-1] if i < nt_PDHG - 1 else phi_c))
            out[q][1].append(s.live_rows(rho_c))
            out[q][2].append(np.stack([s.live_rows(a) for a in alp_c], axis=0))
            loc[q] = [phi0 + (phi_c[-1:] - phi0[0:1]), rho_c, alp_c]
    res = [(max_iters, np.concatenate(o[0], axis=0), np.concatenate(o[1], axis=0), np.concatenate(o[2], axis=1))
           for o in out]
    return res, errs_all
