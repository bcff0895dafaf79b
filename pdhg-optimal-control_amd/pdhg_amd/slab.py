"""t-slab decomposition of one PDHG window over P GPUs.

The reference runs one window on one device (README.md:6; utils_pdhg_solver.py:51-88).  Here the T
unknown time rows of a window are split into P contiguous slabs, one SlabContext (one GPU, one
process) each; whole x-y planes stay local, so every FFT stays local.  Per outer iteration a slab
exchanges, over RCCL on xGMI:

* halos, point to point: rho row j1 from the next slab (the continuity residual's rho_{j+1},
  update_fns_in_pdhg.py:83-96) and phi_bar row j0 from the previous slab (the dual's phi_bar_j,
  :150-165), one plane each, moved on a second stream (over RCCL: on a communicator of their own)
  while the rows that do not read the halo are computed;
* the distributed t-solve of the H1 preconditioner (utils_precond.py:142-178): ONE allgather per
  iteration of two spectral planes per slab (D = the zero-carry forward sweep's last row, S1 =
  sum P'_k b0_k); every slab folds the upstream carry and the downstream X0 values itself
  (oracle/slab_oracle.py restates the algebra and pins it against the monolithic solve);
* allreduces of the 16-double sum vectors behind every stop test (the err of
  update_dual_alternative, err1/err2 of utils_pdhg_solver.py:58-68), so every slab takes the same
  control decisions on its device.

Communicators: DistComm (torch.distributed, one slab per rank: "nccl" = RCCL on the GPUs, "gloo" on
CPU tensors) and LocalComm (P slabs in one process on one device -- the single-GPU rehearsal and the
parity tests; its collectives are copies).
"""
import ctypes

import numpy as np

from . import _native as N
from .context import PDHGContext

RHO_ROW0, PHIBAR_LAST, CARRY_DS, CARRY_LONG = 0, 1, 2, 3   # pdhg_slab_plane_out
RHO_HALO, PHIBAR_ROW0 = 0, 1                             # pdhg_slab_plane_in
INTERIOR, EDGE = 1, 2                                    # pdhg_slab_residual / pdhg_slab_dual parts
LONG_RANGE_DELTA = 2.0 ** -40     # modes whose slab gains are all below this exchange with neighbours only


def slab_bounds(T, P):
    """Contiguous near-equal row ranges [(j0, j1)] of T rows over P slabs (the first T % P get one more)."""
    if P < 1 or P > T:
        raise ValueError("need 1 <= P <= T (P={}, T={})".format(P, T))
    base, extra = divmod(T, P)
    out, j = [], 0
    for q in range(P):
        n = base + (1 if q < extra else 0)
        out.append((j, j + n))
        j += n
    return out


class PhaseOps:
    """Phase functions shared by t-slab and x-slab contexts (pdhg_slab_begin / _primal_finalize / _dual /
    _dual_finalize / _outer / _outer_finalize / _status, pdhg_set_stream).  Tensor arguments are device
    tensors (float64[16] sums)."""

    @property
    def plane_dtype(self):
        """Element type of the device planes / halos / wires exchanged between slabs (the context's precision)."""
        import torch
        return torch.float64 if self.precision in ("fp64", 8) else torch.float32

    def set_stream(self, stream_handle):
        N.check(self._lib.pdhg_set_stream(self._h, ctypes.c_void_p(stream_handle)))

    def begin(self):
        N.check(self._lib.pdhg_slab_begin(self._h))

    def primal_finalize(self, sums):
        N.check(self._lib.pdhg_slab_primal_finalize(self._h, _ptr(sums)))

    def dual(self, sigma, k, sub, sums, parts=INTERIOR | EDGE):
        N.check(self._lib.pdhg_slab_dual(self._h, float(sigma), int(k), int(sub), _ptr(sums), int(parts)))

    def dual_finalize(self, eps, sub, sums):
        N.check(self._lib.pdhg_slab_dual_finalize(self._h, float(eps), int(sub), _ptr(sums)))

    def outer(self, k, sums):
        N.check(self._lib.pdhg_slab_outer(self._h, int(k), _ptr(sums)))

    def outer_finalize(self, eps, k, sums):
        N.check(self._lib.pdhg_slab_outer_finalize(self._h, float(eps), int(k), _ptr(sums)))

    def status(self):
        st = N.pdhg_stats()
        N.check(self._lib.pdhg_slab_status(self._h, ctypes.byref(st)))
        return {"iters": st.iters_run, "status": st.status, "err1": st.err1, "err2": st.err2,
                "inner_last": st.inner_last, "inner_total": st.inner_total, "nan_seen": st.nan_seen,
                "first_nan_iter": st.first_nan_iter}


class SlabContext(PhaseOps, PDHGContext):
    """The slab [j0, j1) of a window of T_total rows (2-D; precision "fp32", or "fp64" = the reference's
    arithmetic, jaxsrc/update_fns_in_pdhg.py:10).  Arrays at this boundary are the slab's rows: phi [T+1, nx, ny]
    (row 0 = global phi row j0), rho / alp [T, nx, ny(, n_ctrl)].  Device planes exchanged between slabs are in
    the slab's precision (plane_dtype)."""

    def __init__(self, rank, nranks, T_total, egno, nx, ny, dx, dy, dt, xs, ys, device=0, **kw):
        self.rank, self.nranks, self.T_total = int(rank), int(nranks), int(T_total)
        self.j0, self.j1 = slab_bounds(self.T_total, self.nranks)[self.rank]
        kw.setdefault("precision", "fp32")
        super().__init__(egno, 2, nx, ny, self.j1 - self.j0, dx, dy, dt, xs, ys, device=device, **kw)

    def _create(self, prob, device):
        h = ctypes.c_void_p()
        N.check(self._lib.pdhg_create_slab(ctypes.byref(prob), self.j0, self.T_total, device, ctypes.byref(h)))
        return h

    @property
    def last(self):
        return self.rank == self.nranks - 1

    def plane_sizes(self):
        sp, spec = ctypes.c_ulonglong(), ctypes.c_ulonglong()
        N.check(self._lib.pdhg_slab_plane_size(self._h, ctypes.byref(sp), ctypes.byref(spec)))
        return sp.value, spec.value


    # thin wrappers; tensor arguments are device tensors (planes of plane_dtype)
    def carry_gain(self, GS):
        N.check(self._lib.pdhg_slab_carry_gain(self._h, _ptr(GS)))

    def residual(self, parts=INTERIOR | EDGE):
        N.check(self._lib.pdhg_slab_residual(self._h, int(parts)))

    def forward(self, tau):
        N.check(self._lib.pdhg_slab_forward(self._h, float(tau)))

    def fixup(self, allDS, allGS):
        N.check(self._lib.pdhg_slab_fixup(self._h, _ptr(allDS), _ptr(allGS), self.rank, self.nranks))

    def long_modes(self, allGS, delta=LONG_RANGE_DELTA):
        K = ctypes.c_int()
        N.check(self._lib.pdhg_slab_long_modes(self._h, _ptr(allGS), self.nranks, float(delta), ctypes.byref(K)))
        return K.value

    def fixup_nb(self, D_left, S1_right, allLong, allGS):
        N.check(self._lib.pdhg_slab_fixup_nb(self._h, _ptr(D_left), _ptr(S1_right), _ptr(allLong), _ptr(allGS),
                                             self.rank, self.nranks))

    def backward(self, tau, sums):
        N.check(self._lib.pdhg_slab_backward(self._h, float(tau), _ptr(sums)))

    def plane_out(self, which, dst):
        N.check(self._lib.pdhg_slab_plane_out(self._h, int(which), _ptr(dst)))

    # partitioned carry exchange (column-block parts)
    def part_modes(self, part, nparts):
        a, b = ctypes.c_ulonglong(), ctypes.c_ulonglong()
        N.check(self._lib.pdhg_slab_part_modes(self._h, int(part), int(nparts), ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def forward_part(self, tau, part, nparts):
        N.check(self._lib.pdhg_slab_forward_part(self._h, float(tau), int(part), int(nparts)))

    def carry_out_part(self, dst, part, nparts):
        N.check(self._lib.pdhg_slab_carry_out_part(self._h, _ptr(dst), int(part), int(nparts)))

    def fixup_nb_part(self, D_left, S1_right, allLong, allGS, part, nparts):
        N.check(self._lib.pdhg_slab_fixup_nb_part(self._h, _ptr(D_left), _ptr(S1_right), _ptr(allLong), _ptr(allGS),
                                                  self.rank, self.nranks, int(part), int(nparts)))

    def backward_part(self, tau, part, nparts):
        N.check(self._lib.pdhg_slab_backward_part(self._h, float(tau), int(part), int(nparts)))

    def update(self, tau, sums):
        N.check(self._lib.pdhg_slab_update(self._h, float(tau), _ptr(sums)))

    def plane_in(self, which, src):
        N.check(self._lib.pdhg_slab_plane_in(self._h, int(which), _ptr(src)))


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


# ---------------------------------------------------------------------------------------------
# communicators: lists hold one entry per slab living in this process
# ---------------------------------------------------------------------------------------------
class LocalComm:
    """P slabs in one process on one device: every collective is a device copy."""

    def __init__(self, nranks):
        self.nranks = nranks
        self.ranks = list(range(nranks))

    def allgather(self, planes):
        import torch
        out = torch.stack(planes)
        return [out] * len(planes)

    def alltoall(self, sends, recvs):
        """sends[q] / recvs[q]: [P * chunk] wires of slab q; chunk s of slab q's send -> chunk q of slab s's recv."""
        P = self.nranks
        c = sends[0].numel() // P
        for q in range(P):
            for s in range(P):
                recvs[s][q * c:(q + 1) * c].copy_(sends[q][s * c:(s + 1) * c])

    def allreduce(self, vecs):
        tot = vecs[0].clone()
        for v in vecs[1:]:
            tot += v
        for v in vecs:
            v.copy_(tot)

    def shift_down(self, send, recv):     # slab r -> slab r+1
        for r in range(1, self.nranks):
            recv[r].copy_(send[r - 1])

    def shift_up(self, send, recv):       # slab r -> slab r-1
        for r in range(self.nranks - 1):
            recv[r].copy_(send[r + 1])

    def shift_both(self, send_dn, recv_dn, send_up, recv_up):
        self.shift_down(send_dn, recv_dn)
        self.shift_up(send_up, recv_up)


class DistComm:
    """One slab per rank over torch.distributed (backend "nccl" = RCCL on ROCm, or "gloo")."""

    def __init__(self):
        import torch.distributed as dist
        self.dist = dist
        self.rank = dist.get_rank()
        self.nranks = dist.get_world_size()
        self.ranks = [self.rank]
        self.gloo = dist.get_backend() == "gloo"
        # the halo shifts get a communicator of their own: on one communicator RCCL runs operations in
        # issue order, so the sums all-reduce issued behind a halo would wait for it and stall the
        # main stream -- on a second one the halo overlaps the kernels and the small collectives
        self.halo_group = dist.new_group(list(range(self.nranks))) if self.nranks > 1 else None

    # gloo moves host memory: device tensors are staged through the host (functional rehearsal of the
    # multi-rank path; the GPU runs use RCCL on device buffers directly)
    def allgather(self, planes):
        import torch
        (x,) = planes
        if self.gloo:
            h = x.cpu()
            parts = [torch.empty_like(h) for _ in range(self.nranks)]
            self.dist.all_gather(parts, h)
            return [torch.stack(parts).to(x.device)]
        out = torch.empty((self.nranks,) + tuple(x.shape), dtype=x.dtype, device=x.device)
        self.dist.all_gather_into_tensor(out, x)
        return [out]

    def alltoall(self, sends, recvs):
        """Chunk s of this rank's send -> rank s; chunk q of recv <- rank q (equal chunks)."""
        import torch
        (send,), (recv,) = sends, recvs
        if self.gloo and send.is_cuda:
            h = torch.empty(recv.shape, dtype=recv.dtype)
            self.dist.all_to_all_single(h, send.cpu())
            recv.copy_(h)
        else:
            self.dist.all_to_all_single(recv, send)

    def allreduce(self, vecs):
        if self.gloo and vecs[0].is_cuda:
            h = vecs[0].cpu()
            self.dist.all_reduce(h)
            vecs[0].copy_(h)
        else:
            self.dist.all_reduce(vecs[0])

    def _shift(self, pairs):
        """pairs: (send tensor, recv tensor, step): send to rank+step, receive from rank-step; all in one
        batch of point-to-point operations on the halo communicator."""
        ops, back = [], []
        for send, recv, step in pairs:
            dst, src = self.rank + step, self.rank - step
            stage = self.gloo and send.is_cuda
            s_buf = send.cpu() if stage else send
            r_buf = recv.cpu() if stage else recv
            if 0 <= dst < self.nranks:
                ops.append(self.dist.P2POp(self.dist.isend, s_buf, dst, group=self.halo_group))
            if 0 <= src < self.nranks:
                ops.append(self.dist.P2POp(self.dist.irecv, r_buf, src, group=self.halo_group))
                if stage:
                    back.append((recv, r_buf))
        if ops:
            for w in self.dist.batch_isend_irecv(ops):
                w.wait()
        for recv, r_buf in back:
            recv.copy_(r_buf)

    def shift_down(self, send, recv):
        self._shift([(send[0], recv[0], 1)])

    def shift_up(self, send, recv):
        self._shift([(send[0], recv[0], -1)])

    def shift_both(self, send_dn, recv_dn, send_up, recv_up):
        self._shift([(send_dn[0], recv_dn[0], 1), (send_up[0], recv_up[0], -1)])


# ---------------------------------------------------------------------------------------------
# the iteration
# ---------------------------------------------------------------------------------------------
class SlabRunner:
    """Drives the slabs of this process through outer iterations (pdhg_iterate's loop, split at
    every point where slabs exchange data)."""

    def __init__(self, slabs, comm, overlap=True, exchange="neighbour", delta=LONG_RANGE_DELTA, parts=2):
        """overlap: halos on a second stream while the interior rows compute.  exchange: "neighbour"
        (D / S1 planes to the adjacent slabs + an allgather of the long-range modes only) or
        "allgather" (every slab's full [D, S1] planes).  parts (neighbour exchange with overlap): the column
        blocks are swept in `parts` parts so each part's carry planes travel while the next part sweeps."""
        import torch
        if exchange not in ("neighbour", "allgather"):
            raise ValueError("exchange must be 'neighbour' or 'allgather'")
        self.torch = torch
        self.slabs, self.comm = list(slabs), comm
        self.exchange = exchange
        self.timing = False      # record HIP events around every exchange (exchange_times())
        self._tev = {}
        self.side = torch.cuda.Stream() if overlap else None   # halo stream
        self.parts = int(parts) if (exchange == "neighbour" and overlap) else 1
        dev = torch.device("cuda", torch.cuda.current_device())
        sp, spec = self.slabs[0].plane_sizes()
        f32, f64 = self.slabs[0].plane_dtype, torch.float64   # planes in the slabs' precision; sums fp64
        if any(s.plane_dtype != f32 for s in self.slabs):
            raise ValueError("slabs of one runner must share a precision")
        self.b = []
        handle = torch.cuda.current_stream().cuda_stream
        for s in self.slabs:
            s.set_stream(handle)
            self.b.append({k: torch.zeros(n, dtype=f32, device=dev) for k, n in
                           (("rho_send", sp), ("rho_recv", sp), ("pb_send", sp), ("pb_recv", sp),
                            ("DS", 2 * spec), ("GS", 2 * spec))})
            self.b[-1]["sums"] = torch.zeros(16, dtype=f64, device=dev)
        for s, b in zip(self.slabs, self.b):
            s.carry_gain(b["GS"])
        self.allGS = comm.allgather([b["GS"] for b in self.b])   # iteration-invariant
        self.n_long = None
        self.part_modes = [self.slabs[0].part_modes(q, self.parts) for q in range(self.parts)]
        if exchange == "neighbour":
            Ks = [s.long_modes(self.allGS[i], delta) for i, s in enumerate(self.slabs)]
            self.n_long = Ks[0]
            for b in self.b:
                b["Dl"] = torch.zeros(spec, dtype=f32, device=dev)
                b["S1r"] = torch.zeros(spec, dtype=f32, device=dev)
                b["LONG"] = torch.zeros(max(1, 2 * self.n_long), dtype=f32, device=dev)

    def _each(self, name, *args):
        for s in self.slabs:
            getattr(s, name)(*args)

    def _timed(self, cat, fn, stream=None):
        """fn() bracketed by timing events on `stream` (default: the current stream) when timing is on."""
        if not self.timing:
            return fn()
        torch = self.torch
        stream = stream or torch.cuda.current_stream()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        r = fn()
        b.record(stream)
        self._tev.setdefault(cat, []).append((a, b))
        return r

    def exchange_times(self, reset=True):
        """{category: total ms} of the exchanges since timing was switched on (halo_rho, halo_phibar,
        carry_planes, carry_long, allreduce); side-stream exchanges overlap the kernels of the main stream, and
        exposed_<cat> is the time the main stream waited for them (halo_rho, halo_phibar, carry_planes)."""
        self.torch.cuda.synchronize()
        out = {c: sum(a.elapsed_time(b) for a, b in evs) for c, evs in self._tev.items()}
        if reset:
            self._tev = {}
        return out

    def _halo(self, shift, *planes, cat="halo"):
        """Run a halo shift on the side stream after everything enqueued so far on the main stream;
        returns at once (join with _join before the halo plane is used)."""
        torch = self.torch
        if self.side is None:
            self._timed(cat, lambda: shift(*planes))
            return
        self.side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.side):
            self._timed(cat, lambda: shift(*planes), self.side)

    def _join(self, cat=None):
        """Main stream waits for the side stream.  With timing on, events on the main stream either side of the
        wait measure how long the kernels stood still for the exchange: the exposed part of `cat`
        (exchange_times() key "exposed_<cat>")."""
        if self.side is None:
            return
        main = self.torch.cuda.current_stream()
        if cat is not None and self.timing:
            self._timed("exposed_" + cat, lambda: main.wait_stream(self.side), main)
        else:
            main.wait_stream(self.side)

    def step(self, tau, sigma, eps, k):
        S, B, C = self.slabs, self.b, self.comm
        # rho halo (row 0 of slab r+1 -> slab r: the residual's rho_{j+1} on its last row), overlapped
        # with the residual of the rows that do not read it
        for s, b in zip(S, B):
            s.plane_out(RHO_ROW0, b["rho_send"])
        self._halo(C.shift_up, [b["rho_send"] for b in B], [b["rho_recv"] for b in B], cat="halo_rho")
        for s in S:
            s.residual(INTERIOR)
        self._join("halo_rho")
        for s, b in zip(S, B):
            if not s.last:
                s.plane_in(RHO_HALO, b["rho_recv"])
            s.residual(EDGE)
        # primal: zero-carry forward sweeps, ONE allgather of [D, S1], carry folds, backward sweeps + update
        if self.exchange == "neighbour" and self.parts > 1:
            self._primal_parts(tau)
            return self._after_primal(sigma, eps, k)
        self._each("forward", tau)
        for s, b in zip(S, B):
            s.plane_out(CARRY_DS, b["DS"])
        if self.exchange == "neighbour":
            # D -> next slab, S1 -> previous slab (point to point) || allgather of the long-range modes
            spec = B[0]["Dl"].numel()
            for s, b in zip(S, B):
                s.plane_out(CARRY_LONG, b["LONG"])
            self._halo(C.shift_both, [b["DS"][:spec] for b in B], [b["Dl"] for b in B],
                       [b["DS"][spec:] for b in B], [b["S1r"] for b in B], cat="carry_planes")
            allLong = self._timed("carry_long", lambda: C.allgather([b["LONG"] for b in B]))
            self._join("carry_planes")
            for i, s in enumerate(S):
                s.fixup_nb(B[i]["Dl"], B[i]["S1r"], allLong[i], self.allGS[i])
                s.backward(tau, B[i]["sums"])
        else:
            allDS = self._timed("carry_planes", lambda: C.allgather([b["DS"] for b in B]))
            for i, s in enumerate(S):
                s.fixup(allDS[i], self.allGS[i])
                s.backward(tau, B[i]["sums"])
        self._after_primal(sigma, eps, k)

    def _primal_parts(self, tau):
        """Forward sweep, carry exchange and backward sweep in column-block parts: part q's D / S1 planes
        go to the neighbours on the side stream while part q+1 sweeps forward (and part q-1 backward)."""
        torch = self.torch
        S, B, C = self.slabs, self.b, self.comm
        spec = B[0]["Dl"].numel()
        done = []
        for q in range(self.parts):
            lo, hi = self.part_modes[q]
            for s, b in zip(S, B):
                s.forward_part(tau, q, self.parts)
                s.carry_out_part(b["DS"], q, self.parts)
            self._halo(C.shift_both, [b["DS"][lo:hi] for b in B], [b["Dl"][lo:hi] for b in B],
                       [b["DS"][spec + lo:spec + hi] for b in B], [b["S1r"][lo:hi] for b in B], cat="carry_planes")
            ev = torch.cuda.Event()
            ev.record(self.side)
            done.append(ev)
        for s, b in zip(S, B):
            s.plane_out(CARRY_LONG, b["LONG"])
        allLong = self._timed("carry_long", lambda: C.allgather([b["LONG"] for b in B]))
        main = torch.cuda.current_stream()
        for q in range(self.parts):
            if self.timing:
                self._timed("exposed_carry_planes", lambda: main.wait_event(done[q]), main)
            else:
                main.wait_event(done[q])
            for i, s in enumerate(S):
                s.fixup_nb_part(B[i]["Dl"], B[i]["S1r"], allLong[i], self.allGS[i], q, self.parts)
                s.backward_part(tau, q, self.parts)
        for s, b in zip(S, B):
            s.update(tau, b["sums"])

    def _after_primal(self, sigma, eps, k):
        S, B, C = self.slabs, self.b, self.comm
        # phi_bar halo (row T of slab r -> row 0 of slab r+1: the dual's phi_bar_j), overlapped with the
        # primal sums all-reduce and the dual of the rows that do not read it
        for s, b in zip(S, B):
            s.plane_out(PHIBAR_LAST, b["pb_send"])
        self._halo(C.shift_down, [b["pb_send"] for b in B], [b["pb_recv"] for b in B], cat="halo_phibar")
        self._timed("allreduce", lambda: C.allreduce([b["sums"] for b in B]))
        for s, b in zip(S, B):
            s.primal_finalize(b["sums"])
        # dual sub-iterations (device-side early exit once the global inner error is below eps)
        for sub in range(k):
            for s, b in zip(S, B):
                s.dual(sigma, k, sub, b["sums"], INTERIOR if sub == 0 else INTERIOR | EDGE)
            if sub == 0:
                self._join("halo_phibar")
                for s, b in zip(S, B):
                    if s.rank > 0:
                        s.plane_in(PHIBAR_ROW0, b["pb_recv"])
                    s.dual(sigma, k, sub, b["sums"], EDGE)
            self._timed("allreduce", lambda: C.allreduce([b["sums"] for b in B]))
            for s, b in zip(S, B):
                s.dual_finalize(eps, sub, b["sums"])
        for s, b in zip(S, B):
            s.outer(k, b["sums"])
        if k > 1:
            self._timed("allreduce", lambda: C.allreduce([b["sums"] for b in B]))
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


def split_state(phi, rho, alp, bounds):
    """Slice a window's state (reference layouts) into per-slab states."""
    out = []
    for (j0, j1) in bounds:
        out.append((phi[j0:j1 + 1], rho[j0:j1], tuple(a[j0:j1] for a in alp)))
    return out


def join_state(parts):
    """Inverse of split_state: phi rows j0..j1 of every slab (row 0 of slab r > 0 is the halo)."""
    phi = np.concatenate([parts[0][0]] + [p[0][1:] for p in parts[1:]], axis=0)
    rho = np.concatenate([p[1] for p in parts], axis=0)
    alp = tuple(np.concatenate([p[2][a] for p in parts], axis=0) for a in range(len(parts[0][2])))
    return phi, rho, alp
