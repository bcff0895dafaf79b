"""The N > 1 path on CPU: processes over torch.distributed "gloo" (world sizes 2 and 3).

DistComm (pdhg_amd/slab.py) is the communicator the multi-GPU run uses over RCCL; here it moves CPU
tensors.  Checked: the halo shifts, allgather and allreduce semantics, and the distributed t-solve
(oracle/slab_oracle.py algebra) driven through those collectives reproduces the monolithic solve."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, paths):
    import sys
    sys.path[:0] = paths
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:{}".format(port), rank=rank, world_size=world)
    try:
        from pdhg_amd.slab import DistComm, slab_bounds
        import slab_oracle as S
        comm = DistComm()
        assert comm.rank == rank and comm.nranks == world
        # --- halo shifts: rank r sends r+1 (down) / r-1 (up)
        send = [torch.full((5,), float(rank + 1))]
        recv = [torch.zeros(5)]
        comm.shift_down(send, recv)
        assert float(recv[0][0]) == (rank if rank > 0 else 0.0)
        recv = [torch.zeros(5)]
        comm.shift_up(send, recv)
        assert float(recv[0][0]) == (rank + 2 if rank < world - 1 else 0.0)
        # --- allgather / allreduce
        (g,) = comm.allgather([torch.arange(3, dtype=torch.float32) + 10 * rank])
        assert g.shape == (world, 3) and all(float(g[q, 0]) == 10 * q for q in range(world))
        v = [torch.full((16,), float(rank + 1), dtype=torch.float64)]
        comm.allreduce(v)
        assert float(v[0][3]) == sum(range(1, world + 1))
        # --- distributed Thomas over the real collectives
        rng = np.random.default_rng(3)           # same data on every rank
        T, M = 11, 9
        ae = 1.0 / 0.04 ** 2
        diag = np.tile(1.0 + rng.uniform(0, 3e3, M) + 2 * ae, (T, 1))
        diag[-1] -= ae
        r = rng.standard_normal((T, M))
        ref = S.monolithic_tridiag(diag, r, ae)
        j0, j1 = slab_bounds(T, world)[rank]
        gp = S.pivots(diag, ae)
        b0, D, G = S.local_forward(r, gp, ae, j0, j1)
        (allD,) = comm.allgather([torch.from_numpy(D)])
        (allG,) = comm.allgather([torch.from_numpy(G)])
        c = S.carry_in(list(allD.numpy()), list(allG.numpy()), rank)
        b, X0 = S.fixup(b0, gp, j0, c)
        (allX0,) = comm.allgather([torch.from_numpy(X0)])
        y = S.right_carry(list(allX0.numpy()), list(allG.numpy()), rank)
        x = S.local_backward(b, gp, j0, y)
        assert np.allclose(x, ref[j0:j1], rtol=1e-11, atol=1e-12 * np.abs(ref).max())
        # --- the neighbour exchange (the multi-GPU default): D -> next slab, S1 -> previous slab in one
        # batch of point-to-point operations, an allgather of the long-range modes only
        T, M = 12, 64
        ae = 1.0 / (1.0 / T) ** 2
        lam = -4.0 * np.sin(np.pi * np.arange(M) / (2 * M)) ** 2 * (M / 0.05) ** 2
        diag = np.tile(1.0 - lam + 2 * ae, (T, 1))
        diag[-1] -= ae
        r = rng.standard_normal((T, M))
        ref = S.monolithic_tridiag(diag, r, ae)
        j0, j1 = slab_bounds(T, world)[rank]
        gp = S.pivots(diag, ae)
        b0, D, G = S.local_forward(r, gp, ae, j0, j1)
        s1, s2 = S.s_sums(b0, gp, j0)
        (allGS,) = comm.allgather([torch.from_numpy(np.concatenate([G, s2]))])
        Gs, S2s = [a[:M] for a in allGS.numpy()], [a[M:] for a in allGS.numpy()]
        mask = S.long_range_mask(Gs, 2.0 ** -40)
        assert 0 < mask.sum() < M
        Dl, S1r = [torch.zeros(M, dtype=torch.float64)], [torch.zeros(M, dtype=torch.float64)]
        comm.shift_both([torch.from_numpy(D)], Dl, [torch.from_numpy(s1)], S1r)
        (allLong,) = comm.allgather([torch.from_numpy(np.concatenate([D[mask], s1[mask]]))])
        K = int(mask.sum())
        Ds, S1s = [np.zeros(M) for _ in range(world)], [np.zeros(M) for _ in range(world)]
        for q in range(world):
            Ds[q][mask], S1s[q][mask] = allLong.numpy()[q][:K], allLong.numpy()[q][K:]
        if rank > 0:
            Ds[rank - 1][~mask] = Dl[0].numpy()[~mask]
        if rank + 1 < world:
            S1s[rank + 1][~mask] = S1r[0].numpy()[~mask]
        Ds[rank] = D
        c, y = S.carries_neighbour(Ds, S1s, Gs, S2s, rank, mask)
        b, _ = S.fixup(b0, gp, j0, c)
        x = S.local_backward(b, gp, j0, y)
        assert np.allclose(x, ref[j0:j1], rtol=1e-10, atol=1e-11 * np.abs(ref).max())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_slab_exchanges(world):
    paths = [os.path.join(HERE, "..", "pdhg-optimal-control_amd"), os.path.join(HERE, "..", "oracle")]
    mp.spawn(_worker, args=(world, _free_port(), [os.path.abspath(p) for p in paths]), nprocs=world, join=True)


def _xslab_worker(rank, world, port, paths):
    """x-slab exchanges over gloo: the halo ring (allgather of the first / last live rows) and the
    preconditioner's two all-to-all transposes, restated in oracle/xslab_oracle.py, must reproduce the
    monolithic H1_precond_2d (utils_precond.py:142-178) on this rank's rows."""
    import sys
    sys.path[:0] = paths
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:{}".format(port), rank=rank, world_size=world)
    try:
        from pdhg_amd.slab import DistComm
        import pdhg_oracle as O
        import xslab_oracle as X
        comm = DistComm()
        nx, ny, T, B, dt = 48, 24, 3, 4, 0.05
        dx, dy = 2.0 / nx, 2.0 / ny
        nloc = nx // world
        x0 = rank * nloc
        rng = np.random.default_rng(11)           # same data on every rank
        R = rng.standard_normal((T, nx, ny))
        idx = X.local_index(x0, nloc, nx)
        # --- halo ring: ghost rows from the neighbours' live edge rows
        A = R[:, idx].copy()
        A[:, X.XL0 - 1] = 0.0
        A[:, X.XL0 + nloc] = 0.0
        (allh,) = comm.allgather([torch.from_numpy(X.halo_out(A, nloc))])
        X.halo_in(A, nloc, allh[(rank - 1) % world].numpy(), allh[(rank + 1) % world].numpy())
        assert np.array_equal(A[:, X.XL0 - 1], R[:, (x0 - 1) % nx])
        assert np.array_equal(A[:, X.XL0 + nloc], R[:, (x0 + nloc) % nx])

        # --- preconditioner over the all-to-all transposes
        def a2a(send):
            recv = torch.empty(send.shape, dtype=torch.float64)
            comm.alltoall([torch.from_numpy(np.ascontiguousarray(send))], [recv])
            return recv.numpy()

        lx, ly = X.symbols(nx, ny, dx, dy)
        U = X.precond_rank(R[:, idx], rank, world, nloc, B, a2a, lx, ly, dt)
        fv = O.compute_Dxx_fft_fv(2, (nx, ny), (dx, dy), (0, 0))
        ref = O.H1_precond_2d(np.concatenate([np.zeros((1, nx, ny)), R]), fv, dt, (0, 0))[1:]
        assert np.allclose(U, ref[:, x0:x0 + nloc], rtol=1e-10, atol=1e-12 * np.abs(ref).max())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_xslab_exchanges(world):
    paths = [os.path.join(HERE, "..", "pdhg-optimal-control_amd"), os.path.join(HERE, "..", "oracle")]
    mp.spawn(_xslab_worker, args=(world, _free_port(), [os.path.abspath(p) for p in paths]), nprocs=world, join=True)
