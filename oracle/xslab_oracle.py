"""CPU restatement of the x-slab decomposition (TEST INFRASTRUCTURE: imported only by tests/).

The x-slab path (pdhg-optimal-control_amd/csrc/kernels_xslab.hpp, pdhg_amd/xslab.py) changes no
arithmetic of the reference; it moves data so that the H1 preconditioner of utils_precond.py:142-178
(FFT2 -> tridiagonal solve in t per mode -> iFFT2, bc (0,0)) can run on x rows split over ranks:

* every rank holds nloc = nx / P live rows plus padding (local row i = global row (x0 - XL0 + i) mod nx,
  XL0 = 8 leading rows, 16 extra rows in all); the stencils reach +-1 row, so ghost rows XL0 - 1 and
  XL0 + nloc are refreshed from the neighbours (periodic ring);
* the spatial operator C - Dxx - Dyy is a real symmetric circulant, so the separable discrete Hartley
  transform DHT_y o DHT_x diagonalises it with the reference's symbol fv = lam_x + lam_y
  (utils_precond.py:42-71), and the inverse is the same transform / (nx ny);
* DHT_y runs on the local rows, the spectrum goes to the blocked rows layout W [T][nb][nxl][B], is packed
  into the wire [P][T][nbs][nloc][B] (chunk q for rank q, nbs = nb / P), exchanged all-to-all, unpacked
  into whole x lines Cw [T][nbs][nx][B], transformed along x and solved in t per mode, and sent back the
  same way.

These functions restate those index maps and the per-rank steps in NumPy so a test can run them over real
collectives (gloo) and compare with the monolithic pdhg_oracle.H1_precond_2d.
"""
import numpy as np

import pdhg_oracle as O

XL0 = 8     # leading padding rows (the last one is the left ghost); 8 trailing rows (the first is the right ghost)


def local_index(x0, nloc, nx):
    """Global row of every local row (kernels_xslab.hpp header; pdhg_create_xslab)."""
    return (x0 - XL0 + np.arange(nloc + 16)) % nx


def dht(a, axis):
    """Discrete Hartley transform: Re F - Im F (its own inverse up to 1/n)."""
    f = np.fft.fft(a, axis=axis)
    return f.real - f.imag


def to_blocked(rows, B):
    """[T][nxl][ny] -> W [T][nb][nxl][B] (the residual kernel's spectral output layout)."""
    T, nxl, ny = rows.shape
    return rows.reshape(T, nxl, ny // B, B).transpose(0, 2, 1, 3).copy()


def from_blocked(W):
    T, nb, nxl, B = W.shape
    return W.transpose(0, 2, 1, 3).reshape(T, nxl, nb * B)


def pack_rows(W, P, nloc):
    """k_xs_rows_wire dir 0: live rows of W -> wire [P][T][nbs][nloc][B]."""
    T, nb, nxl, B = W.shape
    nbs = nb // P
    return W[:, :, XL0:XL0 + nloc, :].reshape(T, P, nbs, nloc, B).transpose(1, 0, 2, 3, 4).copy()


def unpack_rows(S, W):
    """k_xs_rows_wire dir 1: wire [P][T][nbs][nloc][B] -> live rows of W (in place)."""
    P, T, nbs, nloc, B = S.shape
    W[:, :, XL0:XL0 + nloc, :] = S.transpose(1, 0, 2, 3, 4).reshape(T, P * nbs, nloc, B)


def unpack_cols(S):
    """k_xs_cols_wire dir 1: wire [P][T][nbs][nloc][B] (chunk q = rank q's rows) -> Cw [T][nbs][nx][B]."""
    P, T, nbs, nloc, B = S.shape
    return S.transpose(1, 2, 0, 3, 4).reshape(T, nbs, P * nloc, B).copy()


def pack_cols(Cw, P):
    """k_xs_cols_wire dir 0: Cw [T][nbs][nx][B] -> wire [P][T][nbs][nloc][B] (chunk q = rank q's rows)."""
    T, nbs, nx, B = Cw.shape
    return Cw.reshape(T, nbs, P, nx // P, B).transpose(2, 0, 1, 3, 4).copy()


def symbols(nx, ny, dx, dy):
    """Periodic Laplacian symbols per mode (the analytic form of compute_Dxx_fft_fv, utils_precond.py:42-71)."""
    lx = -2.0 * (1.0 - np.cos(2.0 * np.pi * np.arange(nx) / nx)) / dx ** 2
    ly = -2.0 * (1.0 - np.cos(2.0 * np.pi * np.arange(ny) / ny)) / dy ** 2
    return lx, ly


def precond_cols(Cw, ky0, lx, ly, dt, C=1.0):
    """x transform, tridiagonal solve in t per mode (utils_precond.py:164-169: diag C - fv + Lap_t),
    inverse x transform, of one rank's column blocks Cw [T][nbs][nx][B]; ky0 = its first global column."""
    T, nbs, nx, B = Cw.shape
    v = dht(Cw, axis=2)
    ky = ky0 + np.arange(nbs * B).reshape(nbs, B)
    fv = lx[None, :, None] + ly[ky][:, None, :]                  # [nbs][nx][B]
    dl, du, diag = O._lap_t(T, dt)
    thomas_b = -fv[None] + diag[:, None, None, None] + C
    part = O.tridiagonal_solve(dl, thomas_b, du, v).real     # real data, real system
    return dht(part, axis=2)


def precond_rank(R_local, rank, P, nloc, B, comm_alltoall, lx, ly, dt, C=1.0):
    """One rank's x-slab H1 preconditioner of its local residual rows R_local [T][nxl][ny]; returns U on the
    live rows [T][nloc][ny].  comm_alltoall(send_flat) -> recv_flat exchanges equal chunks."""
    T, nxl, ny = R_local.shape
    nx = nloc * P
    W = to_blocked(dht(R_local, axis=2), B)
    S = pack_rows(W, P, nloc)
    Rw = comm_alltoall(S.reshape(-1)).reshape(S.shape)
    Cw = unpack_cols(Rw)
    nbs = Cw.shape[1]
    Cw = precond_cols(Cw, rank * nbs * B, lx, ly, dt, C)
    S = pack_cols(Cw, P)
    Rw = comm_alltoall(S.reshape(-1)).reshape(S.shape)
    unpack_rows(Rw, W)
    U = dht(from_blocked(W), axis=2) / (nx * ny)
    return U[:, XL0:XL0 + nloc]


def halo_out(A, nloc):
    """k_xs_halo_out for one array [R][nxl][ny]: [2][R][ny], side 0 = first live row, side 1 = last."""
    return np.stack([A[:, XL0], A[:, XL0 + nloc - 1]])


def halo_in(A, nloc, from_left, from_right):
    """k_xs_halo_in: the left ghost from the left neighbour's side 1, the right ghost from the right's side 0."""
    A[:, XL0 - 1] = from_left[1]
    A[:, XL0 + nloc] = from_right[0]
