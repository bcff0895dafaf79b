// x-slab decomposition: data movement kernels.
//
// A rank owns x rows [x0, x0 + nloc) of the global grid.  Its spatial arrays hold nxl = nloc + 16 rows:
// 8 leading rows (the last of them, xl0 - 1, is the left ghost), the nloc live rows [xl0, xl1) and 8
// trailing rows (the first, xl1, is the right ghost).  The row kernels run unchanged over all nxl rows
// (padding rows are never stored by the dual / update); the x transform of the preconditioner
// (utils_precond.py:142-178) needs whole x lines, so the spectrum is transposed over the ranks:
//   rows layout  W [T][nb][nxl][B]       (the y-DHT output of this rank's rows)
//   wire layout  S [P][T][nbs][nloc][B]  (chunk q: the part for / from rank q; nbs = nb / P)
//   cols layout  Cw [T][nbs][nx][B]      (this rank's column blocks, whole x lines)
// Every move is a set of runs of L = nloc*B contiguous floats, copied as float4.
#pragma once
#include "params.hpp"

namespace pdhg {

// rows <-> wire.  dir 0: W (live rows) -> S; dir 1: S -> W (live rows).  Run r = (q*T + j)*nbs + bl.
template <typename R>
__global__ void __launch_bounds__(256) k_xs_rows_wire(R* __restrict__ W, R* __restrict__ S, int dir, int P, int T,
                                                      int nb, int nbs, int nxl, int xl0, int B, size_t L) {
  const size_t L4 = L / 4, total = (size_t)P * T * nbs * L4;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const size_t run = i / L4, e = (i - run * L4) * 4;
    const int bl = (int)(run % nbs);
    const size_t qj = run / nbs;
    const int j = (int)(qj % T), q = (int)(qj / T);
    R* w = W + (((size_t)j * nb + (size_t)q * nbs + bl) * nxl + xl0) * B + e;
    R* s = S + run * L + e;
    if (dir == 0) {
      for (int k = 0; k < 4; ++k) s[k] = w[k];
    } else {
      for (int k = 0; k < 4; ++k) w[k] = s[k];
    }
  }
}

// cols <-> wire.  dir 0: Cw -> S (chunk q = x rows [q*nloc, (q+1)*nloc)); dir 1: S -> Cw.
template <typename R>
__global__ void __launch_bounds__(256) k_xs_cols_wire(R* __restrict__ Cw, R* __restrict__ S, int dir, int P, int T,
                                                      int nbs, int nx, int nloc, int B, size_t L) {
  const size_t L4 = L / 4, total = (size_t)P * T * nbs * L4;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const size_t run = i / L4, e = (i - run * L4) * 4;
    const int bl = (int)(run % nbs);
    const size_t qj = run / nbs;
    const int j = (int)(qj % T), q = (int)(qj / T);
    R* c = Cw + (((size_t)j * nbs + bl) * nx + (size_t)q * nloc) * B + e;
    R* s = S + run * L + e;
    if (dir == 0) {
      for (int k = 0; k < 4; ++k) s[k] = c[k];
    } else {
      for (int k = 0; k < 4; ++k) c[k] = s[k];
    }
  }
}

// Halo rows out: which 0 = rho and the live controls of the current set (the continuity residual's x
// neighbours, update_fns_in_pdhg.py:83-96), which 1 = phi_bar rows 1..T (the dual's x differences,
// utils_diff_op.py:9-91).  dst [2][nq][nr][ny]: side 0 = the first live row (the left neighbour's right
// ghost), side 1 = the last live row (the right neighbour's left ghost).
template <typename R>
__global__ void __launch_bounds__(256) k_xs_halo_out(KP<R> p, int which, R* __restrict__ dst) {
  const int cur = p.ctrl->cur;
  const int nq = which == 0 ? 1 + p.na : 1, nr = p.T;
  const int roff = which == 0 ? 0 : 1;
  const size_t ny = p.ny, plane = (size_t)p.nx * ny, total = (size_t)2 * nq * nr * ny;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const size_t y = i % ny, t = i / ny;
    const int j = (int)(t % nr), q = (int)((t / nr) % nq), side = (int)(t / ((size_t)nr * nq));
    const R* a = which == 1 ? p.phibar : (q == 0 ? p.rho[cur] : p.alp[cur][q - 1]);
    const int x = side == 0 ? p.xl0 : p.xl1 - 1;
    dst[i] = a[(size_t)(j + roff) * plane + (size_t)x * ny + y];
  }
}

// Halo rows in: the left ghost row (xl0 - 1) from the left neighbour's side 1, the right ghost row (xl1)
// from the right neighbour's side 0 (layouts of k_xs_halo_out).  own_l / own_r (Neumann x edge of the global grid,
// nb_index bc 1): that ghost replicates the slab's own edge row instead.
template <typename R>
__global__ void __launch_bounds__(256) k_xs_halo_in(KP<R> p, int which, const R* __restrict__ from_left,
                                                    const R* __restrict__ from_right, int own_l, int own_r) {
  const int cur = p.ctrl->cur;
  const int nq = which == 0 ? 1 + p.na : 1, nr = p.T;
  const int roff = which == 0 ? 0 : 1;
  const size_t ny = p.ny, plane = (size_t)p.nx * ny, half = (size_t)nq * nr * ny, total = 2 * half;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int side = i >= half ? 1 : 0;   // 0: left ghost, 1: right ghost
    const size_t k = i - side * half;
    const size_t y = k % ny, t = k / ny;
    const int j = (int)(t % nr), q = (int)(t / nr);
    R* a = which == 1 ? p.phibar : (q == 0 ? p.rho[cur] : p.alp[cur][q - 1]);
    const int x = side == 0 ? p.xl0 - 1 : p.xl1;
    const size_t rowoff = (size_t)(j + roff) * plane + y;
    R v;
    if (side == 0) v = own_l ? a[rowoff + (size_t)p.xl0 * ny] : from_left[half + k];
    else v = own_r ? a[rowoff + (size_t)(p.xl1 - 1) * ny] : from_right[k];
    a[rowoff + (size_t)x * ny] = v;
  }
}

}  // namespace pdhg
