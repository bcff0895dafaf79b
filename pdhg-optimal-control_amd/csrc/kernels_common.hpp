// Reductions-to-scalars and device-side loop control (utils_pdhg_solver.py:58-80,
// update_fns_in_pdhg.py:162-176) plus state initialisation kernels.
#pragma once
#include "params.hpp"

namespace pdhg {

// Fixed-order reduction of nrows partial rows (ns sums each) into out[0..ns).
// The table is read as a flat array of double2: thread i accumulates column pair i % 8 of rows i/8,
// i/8 + blockDim/8, ... (every load instruction of a wave reads 1 KiB of consecutive rows, 8 of them in
// flight per thread), then the 8 threads of each column pair are reduced across the wave (shuffles) and
// across the waves (LDS), both in fixed order.  Call with blockDim.x a multiple of 64, at most 1024 (the
// finalize kernels run one 1024-thread block); out is visible to every thread on return.
__device__ void reduce_partials(const double* __restrict__ partials, int nrows, int ns, double* out) {
  static_assert(kNumSums == 16, "rows of 8 double2");
  __shared__ double red[16][kNumSums];
  const int c = threadIdx.x & 7;
  const int rstep = blockDim.x >> 3;
  const double2* P = reinterpret_cast<const double2*>(partials);
  double ax = 0.0, ay = 0.0;
  if (2 * c < ns) {   // entries >= ns are never written out
#pragma unroll 8
    for (int r = threadIdx.x >> 3; r < nrows; r += rstep) {
      const double2 v = P[(size_t)r * 8 + c];
      ax += v.x;
      ay += v.y;
    }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int o = 32; o >= 8; o >>= 1) {
    ax += __shfl_down(ax, o, 64);
    ay += __shfl_down(ay, o, 64);
  }
  if (lane < 8) {
    red[w][2 * lane] = ax;
    red[w][2 * lane + 1] = ay;
  }
  __syncthreads();
  if ((int)threadIdx.x < ns) {
    double t = 0.0;
    for (int i = 0; i < nw; ++i) t += red[i][threadIdx.x];
    out[threadIdx.x] = t;
  }
  __syncthreads();
}

// First level of a two-level fold for long partial tables: workgroup b reduces rows [b chunk, (b+1) chunk)
// into row b of out (fixed order, as reduce_partials); the finalize kernels then read gridDim.x rows.
// ctrl (optional): skip the fold once the dual loop has exited (the per-sub-iteration kernels still launch and
// return at once; their tables are not read)
__global__ void __launch_bounds__(1024) k_fold_partials(const double* __restrict__ partials, int nrows, int ns,
                                                       int chunk, double* __restrict__ out, const Ctrl* ctrl) {
  if (ctrl && (ctrl->done || ctrl->inner_done)) return;
  __shared__ double o[kNumSums];
  const int r0 = blockIdx.x * chunk;
  reduce_partials(partials + (size_t)r0 * kNumSums, max(0, min(chunk, nrows - r0)), ns, o);
  if ((int)threadIdx.x < ns) out[(size_t)blockIdx.x * kNumSums + threadIdx.x] = o[threadIdx.x];
}

// After the primal update: err1 sums (utils_pdhg_solver.py:58).  ctrl->row0_sq = sum phi_0^2
// (row 0 never changes: utils_precond.py:139/177).  Read from the control block, not passed by value, so a
// replayed graph sees the row 0 of the state set after the capture (window marching re-seeds it).
__global__ void __launch_bounds__(1024) k_finalize_primal(const double* partials, int nrows, int add_row0, Ctrl* ctrl) {
  if (ctrl->done) return;
  __shared__ double out[3];
  reduce_partials(partials, nrows, 3, out);
  if (threadIdx.x == 0) {
    const double row0_sq = add_row0 ? ctrl->row0_sq : 0.0;   // t-slab sums carry it already (k_reduce_vec)
    ctrl->s_dphi = out[0];
    ctrl->s_phi_old = out[1] + row0_sq;
    ctrl->s_phi_new = out[2] + row0_sq;
    ctrl->primal_valid = 1;
  }
}

// After dual sub-iteration `sub`: err = sum (drho)^2/sum rho'^2 + sum_a sum (dalp)^2/sum alp'^2
// (update_fns_in_pdhg.py:162-164); early exit flag when err < eps (:176).  n_dead reference
// arrays that are not stored (egno 3's y controls, identically zero) contribute 0/0 = NaN.
// spec (the speculative one-sub-iteration schedule of iterate(), pdhg_api.hip): a loop that does not exit here halts
// the iteration instead (done = kHaltTail: every later kernel returns at entry) and the host runs the rest of the loop
__device__ __forceinline__ void finalize_dual_sums(const double* out, int na, int n_dead, double eps, int sub,
                                                   Ctrl* ctrl, int spec = 0) {
  const int ns = 3 + 3 * na;
  if (threadIdx.x == 0) {
    double err = out[0] / out[1];
    for (int a = 0; a < na; ++a) err += out[3 + 3 * a] / out[4 + 3 * a];
    for (int a = 0; a < n_dead; ++a) {
      volatile double z = 0.0;
      err += z / z;
    }
    for (int s = 0; s < ns; ++s) ctrl->dual_sums[s] = out[s];
    if (sub == 0) {
      for (int s = 0; s < ns; ++s) ctrl->outer_sums[s] = out[s];
    }
    ctrl->err_inner = err;
    ctrl->inner_count = sub + 1;
    if (err < eps) ctrl->inner_done = 1;
    else if (spec) ctrl->done = kHaltTail;
  }
}
__global__ void __launch_bounds__(1024) k_finalize_dual(const double* partials, int nrows, int na, int n_dead,
                                                       double eps, int sub, Ctrl* ctrl, int spec = 0) {
  if (ctrl->done || ctrl->inner_done) return;
  __shared__ double out[kNumSums];
  reduce_partials(partials, nrows, 3 + 3 * na, out);
  finalize_dual_sums(out, na, n_dead, eps, sub, ctrl, spec);
}

// The fold and the finalize of a dual sub-iteration in one launch: workgroup b folds its chunk of the table into
// row b of fold (as k_fold_partials); the last workgroup to finish (ticket in ctrl->fold_ticket, device-scope
// fences on both sides of it) reduces the gridDim.x rows in fixed order and finalizes (as k_finalize_dual), then
// re-arms the ticket.  Same sums, same order as the two-launch form; one launch fewer per sub-iteration.
__global__ void __launch_bounds__(1024) k_fold_finalize_dual(const double* __restrict__ partials, int nrows,
                                                            int chunk, double* fold, int na, int n_dead, double eps,
                                                            int sub, Ctrl* ctrl) {
  if (ctrl->done || ctrl->inner_done) return;
  __shared__ double o[kNumSums];
  __shared__ int last;
  const int ns = 3 + 3 * na;
  const int r0 = blockIdx.x * chunk;
  reduce_partials(partials + (size_t)r0 * kNumSums, max(0, min(chunk, nrows - r0)), ns, o);
  if ((int)threadIdx.x < ns) fold[(size_t)blockIdx.x * kNumSums + threadIdx.x] = o[threadIdx.x];
  __threadfence();      // release the row before taking a ticket
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(&ctrl->fold_ticket, 1) == (int)gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  __threadfence();      // acquire the other workgroups' rows
  reduce_partials(fold, gridDim.x, ns, o);
  finalize_dual_sums(o, na, n_dead, eps, sub, ctrl);
  if (threadIdx.x == 0) ctrl->fold_ticket = 0;
}

// Chunked dual loop (kernels_dual_multi.hpp): after the chunk of sub-iterations slo .. slo + nsub - 1, the first
// one whose err (as k_finalize_dual, from the table of its sums) is below eps -- or the loop's last,
// sub-iteration kmax - 1 -- fixes k* = s + 1; the bookkeeping of k_finalize_dual for that sub-iteration follows
// (inner_count, err_inner, dual_sums [0, 1, 3+3a, 4+3a]).  kstored = slo + nsub: the state the chunk stored.
__global__ void __launch_bounds__(1024) k_finalize_dual_multi(const double* partials, int table_rows, int nsub,
                                                             int slo, int kmax, int na, int n_dead, double eps,
                                                             Ctrl* ctrl) {
  if (ctrl->done || ctrl->kstar_found || ctrl->inner_done) return;   // inner_done alone: the head's sub-iteration 0
  __shared__ double out[kNumSums];
  __shared__ int stop;
  const int sp = 2 + 2 * na;
  if (threadIdx.x == 0) ctrl->kstored = slo + nsub;
  for (int i = 0; i < nsub; ++i) {
    reduce_partials(partials + (size_t)i * table_rows * kNumSums, table_rows, sp, out);
    if (threadIdx.x == 0) {
      double err = out[0] / out[1];
      for (int a = 0; a < na; ++a) err += out[2 + 2 * a] / out[3 + 2 * a];
      for (int a = 0; a < n_dead; ++a) {
        volatile double z = 0.0;
        err += z / z;
      }
      const int s = slo + i;
      stop = (err < eps || s + 1 >= kmax) ? 1 : 0;
      if (stop) {
        ctrl->kstar = s + 1;
        ctrl->kstar_found = 1;
        ctrl->inner_count = s + 1;
        ctrl->err_inner = err;
        ctrl->dual_sums[0] = out[0];
        ctrl->dual_sums[1] = out[1];
        for (int a = 0; a < na; ++a) {
          ctrl->dual_sums[3 + 3 * a] = out[2 + 2 * a];
          ctrl->dual_sums[4 + 3 * a] = out[3 + 2 * a];
        }
        if (err < eps) ctrl->inner_done = 1;
      }
    }
    __syncthreads();
    if (stop) break;
  }
}

// k > 1: sums between the outer iteration's initial (cur) and final (1-cur) dual state.
// partial rows: [0] sum (rho_f - rho_i)^2 [1] unused [2] sum rho_i^2, [3+3a] sum (da)^2, [5+3a] sum a_i^2
template <typename R>
// k1_skip: a loop that exited after its first sub-iteration (inner_count == 1) left the initial-vs-final sums in
// ctrl->outer_sums already (sub-iteration 0 reads the initial state and writes the final one), so the pass is
// skipped and k_finalize_outer takes those (the same sums up to summation order)
__global__ void __launch_bounds__(256) k_outer_sums(KP<R> p, size_t n, int k1_skip) {
  if (p.ctrl->done || (k1_skip && p.ctrl->inner_count == 1)) return;
  const int cur = p.ctrl->cur;
  double s[kNumSums];
  for (int i = 0; i < kNumSums; ++i) s[i] = 0.0;
  const bool all_rows = p.xl0 == 0 && p.xl1 == p.nx;   // else x-slab: live rows [xl0, xl1) only
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    if (!all_rows) {
      const int x = (int)((i / p.ny) % p.nx);
      if (x < p.xl0 || x >= p.xl1) continue;
    }
    const double ri = p.rho[cur][i], rf = p.rho[1 - cur][i];
    s[0] += (rf - ri) * (rf - ri);
    s[2] += ri * ri;
    for (int a = 0; a < p.na; ++a) {
      const double ai = p.alp[cur][a][i], af = p.alp[1 - cur][a][i];
      s[3 + 3 * a] += (af - ai) * (af - ai);
      s[5 + 3 * a] += ai * ai;
    }
  }
  block_reduce_store<kNumSums>(s, p.partials, blockIdx.x);
}

// End of an outer iteration: err1, err2 (utils_pdhg_solver.py:58-68), stop tests (:74-80).
// outer_rows > 0: reduce k_outer_sums partials first (k > 1); else use the sub-iteration-0 sums (also with k1_skip
// when the dual loop ran one sub-iteration: k_outer_sums skipped).
// thread 0's part (os: the outer sums)
__device__ __forceinline__ void finalize_outer_sums(const double* os, int na, double eps, int flip, int stop_conv,
                                                    int stop_nan, Ctrl* ctrl) {
  {
    const double err1 = sqrt(ctrl->s_dphi) / sqrt(ctrl->s_phi_old);
    double err2 = sqrt(os[0]) / sqrt(os[2]);
    for (int a = 0; a < na; ++a) {
      const double norm_alp = sqrt(os[5 + 3 * a]);
      const double norm_err = sqrt(os[3 + 3 * a]);
      if (norm_alp < 1e-6 && norm_err > 1e-6) err2 += norm_err;
      else if (norm_alp >= 1e-6) err2 += norm_err / norm_alp;
    }
    ctrl->err1 = err1;
    ctrl->err2 = err2;
    ctrl->iters += 1;
    ctrl->inner_total += ctrl->inner_count;
    const double rho_new_sq = ctrl->dual_sums[1];
    if (err1 < eps && err2 < eps) {
      if (stop_conv) ctrl->done = 1;
    } else if (ctrl->s_phi_new != ctrl->s_phi_new || rho_new_sq != rho_new_sq) {
      if (stop_nan) ctrl->done = 2;
      if (!ctrl->nan_seen) ctrl->first_nan = ctrl->iters;
      ctrl->nan_seen = 1;
    }
    if (flip) ctrl->cur = 1 - ctrl->cur;
    ctrl->inner_done = 0;
    ctrl->kstar_found = 0;
    ctrl->primal_valid = 0;
  }
}
__global__ void __launch_bounds__(1024) k_finalize_outer(const double* partials, int outer_rows, int na, double eps,
                                                        int flip, int stop_conv, int stop_nan, Ctrl* ctrl,
                                                        int k1_skip = 0) {
  if (ctrl->done) return;
  __shared__ double out[kNumSums];
  if (k1_skip && ctrl->inner_count == 1) outer_rows = 0;   // uniform: inner_count is not written below
  if (outer_rows > 0) reduce_partials(partials, outer_rows, kNumSums, out);
  if (threadIdx.x == 0) finalize_outer_sums((outer_rows > 0) ? out : ctrl->outer_sums, na, eps, flip, stop_conv,
                                           stop_nan, ctrl);
}

// A speculative iteration's sub-iteration-0 finalize and its outer finalize in one launch (iterate()'s speculative
// schedule, pdhg_api.hip): the two were adjacent launches there -- k_finalize_dual(spec) then k_finalize_outer with
// the one-sub-iteration skip (inner_count == 1, sums from ctrl->outer_sums) -- and thread 0 runs both bodies in that
// order, so the control block ends the same.  A loop that does not exit halts (done = kHaltTail) and the outer part
// is not run, as k_finalize_outer returned at entry then.
// prim_rows > 0: the iteration's primal finalize too (k_finalize_primal's reduction of the update's rows, first: a
// halted iteration's outer tests, run later by the host, read its sums)
__global__ void __launch_bounds__(1024) k_finalize_dual_outer(const double* prim_partials, int prim_rows,
                                                             const double* partials, int nrows, int na, int n_dead,
                                                             double eps, int flip, int stop_conv, int stop_nan,
                                                             Ctrl* ctrl) {
  if (ctrl->done || ctrl->inner_done) return;
  __shared__ double out[kNumSums];
  if (prim_rows > 0) {
    reduce_partials(prim_partials, prim_rows, 3, out);
    if (threadIdx.x == 0) {
      const double row0_sq = ctrl->row0_sq;
      ctrl->s_dphi = out[0];
      ctrl->s_phi_old = out[1] + row0_sq;
      ctrl->s_phi_new = out[2] + row0_sq;
      ctrl->primal_valid = 1;
    }
  }
  reduce_partials(partials, nrows, 3 + 3 * na, out);
  finalize_dual_sums(out, na, n_dead, eps, 0, ctrl, 1);
  if (threadIdx.x == 0 && ctrl->done == 0) finalize_outer_sums(ctrl->outer_sums, na, eps, flip, stop_conv, stop_nan, ctrl);
}

// ---- state initialisation / conversion ----
template <typename R>
__global__ void k_fill(R* __restrict__ p, size_t n, R v) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}

// every row of dst [rows][plane] = src [plane]
template <typename R>
__global__ void k_bcast_rows(R* __restrict__ dst, const R* __restrict__ src, size_t plane, int rows) {
  const size_t n = plane * (size_t)rows;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i % plane];
}

template <typename R>
__global__ void k_copy(R* __restrict__ dst, const R* __restrict__ src, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

}  // namespace pdhg

// ---------------- t-slab decomposition (multi-GPU), see oracle/slab_oracle.py ----------------
namespace pdhg {

// Fold a partial-sum table into one row of kNumSums doubles (the vector the ranks all-reduce);
// add0 is added to sums 1 and 2 (the fixed phi row 0 in the primal sums, first slab only).
__global__ void __launch_bounds__(1024) k_reduce_vec(const double* partials, int nrows, int ns, double add0,
                                                    double* out) {
  __shared__ double o[kNumSums];
  reduce_partials(partials, nrows, ns, o);
  if (threadIdx.x < kNumSums) out[threadIdx.x] = (threadIdx.x < ns ? o[threadIdx.x] : 0.0) +
                                                 ((threadIdx.x == 1 || threadIdx.x == 2) ? add0 : 0.0);
}

// Per spectral mode m of the work-row layout (2-D: m = (b*nx + kx)*B + c, ky = b*B + c; half_real:
// item k of block b holds kx = k, k + nx/2): dd = d0/ae and the pivot state entering row j0.
template <typename R>
__device__ __forceinline__ void slab_mode(const KP<R>& p, size_t m, double& dd, double& h) {
  const int nx = p.nx, B = p.B;
  int kx, ky;
  if (p.half_real) {
    const int w = (int)(m % nx);
    ky = (int)(m / nx);
    kx = (w >> 1) + (w & 1) * (nx >> 1);
  } else {
    const int c = (int)(m % B);
    const size_t bx = m / B;
    kx = (int)(bx % nx);
    ky = (int)(bx / nx) * B + c;
  }
  dd = ((double)p.C - (double)p.lamx[kx] - (double)p.cx[kx] * (double)p.lamy[ky]) / (double)p.ae;
  h = 1.0;
  if (p.j0 > 0) {   // closed form h_{j0-1} (see h_entry)
    const double dl = 0.5 * dd;
    const double th = fmax(log1p(dl + sqrt(dl * (dl + 2.0))), 1e-300);
    h = expm1(-th) * (1.0 + exp(-th * (2.0 * p.j0 + 1.0))) / expm1(-2.0 * th * (p.j0 + 1.0));
  }
}
// pivot g_k of local row k (recurrence s = dd + h, g = 1/(1+s), h = s g; Neumann window end: g = 1/s)
template <typename R>
__device__ __forceinline__ double slab_pivot(const KP<R>& p, int k, double dd, double& h) {
  const double s = dd + h;
  const double g = (p.last_slab && k == p.T - 1) ? 1.0 / s : 1.0 / (1.0 + s);
  h = s * g;
  return g;
}

// Exchange planes of a slab (oracle/slab_oracle.py, single-exchange variant), 2 planes of M each:
//   data = 0 (once per context):  out = [G, S2],  G = prod_k g_k,  S2 = sum_k P'_k P_k
//   data = 1 (every iteration):   out = [D, S1],  D = b0 of the last local row,  S1 = sum_k P'_k b0_k
// (P'_k = prod g_{j0..k-1}, P_k = P'_k g_k; b0 = the zero-carry forward sweep stored in work).
// The products only decrease (0 < g <= 1); once P'_k < kSlabDrop the remaining terms of S1 are below that
// relative weight and the row sweep stops (the high-frequency modes decay within a few rows), the same
// bound as the neighbour exchange's short-range classification (LONG_RANGE_DELTA = 2^-40).
constexpr double kSlabDrop = 9.094947017729282e-13;   // 2^-40
template <typename R>
__global__ void __launch_bounds__(256) k_slab_sums(KP<R> p, int data, R* __restrict__ out, size_t m0, size_t m1) {
  if (data && p.ctrl->done) return;
  const size_t M = (size_t)p.nb * p.nx * p.B;
  const size_t m = m0 + (size_t)blockIdx.x * blockDim.x + threadIdx.x;   // modes [m0, m1)
  if (m >= m1) return;
  double dd, h;
  slab_mode(p, m, dd, h);
  double P = 1.0, s = 0.0;
  for (int k = 0; k < p.T; ++k) {
    if (data && P < kSlabDrop) break;
    const double g = slab_pivot(p, k, dd, h);
    if (data) {
      s += P * (double)p.work[(size_t)k * M + m];
    } else {
      s += P * P * g;
    }
    P *= g;
  }
  out[m] = data ? p.work[(size_t)(p.T - 1) * M + m] : (R)P;
  out[M + m] = (R)s;
}

// Carries of slab `rank` from everybody's planes (allDS[q] = [D_q, S1_q], allGS[q] = [G_q, S2_q]):
//   c_in(q) = D_{q-1} + G_{q-1} c_in(q-1)              (carry INTO slab q; c_in(0) = 0)
//   X0_q    = S1_q + c_in(q) S2_q                       (slab q's zero-right-carry backward value)
//   y       = sum_{q > rank} (prod_{rank < s < q} G_s) X0_q   (= x at this slab's j1; written to carry_y)
// then the own rows' forward fix-up b_k += P_k c_in(rank).
template <typename R>
__global__ void __launch_bounds__(256) k_slab_fix(KP<R> p, const R* __restrict__ allDS, const R* __restrict__ allGS,
                                                  int rank, int nranks, R* __restrict__ carry_y) {
  if (p.ctrl->done) return;
  const size_t M = (size_t)p.nb * p.nx * p.B;
  const size_t m = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  double c = 0.0, c_own = 0.0, y = 0.0, W = 1.0;
  for (int q = 0; q < nranks; ++q) {
    const size_t o = (size_t)q * 2 * M + m;
    if (q == rank) c_own = c;
    if (q > rank) {
      y += W * ((double)allDS[o + M] + c * (double)allGS[o + M]);
      W *= (double)allGS[o];
    }
    c = (double)allDS[o] + (double)allGS[o] * c;
  }
  carry_y[m] = (R)y;
  if (rank > 0) {
    double dd, h;
    slab_mode(p, m, dd, h);
    double P = 1.0;
    for (int k = 0; k < p.T; ++k) {
      P *= slab_pivot(p, k, dd, h);
      if (P < kSlabDrop) break;   // decreasing: the carry's weight on the remaining rows is below 2^-40
      R* w = p.work + (size_t)k * M + m;
      *w = (R)((double)*w + P * c_own);
    }
  }
}

// Neighbour-exchange variant of k_slab_fix.  The gain G_q = prod g over slab q's rows depends only on
// the mode and the slab length; where every slab's G_q < delta (pos[m] < 0: "short-range" modes, all
// but a few thousand low frequencies) the far terms G_{q-1} c_in(q-1) and G_{q+1} y_{q+1} are below
// delta relative and
//   c_in(rank) = D_{rank-1},   y = X0_{rank+1} = S1_{rank+1} + (D_rank + G_rank c_in(rank)) S2_{rank+1},
// so only the neighbours' D (from the left) and S1 (from the right) are needed.  The long-range modes
// (pos[m] = their index in the compact list of K) fold exactly as k_slab_fix from everybody's compact
// [D, S1] (allLong[q] = [D_q(K), S1_q(K)]).  oracle/slab_oracle.py: thomas_slabs_neighbour.
template <typename R>
__global__ void __launch_bounds__(256) k_slab_fix_nb(KP<R> p, const R* __restrict__ ownDS, const R* __restrict__ D_left,
                                                     const R* __restrict__ S1_right, const R* __restrict__ allLong,
                                                     const int* __restrict__ pos, int K, const R* __restrict__ allGS,
                                                     int rank, int nranks, R* __restrict__ carry_y, size_t m0,
                                                     size_t m1) {
  if (p.ctrl->done) return;
  const size_t M = (size_t)p.nb * p.nx * p.B;
  const size_t m = m0 + (size_t)blockIdx.x * blockDim.x + threadIdx.x;   // modes [m0, m1)
  if (m >= m1) return;
  double c_own = 0.0, y = 0.0;
  const int q = pos[m];
  if (q >= 0) {
    double c = 0.0, W = 1.0;
    for (int s = 0; s < nranks; ++s) {
      const R* L = allLong + (size_t)s * 2 * K;
      const size_t o = (size_t)s * 2 * M + m;
      if (s == rank) c_own = c;
      if (s > rank) {
        y += W * ((double)L[K + q] + c * (double)allGS[o + M]);
        W *= (double)allGS[o];
      }
      c = (double)L[q] + (double)allGS[o] * c;
    }
  } else {
    if (rank > 0) c_own = (double)D_left[m];
    if (rank + 1 < nranks) {
      const size_t o = (size_t)rank * 2 * M + m;
      const double cn = (double)ownDS[m] + (double)allGS[o] * c_own;   // carry into slab rank+1
      y = (double)S1_right[m] + cn * (double)allGS[o + 3 * M];         // S2 of slab rank+1
    }
  }
  carry_y[m] = (R)y;
  if (rank > 0) {
    double dd, h;
    slab_mode(p, m, dd, h);
    double P = 1.0;
    for (int k = 0; k < p.T; ++k) {
      P *= slab_pivot(p, k, dd, h);
      if (P < kSlabDrop) break;   // decreasing: the carry's weight on the remaining rows is below 2^-40
      R* w = p.work + (size_t)k * M + m;
      *w = (R)((double)*w + P * c_own);
    }
  }
}

// max over slabs of the gain G_q of every mode (classifies long-range modes once)
template <typename R>
__global__ void __launch_bounds__(256) k_slab_gmax(const R* __restrict__ allGS, size_t M, int nranks,
                                                   R* __restrict__ out) {
  const size_t m = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  R g = 0;
  for (int s = 0; s < nranks; ++s) g = fmax(g, fabs(allGS[(size_t)s * 2 * M + m]));
  out[m] = g;
}

// compact [D(K), S1(K)] of the long-range modes from this slab's [D, S1] planes
template <typename R>
__global__ void __launch_bounds__(256) k_slab_gather_long(const R* __restrict__ DS, size_t M, const int* __restrict__ idx,
                                                          int K, R* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= K) return;
  out[i] = DS[idx[i]];
  out[K + i] = DS[M + idx[i]];
}

// rho row 0 of the current buffer set (the set index lives on the device)
template <typename R>
__global__ void __launch_bounds__(256) k_copy_cur_rho(KP<R> p, R* __restrict__ dst, size_t n) {
  const R* src = p.rho[p.ctrl->cur];
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

}  // namespace pdhg
