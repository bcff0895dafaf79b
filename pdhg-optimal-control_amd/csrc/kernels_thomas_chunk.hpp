// 1-D H1 preconditioner t-solve split over chunks of CL time rows per mode (fp32 / fp64; H1_precond_1d,
// utils_precond.py:105-140: (C - lam)^pow u - Ct Dtt u = v per Fourier mode, u_0 = 0, Neumann at t = T).
//
// k_thomas_1d runs one thread per mode through all T rows twice: 65536 threads at C1 (one wave per SIMD),
// each step a dependent load -> recurrence -> store, so the kernel is latency-bound (0.23 ms for 0.21 GB).
// Here a workgroup owns 64 modes (one per lane) and all P = ceil(T/CL) chunks of their rows (one wave
// per chunk).  Both recurrences of the Thomas solve are affine in the value carried into a chunk, with
// data-independent coefficients, so (the algebra of the t-slab decomposition, oracle/slab_oracle.py):
//   forward   b'_k = b0_k + G_k c,   G_k = prod_{m=j0..k} g_m   (b0: the chunk's sweep from a zero carry)
//   backward  x_k  = x0_k + H_k y,   H_k = prod_{m=k..j1-1} g_m (x0: from a zero right carry y = x_{j1})
// Each wave loads its chunk's CL rows into registers at once (CL rows of loads in flight), sweeps forward
// from zero with pivots starting at the closed-form h_{j0-1}, and leaves (b0_last, G_last) in LDS; one wave
// scans the P chunk carries c_q = b'_{j0-1} per mode; every wave folds its carry in, sweeps backward from
// zero, leaves (x0_first, H_first); one wave scans the right carries; every wave folds y in and stores its
// rows.  HBM traffic: each spectrum row read once and written once (8 B per point), no intermediate rows.
// Pivots (cancellation-free, as the other Thomas kernels): s = dd + h_{k-1}, g_k = 1/(1+s), h_k = s g_k,
// b'_k = (v_k/ae + b'_{k-1}) g_k; last row of the window: b'_{T-1} = (v/ae + b'_{T-2}) / (dd + h_{T-2}),
// x_{T-1} = b'_{T-1}; x_k = b'_k + g_k x_{k+1}.  dd = d0/ae, d0 = (C - lam)^pow, ae = Ct/dt^2 > 0.
// grid: ceil(nx/64); block 64 * P (P <= 16); LDS 3 * 16 * 64 reals.  fp32 pivots through v_rcp_f32 (1 ulp, the
// recurrence is contractive), fp64 through correctly rounded divisions (layout for fp64 below).
#pragma once
#include "kernels_2d_fast.hpp"

namespace pdhg {

// fp64 (CPW = 2 chunks per wave): v[CL] and g[CL] in doubles at CL = 32 exceed the 128 VGPRs a 1024-thread
// block allows, so each half-wave owns one chunk of CL = 16 rows for 32 modes (a half-wave still reads 256 B
// contiguous per row): up to 32 chunks, T <= 512, 64 VGPRs of rows and multipliers.
// grid: ceil(nx / (64 / CPW)); block 64 * ceil(P / CPW) (P = ceil(T / CL) <= 16 * CPW).
template <int CL, int CPW = 1, typename R = float>
__global__ void __launch_bounds__(1024) k_thomas_chunk_1d(KP<R> p) {
  if (p.ctrl->done) return;
  constexpr int W = 64 / CPW;                         // modes per workgroup
  __shared__ R sA[16 * CPW][W], sB[16 * CPW][W], sC[16 * CPW][W];
  auto rcp = [](R x) {
    if constexpr (sizeof(R) == 4) return rcp_fast(x);
    else return (R)1 / x;
  };
  const int lane = threadIdx.x & (W - 1);
  const int q = (threadIdx.x >> 6) * CPW + ((threadIdx.x & 63) / W), P = (blockDim.x >> 6) * CPW;
  const int nx = p.nx, T = p.T;
  const int kx = blockIdx.x * W + lane;
  const bool live = kx < nx;
  const int j0 = q * CL, j1 = min(j0 + CL, T);        // j1 <= j0: an empty chunk (carry passes through)
  const int kxc = live ? kx : nx - 1;                 // loads stay in range; stores only for live modes
  R* w = p.work + kxc;
  const R ae = p.ae, inv_ae = (R)1 / ae;
  const R dd = p.d0_1d[kxc] * inv_ae;
  R v[CL], g[CL];
#pragma unroll
  for (int i = 0; i < CL; ++i)
    if (j0 + i < j1) v[i] = w[(size_t)(j0 + i) * nx];
  // ---- forward from a zero carry ----
  R h = h_entry(dd, j0), b = (R)0, G = (R)1;
#pragma unroll
  for (int i = 0; i < CL; ++i) {
    if (j0 + i < j1) {
      const R s = dd + h;
      R gi;
      if (j0 + i < T - 1) {
        gi = rcp((R)1 + s);
        h = s * gi;
      } else {                                        // Neumann row of the window
        gi = (R)1 / s;
      }
      b = (v[i] * inv_ae + b) * gi;
      G *= gi;
      v[i] = b;
      g[i] = gi;                                      // forward multiplier (the backward skips row T-1)
    }
  }
  sA[q][lane] = b;
  sB[q][lane] = G;
  __syncthreads();
  if (q == 0) {                                       // carries into each chunk: c_0 = 0, c_{q+1} = D_q + G_q c_q
    R c = (R)0;
    for (int r = 0; r < P; ++r) {
      sC[r][lane] = c;
      c = sA[r][lane] + sB[r][lane] * c;
    }
  }
  __syncthreads();
  {                                                   // fold the carry in: b'_k = b0_k + G_k c
    const R c = sC[q][lane];
    R Gk = (R)1;
#pragma unroll
    for (int i = 0; i < CL; ++i) {
      if (j0 + i < j1) {
        Gk *= g[i];
        v[i] += Gk * c;
        if (j0 + i == T - 1) g[i] = (R)0;             // x_{T-1} = b'_{T-1}
      }
    }
  }
  // ---- backward from a zero right carry ----
  R x = (R)0, H = (R)1;
#pragma unroll
  for (int i = CL - 1; i >= 0; --i) {
    if (j0 + i < j1) {
      x = v[i] + g[i] * x;
      H *= g[i];
      v[i] = x;                                       // x0_k
    }
  }
  __syncthreads();
  sA[q][lane] = x;                                    // x0 of the chunk's first row
  sB[q][lane] = H;                                    // prod of g over the chunk
  __syncthreads();
  if (q == 0) {                                       // right carries: y_{P-1} = 0, y_q = X0_{q+1} + H_{q+1} y_{q+1}
    R y = (R)0;
    for (int r = P - 1; r >= 0; --r) {
      sC[r][lane] = y;
      y = sA[r][lane] + sB[r][lane] * y;
    }
  }
  __syncthreads();
  const R y = sC[q][lane];
  R Hk = (R)1;
#pragma unroll
  for (int i = CL - 1; i >= 0; --i) {
    if (j0 + i < j1) {
      Hk *= g[i];
      if (live) w[(size_t)(j0 + i) * nx] = v[i] + Hk * y;
    }
  }
}

}  // namespace pdhg
