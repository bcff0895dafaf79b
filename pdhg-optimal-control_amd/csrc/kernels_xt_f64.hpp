// fp64 x-transform + Thomas in t for power-of-two nx = N >= 4096 (the reference's own precision at C3's grid:
// jaxsrc runs float64 / complex128 throughout, solver.py:11, update_fns_in_pdhg.py:10).
//
// Same preconditioner as the fp32 kernels (H1_precond_2d, utils_precond.py:142-178: DHT_x of the spectral
// rows, the tridiagonal solve in t per mode, inverse DHT_x) and the same Thomas algebra as
// k_precond_xt_fast_2d (cancellation-free pivot recurrence forward, closed-form pivots backward), in double.
// The generic runtime-radix kernel keeps two FFT buffers and three per-mode carry arrays in LDS (5 M reals:
// 320 KiB for a 4096-point column pair in fp64), so it stops at nx = 2048 in fp64.  Here the block's one
// complex line (B = 2 real columns packed as z = a + i b) is transformed in place in a padded LDS line
// (68 KiB + 13 KiB of twiddle seeds); a thread owns IT = N/NT items (kx), each carrying the two modes
// (kx, 2b) and (kx, 2b + 1): the dd of the mode pair (then theta) and the forward pivot state h (then E) stay
// in registers, b' / x in a 64 KiB LDS array (148 KiB in all; registers for all three spilled).  The next row
// is prefetched into registers before the transform (loads in flight across the LDS passes).
// Single context only (no t-slab phases: the slab decomposition is fp32).
// grid: nb column blocks; block NT; LDS (N + N/16 + TwLds<N> + N) * 16 B.
#pragma once
#include "kernels_2d_fast.hpp"

namespace pdhg {

template <int N, int NT>
__global__ void __launch_bounds__(NT) k_precond_xt_f64_2d(KP<double> p, const double2* __restrict__ twx) {
  using C = double2;
  constexpr int IT = N / NT;
  constexpr int LINE = Pad<N>::LINE;
  constexpr int M = 2 * N;   // B = 2 real columns per block
  static_assert(N % NT == 0 && N <= 4096, "one padded complex line and its twiddle seeds in LDS");
  if (p.ctrl->done) return;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  C* A = reinterpret_cast<C*>(smem_raw);
  C* twl = A + LINE;
  C* bp = twl + TwLds<N>::SIZE;   // b' / x per item
  fill_twlds<C, N>(twl, twx);
  const int T = p.T, tid = threadIdx.x;
  const int b = blockIdx.x;
  double* wb = p.work + (size_t)b * M;
  const size_t kstride = (size_t)p.nb * M;
  const double inv_ae = 1.0 / p.ae;
  const double ly0 = p.lamy[2 * b], ly1 = p.lamy[2 * b + 1];
  // per item: dd = (C - lam)/ae of the two modes, then theta; h = 1 - g, then E; b', then x
  C dd[IT], h[IT], pf[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int kx = tid + i * NT;
    const double lx = p.lamx[kx];
    dd[i] = make_double2((p.C - lx - ly0) * inv_ae, (p.C - lx - ly1) * inv_ae);
    h[i] = make_double2(1.0, 1.0);   // h_{-1} = 1: the first row's pivot is dd + 2
    bp[kx] = make_double2(0.0, 0.0);
  }
  auto ldrow = [&](int k) {
    const C* s = reinterpret_cast<const C*>(wb + (size_t)k * kstride);
#pragma unroll
    for (int i = 0; i < IT; ++i) pf[i] = s[tid + i * NT];
  };
  // ---------------- forward: DHT_x + elimination ----------------
  //   s = dd + h_{k-1},  g_k = 1/(1+s),  h_k = s g_k,  b'_k = (rhs/ae + b'_{k-1}) g_k
  //   last (Neumann) row: x_{T-1} = (rhs/ae + b'_{T-2}) / (dd + h_{T-2})
  ldrow(0);
  for (int k = 0; k < T; ++k) {
#pragma unroll
    for (int i = 0; i < IT; ++i) A[pix(tid + i * NT)] = pf[i];
    if (k + 1 < T) ldrow(k + 1);
    lds_sync();
    lds_fft_inplace_tl<C, N, 1, NT>(A, twl);
    C* dst = reinterpret_cast<C*>(wb + (size_t)k * kstride);
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int kx = tid + i * NT;
      double ha, hb;
      hartley_padded<C, double>(A, N, kx, ha, hb);
      const C b0 = bp[kx];
      if (k < T - 1) {
        const double s0 = dd[i].x + h[i].x, s1 = dd[i].y + h[i].y;
        const double g0 = 1.0 / (1.0 + s0), g1 = 1.0 / (1.0 + s1);
        const C bn = make_double2((ha * inv_ae + b0.x) * g0, (hb * inv_ae + b0.y) * g1);
        h[i] = make_double2(s0 * g0, s1 * g1);
        bp[kx] = bn;
        dst[kx] = bn;
      } else {
        bp[kx] = make_double2((ha * inv_ae + b0.x) / (dd[i].x + h[i].x), (hb * inv_ae + b0.y) / (dd[i].y + h[i].y));
      }
    }
    lds_sync();
  }
  // ---------------- backward: substitution + inverse DHT_x ----------------
  //   x_k = b'_k + g_k x_{k+1},  g_k = e^-th E_{k+1}/E_{k+2},  E_m = expm1(-2 th m),  cosh th = 1 + dd/2
  //   (th -> 0: g_k -> (k+1)/(k+2))
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const double d0 = 0.5 * dd[i].x, d1 = 0.5 * dd[i].y;
    dd[i] = make_double2(log1p(d0 + sqrt(d0 * (d0 + 2.0))), log1p(d1 + sqrt(d1 * (d1 + 2.0))));   // theta
    h[i] = make_double2(expm1(-2.0 * dd[i].x * T), expm1(-2.0 * dd[i].y * T));                      // E_{k+2}, k = T-2
  }
  if (T >= 2) ldrow(T - 2);
  auto gk = [](double th, double e1, double e2, int k) {
    return th > 1e-150 ? exp(-th) * e1 / e2 : (double)(k + 1) / (double)(k + 2);
  };
  for (int k = T - 1; k >= 0; --k) {
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int kx = tid + i * NT;
      C x = bp[kx];
      if (k < T - 1) {
        const double e1x = expm1(-2.0 * dd[i].x * (k + 1)), e1y = expm1(-2.0 * dd[i].y * (k + 1));
        x = make_double2(pf[i].x + gk(dd[i].x, e1x, h[i].x, k) * x.x, pf[i].y + gk(dd[i].y, e1y, h[i].y, k) * x.y);
        h[i] = make_double2(e1x, e1y);
        bp[kx] = x;
      }
      A[pix(kx)] = x;
    }
    if (k < T - 1 && k >= 1) ldrow(k - 1);
    lds_sync();
    lds_fft_inplace_tl<C, N, 1, NT>(A, twl);
    C* wk = reinterpret_cast<C*>(wb + (size_t)k * kstride);
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int kx = tid + i * NT;
      double ha, hb;
      hartley_padded<C, double>(A, N, kx, ha, hb);
      wk[kx] = make_double2(ha, hb);
    }
    lds_sync();
  }
}

}  // namespace pdhg
