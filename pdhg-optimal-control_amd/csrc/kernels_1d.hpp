// 1-D PDHG kernels (ndim = 1), same pass structure as 2-D (kernels_2d.hpp):
//   k_res_fwdx_1d    continuity residual (update_fns_in_pdhg.py:72-81) + forward DHT along x
//                    of two time rows packed as one complex line
//   k_thomas_1d      tridiagonal solve in t per mode, closed-form pivots (utils_precond.py:125-132)
//   k_invx_update_1d inverse DHT along x + phi update / phi_bar / err1 sums
//   k_dual_1d        alpha / rho prox + err sums (update_fns_in_pdhg.py:99-113, 150-165)
// Spectral work layout: work[k][kx] (natural order).
#pragma once
#include "params.hpp"

namespace pdhg {

template <typename R, int EGNO>
__device__ __forceinline__ R cont_residual_1d(const KP<R>& p, const R* __restrict__ rho, const R* __restrict__ a1,
                                              const R* __restrict__ a2, int j, int x) {
  const int nx = p.nx;
  const R* rj = rho + (size_t)j * nx;
  const R* b1 = a1 + (size_t)j * nx;
  const R* b2 = a2 + (size_t)j * nx;
  const int xm = nb_index(x - 1, nx, p.bcx), xp = nb_index(x + 1, nx, p.bcx);
  const R eps = (R)1e-4;
  const R r0 = rj[x];
  const R rnext = (j + 1 < p.T) ? rho[(size_t)(j + 1) * nx + x] : (R)0;
  R res = (rnext - r0) * p.inv_dt;                                     // Dt_increasedim
  if (p.epsl != (R)0) {
    const R rxm = (xm >= 0) ? rj[xm] : (R)0;
    const R rxp = (xp >= 0) ? rj[xp] : (R)0;
    res = res + p.epsl * ((rxp + rxm - (R)2 * r0) * p.inv_dx2);        // Dxx_increasedim
  }
  const R a = p.ax[x];
  const R m1c = (r0 + eps) * fpos<R>(fval<R, EGNO>(b1[x], a));
  const R m1m = (xm >= 0) ? (rj[xm] + eps) * fpos<R>(fval<R, EGNO>(b1[xm], p.ax[xm])) : (R)0;
  const R m2c = (r0 + eps) * fneg<R>(fval<R, EGNO>(b2[x], a));
  const R m2p = (xp >= 0) ? (rj[xp] + eps) * fneg<R>(fval<R, EGNO>(b2[xp], p.ax[xp])) : (R)0;
  res = res - ((m1c - m1m) * p.inv_dx + (m2p - m2c) * p.inv_dx);      // Dx_left_inc(m1) + Dx_right_inc(m2)
  if (j == p.T - 1) res = res + p.c_over_dt;
  return res;
}

// grid: ceil(T/2) row pairs; block 256; LDS 2 * nx complex
template <typename R, int EGNO, class F>
__global__ void __launch_bounds__(1024) k_res_fwdx_1d(KP<R> p, F plx, const cplx<R>* __restrict__ twx) {
  using C = cplx<R>;
  if (p.ctrl->done) return;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  C* A = plx.template buffer<C>(reinterpret_cast<C*>(smem_raw), reinterpret_cast<C*>(p.gscr), blockIdx.x);
  C* Bf = A + plx.n();
  const int cur = p.ctrl->cur;
  const R* rho = p.rho[cur];
  const R* a1 = p.alp[cur][0];
  const R* a2 = p.alp[cur][1];
  const int nx = p.nx;
  const int j = blockIdx.x * 2;
  const bool has2 = (j + 1) < p.T;
  for (int x = threadIdx.x; x < nx; x += blockDim.x) {
    const R r0 = cont_residual_1d<R, EGNO>(p, rho, a1, a2, j, x);
    const R r1 = has2 ? cont_residual_1d<R, EGNO>(p, rho, a1, a2, j + 1, x) : (R)0;
    A[x] = cmk<C>(r0, r1);
  }
  __syncthreads();
  const C* Z = plx.template run<C>(A, Bf, twx);
  R* w0 = p.work + (size_t)j * nx;
  for (int k = threadIdx.x; k < nx; k += blockDim.x) {
    R ha, hb;
    hartley_pair<C, R>(Z, nx, 1, k, 0, ha, hb);
    w0[k] = ha;
    if (has2) w0[nx + k] = hb;
  }
}

// ---- four-step DHT of row pairs for nx = 65536 = 256 x 256 (fp32; C1, BASELINE configs[1]) ----
// x = 256 n1 + n2, k = k1 + 256 k2:  X[k] = sum_n2 W_256^{n2 k2} W_65536^{n2 k1} sum_n1 W_256^{n1 k1} z[256 n1 + n2].
// A line that does not fit in LDS is split over 16 + 9 workgroups per row pair instead of one workgroup
// per pair (T = 400 rows gave 200 workgroups for 256 CUs).
// Stage 1 (grid 16 x pairs): 16 columns n2 per workgroup, 256-point FFTs over n1 in LDS, times
// W_65536^{n2 k1}, to Y[pair][k1][n2] (global scratch).  MODE 0: z = residual rows j, j+1
// (update_fns_in_pdhg.py:72-81); MODE 1: z = spectrum rows j, j+1 of work (the inverse DHT).
constexpr int kFsN1 = 256, kFsL = 16;
template <int MODE, int EGNO>
__global__ void __launch_bounds__(1024) k_fs1_1d(KP<float> p, const float2* __restrict__ tw256,
                                                const float2* __restrict__ twN, float2* __restrict__ Y) {
  using C = float2;
  if (p.ctrl->done) return;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  C* A = reinterpret_cast<C*>(smem_raw);
  C* Bf = A + kFsN1 * kFsL;
  const int nx = p.nx, tile = blockIdx.x, pair = blockIdx.y;
  const int j = 2 * pair;
  const bool has2 = (j + 1) < p.T;
  const int cur = p.ctrl->cur;
  for (int i = threadIdx.x; i < kFsN1 * kFsL; i += blockDim.x) {
    const int n1 = i >> 4, l = i & (kFsL - 1);
    const int x = kFsN1 * n1 + kFsL * tile + l;
    float r0, r1 = 0.f;
    if constexpr (MODE == 0) {
      r0 = cont_residual_1d<float, EGNO>(p, p.rho[cur], p.alp[cur][0], p.alp[cur][1], j, x);
      if (has2) r1 = cont_residual_1d<float, EGNO>(p, p.rho[cur], p.alp[cur][0], p.alp[cur][1], j + 1, x);
    } else {
      r0 = p.work[(size_t)j * nx + x];
      if (has2) r1 = p.work[(size_t)(j + 1) * nx + x];
    }
    A[i] = make_float2(r0, r1);   // line l (column n2), element n1
  }
  __syncthreads();
  const C* Z = lds_fft_fixed<C, kFsN1, kFsL>(A, Bf, tw256);
  C* Yp = Y + (size_t)pair * nx;
  for (int i = threadIdx.x; i < kFsN1 * kFsL; i += blockDim.x) {
    const int k1 = i >> 4, l = i & (kFsL - 1);
    const int n2 = kFsL * tile + l;
    Yp[(size_t)k1 * kFsN1 + n2] = cmul(Z[i], twN[(n2 * k1) & (nx - 1)]);
  }
}

// Stage 2 (grid 9 x pairs): rows k1 = 16 g + l (k1 <= 128) and their Hartley partners (256 - k1) mod 256,
// 256-point FFTs over n2, then the Hartley unpack of the two packed real lines: H[k] = (Z_k + Z_{N-k})/2 ...
// (hartley_pair).  MODE 0: the DHT rows go to work (spectral rows j, j+1); MODE 1: they are the inverse
// transform -- phi' = phi + tau/nx U, phi_bar = 2 phi' - phi and the err1 sums (k_invx_update_1d).
template <int MODE>
__global__ void __launch_bounds__(1024) k_fs2_1d(KP<float> p, const float2* __restrict__ tw256,
                                                const float2* __restrict__ Y) {
  using C = float2;
  double s[3] = {0.0, 0.0, 0.0};
  const int nx = p.nx, g = blockIdx.x, pair = blockIdx.y;
  const int row = blockIdx.y * gridDim.x + blockIdx.x;
  if (p.ctrl->done) {
    block_reduce_store<3>(s, p.partials, row);
    return;
  }
  extern __shared__ __align__(16) unsigned char smem_raw[];
  C* A = reinterpret_cast<C*>(smem_raw);     // rows k1 (lines l)
  C* Ab = A + kFsN1 * kFsL;
  C* Bm = Ab + kFsN1 * kFsL;                  // partner rows (256 - k1) mod 256
  C* Bb = Bm + kFsN1 * kFsL;
  const int j = 2 * pair;
  const bool has2 = (j + 1) < p.T;
  const C* Yp = Y + (size_t)pair * nx;
  for (int i = threadIdx.x; i < kFsN1 * kFsL; i += blockDim.x) {
    const int l = i >> 8, n2 = i & (kFsN1 - 1);   // consecutive threads read consecutive n2
    const int k1 = kFsL * g + l;
    const int k1b = (kFsN1 - k1) & (kFsN1 - 1);
    const bool ok = k1 <= kFsN1 / 2;
    A[n2 * kFsL + l] = ok ? Yp[(size_t)k1 * kFsN1 + n2] : make_float2(0.f, 0.f);
    Bm[n2 * kFsL + l] = ok ? Yp[(size_t)k1b * kFsN1 + n2] : make_float2(0.f, 0.f);
  }
  __syncthreads();
  const C* ZA = lds_fft_fixed<C, kFsN1, kFsL>(A, Ab, tw256);
  const C* ZB = lds_fft_fixed<C, kFsN1, kFsL>(Bm, Bb, tw256);
  const float scale = p.tau * p.inv_n;
  for (int i = threadIdx.x; i < kFsN1 * kFsL; i += blockDim.x) {
    const int k2 = i >> 4, l = i & (kFsL - 1);   // consecutive threads: consecutive k1 (64-B segments)
    const int k1 = kFsL * g + l;
    if (k1 > kFsN1 / 2) continue;
    const bool self = (k1 == 0) || (k1 == kFsN1 / 2);   // the partner row is the row itself
    const int k2m = (k1 == 0) ? ((kFsN1 - k2) & (kFsN1 - 1)) : (kFsN1 - 1 - k2);
    const C z = ZA[k2 * kFsL + l], w = ZB[k2m * kFsL + l];   // Z_k, Z_{N-k}
    const int k = k1 + kFsN1 * k2, km = (nx - k) & (nx - 1);
    // DHT pair at k (from Z_k, Z_{N-k}) and at N-k (roles swapped); a self-paired row writes k only
    const float ha = 0.5f * ((z.x + w.x) - (z.y - w.y)), hb = 0.5f * ((z.y + w.y) - (w.x - z.x));
    const float ma = 0.5f * ((w.x + z.x) - (w.y - z.y)), mb = 0.5f * ((w.y + z.y) - (z.x - w.x));
    const int nout = self ? 1 : 2;
    for (int o = 0; o < nout; ++o) {
      const int kk = o ? km : k;
      const float va = o ? ma : ha, vb = o ? mb : hb;
      if constexpr (MODE == 0) {
        p.work[(size_t)j * nx + kk] = va;
        if (has2) p.work[(size_t)(j + 1) * nx + kk] = vb;
      } else {
        for (int r = 0; r < 2; ++r) {
          if (r == 1 && !has2) break;
          const size_t idx = (size_t)(j + 1 + r) * nx + kk;
          const float old = p.phi[idx];
          const float nw = old + scale * (r ? vb : va);
          p.phi[idx] = nw;
          p.phibar[idx] = 2.f * nw - old;
          const double d = (double)nw - (double)old;
          s[0] += d * d;
          s[1] += (double)old * (double)old;
          s[2] += (double)nw * (double)nw;
        }
      }
    }
  }
  if constexpr (MODE == 1) block_reduce_store<3>(s, p.partials, row);
}

// grid: ceil(nx/256); one thread per mode, sequential in t.
// (C - lam)^pow u - Ct Dtt u = v with u_0 = 0, Neumann at t = T  (utils_precond.py:105-140)
template <typename R>
__global__ void __launch_bounds__(256) k_thomas_1d(KP<R> p) {
  if (p.ctrl->done) return;
  const int kx = blockIdx.x * blockDim.x + threadIdx.x;
  const int nx = p.nx, T = p.T;
  if (kx >= nx) return;
  R* w = p.work + kx;
  const R d0 = p.d0_1d[kx];
  const R ae = p.ae;
  if (ae == (R)0) {            // Ct == 0: v / thomas_b (utils_precond.py:133-134)
    for (int k = 0; k < T; ++k) w[(size_t)k * nx] = w[(size_t)k * nx] / d0;
    return;
  }
  const R inv_ae = (R)1 / ae;
  const R delta = d0 / ((R)2 * ae);
  const R th = log1p(delta + sqrt(delta * (delta + (R)2)));
  const R em = exp(-th);
  R E = expm1((R)-2 * th);
  R bp = (R)0;
  // each row's load is issued one step ahead (the rows are independent addresses; without the explicit
  // prefetch the store to row k keeps the load of row k+1 behind it)
  R hn = w[0];
  for (int k = 0; k < T; ++k) {
    const R h = hn;
    if (k + 1 < T) hn = w[(size_t)(k + 1) * nx];
    if (k < T - 1) {
      const R E2 = expm1((R)-2 * th * (R)(k + 2));
      const R g = (th > (R)0) ? em * E / E2 : (R)(k + 1) / (R)(k + 2);
      bp = (h * inv_ae + bp) * g;
      E = E2;
      w[(size_t)k * nx] = bp;
    } else {
      R u;
      if (th > (R)0) {
        const R ET = expm1((R)-2 * th * (R)T);
        u = d0 + ae * expm1(-th) * ((R)1 + exp(-th * (R)(2 * T - 1))) / ET;
      } else {
        u = d0 + ae / (R)T;
      }
      bp = (h + ae * bp) / u;
      w[(size_t)k * nx] = bp;
    }
  }
  E = expm1((R)-2 * th * (R)T);
  R wn = (T >= 2) ? w[(size_t)(T - 2) * nx] : (R)0;
  for (int k = T - 2; k >= 0; --k) {
    const R wk = wn;
    if (k > 0) wn = w[(size_t)(k - 1) * nx];
    const R E1 = expm1((R)-2 * th * (R)(k + 1));
    const R g = (th > (R)0) ? em * E1 / E : (R)(k + 1) / (R)(k + 2);
    bp = wk + g * bp;
    E = E1;
    w[(size_t)k * nx] = bp;
  }
}

// grid: G workgroups striding over the ceil(T/2) row pairs; block 256; LDS 2 * nx complex
template <typename R, class F>
__global__ void __launch_bounds__(1024) k_invx_update_1d(KP<R> p, F plx, const cplx<R>* __restrict__ twx) {
  using C = cplx<R>;
  if (p.ctrl->done) return;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  C* A = plx.template buffer<C>(reinterpret_cast<C*>(smem_raw), reinterpret_cast<C*>(p.gscr), blockIdx.x);
  C* Bf = A + plx.n();
  const int nx = p.nx;
  const R scale = p.tau * p.inv_n;
  double s[3] = {0.0, 0.0, 0.0};
  const int npairs = (p.T + 1) / 2;
  for (int pr = blockIdx.x; pr < npairs; pr += gridDim.x) {
    const int j = 2 * pr;
    const bool has2 = (j + 1) < p.T;
    const R* w0 = p.work + (size_t)j * nx;
    for (int k = threadIdx.x; k < nx; k += blockDim.x) A[k] = cmk<C>(w0[k], has2 ? w0[nx + k] : (R)0);
    __syncthreads();
    const C* Z = plx.template run<C>(A, Bf, twx);
    for (int x = threadIdx.x; x < nx; x += blockDim.x) {
      R u0, u1;
      hartley_pair<C, R>(Z, nx, 1, x, 0, u0, u1);
      for (int r = 0; r < 2; ++r) {
        if (r == 1 && !has2) break;
        const size_t idx = (size_t)(j + 1 + r) * nx + x;
        const R old = p.phi[idx];
        const R nw = old + scale * (r ? u1 : u0);
        p.phi[idx] = nw;
        p.phibar[idx] = (R)2 * nw - old;
        const double d = (double)nw - (double)old;
        s[0] += d * d;
        s[1] += (double)old * (double)old;
        s[2] += (double)nw * (double)nw;
      }
    }
    __syncthreads();
  }
  block_reduce_store<3>(s, p.partials, blockIdx.x);
}

// grid: (ceil(nx/256), G) striding over the T time rows; block 256.  Sums as k_dual_2d with NA = 2.
template <typename R, int EGNO>
__global__ void __launch_bounds__(256) k_dual_1d(KP<R> p) {
  if (p.ctrl->done || p.ctrl->inner_done) return;
  const int cur = p.ctrl->cur;
  const int src_set = (p.inplace || p.sub == 0) ? cur : 1 - cur;
  const int dst_set = p.inplace ? cur : 1 - cur;
  const int nx = p.nx;
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  constexpr int NS = 9;
  double s[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) s[i] = 0.0;
  if (x < nx) {
    const int xm = nb_index(x - 1, nx, p.bcx), xp = nb_index(x + 1, nx, p.bcx);
    const R a = p.ax[x];
    for (int j = blockIdx.y; j < p.T; j += gridDim.y) {
      const R* f1 = p.phibar + (size_t)(j + 1) * nx;
      const R* f0 = p.phibar + (size_t)j * nx;
      const R pc = f1[x];
      const R pxm = (xm >= 0) ? f1[xm] : (R)0;
      const R pxp = (xp >= 0) ? f1[xp] : (R)0;
      const R DxR = (pxp - pc) * p.inv_dx;
      const R DxL = (pc - pxm) * p.inv_dx;
      const size_t o = (size_t)j * nx + x;
      const R rho = p.rho[src_set][o];
      const R pinv = (rho + (R)1e-4) / p.sigma;
      const R ao0 = p.alp[src_set][0][o], ao1 = p.alp[src_set][1][o];
      const R q = prox_recip<R, EGNO>(rho, p.sigma, pinv);
      const R an0 = alp_prox<R, EGNO>(ao0, DxR, a, pinv, q, true);
      const R an1 = alp_prox<R, EGNO>(ao1, DxL, a, pinv, q, false);
      const R f1v = fpos<R>(fval<R, EGNO>(an0, a));
      const R f2v = fneg<R>(fval<R, EGNO>(an1, a));
      const R L = lag<R, EGNO>(an0 * an0) + lag<R, EGNO>(an1 * an1);
      R vec = (pc - f0[x]) * p.inv_dt;
      if (p.epsl != (R)0) vec = vec - p.epsl * ((pxp + pxm - (R)2 * pc) * p.inv_dx2);
      vec = vec - (DxR * f1v + DxL * f2v);
      vec = vec - L;
      const R rn = nmax<R>(rho + p.sigma * vec, (R)0);
      p.rho[dst_set][o] = rn;
      p.alp[dst_set][0][o] = an0;
      p.alp[dst_set][1][o] = an1;
      const double dr = (double)rn - (double)rho;
      s[0] += dr * dr;
      s[1] += (double)rn * (double)rn;
      s[2] += (double)rho * (double)rho;
      const double d0 = (double)an0 - (double)ao0, d1 = (double)an1 - (double)ao1;
      s[3] += d0 * d0;
      s[4] += (double)an0 * (double)an0;
      s[5] += (double)ao0 * (double)ao0;
      s[6] += d1 * d1;
      s[7] += (double)an1 * (double)an1;
      s[8] += (double)ao1 * (double)ao1;
    }
  }
  block_reduce_store<NS>(s, p.partials, blockIdx.y * gridDim.x + blockIdx.x);
}

}  // namespace pdhg
