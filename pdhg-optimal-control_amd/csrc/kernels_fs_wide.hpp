// Four-step DHT of row pairs for nx = 65536 = 256 x 256 (fp32, C1: BASELINE configs[1]) with wide tiles.
//
// Same transform as k_fs1_1d / k_fs2_1d (x = 256 n1 + n2, k = k1 + 256 k2; stage 1: 256-point FFTs over n1
// of a tile of columns n2, times W_65536^{n2 k1}, to Y[pair][k1][n2]; stage 2: 256-point FFTs over n2 of
// rows k1 and their Hartley partners 256 - k1, then the Hartley unpack), with every global access made of
// whole 128-B lines: the 16-column tiles of k_fs1_1d read 64-B pieces (and their +-1 neighbours), which
// fetched 3.5x the residual's input bytes (rocprofv3 FETCH_SIZE 1.10 GB for 0.31 GB at C1).
//   k_fs1w_1d: 64 columns n2 per workgroup (one wave = one n1 row of the tile: 256 B per array per wave;
//              x +- 1 from the neighbouring lanes by DPP, one uniform load at each wave edge);
//   k_fs2w_1d: 32 rows k1 + their 32 partners per workgroup (writes / phi reads of 32 consecutive k: 128 B).
// Both transform in place in LDS (padded lines, radix 16 x 16, twiddle seeds in LDS), with LINE = 273 complex
// per line so that reading element e of 64 consecutive lines (the output / unpack loops) hits distinct banks.
#pragma once
#include "kernels_1d.hpp"
#include "kernels_2d_fast.hpp"

namespace pdhg {

constexpr int kFwLine = 256 + 16 + 1;   // padded line (pix) + 1: consecutive lines 34 banks apart

// one radix-R pass of the padded in-place schedule on NL lines of 256 points, line stride kFwLine
template <int NL, int NT, int LS, int R>
__device__ __forceinline__ void fw_pass(float2* __restrict__ a, const float2* twl) {
  using C = float2;
  constexpr int N = 256, nR = N / R, total = nR * NL, PER = (total + NT - 1) / NT;
  static_assert(R == 16, "256 = 16 x 16");
  C v[PER][R];
  int base[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int idx = threadIdx.x + q * NT;
    base[q] = -1;
    if (total % NT == 0 || idx < total) {
      const int l = idx / nR, j = idx - l * nR, k = j & (LS - 1);
      const C* s = a + l * kFwLine + pix(j);
#pragma unroll
      for (int r = 0; r < R; ++r) v[q][r] = s[r * (nR + nR / 16)];
      if (LS > 1 && k != 0) {
        const C* t3 = twl + twlds_off(LS) + 3 * k;
        const C w1 = t3[0], w2 = cmul(w1, w1), w3 = cmul(w2, w1), w4 = t3[1];
        const C w5 = cmul(w4, w1), w6 = cmul(w4, w2), w7 = cmul(w4, w3), w8 = t3[2];
        const C w[16] = {make_float2(1.f, 0.f), w1, w2, w3, w4, w5, w6, w7, w8, cmul(w8, w1), cmul(w8, w2),
                         cmul(w8, w3), cmul(w8, w4), cmul(w8, w5), cmul(w8, w6), cmul(w8, w7)};
#pragma unroll
        for (int r = 1; r < R; ++r) v[q][r] = cmul(v[q][r], w[r]);
      }
      base[q] = l * kFwLine + pix((j - k) * R + k);
    }
  }
  lds_sync();
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    if (base[q] >= 0) {
      dft_any<C, R>(v[q]);
      C* d = a + base[q];
#pragma unroll
      for (int r = 0; r < R; ++r) d[(LS == 1) ? r : r * (LS + LS / 16)] = v[q][r];
    }
  }
  lds_sync();
}

template <int NL, int NT>
__device__ __forceinline__ void fw_fft256(float2* a, const float2* twl) {
  fw_pass<NL, NT, 1, 16>(a, twl);
  fw_pass<NL, NT, 16, 16>(a, twl);
}

// continuity residual at x from the centre values and the x +- 1 neighbours (update_fns_in_pdhg.py:72-81;
// cont_residual_1d with the loads done by the caller)
template <int EGNO, typename R>
__device__ __forceinline__ R res1d(const KP<R>& p, R r0, R rm, R rp, R rnext, R b1c, R b1m, R b2c, R b2p, R ac, R am,
                                   R ap, bool last) {
  const R eps = (R)1e-4;
  // branch-free (the callers unroll 16 rows): epsl * Dxx is added as the reference does, even for epsl = 0
  R res = (rnext - r0) * p.inv_dt;
  res = res + p.epsl * ((rp + rm - (R)2 * r0) * p.inv_dx2);
  const R m1c = (r0 + eps) * fpos<R>(fval<R, EGNO>(b1c, ac));
  const R m1m = (rm + eps) * fpos<R>(fval<R, EGNO>(b1m, am));
  const R m2c = (r0 + eps) * fneg<R>(fval<R, EGNO>(b2c, ac));
  const R m2p = (rp + eps) * fneg<R>(fval<R, EGNO>(b2p, ap));
  res = res - ((m1c - m1m) * p.inv_dx + (m2p - m2c) * p.inv_dx);
  return res + (last ? p.c_over_dt : (R)0);
}

// Stage 1.  grid (256/64, pairs); block 1024 (16 waves: wave w handles n1 rows w, w + 16, ...); LDS 64 lines.
// MODE 0: z = residual rows j, j+1 (periodic x: bc 0 only); MODE 1: z = spectrum rows j, j+1 of work.
template <int MODE, int EGNO>
__global__ void __launch_bounds__(1024) k_fs1w_1d(KP<float> p, const float2* __restrict__ tw256,
                                                 const float2* __restrict__ twN, float2* __restrict__ Y) {
  using C = float2;
  constexpr int L = 64, NT = 1024;
  if (p.ctrl->done) return;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  C* A = reinterpret_cast<C*>(smem_raw);
  C* twl = A + L * kFwLine;
  fill_twlds<C, 256>(twl, tw256);
  const int nx = p.nx, tile = blockIdx.x, pair = blockIdx.y;
  const int j = 2 * pair, T = p.T;
  const bool has2 = (j + 1) < T;
  const int cur = p.ctrl->cur;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll 4
  for (int n1 = wv; n1 < 256; n1 += NT / 64) {
    const int x0 = 256 * n1 + L * tile;          // first column of this wave's 64
    const int x = x0 + lane;
    float r0, r1 = 0.f;
    if constexpr (MODE == 0) {
      const float* rho = p.rho[cur];
      const float* a1 = p.alp[cur][0];
      const float* a2 = p.alp[cur][1];
      const int xm = (x0 - 1) & (nx - 1), xp = (x0 + L) & (nx - 1);   // wave-edge neighbours (periodic)
      const size_t o0 = (size_t)j * nx, o1 = o0 + nx;
      const int j1c = has2 ? j + 1 : j, j2 = min(j + 2, T - 1);
      const float* r_j = rho + o0;
      const float* r_j1 = rho + (size_t)j1c * nx;
      const float* r_j2 = rho + (size_t)j2 * nx;
      const float ac = p.ax[x];
      const float am = lane_from_prev(ac, p.ax[xm]), ap = lane_from_next(ac, p.ax[xp]);
      {   // row j
        const float c = r_j[x], n = (j + 1 < T) ? r_j1[x] : 0.f;
        const float b1 = a1[o0 + x], b2 = a2[o0 + x];
        const float rm = lane_from_prev(c, r_j[xm]), rp = lane_from_next(c, r_j[xp]);
        const float b1m = lane_from_prev(b1, a1[o0 + xm]), b2p = lane_from_next(b2, a2[o0 + xp]);
        r0 = res1d<EGNO>(p, c, rm, rp, n, b1, b1m, b2, b2p, ac, am, ap, j == T - 1);
      }
      if (has2) {   // row j + 1
        const float c = r_j1[x], n = (j + 2 < T) ? r_j2[x] : 0.f;
        const float b1 = a1[o1 + x], b2 = a2[o1 + x];
        const float rm = lane_from_prev(c, r_j1[xm]), rp = lane_from_next(c, r_j1[xp]);
        const float b1m = lane_from_prev(b1, a1[o1 + xm]), b2p = lane_from_next(b2, a2[o1 + xp]);
        r1 = res1d<EGNO>(p, c, rm, rp, n, b1, b1m, b2, b2p, ac, am, ap, j + 1 == T - 1);
      }
    } else {
      r0 = p.work[(size_t)j * nx + x];
      if (has2) r1 = p.work[(size_t)(j + 1) * nx + x];
    }
    A[lane * kFwLine + pix(n1)] = make_float2(r0, r1);   // line = column n2, element n1
  }
  lds_sync();
  fw_fft256<L, NT>(A, twl);
  C* Yp = Y + (size_t)pair * nx;
#pragma unroll 4
  for (int k1 = wv; k1 < 256; k1 += NT / 64) {
    const int n2 = L * tile + lane;
    Yp[(size_t)k1 * 256 + n2] = cmul(A[lane * kFwLine + pix(k1)], twN[(n2 * k1) & (nx - 1)]);
  }
}

// Stage 2.  grid (5, pairs): rows k1 = 32 g + l (k1 <= 128) and partners (256 - k1) mod 256; block 1024;
// LDS 64 lines (rows in lines 0..31, partners in 32..63).  MODE 0: DHT rows to work; MODE 1: the inverse
// transform -- phi' = phi + tau/nx U, phi_bar = 2 phi' - phi and the err1 sums (one partial row per workgroup).
template <int MODE>
__global__ void __launch_bounds__(1024) k_fs2w_1d(KP<float> p, const float2* __restrict__ tw256,
                                                 const float2* __restrict__ Y) {
  using C = float2;
  constexpr int L = 32, NT = 1024;
  double s[3] = {0.0, 0.0, 0.0};
  const int nx = p.nx, g = blockIdx.x, pair = blockIdx.y;
  const int row = blockIdx.y * gridDim.x + blockIdx.x;
  if (p.ctrl->done) {
    if constexpr (MODE == 1) block_reduce_store<3>(s, p.partials, row);
    return;
  }
  extern __shared__ __align__(16) unsigned char smem_raw[];
  C* A = reinterpret_cast<C*>(smem_raw);
  C* twl = A + 2 * L * kFwLine;
  fill_twlds<C, 256>(twl, tw256);
  const int j = 2 * pair;
  const bool has2 = (j + 1) < p.T;
  const C* Yp = Y + (size_t)pair * nx;
  const int tid = threadIdx.x;
  // 64 lines x 256 elements: line l < 32 is row k1 = 32 g + l, line 32 + l its partner
#pragma unroll 4
  for (int i = tid; i < 2 * L * 256; i += NT) {
    const int ln = i >> 8, n2 = i & 255;            // consecutive threads: consecutive n2 (2 KB per row)
    const int l = ln & (L - 1);
    const int k1 = L * g + l;
    const int kr = (ln < L) ? k1 : ((256 - k1) & 255);
    A[ln * kFwLine + pix(n2)] = (k1 <= 128) ? Yp[(size_t)kr * 256 + n2] : make_float2(0.f, 0.f);
  }
  lds_sync();
  fw_fft256<2 * L, NT>(A, twl);
  const float scale = p.tau * p.inv_n;
#pragma unroll 2
  for (int i = tid; i < L * 256; i += NT) {
    const int k2 = i >> 5, l = i & (L - 1);         // consecutive threads: consecutive k1 (128-B pieces)
    const int k1 = L * g + l;
    if (k1 > 128) continue;
    const bool self = (k1 == 0) || (k1 == 128);     // the partner row is the row itself
    const int k2m = (k1 == 0) ? ((256 - k2) & 255) : (255 - k2);
    const C z = A[l * kFwLine + pix(k2)];
    const C w = self ? A[l * kFwLine + pix(k2m)] : A[(L + l) * kFwLine + pix(k2m)];   // Z_k, Z_{N-k}
    const int k = k1 + 256 * k2, km = (nx - k) & (nx - 1);
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

}  // namespace pdhg
