// Fast 2-D row-transform kernels (fp32, ny = N a power of two, nx % RW == 0).
//
//   k_res_fwdy_fast_2d     continuity residual + forward DHT along y for RW rows at once
//   k_invy_update_fast_2d  inverse DHT along y + phi update for RW rows at once
//
// One workgroup owns an RW-row group of one time row: the RW/2 row pairs are RW/2 complex
// lines (line-major in LDS) transformed together in place (lds_fft_inplace, RW/2 * N complex).  The
// blocked spectral layout work[k][b][x][c] then has one contiguous RW*B-float chunk per
// column block and row group, written / read by RW*B/4 neighbouring lanes with float4
// (whole 64-B pieces instead of 8-B scattered stores).  The residual reads each input row
// once per group with float4 loads over a sliding 3-row window (rows x-1, x, x+1).
#pragma once
#include <type_traits>
#include "params.hpp"

namespace pdhg {

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ float f4(const float4& v, int e) { return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w; }
__device__ __forceinline__ void f4set(float4& v, int e, float x) {
  if (e == 0) v.x = x; else if (e == 1) v.y = x; else if (e == 2) v.z = x; else v.w = x;
}
__device__ __forceinline__ float4 z4() { return make_float4(0.f, 0.f, 0.f, 0.f); }

// fp64 counterparts (4 consecutive y per lane as two 16-B accesses), for the kernels templated on R
struct dbl4 {
  double x, y, z, w;
};
template <typename R> struct V4s { using type = float4; };
template <> struct V4s<double> { using type = dbl4; };
template <typename R> using V4 = typename V4s<R>::type;
__device__ __forceinline__ dbl4 ld4(const double* p) {
  const double2 a = reinterpret_cast<const double2*>(p)[0], b = reinterpret_cast<const double2*>(p)[1];
  return dbl4{a.x, a.y, b.x, b.y};
}
__device__ __forceinline__ void st4(double* p, dbl4 v) {
  reinterpret_cast<double2*>(p)[0] = make_double2(v.x, v.y);
  reinterpret_cast<double2*>(p)[1] = make_double2(v.z, v.w);
}
__device__ __forceinline__ double f4(const dbl4& v, int e) { return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w; }
__device__ __forceinline__ void f4set(dbl4& v, int e, double x) {
  if (e == 0) v.x = x; else if (e == 1) v.y = x; else if (e == 2) v.z = x; else v.w = x;
}
template <typename R> __device__ __forceinline__ V4<R> z4r() { return z4(); }
template <> __device__ __forceinline__ dbl4 z4r<double>() { return dbl4{0.0, 0.0, 0.0, 0.0}; }
// YPL consecutive y per lane: 4 (float4 / dbl4) or 2 (float2 / double2, one 16-B access per lane in fp64)
template <typename R, int YPL> struct VYs { using type = V4<R>; };
template <typename R> struct VYs<R, 2> { using type = cplx<R>; };
template <typename R, int YPL> using VY = typename VYs<R, YPL>::type;
__device__ __forceinline__ float f4(const float2& v, int e) { return e == 0 ? v.x : v.y; }
__device__ __forceinline__ double f4(const double2& v, int e) { return e == 0 ? v.x : v.y; }
__device__ __forceinline__ void f4set(float2& v, int e, float x) { if (e == 0) v.x = x; else v.y = x; }
__device__ __forceinline__ void f4set(double2& v, int e, double x) { if (e == 0) v.x = x; else v.y = x; }
template <int YPL, typename R> __device__ __forceinline__ VY<R, YPL> ldy(const R* p) {
  if constexpr (YPL == 4) return ld4(p);
  else return *reinterpret_cast<const cplx<R>*>(p);
}
template <int YPL, typename R> __device__ __forceinline__ void sty(R* p, VY<R, YPL> v) {
  if constexpr (YPL == 4) st4(p, v);
  else *reinterpret_cast<cplx<R>*>(p) = v;
}
template <typename R, int YPL> __device__ __forceinline__ VY<R, YPL> zy() {
  if constexpr (YPL == 4) return z4r<R>();
  else return cmk<cplx<R>>((R)0, (R)0);
}
__device__ __forceinline__ float4 mk4(float a, float b, float c, float d) { return make_float4(a, b, c, d); }
__device__ __forceinline__ dbl4 mk4(double a, double b, double c, double d) { return dbl4{a, b, c, d}; }
// the float lane shifts (common.hpp) on the two halves of a double
__device__ __forceinline__ double lane_from_prev(double v, double edge) {
  const long long vi = __builtin_bit_cast(long long, v), ei = __builtin_bit_cast(long long, edge);
  const float lo = lane_from_prev(__builtin_bit_cast(float, (int)vi), __builtin_bit_cast(float, (int)ei));
  const float hi = lane_from_prev(__builtin_bit_cast(float, (int)(vi >> 32)), __builtin_bit_cast(float, (int)(ei >> 32)));
  return __builtin_bit_cast(double, (long long)(unsigned)__builtin_bit_cast(int, lo) |
                                        ((long long)__builtin_bit_cast(int, hi) << 32));
}
__device__ __forceinline__ double lane_from_next(double v, double edge) {
  const long long vi = __builtin_bit_cast(long long, v), ei = __builtin_bit_cast(long long, edge);
  const float lo = lane_from_next(__builtin_bit_cast(float, (int)vi), __builtin_bit_cast(float, (int)ei));
  const float hi = lane_from_next(__builtin_bit_cast(float, (int)(vi >> 32)), __builtin_bit_cast(float, (int)(ei >> 32)));
  return __builtin_bit_cast(double, (long long)(unsigned)__builtin_bit_cast(int, lo) |
                                        ((long long)__builtin_bit_cast(int, hi) << 32));
}

__device__ __forceinline__ float fmar(float a, float b, float c) { return fmaf(a, b, c); }
__device__ __forceinline__ double fmar(double a, double b, double c) { return fma(a, b, c); }

template <int EGNO, typename R = float>
__device__ __forceinline__ R m1f(R rho, R alp, R a) {   // (rho + 1e-4) f(alp)^+
  return (rho + (R)1e-4) * fpos<R>(fval<R, EGNO>(alp, a));
}
template <int EGNO, typename R = float>
__device__ __forceinline__ R m2f(R rho, R alp, R a) {   // (rho + 1e-4) f(alp)^-
  return (rho + (R)1e-4) * fneg<R>(fval<R, EGNO>(alp, a));
}

// grid: T * nx/RW row-group tasks (XCD-aware); block NT = min(1024, N/4); LDS RW/2 * (N + N/16) * 8 B.
// float4 number `part` of the blocked-layout chunk of column block b (RW rows x B columns, row-major) from
// the task's RW/2 transformed lines in LDS (line l = rows 2l, 2l+1 as real / imaginary part, stride LINE).
// B = 2: the float4 holds rows 2 part, 2 part + 1 at columns 2b, 2b + 1, i.e. the Hartley values of line
// `part` at ky = 2b, 2b+1 -- two element pairs read once for both rows (the generic path reads them per row).
template <int N, int LINE, typename R = float>
__device__ __forceinline__ V4<R> unpack_chunk4(const cplx<R>* A, int b, int part, int B, int lB) {
  using C = cplx<R>;
  if (B == 2) {   // ky = 2b + 1 < N always (N even)
    const C* Z = A + part * LINE;
    R a0, b0, a1, b1;
    hartley_padded<C, R>(Z, N, 2 * b, a0, b0);
    hartley_padded<C, R>(Z, N, 2 * b + 1, a1, b1);
    return mk4(a0, a1, b0, b1);
  }
  V4<R> v;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int f = part * 4 + e;
    const int r = f >> lB, c = f & (B - 1);
    const int ky = b * B + c;
    R ha = (R)0, hb = (R)0;
    if (ky < N) hartley_padded<C, R>(A + (r >> 1) * LINE, N, ky, ha, hb);
    f4set(v, e, (r & 1) ? hb : ha);
  }
  return v;
}

template <int EGNO, int N, int RW, int NT, typename R = float>
__global__ void __launch_bounds__(NT) k_res_fwdy_fast_2d(KP<R> p, const cplx<R>* __restrict__ twy) {
  using C = cplx<R>;
  using V = V4<R>;
  constexpr int NL = RW / 2;
  constexpr int GPT = (N / 4) / NT;   // V y-groups per thread
  if (p.ctrl->done) return;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  C* A = reinterpret_cast<C*>(smem_raw);
  const int cur = p.ctrl->cur;
  const int nx = p.nx, T = p.T;
  const int ngx = nx / RW;
  const int task = xcd_remap(blockIdx.x, gridDim.x);
  // this launch covers time rows [row_base, row_base + row_cnt) (the t-slab path launches the rows
  // that need the next slab's rho separately, so the halo exchange overlaps the others)
  int j, gx;
  const int TJ = p.tile_j, ntiled = (p.row_cnt / TJ) * TJ * ngx;
  if (TJ > 1 && task < ntiled) {
    // tiles of TW row groups x TJ time rows: the ~32 tasks an XCD runs together share rho row j+1
    // and the x-halo rows in that XCD's L2 (needs ngx % 4 == 0, checked on the host); the rows
    // after the last whole tile fall back to the row-major order below.  Chunks of < 64 B (C4's half-real
    // spectrum, B = 1): 8 row groups per tile, so one XCD writes whole 128-B lines of the spectrum
    // (PDHG_DBG 2048: 4 groups, A/B timing only)
    const int lTW = (RW * p.B * (int)sizeof(R) < 64 && (ngx & 7) == 0 && !(p.dbg & 2048)) ? 3 : 2;
    const int tsz = TJ << lTW, ngt = ngx >> lTW;
    const int tile = task / tsz, w = task - tile * tsz;
    const int tjx = tile / ngt, tg = tile - tjx * ngt;
    j = tjx * TJ + (w >> lTW);
    gx = (tg << lTW) + (w & ((1 << lTW) - 1));
  } else {
    const int t2 = task - (TJ > 1 ? ntiled : 0);
    j = t2 / ngx;
    gx = t2 - j * ngx;
    if (TJ > 1) j += (p.row_cnt / TJ) * TJ;
  }
  j += p.row_base;
  const int x0 = gx * RW;
  const size_t plane = (size_t)nx * N;
  const R* rj = p.rho[cur] + (size_t)j * plane;
  const R* a1x = p.alp[cur][0] + (size_t)j * plane;
  const R* a2x = p.alp[cur][1] + (size_t)j * plane;
  const R* a1y = (EGNO == 3) ? nullptr : p.alp[cur][2] + (size_t)j * plane;
  const R* a2y = (EGNO == 3) ? nullptr : p.alp[cur][3] + (size_t)j * plane;
  const R cdt = (j == T - 1 && p.last_slab) ? p.c_over_dt : (R)0;   // +c/dt on the window's last row
  const bool use_eps = p.epsl != (R)0;

  // Branch-free row loop: every load reads a valid address (rows/columns outside a Dirichlet edge
  // are clamped and zeroed by a select afterwards), so the loads of consecutive rows stay in
  // flight together instead of each conditional load draining the queue.
  const int xm0 = nb_index(x0 - 1, nx, p.bcx);          // row above the group (uniform)
  const int xpl = nb_index(x0 + RW, nx, p.bcx);         // row below the group (uniform)
  const bool zm = xm0 < 0, zpl = xpl < 0;
  const int xm0c = zm ? x0 : xm0, xplc = zpl ? x0 + RW - 1 : xpl;
  // rho row j+1: local, or the next slab's first row (halo), or zero after the window's last row
  const bool halo_j = (j + 1 >= T) && !p.last_slab;
  const bool last_j = (j + 1 >= T) && p.last_slab;
  const R* rnx = last_j ? rj : halo_j ? p.rho_halo : p.rho[cur] + (size_t)(j + 1) * plane;
  const int lane = threadIdx.x & (kWave - 1);
#pragma unroll
  for (int gi = 0; gi < GPT; ++gi) {
    const int y = 4 * (threadIdx.x + gi * NT);
    // wave-edge y neighbours (uniform per wave): y0-1 for lane 0, y63+4 for lane 63
    const int yw0 = __builtin_amdgcn_readfirstlane(y);
    const int ywm = nb_index(yw0 - 1, N, p.bcy), ywp = nb_index(yw0 + 4 * kWave, N, p.bcy);
    const bool zym = ywm < 0, zyp = ywp < 0;
    const int ywmc = zym ? 0 : ywm, ywpc = zyp ? 0 : ywp;
    V ay4 = z4r<R>();
    R aym = (R)0, ayp = (R)0;
    if constexpr (EGNO != 3) {
      ay4 = ld4(p.ay + y);
      aym = lane_from_prev(ay4.w, zym ? (R)0 : p.ay[ywmc]);
      ayp = lane_from_next(ay4.x, zyp ? (R)0 : p.ay[ywpc]);
    }
    V r_m = ld4(rj + (size_t)xm0c * N + y);
    V a1_m = ld4(a1x + (size_t)xm0c * N + y);
    R ax_m = p.ax[xm0c];
    if (zm) {
      r_m = z4r<R>();
      a1_m = z4r<R>();
      ax_m = (R)0;
    }
    V r_c = ld4(rj + (size_t)x0 * N + y);
    V a2_c = ld4(a2x + (size_t)x0 * N + y);
    R ax_c = p.ax[x0];
    // flux carries: m1x at the row above, m2x at the current row
    R m1x_prev[4], m2x_cur[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      m1x_prev[e] = zm ? (R)0 : m1f<EGNO, R>(f4(r_m, e), f4(a1_m, e), ax_m);
      m2x_cur[e] = m2f<EGNO, R>(f4(r_c, e), f4(a2_c, e), ax_c);
    }
    // software pipeline: the loads of row r+1 are issued before row r is computed
    struct RowIn {
      V r_p, a2_p, a1_c, rn4, a1y4, a2y4;
      R ax_p, e_rm, e_rp, e_a1m, e_a2p;
    };
    auto load_row = [&](int r) {
      RowIn in;
      const int x = x0 + r;
      const int xpc = (r + 1 == RW) ? xplc : x + 1;
      const size_t ro = (size_t)x * N;
      in.r_p = ld4(rj + (size_t)xpc * N + y);
      in.a2_p = ld4(a2x + (size_t)xpc * N + y);
      in.ax_p = p.ax[xpc];
      in.a1_c = ld4(a1x + ro + y);
      in.rn4 = ld4(rnx + ro + y);
      in.e_rm = rj[ro + ywmc];
      in.e_rp = rj[ro + ywpc];
      if constexpr (EGNO != 3) {
        in.a1y4 = ld4(a1y + ro + y);
        in.a2y4 = ld4(a2y + ro + y);
        in.e_a1m = a1y[ro + ywmc];
        in.e_a2p = a2y[ro + ywpc];
      } else {
        in.a1y4 = in.a2y4 = z4r<R>();
        in.e_a1m = in.e_a2p = (R)0;
      }
      return in;
    };
    RowIn nxt = load_row(0);
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const RowIn in = nxt;
      if (r + 1 < RW) nxt = load_row(r + 1);
      const bool zp = (r + 1 == RW) && zpl;
      V r_p = in.r_p, a2_p = in.a2_p, rn4 = in.rn4;
      R ax_p = in.ax_p;
      const V a1_c = in.a1_c;
      if (zp) {
        r_p = z4r<R>();
        a2_p = z4r<R>();
        ax_p = (R)0;
      }
      if (last_j) rn4 = z4r<R>();
      const V a1y4 = in.a1y4, a2y4 = in.a2y4;
      R a1y_m = (R)0, a2y_p = (R)0;
      // y neighbours: from the adjacent lanes (DPP); the wave-edge values are uniform loads
      if constexpr (EGNO != 3) {
        a1y_m = lane_from_prev(a1y4.w, zym ? (R)0 : in.e_a1m);
        a2y_p = lane_from_next(a2y4.x, zyp ? (R)0 : in.e_a2p);
      }
      const R r_ym = lane_from_prev(r_c.w, zym ? (R)0 : in.e_rm);
      const R r_yp = lane_from_next(r_c.x, zyp ? (R)0 : in.e_rp);
      const bool edge_m = zym && lane == 0, edge_p = zyp && lane == kWave - 1;
      R m1y[6], m2y[6], rr[6];   // index e+1 for e = -1..4
      rr[0] = r_ym;
      rr[5] = r_yp;
#pragma unroll
      for (int e = 0; e < 4; ++e) rr[e + 1] = f4(r_c, e);
      if constexpr (EGNO == 3) {
        const R f1 = fpos<R>(ax_c), f2 = fneg<R>(ax_c);
#pragma unroll
        for (int e = 0; e < 6; ++e) {
          m1y[e] = (rr[e] + (R)1e-4) * f1;
          m2y[e] = (rr[e] + (R)1e-4) * f2;
        }
      } else {
        m1y[0] = m1f<EGNO, R>(r_ym, a1y_m, aym);
        m2y[5] = m2f<EGNO, R>(r_yp, a2y_p, ayp);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          m1y[e + 1] = m1f<EGNO, R>(rr[e + 1], f4(a1y4, e), f4(ay4, e));
          m2y[e + 1] = m2f<EGNO, R>(rr[e + 1], f4(a2y4, e), f4(ay4, e));
        }
      }
      if (edge_m) m1y[0] = (R)0;   // zero flux outside a Dirichlet edge
      if (edge_p) m2y[5] = (R)0;
      R out[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const R r0 = rr[e + 1];
        R res = (f4(rn4, e) - r0) * p.inv_dt;
        if (use_eps) {
          res = res + p.epsl * ((f4(r_p, e) + f4(r_m, e) - (R)2 * r0) * p.inv_dx2);
          res = res + p.epsl * ((rr[e + 2] + rr[e] - (R)2 * r0) * p.inv_dy2);
        }
        const R m1x_c = m1f<EGNO, R>(r0, f4(a1_c, e), ax_c);
        const R m2x_p = zp ? (R)0 : m2f<EGNO, R>(f4(r_p, e), f4(a2_p, e), ax_p);
        const R div = (m1x_c - m1x_prev[e]) * p.inv_dx + (m2x_p - m2x_cur[e]) * p.inv_dx +
                          (m1y[e + 1] - m1y[e]) * p.inv_dy + (m2y[e + 2] - m2y[e + 1]) * p.inv_dy;
        out[e] = res - div + cdt;
        m1x_prev[e] = m1x_c;
        m2x_cur[e] = m2x_p;
      }
      // residual row x -> line r/2, real (even r) or imaginary (odd r) part; 4 contiguous elements
      R* Af = reinterpret_cast<R*>(A + (r >> 1) * Pad<N>::LINE + pix(y)) + (r & 1);
#pragma unroll
      for (int e = 0; e < 4; ++e) Af[2 * e] = out[e];
      // slide the window
      r_m = r_c;
      r_c = r_p;
      ax_c = ax_p;
    }
  }
  __syncthreads();
  if (!(p.dbg & 8)) lds_fft_inplace<C, N, NL, NT>(A, twy);
  // Hartley unpack -> blocked layout: chunk (j, b, x0..x0+RW-1, 0..B-1) = RW*B contiguous floats
  const int B = p.B;
  const int CS4 = RW * B / 4;                 // V per chunk
  const int lCS4 = p.lB + (RW == 8 ? 1 : RW == 4 ? 0 : RW == 2 ? -1 : -2);   // log2(CS4), B power of two
  const int nb = p.nb;
  if (p.rspec) {   // task order (tc_spec): the task's RW rows x all ky, one contiguous run
    R* wt = p.rspec + (size_t)j * nb * nx * B + (size_t)x0 * nb * B;
    for (int t = threadIdx.x; t < nb * CS4; t += NT)
      st4(wt + 4 * t, unpack_chunk4<N, Pad<N>::LINE, R>(A, t >> lCS4, t & (CS4 - 1), B, p.lB));
    return;
  }
  R* wk = p.work + (size_t)j * nb * nx * B;
  for (int t = threadIdx.x; t < nb * CS4; t += NT) {
    const int b = t >> lCS4, part = t & (CS4 - 1);
    st4(wk + ((size_t)b * nx + x0) * B + part * 4, unpack_chunk4<N, Pad<N>::LINE, R>(A, b, part, B, p.lB));
  }
}

// Residual rows formed by the fused dual sweep (k_dual_lds_2d<.., FR = true>, 8-row x 256-column tiles)
// + forward DHT along y.  Adds the terms the sweep could not form inside its tile
// (update_fns_in_pdhg.py:83-96), which the neighbouring tiles' sweeps wrote for it: p.ex holds, per tile,
// eps*rho'(x0-1)/dx^2 + m1x(x0-1)/dx for row x0 and eps*rho'(x0+RW)/dx^2 - m2x(x0+RW)/dx for row x0+RW-1
// (periodic wrap); p.ey holds eps*rho'/dy^2 +- m/dy of the neighbouring strip's edge column for the first /
// last column of every 256-wide strip.  Then the same in-place 4-line FFT and blocked-layout unpack as
// k_res_fwdy_fast_2d.  Needs RW = 8 (the sweep's tile height), bc (0, 0), ny % 256 == 0.
// Persistent: G workgroups (one per CU: the 4 lines take 139 KiB of LDS) stride over the T * nx/RW
// row-group tasks.  The next task's rows are loaded into registers before the current FFT and its edge rows
// after it, so the CU's memory pipe is not idle during the transform; its strip-edge terms (RW * ny/256 * 2
// floats) go through a small LDS double buffer, so only the edge lanes read them.
// fp64 (R = double): the sweep's strips are 128 columns wide (k_dual_lds_2d<.., double, YPL = 2>) and 4 rows of
// complex double fill the LDS, so a task is half a sweep tile (RW = 4, NH = 2): the first half adds row x0's
// p.ex term, the second row x0+RW-1's.  fp32 at ny = 8192 (C4) likewise: 4 rows of 8192 floats fill the LDS.
// fp64 at ny = 8192 (C4's grid in the reference's precision): one line of 8192 complex doubles (136 KiB) per task,
// i.e. a quarter of a sweep tile (RW = 2, NH = 4; the first quarter adds row x0's p.ex term, the last row x0+7's);
// with C4's half-real spectrum (B = 1) a chunk is the two rows' values at one ky (one 16-B store).
// grid: G <= T * nx/RW; block NT (N/4 % NT == 0); LDS RW/2 * (N + N/16) * sizeof(C) (+ 2 * RW * N/YW reals).
template <int EGNO, int N, int RW, int NT, typename R = float>
__global__ void __launch_bounds__(NT) k_res_fwdy_fused_2d(KP<R> p, const cplx<R>* __restrict__ twy) {
  using C = cplx<R>;
  using V = V4<R>;
  constexpr int TH = 8;                  // tile height of the sweep (k_dual_lds_2d RX)
  constexpr int NH = TH / RW;            // tasks per sweep tile
  constexpr int NL = RW / 2;
  constexpr int LN = Pad<N>::LINE;
  constexpr int GPT = (N / 4) / NT;
  constexpr int YW = sizeof(R) == 4 ? 256 : 128, NSTRIP = N / YW;
  constexpr int NEY = RW * NSTRIP * 2;   // strip-edge terms of one task
  static_assert((RW == 8 || RW == 4 || RW == 2) && (sizeof(R) == 4 || RW <= 4) && (RW != 2 || (sizeof(R) == 8 &&
                N == 8192)) && N % YW == 0 && (N / 4) % NT == 0,
                "fused residual tasks: 8, 4 (fp64, fp32 ny = 8192) or 2 (fp64 ny = 8192) rows of the sweep's 8-row x "
                "YW-column tiles");
  static_assert(NEY <= NT, "one strip-edge term per thread");
  if (p.ctrl->done) return;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  __shared__ R eyl[2][NEY];
  C* A = reinterpret_cast<C*>(smem_raw);
  // twiddle seeds in LDS behind the lines (N <= 4096): the passes then issue no global loads, so the next
  // task's rows stay in flight across the whole transform (vmcnt drains in order)
  constexpr bool TWL = N <= 4096;
  C* twl = A + NL * LN;
  if constexpr (TWL) fill_twlds<C, N>(twl, twy);
  const int nx = p.nx;
  const int ngx = nx / RW;
  const int ntask = ngx * p.row_cnt;   // time rows [row_base, row_base + row_cnt) (t-slab: halo row apart)
  const size_t plane = (size_t)nx * N;
  const int B = p.B;
  const int CS4 = RW * B / 4;
  const int lCS4 = p.lB + (RW == 8 ? 1 : RW == 4 ? 0 : RW == 2 ? -1 : -2);   // log2(CS4), B power of two
  const int nb = p.nb;
  const int tid = threadIdx.x;
  V rows[GPT][RW];             // next task's residual rows x0 .. x0+RW-1
  V e0[GPT], e1[NH == 1 ? GPT : 1];   // next task's edge-row terms (row x0, row x0+RW-1; NH = 2: the half's one)
  R ev = (R)0;                 // next task's strip-edge term number tid
  // rows [r0, r1) of a task (NT = 1024: half before the transform, half after, so that only 4 rows of
  // loads are live across the FFT's registers)
  auto load_rows = [&](int task, int r0, int r1) {
    const int jt = task / ngx, j = p.row_base + jt, x0 = (task - jt * ngx) * RW;
    if (r0 == 0 && tid < NEY) ev = p.ey[((size_t)j * nx + x0) * NSTRIP * 2 + tid];   // first: waited for alone
    const R* R0 = p.res + (size_t)j * plane + (size_t)x0 * N;
#pragma unroll
    for (int gi = 0; gi < GPT; ++gi) {
      const int y = 4 * (tid + gi * NT);
#pragma unroll
      for (int r = 0; r < RW; ++r)
        if (r >= r0 && r < r1) rows[gi][r] = ld4(R0 + (size_t)r * N + y);
    }
  };
  // (N = 8192: none -- the 8192-point transform's registers leave no room for rows held across it)
  constexpr int RSPLIT = (N > 4096) ? 0 : (NT >= 1024) ? RW / 2 : RW;
  auto load_edges = [&](int task) {
    const int jt = task / ngx, j = p.row_base + jt, tk = task - jt * ngx, tile = tk / NH, sub = tk & (NH - 1);
    const R* E = p.ex + ((size_t)j * (ngx / NH) + tile) * 2 * N;
    if (NH > 2 && sub != 0 && sub != NH - 1) return;   // inner quarters of a tile: no edge row (uniform)
#pragma unroll
    for (int gi = 0; gi < GPT; ++gi) {
      const int y = 4 * (tid + gi * NT);
      if constexpr (NH == 1) {
        e0[gi] = ld4(E + y);
        e1[gi] = ld4(E + N + y);
      } else {
        e0[gi] = ld4(E + (sub == NH - 1 ? N : 0) + y);
      }
    }
  };
  // C4 (B = 1: 16-B chunks, 8 tasks per 128-B line of the spectrum; fp64 2-row, fp32 4-row tasks): XCD-aware order, the
  // G / 8 workgroups of one XCD take consecutive tasks in every round, so a line's chunks are written through one
  // L2.  Interleaved A/B (round 5, c4w50 fp64): residual 73.2 -> 60.4 ms; at C3's 64-B chunks (2 tasks per line)
  // the same order measured slower (fp64 15.5 -> 17.8 ms, fp32 neutral), so only the 2-row tasks take it.
  // (PDHG_DBG 1024: round-robin order, A/B timing only)
  const bool xcdo = RW * p.B * (int)sizeof(R) < 64;   // 16-B chunks (B = 1, half-real x blocks)
  int task = (xcdo && (gridDim.x & 7) == 0 && !(p.dbg & 1024)) ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  int buf = 0;
  if (task < ntask) {
    load_rows(task, 0, RW);
    load_edges(task);
    if (tid < NEY) eyl[0][tid] = ev;
  }
  __syncthreads();
  for (; task < ntask; task += gridDim.x, buf ^= 1) {
    const int jt = task / ngx, j = p.row_base + jt, x0 = (task - jt * ngx) * RW;
    // t-slab, last row: the dual stored it without the time difference; the next slab's rho row 0 (the halo)
    // completes it, (rho_T - rho_{T-1})/dt added with the fma k_dual_lds_2d's finish_res uses inside a window
    const bool hal = p.rho_halo != nullptr && j == p.T - 1;
#pragma unroll
    for (int gi = 0; gi < GPT; ++gi) {
      const int y = 4 * (tid + gi * NT);
      V v[RW];
#pragma unroll
      for (int r = 0; r < RW; ++r) v[r] = rows[gi][r];
      if (hal) {
        const R* rl = p.rho[p.ctrl->cur] + (size_t)j * plane + (size_t)x0 * N;
#pragma unroll
        for (int r = 0; r < RW; ++r) {
          const V hv = ld4(p.rho_halo + (size_t)(x0 + r) * N + y), rv = ld4(rl + (size_t)r * N + y);
#pragma unroll
          for (int e = 0; e < 4; ++e) f4set(v[r], e, fmar(f4(hv, e) - f4(rv, e), p.inv_dt, f4(v[r], e)));
        }
      }
      if constexpr (NH == 1) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          f4set(v[0], e, f4(v[0], e) + f4(e0[gi], e));
          f4set(v[RW - 1], e, f4(v[RW - 1], e) + f4(e1[gi], e));
        }
      } else if (((task - jt * ngx) & (NH - 1)) == 0) {
#pragma unroll
        for (int e = 0; e < 4; ++e) f4set(v[0], e, f4(v[0], e) + f4(e0[gi], e));
      } else if (((task - jt * ngx) & (NH - 1)) == NH - 1) {
#pragma unroll
        for (int e = 0; e < 4; ++e) f4set(v[RW - 1], e, f4(v[RW - 1], e) + f4(e0[gi], e));
      }
      const int s = y / YW, yo = y - s * YW;
      if (yo == 0) {
#pragma unroll
        for (int r = 0; r < RW; ++r) v[r].x += eyl[buf][(r * NSTRIP + s) * 2];
      } else if (yo == YW - 4) {
#pragma unroll
        for (int r = 0; r < RW; ++r) v[r].w += eyl[buf][(r * NSTRIP + s) * 2 + 1];
      }
#pragma unroll
      for (int l = 0; l < RW / 2; ++l) {   // rows 2l, 2l+1 -> line l (real, imaginary): one 8-B LDS store each
        C* Al = A + l * LN + pix(y);
#pragma unroll
        for (int e = 0; e < 4; ++e) Al[e] = cmk<C>(f4(v[2 * l], e), f4(v[2 * l + 1], e));
      }
    }
    // the next task's loads are unconditional (the last task re-loads its own rows): a conditional load
    // keeps the previous registers live across the transform on the not-taken path (spills at NT = 1024)
    const int nxt = min(task + (int)gridDim.x, ntask - 1);
    load_rows(nxt, 0, RSPLIT);
    lds_sync();
    if (!(p.dbg & 16)) {   // timing experiments only (PDHG_DBG): 16 skips the transform
      if constexpr (TWL) lds_fft_inplace_tl<C, N, NL, NT>(A, twl);
      else lds_fft_inplace<C, N, NL, NT>(A, twy);
    }
    if (tid < NEY) eyl[buf ^ 1][tid] = ev;   // read one barrier after its last use two tasks ago
    if constexpr (RSPLIT < RW) load_rows(nxt, RSPLIT, RW);
    load_edges(nxt);
    R* wk = p.work + (size_t)j * nb * nx * B;
    if (p.rspec) {   // task order (tc_spec; C4's to_c4): one contiguous run per task
      R* wt = p.rspec + (size_t)j * nb * nx * B + (size_t)x0 * nb * B;
      if (RW * B < 4) {   // RW = 2, B = 1 (fp64 C4): element b = rows x0, x0+1 at ky = b, 16 B, consecutive in b
        for (int b = tid; b < nb; b += NT) {
          R ha, hb;
          hartley_padded<C, R>(A, N, b, ha, hb);
          *reinterpret_cast<C*>(wt + 2 * (size_t)b) = cmk<C>(ha, hb);
        }
      } else {
        for (int t = tid; t < nb * CS4; t += NT)
          st4(wt + 4 * t, unpack_chunk4<N, LN, R>(A, t >> lCS4, t & (CS4 - 1), B, p.lB));
      }
    } else if (RW * B < 4) {   // RW = 2, B = 1 (fp64 C4): chunk b = rows x0, x0+1 at ky = b, one 16-B store
      for (int b = tid; b < nb; b += NT) {
        R ha, hb;
        hartley_padded<C, R>(A, N, b, ha, hb);
        *reinterpret_cast<C*>(wk + (size_t)b * nx + x0) = cmk<C>(ha, hb);
      }
    } else {
      for (int t = tid; t < nb * CS4 && !(p.dbg & 32); t += NT) {   // PDHG_DBG 32: no unpack / stores (timing)
        const int b = t >> lCS4, part = t & (CS4 - 1);
        const V v = unpack_chunk4<N, LN, R>(A, b, part, B, p.lB);
        if (p.dbg & 512) st4(wk + (size_t)x0 * N + 4 * t, v);   // PDHG_DBG 512: task-contiguous stores (timing)
        else st4(wk + ((size_t)b * nx + x0) * B + part * 4, v);
      }
    }
    lds_sync();
  }
}

// C4's task-order spectrum (to_c4) into the x kernel's blocked layout.  With half-real x blocks (B = 1) a blocked
// chunk is one row task's RW values at one ky: 16 B (fp64 RW = 2, fp32 RW = 4), so the fused residual writing the
// blocked layout directly stores 16 B per 64-KiB stride (round 5: fp64 c4w50 residual 55-60 ms for 61 GB, PMC 1.5x).
// It now stores each task's spectrum as one contiguous run, [row j][task xq][ky] of 16-B elements, and this kernel
// transposes every row's [XQ][NK] element matrix into [NK][XQ] (the blocked [j][b = ky][x]): 32 x 64 element tiles
// through LDS, 1-KiB contiguous reads (a wave = one task row of 64 ky) and 512-B contiguous writes (32 tasks of one
// ky).  2N reals of extra traffic (one read + one write of the spectrum) for full-line accesses on both sides.
// grid (NK/64, XQ/32, row_cnt); block 256; rows [row_base, row_base + row_cnt).
template <typename R>
__global__ void __launch_bounds__(256) k_res_fwdy_fused_transpose_2d(KP<R> p, int XQ, int NK) {
  if (p.ctrl->done) return;
  __shared__ uint4 tile[32][65];
  const int k0 = blockIdx.x * 64, q0 = blockIdx.y * 32;
  const size_t rowsz = (size_t)XQ * NK;
  const size_t j = (size_t)p.row_base + blockIdx.z;
  const uint4* in = reinterpret_cast<const uint4*>(p.rspec) + j * rowsz;
  uint4* out = reinterpret_cast<uint4*>(p.work) + j * rowsz;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint4 v[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) v[r] = in[(size_t)(q0 + w + 4 * r) * NK + k0 + lane];
#pragma unroll
  for (int r = 0; r < 8; ++r) tile[w + 4 * r][lane] = v[r];
  __syncthreads();
  const int q = threadIdx.x & 31, kb = threadIdx.x >> 5;
#pragma unroll
  for (int r = 0; r < 8; ++r) out[(size_t)(k0 + kb + 8 * r) * XQ + q0 + q] = tile[q][kb + 8 * r];
}

// G workgroups striding over the T * nx/RW row-group tasks; block NT; LDS RW/2 * (N + N/16) * 8 B.
// sums: [0] sum (phi'-phi)^2, [1] sum phi^2 (old), [2] sum phi'^2
// RW = 2 with B = 1 (fp64 at C4's ny = 8192 with the half-real x blocks): one line, 16-B chunks.
// G16: only the first twiddled pass's seeds in LDS, the later passes' from twy (bitwise the same transform; fp64 ny = 2048
// with 256 threads: 70.4 KiB of LDS, two workgroups per CU -- the one-row windows' update)
template <int N, int RW, int NT, int PF = 1, typename R = float, bool G16 = false>
__global__ void __launch_bounds__(NT) k_invy_update_fast_2d(KP<R> p, const cplx<R>* __restrict__ twy) {
  using C = cplx<R>;
  using V = V4<R>;
  constexpr int NL = RW / 2;
  constexpr int GPT = (N / 4) / NT;
  if (p.ctrl->done) return;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  C* A = reinterpret_cast<C*>(smem_raw);
  R* Af = reinterpret_cast<R*>(A);
  constexpr bool TWL = N <= 4096;   // twiddle seeds in LDS (see k_res_fwdy_fused_2d)
  C* twl = A + NL * Pad<N>::LINE;
  if constexpr (TWL) fill_twlds<C, N>(twl, twy, 1, G16 ? 48 : TwLds<N>::SIZE);
  const int nx = p.nx, B = p.B, nb = p.nb;
  const int ngx = nx / RW;
  const int ntask = ngx * p.T;
  const size_t plane = (size_t)nx * N;
  const R scale = p.tau * p.inv_n;
  const int CS4 = RW * B / 4;
  const int lB = p.lB;
  const int lCS4 = lB + (RW == 8 ? 1 : RW == 4 ? 0 : RW == 2 ? -1 : -2);   // log2(CS4), B power of two
  const int tid = threadIdx.x;
  constexpr int NLD = RW * N / 4 / NT, BATCH = NLD < 8 ? NLD : 8;
  static_assert((RW * N / 4) % NT == 0 && NLD % BATCH == 0, "whole spectrum batches per thread");
  double s[3] = {0.0, 0.0, 0.0};
  // Per task: the spectrum goes to LDS, the first old-phi row pair is issued, and the transform runs on
  // LDS only (twiddle seeds in LDS), so that pair stays in flight across it; each pair prefetches the next.
  for (int task = xcd_remap(blockIdx.x, gridDim.x); task < ntask; task += gridDim.x) {
    const int j = task / ngx;
    const int x0 = (task - j * ngx) * RW;
    if (x0 + RW <= p.xl0 || x0 >= p.xl1) continue;   // x-slab padding / ghost rows only (workgroup-uniform)
    const R* wk = p.work + (size_t)j * nb * nx * B;
    // the task's spectrum (RW*B/4 float4 per block, N/B blocks = NLD per thread), in batches of up to 8
    // loads issued together: one memory round trip per batch, not per float4.  The thread index is
    // laundered per task so the 4*BATCH LDS addresses are not hoisted out of the task loop (registers).
    int tl = tid;
    asm volatile("" : "+v"(tl));
    if (RW == 2 && B == 1) {   // fp64 C4 (half-real spectrum): chunk b = rows x0, x0+1 at ky = b, one 16-B load
      constexpr int NC = N / NT, CB = NC < 8 ? NC : 8;
#pragma unroll
      for (int i0 = 0; i0 < NC; i0 += CB) {
        C v[CB];
#pragma unroll
        for (int i = 0; i < CB; ++i) v[i] = *reinterpret_cast<const C*>(wk + (size_t)(tl + (i0 + i) * NT) * nx + x0);
#pragma unroll
        for (int i = 0; i < CB; ++i) A[pix(tl + (i0 + i) * NT)] = v[i];
      }
    } else
#pragma unroll
    for (int i0 = 0; i0 < NLD; i0 += BATCH) {
      V v[BATCH];
#pragma unroll
      for (int i = 0; i < BATCH; ++i) {
        const int t = tl + (i0 + i) * NT;
        v[i] = (p.dbg & 512) ? ld4(wk + (size_t)x0 * N + 4 * t)   // PDHG_DBG 512: task-contiguous (timing)
                             : ld4(wk + ((size_t)(t >> lCS4) * nx + x0) * B + (t & (CS4 - 1)) * 4);
      }
#pragma unroll
      for (int i = 0; i < BATCH; ++i) {
        const int t = tl + (i0 + i) * NT;
        const int b = t >> lCS4, part = t & (CS4 - 1);
        if (B == 2) {   // the float4 holds rows r, r+1 (r = 2 part) at columns 2b, 2b+1: two complex elements
          C* Al = A + part * Pad<N>::LINE;
          Al[pix(2 * b)] = cmk<C>(v[i].x, v[i].z);
          Al[pix(2 * b + 1)] = cmk<C>(v[i].y, v[i].w);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int f = part * 4 + e;
            const int r = f >> lB, c = f & (B - 1);
            Af[((r >> 1) * Pad<N>::LINE + pix(b * B + c)) * 2 + (r & 1)] = f4(v[i], e);
          }
        }
      }
    }
    R* phi = p.phi + (size_t)(j + 1) * plane;
    R* pbar = p.phibar + (size_t)(j + 1) * plane;
    // old-phi row pairs, one per step s = gi * NL + l; PF steps in flight ahead of the one being updated
    // (step 0 before the transform, steps 1 .. PF-1 right after it, when the FFT's registers are free)
    constexpr int NS = GPT * NL;
    V op[NS][2];
    auto ldstep = [&](int s) {
      const size_t idx = (size_t)(x0 + 2 * (s % NL)) * N + 4 * (tid + (s / NL) * NT);
      op[s][0] = ld4(phi + idx);
      op[s][1] = ld4(phi + idx + N);
    };
    ldstep(0);
    lds_sync();
    if (!(p.dbg & 64)) {   // timing experiments only (PDHG_DBG): 64 skips the transform
      if constexpr (TWL && G16) lds_fft_inplace_tl16<C, N, NL, NT, Pad<N>::LINE>(A, twl, twy);
      else if constexpr (TWL) lds_fft_inplace_tl<C, N, NL, NT, Pad<N>::LINE>(A, twl);
      else lds_fft_inplace<C, N, NL, NT>(A, twy);
    }
#pragma unroll
    for (int s = 1; s < PF && s < NS; ++s) ldstep(s);
#pragma unroll
    for (int gi = 0; gi < GPT; ++gi) {
      const int y = 4 * (tid + gi * NT);
#pragma unroll
      for (int l = 0; l < NL; ++l) {   // rows 2l (real part) and 2l+1 (imaginary part) of line l
        const int st = gi * NL + l;
        const V o4[2] = {op[st][0], op[st][1]};
        if (st + PF < NS) ldstep(st + PF);
        const C* Z = A + l * Pad<N>::LINE;
        V u[2];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          R a, b2;
          hartley_padded<C, R>(Z, N, y + e, a, b2);
          f4set(u[0], e, a);
          f4set(u[1], e, b2);
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int xr = x0 + 2 * l + h;
          if (xr < p.xl0 || xr >= p.xl1) continue;   // x-slab ghost row (workgroup-uniform)
          const size_t idx = (size_t)xr * N + y;
          V nw, pb;
          R fs[3] = {(R)0, (R)0, (R)0};   // the 4 points in R (fp32: then one fp64 add per sum)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const R o = f4(o4[h], e);
            const R n = o + scale * f4(u[h], e);
            f4set(nw, e, n);
            f4set(pb, e, (R)2 * n - o);
            const R d = n - o;
            fs[0] = fmar(d, d, fs[0]);
            fs[1] = fmar(o, o, fs[1]);
            fs[2] = fmar(n, n, fs[2]);
          }
#pragma unroll
          for (int i = 0; i < 3; ++i) s[i] += (double)fs[i];
          st4(phi + idx, nw);
          st4(pbar + idx, pb);
        }
      }
    }
    lds_sync();
  }
  block_reduce_store<3>(s, p.partials, blockIdx.x);
}

}  // namespace pdhg

namespace pdhg {

// expm1(x) for x <= 0 in fp32 without libm's range reduction: degree-7 Taylor for x > -1/4
// (relative error < 2e-9), __expf(x) - 1 below (no cancellation there: |e^x - 1| > 0.22).
__device__ __forceinline__ float expm1_neg(float x) {
  const float p = x * (1.f + x * (0.5f + x * (1.f / 6 + x * (1.f / 24 + x * (1.f / 120 + x * (1.f / 720 + x * (1.f / 5040)))))));
  return x > -0.25f ? p : __expf(x) - 1.f;
}

// expm1 of two non-positive arguments: exp path everywhere, the cancellation-free Taylor
// polynomial only in waves where some lane has |x| < 0.25 (the low-frequency modes, a few
// waves) -- the branch is wave-uniform.
__device__ __forceinline__ float2 expm1_neg2(float a, float b) {
  float ea = __expf(a) - 1.f, eb = __expf(b) - 1.f;
  const bool sa = a > -0.25f, sb = b > -0.25f;
  if (__ballot(sa || sb) != 0) {
    auto poly = [](float x) {
      return x * (1.f + x * (0.5f + x * (1.f / 6 + x * (1.f / 24 + x * (1.f / 120 + x * (1.f / 720 + x * (1.f / 5040)))))));
    };
    if (sa) ea = poly(a);
    if (sb) eb = poly(b);
  }
  return make_float2(ea, eb);
}

// Thomas pivot state entering row j0 (t-slab decomposition): h_{j0-1} = 1 - g_{j0-1} in closed form,
// h_k = expm1(-th) (1 + e^{-th (2k+3)}) / E_{k+2} (no cancellation; h_{-1} = 1; theta -> 0: 1/(k+2)).
__device__ __forceinline__ float h_entry(float dd, int j0) {
  if (j0 == 0) return 1.f;
  const float dl = 0.5f * dd;
  const float th = fmaxf(log1pf(dl + sqrtf(dl * (dl + 2.f))), 1e-20f);
  return expm1f(-th) * (1.f + expf(-th * (float)(2 * j0 + 1))) / expm1f(-2.f * th * (float)(j0 + 1));
}
__device__ __forceinline__ double h_entry(double dd, int j0) {
  if (j0 == 0) return 1.0;
  const double dl = 0.5 * dd;
  const double th = fmax(log1p(dl + sqrt(dl * (dl + 2.0))), 1e-300);
  return expm1(-th) * (1.0 + exp(-th * (double)(2 * j0 + 1))) / expm1(-2.0 * th * (double)(j0 + 1));
}

// Column-block x-transform + Thomas in t (fp32, nx = N a power of two).
// A thread owns IT items (kx, l) of the block's NL complex lines; item (kx, l) carries the two
// modes (kx, 2l) and (kx, 2l+1), which are exactly the real and imaginary parts of line l's
// element kx, so the b' / x carries map 1:1 onto the in-place line-major FFT buffer.
// LDS: padded FFT buffer NL*(N + N/16) complex + per-item carries theta, E, b' as float2
// (3 * N*NL * 8 B); N*NL = 4096 -> 130 KiB.  Barriers are LDS-only (lds_sync) so the register prefetch of the
// next plane and the b'/x stores stay in flight across the FFT passes.
// grid: nb; block NT.
template <int N, int NL, int NT>
__global__ void __launch_bounds__(NT) k_precond_xt_fast_2d(KP<float> p, const float2* __restrict__ twx) {
  using C = float2;
  constexpr int IT = N * NL / NT;
  constexpr int B = 2 * NL;
  constexpr int NI = N * NL;            // items per block
  constexpr int LINE = Pad<N>::LINE;
  constexpr int lnl = (NL == 1) ? 0 : (NL == 2) ? 1 : (NL == 4) ? 2 : 3;
  if (p.ctrl->done) return;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  C* A = reinterpret_cast<C*>(smem_raw);
  C* sth = A + NL * LINE;
  C* sE = sth + NI;
  C* sbp = sE + NI;
  const int T = p.T, tid = threadIdx.x;
  const int b = blockIdx.x + p.b0;
  constexpr int M = N * B;
  float* wb = p.work + (size_t)b * M;
  const size_t kstride = (size_t)p.nb * M;
  const float ae = p.ae, inv_ae = 1.f / ae;
  // forward carries per item (2 modes): sth = dd = 2 delta = d0/ae, sE = h = 1 - g (h_{-1} = 1), sbp = b'
  C* twl = sbp + NI;   // TwLds<N> twiddle seeds
  fill_twlds<C, N>(twl, twx);
  // two-step register prefetch (pf: step k+1, pf2: step k+2; row indices clamped, so the loads are
  // branch-free): 64 KiB per CU in flight instead of 32
  C pf[IT], pf2[IT];
  auto ldrow = [&](C (&dstv)[IT], int kk) {
    const C* sn = reinterpret_cast<const C*>(wb + (size_t)kk * kstride);
#pragma unroll
    for (int i = 0; i < IT; ++i) dstv[i] = sn[tid + i * NT];
  };
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int item = tid + i * NT;
    const int kx = item >> lnl, l = item & (NL - 1);
    const float lx = p.lamx[kx];
    const float dd0 = (p.C - lx - p.lamy[b * B + 2 * l]) * inv_ae, dd1 = (p.C - lx - p.lamy[b * B + 2 * l + 1]) * inv_ae;
    sth[item] = make_float2(dd0, dd1);
    sE[item] = make_float2(h_entry(dd0, p.j0), h_entry(dd1, p.j0));
    sbp[item] = make_float2(0.f, 0.f);
  }
  if (p.xt_phase != 2) {
  ldrow(pf, 0);
  ldrow(pf2, min(1, T - 1));
  // ---------------- forward: DHT_x + elimination ----------------
  // Thomas pivots in the cancellation-free form (all terms >= 0, contractive):
  //   s = dd + h_{k-1},  g_k = ae/u_k = 1/(1+s),  h_k = 1 - g_k = s g_k,  b'_k = (rhs/ae + b'_{k-1}) g_k
  //   last (Neumann) row: u_{T-1} = ae (dd + h_{T-2}).
  for (int k = 0; k < T; ++k) {
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int item = tid + i * NT;
      A[(item & (NL - 1)) * LINE + pix(item >> lnl)] = pf[i];
    }
#pragma unroll
    for (int i = 0; i < IT; ++i) pf[i] = pf2[i];
    ldrow(pf2, min(k + 2, T - 1));
    lds_sync();
    if (!(p.dbg & 1)) lds_fft_inplace_tl<C, N, NL, NT>(A, twl);
    C* dst = reinterpret_cast<C*>(wb + (size_t)k * kstride);
    if (k < T - 1 || !p.last_slab) {
#pragma unroll
      for (int i = 0; i < IT; ++i) {
        const int item = tid + i * NT;
        const int kx = item >> lnl, l = item & (NL - 1);
        float ha, hb;
        hartley_padded<C, float>(A + l * LINE, N, kx, ha, hb);
        const C dd = sth[item], h = sE[item], bp = sbp[item];
        const float s0 = dd.x + h.x, s1 = dd.y + h.y;
        const float g0 = rcp_fast(1.f + s0), g1 = rcp_fast(1.f + s1);
        const C bn = make_float2((ha * inv_ae + bp.x) * g0, (hb * inv_ae + bp.y) * g1);
        sE[item] = make_float2(s0 * g0, s1 * g1);
        sbp[item] = bn;
        dst[item] = bn;
      }
    } else {
#pragma unroll
      for (int i = 0; i < IT; ++i) {
        const int item = tid + i * NT;
        const int kx = item >> lnl, l = item & (NL - 1);
        float ha, hb;
        hartley_padded<C, float>(A + l * LINE, N, kx, ha, hb);
        const C dd = sth[item], h = sE[item], bp = sbp[item];
        const C bn = make_float2((ha * inv_ae + bp.x) / (dd.x + h.x), (hb * inv_ae + bp.y) / (dd.y + h.y));
        sbp[item] = bn;
        if (p.slab) dst[item] = bn;   // re-read (after the carry fix-up) by the backward sweep
      }
    }
    lds_sync();
  }
  }   // xt_phase != 2
  if (p.xt_phase == 1) return;   // forward sweep only (t-slab: the carry fix-up runs in between)
  // ---------------- backward: substitution + inverse DHT_x ----------------
  // x_k = b'_k + g_k x_{k+1},  g_k = ae/u_k = e^-th E_{k+1}/E_{k+2}
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int item = tid + i * NT;
    const C dd = sth[item];
    float t2[2];
    const float dl[2] = {0.5f * dd.x, 0.5f * dd.y};
#pragma unroll
    for (int h = 0; h < 2; ++h) t2[h] = fmaxf(log1pf(dl[h] + sqrtf(dl[h] * (dl[h] + 2.f))), 1e-20f);   // cosh(th) = 1 + delta
    sth[item] = make_float2(t2[0], t2[1]);
    // E_{k+2} for the first substituted row: k = T-2 (single context) or T-1 (slab, from the right carry)
    const float e0 = (float)(p.j0 + T + (p.slab ? 1 : 0));
    sE[item] = make_float2(expm1f(-2.f * t2[0] * e0), expm1f(-2.f * t2[1] * e0));
    if (p.slab) sbp[item] = p.carry_y ? reinterpret_cast<const C*>(p.carry_y + (size_t)b * M)[item] : make_float2(0.f, 0.f);
  }
  // backward prefetch: step k consumes pf = b'_k (k < T-1; slab: every k, from the fixed-up rows);
  // after each step pf <- pf2, pf2 <- b'_{k-2}
  if (p.slab) ldrow(pf, T - 1);
  ldrow(pf2, max(T - 2, 0));
  for (int k = T - 1; k >= 0; --k) {
    const float kk1 = (float)(p.j0 + k + 1);   // global row index
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int item = tid + i * NT;
      C x2 = sbp[item];
      if ((k < T - 1 || p.slab) && !(p.dbg & 4)) {
        const C t2 = sth[item];
        const C e2 = sE[item];
        // theta >= 1e-20 (clamped at the sweep start): the closed form tends to (k+1)/(k+2) as theta -> 0
        const float2 E1 = expm1_neg2(-2.f * t2.x * kk1, -2.f * t2.y * kk1);
        const float g0 = __expf(-t2.x) * E1.x * rcp_fast(e2.x);
        const float g1 = __expf(-t2.y) * E1.y * rcp_fast(e2.y);
        x2 = make_float2(pf[i].x + g0 * x2.x, pf[i].y + g1 * x2.y);
        sE[item] = E1;
        sbp[item] = x2;
      }
      A[(item & (NL - 1)) * LINE + pix(item >> lnl)] = x2;
    }
#pragma unroll
    for (int i = 0; i < IT; ++i) pf[i] = pf2[i];
    ldrow(pf2, max(k - 2, 0));
    lds_sync();
    if (!(p.dbg & 2)) lds_fft_inplace_tl<C, N, NL, NT>(A, twl);
    C* wk = reinterpret_cast<C*>(wb + (size_t)k * kstride);
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int item = tid + i * NT;
      float ha, hb;
      hartley_padded<C, float>(A + (item & (NL - 1)) * LINE, N, item >> lnl, ha, hb);
      wk[item] = make_float2(ha, hb);
    }
    lds_sync();
  }
}

// ---- x-transform for a one-row window (T = 1, the reference's marching default; nx = N) ----
// With T = 1 the t-solve is one division per mode (the Neumann row: u = ae (dd + 1), utils_precond.py:164-169),
// so no carries are kept: forward DHT_x of the block's NL packed lines in LDS, scale every item, write it
// back as the packed lines, inverse DHT_x (same transform), store.  LDS = the padded lines + twiddle seeds
// (fp32: 41 KiB at N = 4096, N * NL = 4096; fp64: N * NL = 2048, or N = 4096 with NL = 1, the column pair of
// k_precond_xt_f64_2d).  HIP's second __launch_bounds__ argument is the minimum waves per SIMD: 4 keeps the
// kernel at <= 128 VGPRs, so two 512-thread (four 256-thread) workgroups fit a CU.
// G16: only the LS = 16 pass's seeds in LDS, the later passes' from twx (bitwise the same transform): fp64 N = 2048
// drops 46.75 -> 34.75 KiB of LDS, so four 256-thread workgroups fit a CU instead of three (1024 column pairs at C2:
// one round of 4 per CU instead of 1.33 rounds of 3).
template <int N, int NL, int NT, typename R = float, bool G16 = false>
__global__ void __launch_bounds__(NT, 4) k_precond_x_t1_2d(KP<R> p, const cplx<R>* __restrict__ twx) {
  using C = cplx<R>;
  constexpr int IT = N * NL / NT;
  constexpr int B = 2 * NL;
  constexpr int LINE = Pad<N>::LINE;
  constexpr int lnl = (NL == 1) ? 0 : (NL == 2) ? 1 : (NL == 4) ? 2 : 3;
  static_assert(IT * NT == N * NL, "whole items per thread");
  if (p.ctrl->done) return;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  C* A = reinterpret_cast<C*>(smem_raw);
  C* twl = A + NL * LINE;
  fill_twlds<C, N>(twl, twx, 1, G16 ? 48 : TwLds<N>::SIZE);
  auto fft = [&]() {
    if constexpr (G16) lds_fft_inplace_tl16<C, N, NL, NT>(A, twl, twx);
    else lds_fft_inplace_tl<C, N, NL, NT>(A, twl);
  };
  const int tid = threadIdx.x;
  const int b = blockIdx.x + p.b0;
  constexpr int M = N * B;
  C* wb = reinterpret_cast<C*>(p.work + (size_t)b * M);
  C v[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) v[i] = wb[tid + i * NT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int item = tid + i * NT;
    A[(item & (NL - 1)) * LINE + pix(item >> lnl)] = v[i];
  }
  lds_sync();
  fft();
  const R inv_ae = (R)1 / p.ae;
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int item = tid + i * NT;
    const int kx = item >> lnl, l = item & (NL - 1);
    R ha, hb;
    hartley_padded<C, R>(A + l * LINE, N, kx, ha, hb);
    const R lx = p.lamx[kx];
    const R dd0 = (p.C - lx - p.lamy[b * B + 2 * l]) * inv_ae, dd1 = (p.C - lx - p.lamy[b * B + 2 * l + 1]) * inv_ae;
    v[i] = cmk<C>(ha * inv_ae / (dd0 + (R)1), hb * inv_ae / (dd1 + (R)1));
  }
  lds_sync();   // every item has read its Hartley pair
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int item = tid + i * NT;
    A[(item & (NL - 1)) * LINE + pix(item >> lnl)] = v[i];
  }
  lds_sync();
  fft();
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int item = tid + i * NT;
    const int kx = item >> lnl, l = item & (NL - 1);
    R ha, hb;
    hartley_padded<C, R>(A + l * LINE, N, kx, ha, hb);
    wb[item] = cmk<C>(ha, hb);
  }
}

// ---- x-transform + Thomas, warp-specialised (fp32, nx = N a power of two, N*NL = 4096) ----
// Waves 0-3 (the FFT group, 256 threads) run the three Stockham passes on buffer X while waves 4-7
// (the Thomas group, 256 threads x 16 items) unpack buffer Y -- the previous t-row's transform --,
// do that row's Thomas step, store it, and stage the next row into Y.  X and Y swap every step, so
// a step costs max(FFT, Thomas) instead of their sum.  Each pass is split at its barrier
// (split_read / split_write); both groups execute the same 6 LDS-only barriers per step.
// Forward, step s = 0..T:   FFT(row s) | unpack FFT(row s-1) -> Thomas(s-1) -> b'_{s-1}; stage row s+1.
// Backward, step s = 0..T+1: FFT(x_{T-s}) | unpack FFT(x_{T+1-s}) -> work; x_{T-1-s} = b' + g x -> Y.
// Thomas carries (registers, per item of 2 modes): forward dd = 2 delta, h = 1 - g, b';
// backward theta, E, x (same arithmetic as k_precond_xt_fast_2d).
// LDS: 2 padded FFT buffers NL*(N + N/16) complex + twiddle seeds (~76 KiB).  grid: nb; block 512.
// HR ("half real", nx = 2N): column blocks of ONE real column of 2N points, packed z[m] = x[2m] + i x[2m+1]
// into the N-point FFT and split with realsplit_padded; item k carries modes kx = k and k + N.
// + N-complex split-twiddle table (W_{2N}^k) in LDS.
template <int N, int NL, bool HR = false>
__global__ void __launch_bounds__(512) k_precond_xt_ws_2d(KP<float> p, const float2* __restrict__ twx) {
  using C = float2;
  constexpr int NTF = 256, NTT = 256;
  constexpr int NI = N * NL;
  constexpr int IT = NI / NTT;
  constexpr int B = 2 * NL;
  constexpr int LINE = Pad<N>::LINE;
  constexpr int lnl = (NL == 1) ? 0 : (NL == 2) ? 1 : (NL == 4) ? 2 : 3;
  constexpr int CH0 = (IT + 2) / 3, CH1 = (2 * IT + 2) / 3;   // Thomas chunks [0,CH0) [CH0,CH1) [CH1,IT)
  static_assert(NI == 4096 && IT == 16, "sized for 4096 items per block");
  using P0 = SplitPass<N, NL, NTF, 0>;
  using P1 = SplitPass<N, NL, NTF, 1>;
  using P2 = SplitPass<N, NL, NTF, 2>;
  if (p.ctrl->done) return;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  C* buf0 = reinterpret_cast<C*>(smem_raw);
  C* buf1 = buf0 + NL * LINE;
  C* twl = buf1 + NL * LINE;
  C* rsw = twl + TwLds<N>::SIZE;                 // HR split twiddles W_{2N}^k, k < N
  fill_twlds<C, N>(twl, twx, HR ? 2 : 1);        // HR: twx holds W_{2N}
  if constexpr (HR) {
    static_assert(NL == 1, "one real column per block");
    for (int i = threadIdx.x; i < N; i += blockDim.x) rsw[i] = twx[i];
  }
  const int T = p.T, tid = threadIdx.x;
  const bool fftg = tid < NTF;                 // wave-uniform role
  const int tt = fftg ? 0 : tid - NTF;         // Thomas-group thread
  const int b = blockIdx.x + p.b0;
  constexpr int M = N * B;
  float* wb = p.work + (size_t)b * M;
  const size_t kstride = (size_t)p.nb * M;
  const float ae = p.ae, inv_ae = 1.f / ae;
  const int l = tt & (NL - 1);                 // line of every item of this thread (NTT % NL == 0)
  const int loff = l * LINE;
  auto kx_of = [&](int i) { return (tt + i * NTT) >> lnl; };
  // one register set for both roles: the FFT group's butterfly values live in c1 (16 complex),
  // which the Thomas group uses for its first carry -- each wave only ever takes one role
  C c1[IT], c2[IT], c3[IT], pf[IT];
  C (&vf)[IT] = c1;
  auto ldrow = [&](int kk) {
    const C* sn = reinterpret_cast<const C*>(wb + (size_t)kk * kstride);
#pragma unroll
    for (int i = 0; i < IT; ++i) pf[i] = sn[tt + i * NTT];
  };
  auto stage = [&](C* Y) {
#pragma unroll
    for (int i = 0; i < IT; ++i) Y[loff + pix(kx_of(i))] = pf[i];
  };
  // DHT pair of item i from a transformed buffer: two packed columns (Hartley) or one real column (HR)
  auto unpack2 = [&](const C* Y, int i, float& h0, float& h1) {
    if constexpr (HR)
      realsplit_padded<C, float>(Y, N, kx_of(i), rsw[kx_of(i)], h0, h1);
    else
      hartley_padded<C, float>(Y + loff, N, kx_of(i), h0, h1);
  };
  int bs0[P0::PER], bs1[P1::PER], bs2[P2::PER];

  if (!fftg) {
    const float cm0 = p.C - p.lamy[HR ? b : b * B + 2 * l];
    const float cm1 = HR ? cm0 : p.C - p.lamy[b * B + 2 * l + 1];
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const float lx0 = p.lamx[kx_of(i)], lx1 = HR ? p.lamx[kx_of(i) + N] : lx0;
      c1[i] = make_float2((cm0 - lx0) * inv_ae, (cm1 - lx1) * inv_ae);
    }
    if (p.xt_phase != 2) {
#pragma unroll
      for (int i = 0; i < IT; ++i) {
        c2[i] = make_float2(h_entry(c1[i].x, p.j0), h_entry(c1[i].y, p.j0));
        c3[i] = make_float2(0.f, 0.f);
      }
      ldrow(0);
      stage(buf0);
      ldrow(min(1, T - 1));
    }
  }
  lds_sync();

  // ---------------- forward sweep ----------------
  for (int s = 0; s <= T && p.xt_phase != 2; ++s) {
    C* X = (s & 1) ? buf1 : buf0;
    C* Y = (s & 1) ? buf0 : buf1;
    const bool fft_on = s < T && !(p.dbg & 1);
    const int kr = (p.dbg & 4) ? -1 : s - 1;                        // row finished by the Thomas group this step
    C* dst = reinterpret_cast<C*>(wb + (size_t)max(kr, 0) * kstride);
    // one Thomas chunk [I0, I1): the uniform row test sits outside the item loop, so each chunk is
    // straight-line code (all its LDS reads issue together)
    auto thomas = [&](auto I0c, auto I1c) {
      constexpr int I0 = decltype(I0c)::value, I1 = decltype(I1c)::value;
      float ha[I1 - I0], hb[I1 - I0];
#pragma unroll
      for (int i = I0; i < I1; ++i) unpack2(Y, i, ha[i - I0], hb[i - I0]);
      if (kr < T - 1 || !p.last_slab) {
#pragma unroll
        for (int i = I0; i < I1; ++i) {
          const float s0 = c1[i].x + c2[i].x, s1 = c1[i].y + c2[i].y;
          const float g0 = rcp_fast(1.f + s0), g1 = rcp_fast(1.f + s1);
          c3[i] = make_float2((ha[i - I0] * inv_ae + c3[i].x) * g0, (hb[i - I0] * inv_ae + c3[i].y) * g1);
          c2[i] = make_float2(s0 * g0, s1 * g1);
          dst[tt + i * NTT] = c3[i];
        }
      } else {   // Neumann last row: u_{T-1} = ae (dd + h_{T-2})
#pragma unroll
        for (int i = I0; i < I1; ++i) {
          c3[i] = make_float2((ha[i - I0] * inv_ae + c3[i].x) / (c1[i].x + c2[i].x),
                              (hb[i - I0] * inv_ae + c3[i].y) / (c1[i].y + c2[i].y));
          if (p.slab) dst[tt + i * NTT] = c3[i];   // re-read (after the carry fix-up) by the backward sweep
        }
      }
    };
    using Z0 = std::integral_constant<int, 0>;
    using ZA = std::integral_constant<int, CH0>;
    using ZB = std::integral_constant<int, CH1>;
    using ZC = std::integral_constant<int, IT>;
    // P1
    if (fftg) {
      if (fft_on) split_read<C, N, NL, NTF, 0>(X, twl, tid, vf, bs0);
    } else if (kr >= 0) {
      thomas(Z0{}, ZA{});
    }
    lds_sync();
    // P2
    if (fftg) {
      if (fft_on) split_write<C, N, NL, NTF, 0>(X, vf, bs0);
    } else if (kr >= 0) {
      thomas(ZA{}, ZB{});
    }
    lds_sync();
    // P3
    if (fftg) {
      if (fft_on) split_read<C, N, NL, NTF, 1>(X, twl, tid, vf, bs1);
    } else if (kr >= 0) {
      thomas(ZB{}, ZC{});
    }
    lds_sync();
    // P4: Y is no longer read -> stage row s+1 into it, prefetch row s+2
    if (fftg) {
      if (fft_on) split_write<C, N, NL, NTF, 1>(X, vf, bs1);
    } else if (s + 1 < T) {
      stage(Y);
      ldrow(min(s + 2, T - 1));
    }
    lds_sync();
    // P5
    if (fftg && fft_on) split_read<C, N, NL, NTF, 2>(X, twl, tid, vf, bs2);
    lds_sync();
    // P6
    if (fftg && fft_on) split_write<C, N, NL, NTF, 2>(X, vf, bs2);
    lds_sync();
  }

  // ---------------- backward sweep ----------------
  // x_k = b'_k + g_k x_{k+1},  g_k = ae/u_k = e^-th E_{k+1}/E_{k+2},  E_m = expm1(-2 th m)
  if (p.xt_phase == 1) return;   // forward sweep only (t-slab: the carry fix-up runs in between)
  if (!fftg) {
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const float dl0 = 0.5f * c1[i].x, dl1 = 0.5f * c1[i].y;
      c1[i] = make_float2(fmaxf(log1pf(dl0 + sqrtf(dl0 * (dl0 + 2.f))), 1e-20f),
                          fmaxf(log1pf(dl1 + sqrtf(dl1 * (dl1 + 2.f))), 1e-20f));
      // E_{k+2} for the first substituted row: k = T-2 (single context) or T-1 (slab, from the right carry)
      const float e0 = (float)(p.j0 + T + (p.slab ? 1 : 0));
      c2[i] = make_float2(expm1f(-2.f * c1[i].x * e0), expm1f(-2.f * c1[i].y * e0));
      if (p.slab)
        c3[i] = p.carry_y ? reinterpret_cast<const C*>(p.carry_y + (size_t)b * M)[tt + i * NTT] : make_float2(0.f, 0.f);
    }
    ldrow(p.slab ? T - 1 : max(T - 2, 0));
  }
  for (int s = 0; s <= T + 1; ++s) {
    C* X = (s & 1) ? buf1 : buf0;
    C* Y = (s & 1) ? buf0 : buf1;
    const bool fft_on = s >= 1 && s <= T && !(p.dbg & 1);
    const int ku = T + 1 - s;                    // row unpacked by the Thomas group (if s >= 2)
    const int kn = T - 1 - s;                    // x row computed by the Thomas group (if s <= T-1)
    C* wk = reinterpret_cast<C*>(wb + (size_t)max(min(ku, T - 1), 0) * kstride);
    const float kk1 = (float)(p.j0 + kn + 1);   // global row index
    auto unpack = [&](int i) {
      float ha, hb;
      unpack2(Y, i, ha, hb);
      if constexpr (HR) {   // spatial x = k and k + N of the real column
        float* wf = reinterpret_cast<float*>(wk);
        wf[kx_of(i)] = ha;
        wf[kx_of(i) + N] = hb;
      } else {
        wk[tt + i * NTT] = make_float2(ha, hb);
      }
    };
    auto subst = [&](int i) {
      // theta >= 1e-20 (clamped at the sweep start): the closed form tends to (k+1)/(k+2) as theta -> 0
      const float2 E1 = expm1_neg2(-2.f * c1[i].x * kk1, -2.f * c1[i].y * kk1);
      const float g0 = __expf(-c1[i].x) * E1.x * rcp_fast(c2[i].x);
      const float g1 = __expf(-c1[i].y) * E1.y * rcp_fast(c2[i].y);
      c3[i] = make_float2(pf[i].x + g0 * c3[i].x, pf[i].y + g1 * c3[i].y);
      c2[i] = E1;
    };
    const bool do_unpack = s >= 2 && !(p.dbg & 4), do_subst = (s >= 1 || p.slab) && s <= T - 1 && !(p.dbg & 4),
               do_stage = s <= T - 1;
    // stage x_{kn} of items [I0, I1) into Y (after every unpack read of Y: phases P4-P6)
    auto stage_x = [&](auto I0c, auto I1c) {
      constexpr int I0 = decltype(I0c)::value, I1 = decltype(I1c)::value;
      if constexpr (HR) {   // modes k and k + N -> packed positions (float f at element f/2, part f%2)
        float* Yf = reinterpret_cast<float*>(Y);
#pragma unroll
        for (int i = I0; i < I1; ++i) {
          const int f0 = kx_of(i), f1 = kx_of(i) + N;
          Yf[2 * pix(f0 >> 1) + (f0 & 1)] = c3[i].x;
          Yf[2 * pix(f1 >> 1) + (f1 & 1)] = c3[i].y;
        }
      } else {
#pragma unroll
        for (int i = I0; i < I1; ++i) Y[loff + pix(kx_of(i))] = c3[i];
      }
    };
    using Z0 = std::integral_constant<int, 0>;
    using ZA = std::integral_constant<int, CH0>;
    using ZB = std::integral_constant<int, CH1>;
    using ZC = std::integral_constant<int, IT>;
    // P1-P3: FFT passes 0-1 | unpack of Y (the previous x row's transform) in three chunks
    if (fftg) {
      if (fft_on) split_read<C, N, NL, NTF, 0>(X, twl, tid, vf, bs0);
    } else if (do_unpack) {
#pragma unroll
      for (int i = 0; i < CH0; ++i) unpack(i);
    }
    lds_sync();
    if (fftg) {
      if (fft_on) split_write<C, N, NL, NTF, 0>(X, vf, bs0);
    } else if (do_unpack) {
#pragma unroll
      for (int i = CH0; i < CH1; ++i) unpack(i);
    }
    lds_sync();
    if (fftg) {
      if (fft_on) split_read<C, N, NL, NTF, 1>(X, twl, tid, vf, bs1);
    } else if (do_unpack) {
#pragma unroll
      for (int i = CH1; i < IT; ++i) unpack(i);
    }
    lds_sync();
    // P4-P6: FFT passes 1-2 | substitution x_{kn} = b'_{kn} + g x_{kn+1} in three chunks, staged into Y;
    // the next b' row is prefetched once the last chunk has consumed pf
    if (fftg) {
      if (fft_on) split_write<C, N, NL, NTF, 1>(X, vf, bs1);
    } else if (do_stage) {
      if (do_subst) {
#pragma unroll
        for (int i = 0; i < CH0; ++i) subst(i);
      }
      stage_x(Z0{}, ZA{});
    }
    lds_sync();
    if (fftg) {
      if (fft_on) split_read<C, N, NL, NTF, 2>(X, twl, tid, vf, bs2);
    } else if (do_stage) {
      if (do_subst) {
#pragma unroll
        for (int i = CH0; i < CH1; ++i) subst(i);
      }
      stage_x(ZA{}, ZB{});
    }
    lds_sync();
    if (fftg) {
      if (fft_on) split_write<C, N, NL, NTF, 2>(X, vf, bs2);
    } else if (do_stage) {
      if (do_subst) {
#pragma unroll
        for (int i = CH1; i < IT; ++i) subst(i);
      }
      stage_x(ZB{}, ZC{});
      ldrow(max(kn - 1, 0));
    }
    lds_sync();
  }
}

// ---- dual step, fp32, time-marching (update_fns_in_pdhg.py:150-165) ----
// grid: (nx rows [XCD-aware], ny/4/NT y-chunks, nJ time chunks); block NT = min(256, ny/4), ny % 256 == 0
// (so every wave is fully inside [0, ny)).
// A thread owns 4 consecutive y (float4) of one x row and marches over its chunk of time rows:
// phi_bar row j+1 is loaded once and kept as phi_bar "row j" of the next step, so phi_bar is read
// about once per iteration instead of twice.  The loads of step j+1 are issued before step j is
// computed; every load reads a valid address (rows outside a Dirichlet edge are clamped, then
// zeroed by a select), so nothing drains the load queue.  y neighbours come from the adjacent
// lanes (DPP), the wave-edge ones from uniform loads.  Sums as in k_dual_2d (double per point).
// ONE: every workgroup has exactly one time row (jchunk == 1, e.g. the T = 1 marching windows): the row is loaded
// once, with no prefetch registers (the marching form re-loads its last row to stay branch-free), the same arithmetic.
// ONE = 2: the same with 4 waves per SIMD asked of the compiler (fp64: 128 VGPRs + 28 B of spill, A/B only).
template <int EGNO, typename R = float, int ONE = 0>
__global__ void __launch_bounds__(256, ONE == 2 ? 4 : 1) k_dual_fast_2d(KP<R> p, int jchunk, int jbase, int jend, int zbase) {
  using V = V4<R>;
  if (p.ctrl->done || p.ctrl->inner_done) return;
  constexpr int NA = (EGNO == 3) ? 2 : 4;
  constexpr int NS = 3 + 3 * NA;
  const int cur = p.ctrl->cur;
  const int src_set = (p.inplace || p.sub == 0) ? cur : 1 - cur;
  const int dst_set = p.inplace ? cur : 1 - cur;
  const int nx = p.nx, ny = p.ny;
  const size_t plane = (size_t)nx * ny;
  const int x = xcd_remap(blockIdx.x, gridDim.x);
  const bool live = x >= p.xl0 && x < p.xl1;   // workgroup-uniform (x-slab ghost / padding rows: not stored or summed)
  const int y = 4 * (blockIdx.y * blockDim.x + threadIdx.x);
  // rows [jbase, jend) in chunks of jchunk (blockIdx.z); partials of this launch start at block row zbase
  const int j0 = jbase + blockIdx.z * jchunk;
  const int j1 = min(jend, j0 + jchunk);
  double s[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) s[i] = 0.0;
  if (y < ny) {
    const int yw0 = __builtin_amdgcn_readfirstlane(y);
    const int ywm = nb_index(yw0 - 1, ny, p.bcy), ywp = nb_index(yw0 + 4 * kWave, ny, p.bcy);
    const bool zym = ywm < 0, zyp = ywp < 0;
    const int ywmc = zym ? 0 : ywm, ywpc = zyp ? 0 : ywp;
    const int xm = nb_index(x - 1, nx, p.bcx), xp = nb_index(x + 1, nx, p.bcx);
    const bool zxm = xm < 0, zxp = xp < 0;
    const size_t rxm = (size_t)(zxm ? x : xm) * ny, rxc = (size_t)x * ny, rxp = (size_t)(zxp ? x : xp) * ny;
    const V ay4 = ld4(p.ay + y);
    const R axc = p.ax[x];
    const R* rs = p.rho[src_set];
    R* rd = p.rho[dst_set];
    const R* as[NA];
    R* ad[NA];
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      as[a] = p.alp[src_set][a];
      ad[a] = p.alp[dst_set][a];
    }
    struct In {
      V pm, pc, pp, rho, al[NA];
      R el, er;
    };
    auto load = [&](int j) {
      In in;
      const R* f1 = p.phibar + (size_t)(j + 1) * plane;
      in.pm = ld4(f1 + rxm + y);
      in.pc = ld4(f1 + rxc + y);
      in.pp = ld4(f1 + rxp + y);
      in.el = f1[rxc + ywmc];
      in.er = f1[rxc + ywpc];
      const size_t o = (size_t)j * plane + rxc + y;
      in.rho = ld4(rs + o);
#pragma unroll
      for (int a = 0; a < NA; ++a) in.al[a] = ld4(as[a] + o);
      return in;
    };
    V f0 = ld4(p.phibar + (size_t)j0 * plane + rxc + y);   // phi_bar row j
    auto step = [&](int j, const In& in) {
      const V pm = zxm ? z4r<R>() : in.pm, pp = zxp ? z4r<R>() : in.pp, pc = in.pc;
      const R pyl = lane_from_prev(pc.w, zym ? (R)0 : in.el);
      const R pyr = lane_from_next(pc.x, zyp ? (R)0 : in.er);
      V rn4, an4[NA];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const R c = f4(pc, e);
        const R lft = e == 0 ? pyl : f4(pc, e - 1);
        const R rgt = e == 3 ? pyr : f4(pc, e + 1);
        R ao[4], an[4];
#pragma unroll
        for (int a = 0; a < NA; ++a) ao[a] = f4(in.al[a], e);
        const R rho = f4(in.rho, e);
        const R rn = dual_point<R, EGNO>(p, c, f4(pm, e), f4(pp, e), lft, rgt, f4(f0, e), rho, ao, axc,
                                                 f4(ay4, e), an);
        f4set(rn4, e, rn);
#pragma unroll
        for (int a = 0; a < NA; ++a) f4set(an4[a], e, an[a]);
        if (!live) continue;
        const double dr = (double)rn - (double)rho;
        s[0] += dr * dr;
        s[1] += (double)rn * (double)rn;
        s[2] += (double)rho * (double)rho;
#pragma unroll
        for (int a = 0; a < NA; ++a) {
          const double da = (double)an[a] - (double)ao[a];
          s[3 + 3 * a] += da * da;
          s[4 + 3 * a] += (double)an[a] * (double)an[a];
          s[5 + 3 * a] += (double)ao[a] * (double)ao[a];
        }
      }
      const size_t o = (size_t)j * plane + rxc + y;
      if (live) {
        st4(rd + o, rn4);
#pragma unroll
        for (int a = 0; a < NA; ++a) st4(ad[a] + o, an4[a]);
      }
      f0 = pc;
    };
    if constexpr (ONE) {   // one row per workgroup: no next-row prefetch (half the input registers)
      step(j0, load(j0));
    } else {
      In nxt = load(j0);
#pragma unroll 1
      for (int j = j0; j < j1; ++j) {
        const In in = nxt;
        nxt = load(min(j + 1, j1 - 1));   // (the last step reloads its own row: keeps the loop branch-free)
        step(j, in);
      }
    }
  }
  block_reduce_store<NS>(s, p.partials, ((zbase + (int)blockIdx.z) * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x);
}

}  // namespace pdhg
