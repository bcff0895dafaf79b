// 65536-point DHT of row pairs as 16 x 4096 (nx = 65536: C1, BASELINE configs[1]; fp32 and fp64) with a permuted
// spectrum.
//
// Same preconditioner as the four-step kernels (H1_precond_1d, utils_precond.py:105-140: DHT_x of the
// residual rows, the t-solve per mode, the inverse DHT, phi update), with a split chosen for HBM streaming:
// x = 4096 n1 + n2, k = k1 + 16 k2.
//   forward  (decimation in frequency)  A: per column n2, a 16-point DFT over n1 (registers only: every
//            load / store of a wave is 64 consecutive columns), times W_65536^{n2 k1}, to Y[k1][n2];
//            B: per chunk k1, a 4096-point FFT over n2 in LDS, then the Hartley unpack of the row pair.
//   inverse  (decimation in time)       B': per chunk k1 of the spectrum, a 4096-point FFT;
//            A': per column n2, W_65536^{n2 k1} times the chunk values, a 16-point DFT over k1, the Hartley
//            unpack, phi' = phi + tau/nx U, phi_bar = 2 phi' - phi and the err1 sums.
// The spectrum in p.work is stored chunk-major, mode k = k1 + 16 k2 at position k1 4096 + k2: the t-solve is
// per mode and reads d0 through the same permutation (the host uploads d0 permuted), so no transpose is ever
// made, and the forward leaves / the inverse takes exactly that order.  The Hartley partner of k is
// N - k = (16 - k1) + 16 (4095 - k2) (chunk 16 - k1, reversed) for k1 != 0 and chunk 0 reversed mod 4096 for
// k1 = 0; of x = 4096 n1 + n2 it is 4096 (15 - n1) + 4096 - n2 (column 4096 - n2) for n2 != 0.
// HBM per iteration: A reads the residual inputs and writes Y (8 B/point), B reads Y and writes the spectrum
// rows, B' / A' the same the other way round; every access is a whole 128-B line.
// fp64 (R = double): the same stages on complex doubles; stage B's 2 lines + twiddle seeds take 152 KiB of LDS.
#pragma once
#include "kernels_2d_fast.hpp"
#include "kernels_fs_wide.hpp"

namespace pdhg {

constexpr int kF16N2 = 4096;
constexpr int kF16Line = Pad<kF16N2>::LINE;

// Hartley values of rows a, b at k and N - k from Z_k = z, Z_{N-k} = w (fft_lds.hpp header)
template <typename R>
struct HPair {
  R ha, hb, ma, mb;
};
template <typename C>
__device__ __forceinline__ HPair<decltype(C::x)> hunpack(C z, C w) {
  using R = decltype(C::x);
  const R h = (R)0.5;
  HPair<R> q;
  q.ha = h * ((z.x + w.x) - (z.y - w.y));
  q.hb = h * ((z.y + w.y) - (w.x - z.x));
  q.ma = h * ((w.x + z.x) - (w.y - z.y));
  q.mb = h * ((w.y + z.y) - (z.x - w.x));
  return q;
}

// value of v in lane l (wave-uniform result)
template <typename R>
__device__ __forceinline__ R lane_value(R v, int l) {
  if constexpr (sizeof(R) == 4) {
    return __builtin_bit_cast(R, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
  } else {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
    return __builtin_bit_cast(R, ((unsigned long long)hi << 32) | lo);
  }
}

// Stage A (forward).  grid (4096/256, pairs); block 256: thread = column n2; 16 residual values per row,
// formed in groups of G rows n1 (a scheduling barrier between groups bounds the loads the compiler hoists).
// The x -+ 1 neighbours come from the neighbouring lanes (DPP); the values beyond the wave's 64 columns for
// all 16 rows n1 are fetched by ONE load per array (lane l < 16: column cw - 1 of row n1 = l, lane 16 + l:
// column cw + 64) and picked per row with readlane.
template <int EGNO, int G = 16, typename R = float>
__global__ void __launch_bounds__(256, G == 16 ? 1 : 4) k_f16a_fwd_1d(KP<R> p, const cplx<R>* __restrict__ twN,
                                                     cplx<R>* __restrict__ Y) {
  using C = cplx<R>;
  if (p.ctrl->done) return;
  const int nx = p.nx, T = p.T;
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63, cw = c - lane;   // first column of this wave
  const int pair = blockIdx.y, j = 2 * pair;
  const bool has2 = (j + 1) < T;
  const int cur = p.ctrl->cur;
  const R* rho = p.rho[cur];
  const R* a1 = p.alp[cur][0];
  const R* a2 = p.alp[cur][1];
  const int j1c = has2 ? j + 1 : j, j2 = min(j + 2, T - 1);
  const size_t o0 = (size_t)j * nx, o1 = (size_t)j1c * nx;
  const R* r_j = rho + o0;
  const R* r_j1 = rho + o1;
  const R* r_j2 = rho + (size_t)j2 * nx;
  const int ex = (kF16N2 * (lane & 15) + cw + ((lane & 16) ? 64 : -1)) & (nx - 1);
  const R e_ax = p.ax[ex], e_r0 = r_j[ex], e_r1 = r_j1[ex];
  const R e_b10 = a1[o0 + ex], e_b20 = a2[o0 + ex], e_b11 = a1[o1 + ex], e_b21 = a2[o1 + ex];
  auto edge = [](R v, int l) { return lane_value(v, l); };
  C v[16];
  int cl = c;   // laundered at every group: the group's addresses are formed there, not hoisted to the top
#pragma unroll
  for (int n1 = 0; n1 < 16; ++n1) {
    if (n1 % G == 0) {
      if (n1 > 0) __builtin_amdgcn_sched_barrier(0);
      cl = c;
      asm volatile("" : "+v"(cl));
    }
    const int x = kF16N2 * n1 + cl;
    const R ac = p.ax[x];
    const R am = lane_from_prev(ac, edge(e_ax, n1)), ap = lane_from_next(ac, edge(e_ax, 16 + n1));
    // every load unconditional (rows clamped into [0, T)), the missing row's terms selected away
    const R c0 = r_j[x], c1 = r_j1[x], c2 = r_j2[x];
    const R b10 = a1[o0 + x], b20 = a2[o0 + x], b11 = a1[o1 + x], b21 = a2[o1 + x];
    const R r0 = res1d<EGNO>(p, c0, lane_from_prev(c0, edge(e_r0, n1)), lane_from_next(c0, edge(e_r0, 16 + n1)),
                             has2 ? c1 : (R)0, b10, lane_from_prev(b10, edge(e_b10, n1)), b20,
                             lane_from_next(b20, edge(e_b20, 16 + n1)), ac, am, ap, j == T - 1);
    const R r1 = res1d<EGNO>(p, c1, lane_from_prev(c1, edge(e_r1, n1)), lane_from_next(c1, edge(e_r1, 16 + n1)),
                             (j + 2 < T) ? c2 : (R)0, b11, lane_from_prev(b11, edge(e_b11, n1)), b21,
                             lane_from_next(b21, edge(e_b21, 16 + n1)), ac, am, ap, j + 1 == T - 1);
    v[n1] = cmk<C>(r0, has2 ? r1 : (R)0);
  }
  dft_any<C, 16>(v);
  C w[16];
  twiddles_from3<C, 16>(w, twN, c);   // W_65536^{c k1}
  C* Yp = Y + (size_t)pair * nx + c;
  Yp[0] = v[0];
#pragma unroll
  for (int k1 = 1; k1 < 16; ++k1) Yp[(size_t)k1 * kF16N2] = cmul(v[k1], w[k1]);
}

// Stage B (forward).  grid (8, pairs); block 512; LDS 2 lines of 4096 + TwLds<4096>.
// Workgroup g transforms chunks {g, 16 - g} (g = 0: the self-partnered chunks {0, 8}) and writes the
// Hartley rows j, j+1 of both to p.work at chunk-major positions.
template <typename R = float>
__global__ void __launch_bounds__(512) k_f16b_fwd_1d(KP<R> p, const cplx<R>* __restrict__ twN,
                                                     const cplx<R>* __restrict__ Y) {
  using C = cplx<R>;
  constexpr int NT = 512, L = kF16Line;
  if (p.ctrl->done) return;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  C* A = reinterpret_cast<C*>(smem_raw);
  C* twl = A + 2 * L;
  fill_twlds<C, kF16N2>(twl, twN, 16);   // twN holds W_65536: stride 16 gives W_4096
  const int nx = p.nx, g = blockIdx.x, pair = blockIdx.y, j = 2 * pair;
  const bool has2 = (j + 1) < p.T;
  const int ka = g, kb = (g == 0) ? 8 : 16 - g;
  const C* Yp = Y + (size_t)pair * nx;
  const int tid = threadIdx.x;
#pragma unroll 4
  for (int i = tid; i < 2 * (kF16N2 / 2); i += NT) {   // two complex per load (16 B fp32, 32 B fp64)
    const int ln = i >> 11, e = 2 * (i & 2047);
    const V4<R> q = ld4(reinterpret_cast<const R*>(Yp + (size_t)(ln ? kb : ka) * kF16N2 + e));
    C* d = A + ln * L;
    d[pix(e)] = cmk<C>(q.x, q.y);
    d[pix(e + 1)] = cmk<C>(q.z, q.w);
  }
  lds_sync();
  lds_fft_inplace_tl<C, kF16N2, 2, NT>(A, twl);
  R* w0 = p.work + (size_t)j * nx;
  R* w1 = w0 + nx;
  if (g == 0) {   // chunk 0: partner (4096 - k2) mod 4096; chunk 8: partner 4095 - k2 (one output each)
#pragma unroll 2
    for (int i = tid; i < kF16N2; i += NT) {
      const HPair<R> h0 = hunpack(A[pix(i)], A[pix((kF16N2 - i) & (kF16N2 - 1))]);
      const HPair<R> h8 = hunpack(A[L + pix(i)], A[L + pix(kF16N2 - 1 - i)]);
      w0[i] = h0.ha;
      w0[8 * kF16N2 + i] = h8.ha;
      if (has2) {
        w1[i] = h0.hb;
        w1[8 * kF16N2 + i] = h8.hb;
      }
    }
  } else {        // chunk ka element i pairs with chunk kb element 4095 - i: both outputs
#pragma unroll 2
    for (int i = tid; i < kF16N2; i += NT) {
      const HPair<R> h = hunpack(A[pix(i)], A[L + pix(kF16N2 - 1 - i)]);
      const int P = ka * kF16N2 + i, Pm = kb * kF16N2 + (kF16N2 - 1 - i);
      w0[P] = h.ha;
      w0[Pm] = h.ma;
      if (has2) {
        w1[P] = h.hb;
        w1[Pm] = h.mb;
      }
    }
  }
}

// Stage B' (inverse).  grid (8, pairs); block 512: chunks {2g, 2g+1} of spectrum rows j, j+1 packed as
// z = H_j + i H_{j+1}, 4096-point FFT, to Y[k1][n2].
template <typename R = float>
__global__ void __launch_bounds__(512) k_f16b_inv_1d(KP<R> p, const cplx<R>* __restrict__ twN,
                                                     cplx<R>* __restrict__ Y) {
  using C = cplx<R>;
  constexpr int NT = 512, L = kF16Line;
  if (p.ctrl->done) return;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  C* A = reinterpret_cast<C*>(smem_raw);
  C* twl = A + 2 * L;
  fill_twlds<C, kF16N2>(twl, twN, 16);
  const int nx = p.nx, g = blockIdx.x, pair = blockIdx.y, j = 2 * pair;
  const bool has2 = (j + 1) < p.T;
  const R* w0 = p.work + (size_t)j * nx + 2 * g * kF16N2;   // chunks 2g, 2g+1 are contiguous
  const R* w1 = w0 + nx;
  const int tid = threadIdx.x;
#pragma unroll 4
  for (int i = tid; i < 2 * kF16N2 / 4; i += NT) {   // four points per load of each row
    const int e = 4 * i;
    const V4<R> a = ld4(w0 + e);
    const V4<R> b = has2 ? ld4(w1 + e) : z4r<R>();
    C* d = A + (e >> 12) * L;
    const int el = e & (kF16N2 - 1);
    d[pix(el)] = cmk<C>(a.x, b.x);
    d[pix(el + 1)] = cmk<C>(a.y, b.y);
    d[pix(el + 2)] = cmk<C>(a.z, b.z);
    d[pix(el + 3)] = cmk<C>(a.w, b.w);
  }
  lds_sync();
  lds_fft_inplace_tl<C, kF16N2, 2, NT>(A, twl);
  C* Yp = Y + (size_t)pair * nx + 2 * g * kF16N2;
#pragma unroll 4
  for (int i = tid; i < kF16N2; i += NT) {   // two complex per store
    const int e = 2 * i;
    const C* s = A + (e >> 12) * L;
    const int el = e & (kF16N2 - 1);
    const C u0 = s[pix(el)], u1 = s[pix(el + 1)];
    V4<R> o;
    o.x = u0.x;
    o.y = u0.y;
    o.z = u1.x;
    o.w = u1.y;
    st4(reinterpret_cast<R*>(Yp + e), o);
  }
}

// Stage A' (inverse) + primal update.  grid (2048/256, pairs); block 256: thread t owns columns t and
// 4096 - t (t = 0: the self-partnered columns 0 and 2048).  One partial row of err1 sums per workgroup.
template <typename R = float>
__global__ void __launch_bounds__(256) k_f16a_inv_1d(KP<R> p, const cplx<R>* __restrict__ twN,
                                                     const cplx<R>* __restrict__ Y) {
  using C = cplx<R>;
  double s[3] = {0.0, 0.0, 0.0};
  const int row = blockIdx.y * gridDim.x + blockIdx.x;
  if (p.ctrl->done) {
    block_reduce_store<3>(s, p.partials, row);
    return;
  }
  const int nx = p.nx, pair = blockIdx.y, j = 2 * pair;
  const bool has2 = (j + 1) < p.T;
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int ca = t, cb = (t == 0) ? kF16N2 / 2 : kF16N2 - t;
  const C* Yp = Y + (size_t)pair * nx;
  auto column = [&](int cc, C (&v)[16]) {
#pragma unroll
    for (int k1 = 0; k1 < 16; ++k1) v[k1] = Yp[(size_t)k1 * kF16N2 + cc];
    C w[16];
    twiddles_from3<C, 16>(w, twN, cc);
#pragma unroll
    for (int k1 = 1; k1 < 16; ++k1) v[k1] = cmul(v[k1], w[k1]);
    dft_any<C, 16>(v);
  };
  C fa[16], fb[16];
  column(ca, fa);
  column(cb, fb);
  const R scale = p.tau * p.inv_n;
  R* phi1 = p.phi + (size_t)(j + 1) * nx;   // phi rows j+1, j+2 (row 0 is the fixed initial condition)
  R* pb1 = p.phibar + (size_t)(j + 1) * nx;
  auto upd = [&](R old, R u, R* ph, R* pbar, int n) {
    const R nw = old + scale * u;
    ph[n] = nw;
    pbar[n] = (R)2 * nw - old;
    const double d = (double)nw - (double)old;
    s[0] += d * d;
    s[1] += (double)old * (double)old;
    s[2] += (double)nw * (double)nw;
  };
  // 8 x-positions per half: their phi loads are issued together, before any store of the half
  // (the stores go through the same pointer, so the compiler cannot move later loads above them)
#pragma unroll
  for (int h0 = 0; h0 < 16; h0 += 8) {
    R oa[8][2], ob[8][2];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int n1 = h0 + q;
      const int na = kF16N2 * n1 + ca, nb = kF16N2 * (15 - n1) + cb;
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const R* ph = phi1 + (size_t)r * nx;
        const bool live = r == 0 || has2;
        oa[q][r] = live ? ph[na] : (R)0;
        ob[q][r] = live ? ph[(t == 0) ? kF16N2 * n1 + cb : nb] : (R)0;
      }
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int n1 = h0 + q;
      HPair<R> ha, hb;
      int na, nb;
      if (t != 0) {   // x = 4096 n1 + t pairs with 4096 (15 - n1) + 4096 - t
        ha = hunpack(fa[n1], fb[15 - n1]);
        hb.ha = ha.ma;
        hb.hb = ha.mb;
        na = kF16N2 * n1 + ca;
        nb = kF16N2 * (15 - n1) + cb;
      } else {        // column 0: partner row (16 - n1) mod 16; column 2048: partner row 15 - n1
        ha = hunpack(fa[n1], fa[(16 - n1) & 15]);
        const HPair<R> h2 = hunpack(fb[n1], fb[15 - n1]);
        hb.ha = h2.ha;
        hb.hb = h2.hb;
        na = kF16N2 * n1;
        nb = kF16N2 * n1 + cb;
      }
      upd(oa[q][0], ha.ha, phi1, pb1, na);
      upd(ob[q][0], hb.ha, phi1, pb1, nb);
      if (has2) {
        upd(oa[q][1], ha.hb, phi1 + nx, pb1 + nx, na);
        upd(ob[q][1], hb.hb, phi1 + nx, pb1 + nx, nb);
      }
    }
  }
  block_reduce_store<3>(s, p.partials, row);
}

}  // namespace pdhg

namespace pdhg {

// ---- fused 1-D residual (C1, rho_alp_iters = 1, periodic x) ----
// The dual step of row j (update_fns_in_pdhg.py:99-113, 150-165; k_dual_1d's arithmetic) also forms the NEXT primal's
// continuity residual (update_fns_in_pdhg.py:72-81) from the rho', alp' it has just computed, so stage A of the
// 16 x 4096 transform reads one residual row per row instead of rho rows j .. j+2 and both alp rows (round 5: stage A
// fetched 1.5x its inputs; fp64 C1 0.97 GB per iteration).  A thread owns one x and marches over a chunk of time
// rows (phi_bar row j+1 kept as the next step's row j); the x +- 1 values of the new rho' and fluxes
// m1 = (rho'+1e-4) f+(alp1'), m2 = (rho'+1e-4) f-(alp2') come from the adjacent lanes (DPP), R_{j-1} is completed one
// step later with rho'_j.  What a wave cannot form -- its edge x's neighbour terms -- the neighbouring waves write
// to p.ex ([2][T][nx/64]: the left term eps rho'(x0-1)/dx^2 + m1(x0-1)/dx, the right term eps rho'(x1+1)/dx^2 -
// m2(x1+1)/dx), and a chunk's last row leaves its time difference to stage A (rho rows j, j+1 of the state), which
// adds both.  grid (nx/256, nchunk); block 256; partial rows blockIdx.y * gridDim.x + blockIdx.x.
template <typename R, int EGNO>
__global__ void __launch_bounds__(256) k_dual_1d_fr(KP<R> p, int jchunk) {
  if (p.ctrl->done || p.ctrl->inner_done) return;
  const int cur = p.ctrl->cur;   // in place (rho_alp_iters = 1)
  const int nx = p.nx, T = p.T;
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & (kWave - 1);
  const int w = x >> 6, nw = nx >> 6;
  const int j0 = blockIdx.y * jchunk, j1 = min(T, j0 + jchunk);
  constexpr int NS = 9;
  double s[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) s[i] = 0.0;
  if (j0 < j1) {
    const int xw = x - lane;   // the wave's first x; its neighbours outside the wave (periodic)
    const int el = (xw - 1 + nx) % nx, er = (xw + kWave) % nx;
    const R a = p.ax[x];
    R* rho = p.rho[cur];
    R* a1 = p.alp[cur][0];
    R* a2 = p.alp[cur][1];
    R* exl = p.ex;
    R* exr = p.ex + (size_t)T * nw;
    const int wl = (w - 1 + nw) % nw, wr = (w + 1) % nw;
    struct In {
      R pc, pl, pr, rho, b1, b2;
    };
    auto load = [&](int j) {
      In in;
      const R* f1 = p.phibar + (size_t)(j + 1) * nx;
      in.pc = f1[x];
      in.pl = f1[el];
      in.pr = f1[er];
      const size_t o = (size_t)j * nx + x;
      in.rho = rho[o];
      in.b1 = a1[o];
      in.b2 = a2[o];
      return in;
    };
    R f0 = p.phibar[(size_t)j0 * nx + x];   // phi_bar row j
    In nxt = load(j0);
    R rprev = (R)0, epsp = (R)0, divp = (R)0;   // rho'_{j-1} and row j-1's spatial terms
    const bool use_eps = p.epsl != (R)0;
#pragma unroll 1
    for (int j = j0; j < j1; ++j) {
      const In in = nxt;
      nxt = load(min(j + 1, j1 - 1));
      const R pc = in.pc;
      const R pxm = lane_from_prev(pc, in.pl), pxp = lane_from_next(pc, in.pr);
      const R DxR = (pxp - pc) * p.inv_dx;
      const R DxL = (pc - pxm) * p.inv_dx;
      const R r0 = in.rho;
      const R pinv = (r0 + (R)1e-4) / p.sigma;
      const R q = prox_recip<R, EGNO>(r0, p.sigma, pinv);
      const R an0 = alp_prox<R, EGNO>(in.b1, DxR, a, pinv, q, true);
      const R an1 = alp_prox<R, EGNO>(in.b2, DxL, a, pinv, q, false);
      const R f1v = fpos<R>(fval<R, EGNO>(an0, a));
      const R f2v = fneg<R>(fval<R, EGNO>(an1, a));
      const R L = lag<R, EGNO>(an0 * an0) + lag<R, EGNO>(an1 * an1);
      R vec = (pc - f0) * p.inv_dt;
      if (use_eps) vec = vec - p.epsl * ((pxp + pxm - (R)2 * pc) * p.inv_dx2);
      vec = vec - (DxR * f1v + DxL * f2v);
      vec = vec - L;
      const R rn = nmax<R>(r0 + p.sigma * vec, (R)0);
      const size_t o = (size_t)j * nx + x;
      rho[o] = rn;
      a1[o] = an0;
      a2[o] = an1;
      const double dr = (double)rn - (double)r0;
      s[0] += dr * dr;
      s[1] += (double)rn * (double)rn;
      s[2] += (double)r0 * (double)r0;
      const double d0 = (double)an0 - (double)in.b1, d1 = (double)an1 - (double)in.b2;
      s[3] += d0 * d0;
      s[4] += (double)an0 * (double)an0;
      s[5] += (double)in.b1 * (double)in.b1;
      s[6] += d1 * d1;
      s[7] += (double)an1 * (double)an1;
      s[8] += (double)in.b2 * (double)in.b2;
      // row j's residual terms (cont_residual_1d order: (time difference + eps Dxx rho') - div m)
      const R m1 = (rn + (R)1e-4) * fpos<R>(fval<R, EGNO>(an0, a));
      const R m2 = (rn + (R)1e-4) * fneg<R>(fval<R, EGNO>(an1, a));
      const R rm = lane_from_prev(rn, (R)0), rp = lane_from_next(rn, (R)0);
      const R m1m = lane_from_prev(m1, (R)0), m2p = lane_from_next(m2, (R)0);
      const R epsj = use_eps ? p.epsl * ((rp + rm - (R)2 * rn) * p.inv_dx2) : (R)0;
      const R divj = (m1 - m1m) * p.inv_dx + (m2p - m2) * p.inv_dx;
      if (lane == 0) exr[(size_t)j * nw + wl] = (use_eps ? p.epsl * (rn * p.inv_dx2) : (R)0) - m2 * p.inv_dx;
      if (lane == kWave - 1) exl[(size_t)j * nw + wr] = (use_eps ? p.epsl * (rn * p.inv_dx2) : (R)0) + m1 * p.inv_dx;
      if (j > j0) p.res[(size_t)(j - 1) * nx + x] = ((rn - rprev) * p.inv_dt + epsp) - divp;
      rprev = rn;
      epsp = epsj;
      divp = divj;
      f0 = pc;
    }
    // the chunk's last row: at the window's end rho_T = 0 and + c/dt (update_fns_in_pdhg.py:78-80); inside the window
    // rho'_{j1} belongs to the next chunk -- stage A adds the time difference
    const R last = (j1 == T) ? (((R)0 - rprev) * p.inv_dt + epsp) - divp + p.c_over_dt : epsp - divp;
    p.res[(size_t)(j1 - 1) * nx + x] = last;
  }
  block_reduce_store<NS>(s, p.partials, blockIdx.y * gridDim.x + blockIdx.x);
}

// Stage A (forward) of the fused 1-D residual: the residual rows j, j+1 as k_dual_1d_fr left them plus its wave-edge
// terms (p.ex) and, on a chunk's last row, the time difference (rho_{j+1} - rho_j)/dt from the state; then the same
// 16-point DFT over n1, twiddles and Y layout as k_f16a_fwd_1d.  grid (4096/256, pairs); block 256.
template <typename R = float>
__global__ void __launch_bounds__(256) k_f16a_fwd_fused_1d(KP<R> p, const cplx<R>* __restrict__ twN, cplx<R>* __restrict__ Y,
                                                        int jchunk) {
  using C = cplx<R>;
  if (p.ctrl->done) return;
  const int nx = p.nx, T = p.T;
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int lane = c & (kWave - 1);
  const int pair = blockIdx.y, j = 2 * pair;
  const bool has2 = (j + 1) < T;
  const int jb = has2 ? j + 1 : j;
  const int nw = nx >> 6;
  const R* R0 = p.res + (size_t)j * nx;
  const R* R1 = p.res + (size_t)jb * nx;
  const R* rho = p.rho[p.ctrl->cur];
  const R* exl = p.ex;
  const R* exr = p.ex + (size_t)T * nw;
  const bool fx0 = (j + 1) % jchunk == 0 && j + 1 < T;          // chunk boundaries (uniform)
  const bool fx1 = has2 && (j + 2) % jchunk == 0 && j + 2 < T;
  C v[16];
#pragma unroll
  for (int n1 = 0; n1 < 16; ++n1) {
    const int x = kF16N2 * n1 + c;
    R r0 = R0[x];
    R r1 = has2 ? R1[x] : (R)0;
    if (lane == 0) {
      r0 += exl[(size_t)j * nw + (x >> 6)];
      if (has2) r1 += exl[(size_t)jb * nw + (x >> 6)];
    } else if (lane == kWave - 1) {
      r0 += exr[(size_t)j * nw + (x >> 6)];
      if (has2) r1 += exr[(size_t)jb * nw + (x >> 6)];
    }
    if (fx0) r0 += (rho[(size_t)(j + 1) * nx + x] - rho[(size_t)j * nx + x]) * p.inv_dt;
    if (fx1) r1 += (rho[(size_t)(j + 2) * nx + x] - rho[(size_t)(j + 1) * nx + x]) * p.inv_dt;
    v[n1] = cmk<C>(r0, r1);
  }
  dft_any<C, 16>(v);
  C wv[16];
  twiddles_from3<C, 16>(wv, twN, c);   // W_65536^{c k1}
  C* Yp = Y + (size_t)pair * nx + c;
  Yp[0] = v[0];
#pragma unroll
  for (int k1 = 1; k1 < 16; ++k1) Yp[(size_t)k1 * kF16N2] = cmul(v[k1], wv[k1]);
}

}  // namespace pdhg
