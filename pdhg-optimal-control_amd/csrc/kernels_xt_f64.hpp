// fp64 x-transform + Thomas in t at nx = 4096 (k_precond_xt_f64_2d) and its row-access helpers.
#pragma once
#include "kernels_2d_fast.hpp"

namespace pdhg {

// Rows of a column block through buffer loads / stores: one descriptor per row (wave-uniform base) and the
// per-item offset i * NTT * 16 B as the scalar offset, so the 3 x IT row accesses per step need one VGPR of
// address instead of a 64-bit address per item (64-bit per-item addresses cost the registers that made the round-3 form of this kernel spill).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const double* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(base), 0, bytes, 0x00020000);
}
__device__ __forceinline__ double2 buf_ld2(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
__device__ __forceinline__ void buf_st2(__amdgpu_buffer_rsrc_t r, int voff, int soff, double2 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), r, voff, soff, 0);
}

__device__ __forceinline__ double eth_of(double dd) {   // e^-th, cosh th = 1 + dd/2 (no cancellation)
  return 1.0 / (1.0 + 0.5 * dd + sqrt(dd * (1.0 + 0.25 * dd)));
}
__device__ __forceinline__ double theta_of(double dd) {
  const double dl = 0.5 * dd;
  return fmax(log1p(dl + sqrt(dl * (dl + 2.0))), 1e-300);
}


// fp64 x-transform + Thomas in t for power-of-two nx = N = 4096 (the reference's own precision at C3's grid:
// jaxsrc runs float64 / complex128 throughout, solver.py:11, update_fns_in_pdhg.py:10).
//
// Same preconditioner as the fp32 kernels (H1_precond_2d, utils_precond.py:142-178: DHT_x of the spectral
// rows, the tridiagonal solve in t per mode, inverse DHT_x) and the same Thomas algebra as
// k_precond_xt_fast_2d (cancellation-free pivot recurrence forward, closed-form pivots backward), in double.
// The generic runtime-radix kernel keeps two FFT buffers and three per-mode carry arrays in LDS (5 M reals:
// 320 KiB for a 4096-point column pair in fp64), so it stops at nx = 2048 in fp64.  Here the block's one
// complex line (B = 2 real columns packed as z = a + i b) is transformed in place in a padded LDS line
// (68 KiB + 13 KiB of twiddle seeds); a thread owns IT = N/NT items (kx), each carrying the two modes
// (kx, 2b) and (kx, 2b + 1): the pivot state (two double2) and the prefetched next row stay in registers,
// b' / x in a 64 KiB LDS array (145 KiB in all, one workgroup per CU).
// Converged pivots: the forward pivots are g_k = e^-th E_{k+1}/E_{k+2}, E_m = expm1(-2 th m) (cosh th = 1 +
// dd/2), and |g_k / e^-th - 1| < e^{-2 th (k+1)}; once 2 th (k+1) > 40 for every lane of a wave the ratio is
// 1 to within 4e-18 (below half an fp64 ulp), and the item switches to the constant g = e^-th: no division in
// the forward sweep, no transcendental in the backward one.  The test is wave-uniform per item, so only the
// low-frequency modes (small th: kx near 0 or N in the first / last wave, the first column blocks) keep the
// recurrence / closed form for many rows; every other wave drops them after a few rows.  (Round 3's form of this
// kernel computed two expm1, one exp and two divisions per mode and row in the backward sweep and spilled 51
// VGPRs: 38 ms per launch at C3.)  Row accesses are buffer loads / stores (one descriptor per row, the item
// offset as the scalar offset): one VGPR of address for all IT items.
// HR ("half real", nx = 2N = 8192, C4's x extent; B = 1): a block is ONE real column of 2N points packed as
// z[m] = x[2m] + i x[2m+1] into the N-point FFT and split with realsplit_padded (the fp32 warp-specialised kernel's
// HR form); item k carries the modes kx = k and k + N, and the inverse stages x of both modes at their real positions
// and splits again.  The split twiddles W_{2N}^k come from two 64-entry LDS tables (W^(k mod 64) W^(64 (k/64))).
// t-slab phases (p.slab, xt_phase 1 / 2) as in the fp32 kernels: global-row pivots, zero-carry forward sweep
// storing every row, backward sweep from the right carry (carry_y) -- oracle/slab_oracle.py.
// grid: nb column blocks; block NT; LDS (N + N/16 + TwLds<N> + N (+ 128 HR)) * 16 B.
// BPR: b' / x of the thread's items in registers instead of the LDS array (nx <= 2048: IT <= 4 items leave the
// registers for it, and the smaller LDS footprint admits a second workgroup per CU).
// TC: the forward sweep reads the residual spectrum in task order (p.rspec: per 4-row task, 8 reals per column block
// b = rows x0..x0+3 at columns 2b, 2b+1): item x = tid + i NT sits at 16 B x (x & 3) of its task's 64-B piece, so
// the 4 lanes of a task read one contiguous 64-B piece (16 pieces per wave load instead of 1 KiB runs); b' and x go
// to `work` (blocked) as always.
template <int N, int NT, bool HR = false, bool BPR = false, bool TC = false>
__global__ void __launch_bounds__(NT) k_precond_xt_f64_2d(KP<double> p, const double2* __restrict__ twx) {
  using C = double2;
  constexpr int IT = N / NT;
  constexpr int LINE = Pad<N>::LINE;
  constexpr int M = 2 * N;   // reals per block row: B = 2 columns of N, or (HR) one column of 2N
  static_assert(N % NT == 0 && N <= 4096 && IT <= 32, "one padded complex line and its twiddle seeds in LDS");
  if (p.ctrl->done) return;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  C* A = reinterpret_cast<C*>(smem_raw);
  C* twl = A + LINE;
  C* bp = twl + TwLds<N>::SIZE;   // b' / x per item (BPR: unused, none allocated)
  C* rsw = bp + (BPR ? 0 : N);    // HR: W_{2N}^j and W_{2N}^{64 j}, j < 64
  static_assert(!(BPR && HR), "half-real blocks keep b' in LDS");
  static_assert(!TC || (!HR && !BPR && NT % 4 == 0), "task-order input: column pairs, 4-row tasks");
  fill_twlds<C, N>(twl, twx, HR ? 2 : 1);   // HR: twx holds W_{2N}
  if constexpr (HR) {
    static_assert(N == 4096, "split-twiddle tables sized for 2N = 8192");
    for (int i = threadIdx.x; i < 128; i += blockDim.x) rsw[i] = twx[i < 64 ? i : 64 * (i - 64)];
  }
  const int T = p.T, tid = threadIdx.x;
  // t-slab carry exchange: blocks [b0, b0 + gridDim.x).  TC: XCD-aware order, the gridDim/8 workgroups of one XCD
  // take consecutive column blocks, so the two blocks sharing each 128-B line of the task-order input (64 B each)
  // read it through one L2 (round robin put them on different XCDs: every line fetched twice)
  const int b = ((TC && !(p.dbg & 4096)) ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x) + p.b0;
  double* wb = p.work + (size_t)b * M;
  const size_t kstride = (size_t)p.nb * M;
  const double inv_ae = 1.0 / (double)p.ae;
  const double ly0 = p.lamy[HR ? b : 2 * b], ly1 = p.lamy[HR ? b : 2 * b + 1];
  auto kx_of = [&](int i) { return tid + i * NT; };
  auto dd_of = [&](int i) {
    const double lx0 = p.lamx[kx_of(i)], lx1 = HR ? (double)p.lamx[kx_of(i) + N] : lx0;
    return make_double2(((double)p.C - lx0 - ly0) * inv_ae, ((double)p.C - lx1 - ly1) * inv_ae);
  };
  // the two modes of item i from a transformed line: Hartley pair of the two packed columns, or (HR) the real
  // split of the one column (modes k and k + N)
  auto unpack2 = [&](int i, double& h0, double& h1) {
    if constexpr (HR) {
      const int k = kx_of(i);
      realsplit_padded<C, double>(A, N, k, cmul(rsw[k & 63], rsw[64 + (k >> 6)]), h0, h1);
    } else {
      hartley_padded<C, double>(A, N, kx_of(i), h0, h1);
    }
  };
  // stage item i's pair of mode values into the line (HR: real positions kx and kx + N of the packed column)
  auto stage2 = [&](int i, C x) {
    if constexpr (HR) {
      double* Af = reinterpret_cast<double*>(A);
      const int f0 = kx_of(i), f1 = kx_of(i) + N;
      Af[2 * pix(f0 >> 1) + (f0 & 1)] = x.x;
      Af[2 * pix(f1 >> 1) + (f1 & 1)] = x.y;
    } else {
      A[pix(kx_of(i))] = x;
    }
  };
  // item i of this thread at byte voff + ioff(i) of a blocked row
  const int voff = tid * (int)sizeof(C);
  auto ioff = [&](int i) { return i * NT * (int)sizeof(C); };
  auto rowr = [&](int kk) { return row_rsrc(wb + (size_t)kk * kstride, M * (int)sizeof(double)); };
  // c1: forward dd, then e^-th once converged; backward theta.  c2: forward h = 1 - g; backward E_{k+2}, or
  // e^-th once converged.
  C c1[IT], c2[IT], pf[IT];
  C bpr[BPR ? IT : 1];
  auto bp_ld = [&](int i) -> C {
    if constexpr (BPR) return bpr[i];
    else return bp[kx_of(i)];
  };
  auto bp_st = [&](int i, C v) {
    if constexpr (BPR) bpr[i] = v;
    else bp[kx_of(i)] = v;
  };
  // kf[i]: the first row from which item i uses the converged pivot: th (k+1) > 20 in every lane of the wave
  // (kf = floor(20 / min th) over the wave's two modes per lane); wave-uniform, held in SGPRs
  int kf[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const C dd = dd_of(i);
    double tm = fmin(theta_of(dd.x), theta_of(dd.y));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) tm = fmin(tm, __shfl_xor(tm, o, kWave));
    const double q = 20.0 / tm;
    kf[i] = __builtin_amdgcn_readfirstlane(q < 1e9 ? (int)q : 1000000000);
  }
  auto ldrow = [&](int kk) {
    const auto r = rowr(kk);
#pragma unroll
    for (int i = 0; i < IT; ++i) pf[i] = buf_ld2(r, voff, ioff(i));
  };
  // the forward sweep's input rows: `work` (blocked), or (TC) the task-order residual spectrum: row kk, block b,
  // item x = tid + i NT at reals (x / 4) 4 ny + 8 b + 2 (x % 4)
  const int ny_t = p.nb * 2;
  auto ldrow_in = [&](int kk) {
    if constexpr (TC) {
      const auto r = row_rsrc(p.rspec + (size_t)kk * kstride + (size_t)8 * b, (int)(kstride * sizeof(double)) - 64 * b);
      const int vin = 32 * ny_t * (tid >> 2) + 16 * (tid & 3);
#pragma unroll
      for (int i = 0; i < IT; ++i) pf[i] = buf_ld2(r, vin, 8 * ny_t * NT * i);
    } else {
      ldrow(kk);
    }
  };
  const int j0 = p.j0;
  const bool slab = p.slab != 0;
  if (p.xt_phase != 2) {
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      c1[i] = dd_of(i);
      // h_{j0-1}: 1 entering the window; a t-slab's entry pivot state in closed form (h_entry)
      c2[i] = slab ? make_double2(h_entry(c1[i].x, j0), h_entry(c1[i].y, j0)) : make_double2(1.0, 1.0);
      bp_st(i, make_double2(0.0, 0.0));   // zero carry (a t-slab's carry is folded in by k_slab_fix)
    }
    // ---------------- forward: DHT_x + elimination ----------------
    //   s = dd + h_{k-1},  g_k = 1/(1+s),  h_k = s g_k,  b'_k = (rhs/ae + b'_{k-1}) g_k
    //   last (Neumann) row of the window: x_{T-1} = (rhs/ae + b'_{T-2}) / (dd + h_{T-2})   [converged: dd + h = (1 - g)/g]
    // A t-slab indexes the pivots by the GLOBAL row j0 + k; only the window's last slab has the Neumann row, and
    // a slab stores every row (the backward sweep is a separate launch after the carry fix-up).
    ldrow_in(0);
    for (int k = 0; k < T; ++k) {
      const int kg = j0 + k;
      const bool nrow = k == T - 1 && p.last_slab;   // the window's Neumann row
#pragma unroll
      for (int i = 0; i < IT; ++i) A[pix(kx_of(i))] = pf[i];
      if (k + 1 < T) ldrow_in(k + 1);
      lds_sync();
      lds_fft_inplace_tl<C, N, 1, NT>(A, twl);
#pragma unroll
      for (int i = 0; i < IT; ++i)   // items whose pivots have converged switch to g = e^-th (dd -> e^-th) on
        if (kg == max(kf[i], j0) && !nrow)   // the first converged row of this sweep (a slab may start past kf)
          c1[i] = make_double2(eth_of(c1[i].x), eth_of(c1[i].y));
      const auto dst = rowr(k);
#pragma unroll
      for (int i = 0; i < IT; ++i) {
        double ha, hb;
        unpack2(i, ha, hb);
        const C b0 = bp_ld(i);
        const double r0 = ha * inv_ae + b0.x, r1 = hb * inv_ae + b0.y;
        C bn;
        const int kfj = max(kf[i], j0);
        const bool fast = kg > kfj || (kg == kfj && !nrow);
        if (!nrow) {
          if (fast) {
            bn = make_double2(r0 * c1[i].x, r1 * c1[i].y);
          } else {
            const double s0 = c1[i].x + c2[i].x, s1 = c1[i].y + c2[i].y;
            const double g0 = 1.0 / (1.0 + s0), g1 = 1.0 / (1.0 + s1);
            bn = make_double2(r0 * g0, r1 * g1);
            c2[i] = make_double2(s0 * g0, s1 * g1);
          }
          buf_st2(dst, voff, ioff(i), bn);
        } else {
          if (fast) bn = make_double2(r0 * c1[i].x / (1.0 - c1[i].x), r1 * c1[i].y / (1.0 - c1[i].y));
          else bn = make_double2(r0 / (c1[i].x + c2[i].x), r1 / (c1[i].y + c2[i].y));
          if (slab) buf_st2(dst, voff, ioff(i), bn);   // re-read after the carry fix-up
        }
        bp_st(i, bn);
      }
      lds_sync();
    }
  }
  if (p.xt_phase == 1) return;   // forward sweep only (t-slab: the carry fix-up runs in between)
  // ---------------- backward: substitution + inverse DHT_x ----------------
  //   x_k = b'_k + g_k x_{k+1},  g_k = e^-th E_{k+1}/E_{k+2},  E_m = expm1(-2 th m),  cosh th = 1 + dd/2
  //   (th -> 0: g_k -> (k+1)/(k+2)); converged: g = e^-th
  // single context: from x_{T-1} (the forward's Neumann row, held in bp); t-slab: from the right carry x_{j0+T}
  // (carry_y, written by k_slab_fix), substituting every local row from the fixed-up b' rows in work
  const int ks = slab ? T - 1 : T - 2;   // first substituted local row
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const C dd = dd_of(i);
    c1[i] = make_double2(theta_of(dd.x), theta_of(dd.y));
    if (j0 + ks >= kf[i]) {   // row ks converged
      c2[i] = make_double2(exp(-c1[i].x), exp(-c1[i].y));
    } else {                  // E_{k+2} for the first substituted row, k = ks (global j0 + ks)
      c2[i] = make_double2(expm1(-2.0 * c1[i].x * (j0 + ks + 2)), expm1(-2.0 * c1[i].y * (j0 + ks + 2)));
    }
    if (slab) bp_st(i, p.carry_y ? reinterpret_cast<const C*>(p.carry_y + (size_t)b * M)[kx_of(i)]
                                 : make_double2(0.0, 0.0));
  }
  if (ks >= 0) ldrow(ks);
  for (int k = T - 1; k >= 0; --k) {
    const int kg = j0 + k;
#pragma unroll
    for (int i = 0; i < IT; ++i)   // items leaving the converged regime: E_{k+2} from theta
      if (kg + 1 == kf[i] && k < ks)
        c2[i] = make_double2(expm1(-2.0 * c1[i].x * (kg + 2)), expm1(-2.0 * c1[i].y * (kg + 2)));
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      C x = bp_ld(i);
      if (k <= ks) {
        double g0, g1;
        if (kg >= kf[i]) {
          g0 = c2[i].x;
          g1 = c2[i].y;
        } else {
          const double t0 = c1[i].x, t1 = c1[i].y;
          const double e0 = expm1(-2.0 * t0 * (kg + 1)), e1 = expm1(-2.0 * t1 * (kg + 1));
          g0 = t0 > 1e-150 ? exp(-t0) * e0 / c2[i].x : (double)(kg + 1) / (double)(kg + 2);
          g1 = t1 > 1e-150 ? exp(-t1) * e1 / c2[i].y : (double)(kg + 1) / (double)(kg + 2);
          c2[i] = make_double2(e0, e1);
        }
        x = make_double2(pf[i].x + g0 * x.x, pf[i].y + g1 * x.y);
        bp_st(i, x);
      }
      stage2(i, x);
    }
    if (k <= ks && k >= 1) ldrow(k - 1);
    lds_sync();
    lds_fft_inplace_tl<C, N, 1, NT>(A, twl);
    const auto wk = rowr(k);
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      double ha, hb;
      unpack2(i, ha, hb);
      if constexpr (HR) {   // spatial x = k and k + N of the real column
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, ha), wk, tid * 8, i * NT * 8, 0);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, hb), wk, tid * 8, (i * NT + N) * 8, 0);
      } else {
        buf_st2(wk, voff, ioff(i), make_double2(ha, hb));
      }
    }
    lds_sync();
  }
}

}  // namespace pdhg
