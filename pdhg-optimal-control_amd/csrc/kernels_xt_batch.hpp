// x-transform + Thomas in t, row-batched (fp32, nx = N a power of two, N*NL = 4096 items per block).
//
// Same arithmetic as k_precond_xt_ws_2d / k_precond_xt_fast_2d (H1_precond_2d, utils_precond.py:142-178:
// DHT_x of the column block, Thomas elimination over t per mode, back substitution, inverse DHT_x), with a
// different schedule: RB = 4 time rows are transformed together.  The DHT along x of a row does not depend on
// the t recurrence, only the Thomas step does, so one workgroup of 1024 threads (16 waves, 4 per SIMD) runs
// the three radix-16 passes on the 4*NL lines of a batch at once (one butterfly per thread per pass) and then
// the Thomas steps of the 4 rows back to back from registers.  Against the one-row warp-specialised kernel
// (8 waves, 6 barriers per row, one row of loads in flight) this gives twice the waves per SIMD to hide LDS
// and VALU latency, 7 barriers per 4 rows, and 2-4 rows (64-128 KiB) of loads in flight per CU.
// Thomas state per item (two modes, the real and imaginary parts of line element kx): forward dd = 2 delta,
// h = 1 - g, b'; backward theta, E, x.  Each thread owns IT = 4 items for the whole sweep.
// LDS: 4*NL padded lines (139 KiB) + twiddle seeds (6.4 KiB): one workgroup per CU.  grid: nb; block 1024.
// Supports the t-slab phases like the warp-specialised kernel (xt_phase, j0, last_slab, carry_y).
#pragma once
#include "kernels_2d_fast.hpp"

namespace pdhg {

// One in-place radix-R pass of the padded line-major schedule (as inplace_pass with REG twiddle seeds), with
// each twiddle applied as soon as it is formed: the seeds W^k, W^4k, W^8k and at most W^1..W^7 are live at
// once instead of all fifteen products, which keeps the batched kernel within 128 VGPRs.
// t: the thread index (a caller in a loop passes a laundered copy so the pass's LDS addresses are not
// hoisted out of the loop as loop-invariant registers)
template <typename C, int N, int NLT, int NT, int LS, int R>
__device__ __forceinline__ void batch_pass(C* __restrict__ a, const C* twl, int t = threadIdx.x) {
  constexpr int nR = N / R;
  constexpr int total = nR * NLT;
  constexpr int PER = (total + NT - 1) / NT;
  constexpr int LINE = Pad<N>::LINE;
  static_assert(nR % 16 == 0 && (LS == 1 || LS % 16 == 0) && (LS > 1 || R == 16), "padded schedule");
  C v[PER][R];
  int base[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int idx = t + q * NT;
    base[q] = -1;
    if (total % NT == 0 || idx < total) {
      const int l = idx / nR;
      const int j = idx - l * nR;
      const int k = j & (LS - 1);
      const C* s = a + l * LINE + pix(j);
#pragma unroll
      for (int r = 0; r < R; ++r) v[q][r] = s[r * (nR + nR / 16)];
      if (LS > 1 && k != 0) {
        const C* t3 = twl + twlds_off(LS) + 3 * k;
        const C w1 = t3[0];
        v[q][1] = cmul(v[q][1], w1);
        if constexpr (R > 2) {
          const C w2 = cmul(w1, w1);
          const C w3 = cmul(w2, w1);
          v[q][2] = cmul(v[q][2], w2);
          v[q][3] = cmul(v[q][3], w3);
          if constexpr (R > 4) {
            const C w4 = t3[1];
            const C w5 = cmul(w4, w1), w6 = cmul(w4, w2), w7 = cmul(w4, w3);
            v[q][4] = cmul(v[q][4], w4);
            v[q][5] = cmul(v[q][5], w5);
            v[q][6] = cmul(v[q][6], w6);
            v[q][7] = cmul(v[q][7], w7);
            if constexpr (R > 8) {
              const C w8 = t3[2];
              v[q][8] = cmul(v[q][8], w8);
              v[q][9] = cmul(v[q][9], cmul(w8, w1));
              v[q][10] = cmul(v[q][10], cmul(w8, w2));
              v[q][11] = cmul(v[q][11], cmul(w8, w3));
              v[q][12] = cmul(v[q][12], cmul(w8, w4));
              v[q][13] = cmul(v[q][13], cmul(w8, w5));
              v[q][14] = cmul(v[q][14], cmul(w8, w6));
              v[q][15] = cmul(v[q][15], cmul(w8, w7));
            }
          }
        }
      }
      base[q] = l * LINE + pix((j - k) * R + k);
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

template <typename C, int N, int NLT, int NT, int LS>
__device__ __forceinline__ void batch_fft(C* a, const C* twl, int t = threadIdx.x) {
  if constexpr (LS < N) {
    constexpr int rem = N / LS;
    constexpr int R = (rem >= 16) ? 16 : rem;
    batch_pass<C, N, NLT, NT, LS, R>(a, twl, t);
    batch_fft<C, N, NLT, NT, LS * R>(a, twl, t);
  }
}

// NT = 512, RB = 2: half the LDS (76 KiB) and threads, so two workgroups share a CU and one's transform
// overlaps the other's row traffic; each thread then owns IT = 8 items.
template <int N, int NL, int RB = 4, int RPRE = 0, int NT = 1024>
__global__ void __launch_bounds__(NT, NT == 1024 ? 1 : 4) k_precond_xt_batch_2d(KP<float> p,
                                                                                const float2* __restrict__ twx) {
  using C = float2;
  constexpr int NI = N * NL;             // items per block
  constexpr int IT = NI / NT;            // items per thread
  constexpr int B = 2 * NL;
  constexpr int LINE = Pad<N>::LINE;
  constexpr int lnl = (NL == 1) ? 0 : (NL == 2) ? 1 : (NL == 4) ? 2 : 3;
  static_assert(NI == 4096 && (IT == 4 || IT == 8), "sized for 4096 items per block");
  if (p.ctrl->done) return;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  C* A = reinterpret_cast<C*>(smem_raw);          // RB*NL lines: row r, line l at (r*NL + l) * LINE
  C* twl = A + RB * NL * LINE;
  fill_twlds<C, N>(twl, twx);
  const int T = p.T, tid = threadIdx.x;
  const int b = blockIdx.x + p.b0;
  constexpr int M = N * B;
  float* wb = p.work + (size_t)b * M;
  const size_t kstride = (size_t)p.nb * M;
  const float inv_ae = 1.f / p.ae;
  // the thread index is laundered once per batch (tl), so the unrolled loops' LDS / global addresses are
  // recomputed there instead of being hoisted out of the row loops into registers (which spills)
  int tl = tid;
  auto launder = [&]() {
    tl = tid;
    asm volatile("" : "+v"(tl));
  };
  // items in pairs: item i of this thread is 2 (tl + (i/2) NT) + i%2, so every global access moves two
  // neighbouring items as one 16-B float4 (dwordx4)
  auto item_of = [&](int i) { return 2 * (tl + (i >> 1) * NT) + (i & 1); };
  auto kx_of = [&](int i) { return item_of(i) >> lnl; };
  auto ln_of = [&](int i) { return item_of(i) & (NL - 1); };
  auto ld_pair = [&](const C* src, int j, C& a, C& b2) {
    const float4 v = reinterpret_cast<const float4*>(src)[tl + j * NT];
    a = make_float2(v.x, v.y);
    b2 = make_float2(v.z, v.w);
  };
  auto st_pair = [&](C* dst, int j, C a, C b2) {
    reinterpret_cast<float4*>(dst)[tl + j * NT] = make_float4(a.x, a.y, b2.x, b2.y);
  };
  auto row_ptr = [&](int k) { return reinterpret_cast<C*>(wb + (size_t)k * kstride); };
  C c1[IT], c2[IT], c3[IT];     // dd | theta,  h | E,  b' | x
  // rows of the next batch: the first RPRE rows are loaded before the transform, the others after it
  // (only RPRE rows of loads are live across the FFT's registers: 80 + 24 + 8 RPRE VGPRs; RPRE = 0 spills
  // nothing, each row more costs ~15 spilled VGPRs)
  C pf[RB][IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int l = ln_of(i);
    const float lx = p.lamx[kx_of(i)];
    c1[i] = make_float2((p.C - lx - p.lamy[b * B + 2 * l]) * inv_ae, (p.C - lx - p.lamy[b * B + 2 * l + 1]) * inv_ae);
  }
  auto load_rows = [&](int k_first, int dir, auto half) {   // rows k_first + dir*r of one part, clamped into [0, T)
    constexpr int H = decltype(half)::value;
#pragma unroll
    for (int r = H ? RPRE : 0; r < (H ? RB : RPRE); ++r) {
      const C* src = row_ptr(min(max(k_first + dir * r, 0), T - 1));
#pragma unroll
      for (int j = 0; j < IT / 2; ++j) ld_pair(src, j, pf[r][2 * j], pf[r][2 * j + 1]);
    }
  };
  auto stage = [&](int r, int i, C v) { A[(r * NL + ln_of(i)) * LINE + pix(kx_of(i))] = v; };

  if (p.xt_phase != 2) {
    // ---------------- forward: DHT_x of 4 rows, then their elimination steps ----------------
    // s = dd + h_{k-1},  g_k = 1/(1+s),  h_k = s g_k,  b'_k = (rhs/ae + b'_{k-1}) g_k;
    // last (Neumann) row of the window: u_{T-1} = ae (dd + h_{T-2})
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      c2[i] = make_float2(h_entry(c1[i].x, p.j0), h_entry(c1[i].y, p.j0));
      c3[i] = make_float2(0.f, 0.f);
    }
    load_rows(0, 1, std::integral_constant<int, 0>{});
    load_rows(0, 1, std::integral_constant<int, 1>{});
    for (int k0 = 0; k0 < T; k0 += RB) {
      launder();
#pragma unroll
      for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int i = 0; i < IT; ++i) stage(r, i, pf[r][i]);
      // unconditional (clamped rows after the last batch): a conditional load would keep the old pf live
      // across the transform on the not-taken path
      load_rows(k0 + RB, 1, std::integral_constant<int, 0>{});
      lds_sync();
      __builtin_amdgcn_sched_barrier(0);   // the second half's loads stay below the transform
      if (!(p.dbg & 1)) batch_fft<C, N, RB * NL, NT, 1>(A, twl);
      __builtin_amdgcn_sched_barrier(0);
      launder();
      load_rows(k0 + RB, 1, std::integral_constant<int, 1>{});
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const int k = k0 + r;
        if (k >= T) break;
        C* dst = row_ptr(k);
        if (k < T - 1 || !p.last_slab) {
#pragma unroll
          for (int i = 0; i < IT; ++i) {
            float ha, hb;
            hartley_padded<C, float>(A + (r * NL + ln_of(i)) * LINE, N, kx_of(i), ha, hb);
            const float s0 = c1[i].x + c2[i].x, s1 = c1[i].y + c2[i].y;
            const float g0 = rcp_fast(1.f + s0), g1 = rcp_fast(1.f + s1);
            c3[i] = make_float2((ha * inv_ae + c3[i].x) * g0, (hb * inv_ae + c3[i].y) * g1);
            c2[i] = make_float2(s0 * g0, s1 * g1);
          }
#pragma unroll
          for (int j = 0; j < IT / 2; ++j) st_pair(dst, j, c3[2 * j], c3[2 * j + 1]);
        } else {
#pragma unroll
          for (int i = 0; i < IT; ++i) {
            float ha, hb;
            hartley_padded<C, float>(A + (r * NL + ln_of(i)) * LINE, N, kx_of(i), ha, hb);
            c3[i] = make_float2((ha * inv_ae + c3[i].x) / (c1[i].x + c2[i].x),
                                (hb * inv_ae + c3[i].y) / (c1[i].y + c2[i].y));
          }
          if (p.slab) {   // re-read (after the carry fix-up) by the backward sweep
#pragma unroll
            for (int j = 0; j < IT / 2; ++j) st_pair(dst, j, c3[2 * j], c3[2 * j + 1]);
          }
        }
        // keep the next row's LDS reads below this row's step (hoisting them all needs 64 more VGPRs)
        __builtin_amdgcn_sched_barrier(0);
      }
      lds_sync();
    }
  }
  if (p.xt_phase == 1) return;   // forward sweep only (t-slab: the carry fix-up runs in between)

  // ---------------- backward: 4 substitution steps, then the inverse DHT_x of those rows ----------------
  // x_k = b'_k + g_k x_{k+1},  g_k = e^-th E_{k+1}/E_{k+2},  E_m = expm1(-2 th m),  cosh th = 1 + dd/2
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const float dl0 = 0.5f * c1[i].x, dl1 = 0.5f * c1[i].y;
    c1[i] = make_float2(fmaxf(log1pf(dl0 + sqrtf(dl0 * (dl0 + 2.f))), 1e-20f),
                        fmaxf(log1pf(dl1 + sqrtf(dl1 * (dl1 + 2.f))), 1e-20f));
    // E_{k+2} for the first substituted row: k = T-2 (single context) or T-1 (slab, from the right carry)
    const float e0 = (float)(p.j0 + T + (p.slab ? 1 : 0));
    c2[i] = make_float2(expm1f(-2.f * c1[i].x * e0), expm1f(-2.f * c1[i].y * e0));
    if (p.slab)
      c3[i] = p.carry_y ? reinterpret_cast<const C*>(p.carry_y + (size_t)b * M)[item_of(i)] : make_float2(0.f, 0.f);
  }
  // b' of rows T-1, T-2, ... (single context: row T-1's x is c3 already)
  load_rows(T - 1, -1, std::integral_constant<int, 0>{});
  load_rows(T - 1, -1, std::integral_constant<int, 1>{});
  for (int kt = T - 1; kt >= 0; kt -= RB) {
    launder();
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int k = kt - r;
      if (k < 0) break;
      if ((k < T - 1 || p.slab) && !(p.dbg & 4)) {
        const float kk1 = (float)(p.j0 + k + 1);   // global row index + 1
#pragma unroll
        for (int i = 0; i < IT; ++i) {
          // theta >= 1e-20 (clamped above): the closed form tends to (k+1)/(k+2) as theta -> 0
          const float2 E1 = expm1_neg2(-2.f * c1[i].x * kk1, -2.f * c1[i].y * kk1);
          const float g0 = __expf(-c1[i].x) * E1.x * rcp_fast(c2[i].x);
          const float g1 = __expf(-c1[i].y) * E1.y * rcp_fast(c2[i].y);
          c3[i] = make_float2(pf[r][i].x + g0 * c3[i].x, pf[r][i].y + g1 * c3[i].y);
          c2[i] = E1;
        }
      }
#pragma unroll
      for (int i = 0; i < IT; ++i) stage(r, i, c3[i]);
      __builtin_amdgcn_sched_barrier(0);
    }
    load_rows(kt - RB, -1, std::integral_constant<int, 0>{});
    lds_sync();
    __builtin_amdgcn_sched_barrier(0);
    if (!(p.dbg & 2)) batch_fft<C, N, RB * NL, NT, 1>(A, twl);
    __builtin_amdgcn_sched_barrier(0);
    launder();
    load_rows(kt - RB, -1, std::integral_constant<int, 1>{});
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int k = kt - r;
      if (k < 0) break;
      C* wk = row_ptr(k);
      C o[IT];
#pragma unroll
      for (int i = 0; i < IT; ++i) {
        float ha, hb;
        hartley_padded<C, float>(A + (r * NL + ln_of(i)) * LINE, N, kx_of(i), ha, hb);
        o[i] = make_float2(ha, hb);
      }
#pragma unroll
      for (int j = 0; j < IT / 2; ++j) st_pair(wk, j, o[2 * j], o[2 * j + 1]);
      __builtin_amdgcn_sched_barrier(0);
    }
    lds_sync();
  }
}

}  // namespace pdhg
