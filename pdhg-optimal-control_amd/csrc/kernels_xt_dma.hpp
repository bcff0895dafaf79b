// x-transform + Thomas in t with the row traffic staged by LDS DMA (fp32, nx = N = 4096, one line per block).
//
// Same arithmetic and slab semantics as k_precond_xt_batch_2d (H1_precond_2d, utils_precond.py:142-178),
// different data movement.  The batched kernel loads its next rows into registers, and only after the
// transform (registers live across the FFT spill), so HBM idles while the LDS passes run: 14.2 ms at C3 against
// a 10.3-11 ms floor with the transforms switched off.  Here the next two rows go HBM -> LDS directly
// (global_load_lds_dwordx4: no VGPR destination, 2 instructions per row per thread), issued as soon as the
// staging buffer S is free and retired by a counted vmcnt one batch later, so they stream during the
// transform and the Thomas steps of the current rows.
//   LDS (static): A = 2 padded lines (the transform, 68 KiB) + S = 2 rows lane-linear (64 KiB) + TwLds<4096>.
//   forward batch (rows k0, k0+1): [S landed] the first radix-16 pass reads S (unpadded) and writes A,
//     then S is re-issued with rows k0+2, k0+3; passes 2-3; the two elimination steps read A and store b'.
//   backward batch (rows kt, kt-1): [S landed] the substitution steps read b' from S and stage x in A; S is
//     re-issued with rows kt-2, kt-3; the transform; the inverse-transformed rows are stored.
// vmcnt is in issue order on gfx9: the wait for S leaves only the stores issued after its DMA outstanding.
// Barriers are s_barrier + lgkmcnt only (lds_sync), so the DMA spans them.
// grid: nb; block 1024 (IT = 4 items per thread, the batched kernel's pairing: 16-B global accesses).
//
// HR ("half real", nx = 2N = 8192, C4's x extent; B = 1 real column per block): the block row is ONE real column of
// 2N points, packed as z[m] = x[2m] + i x[2m+1] -- the same N float2 of a row as a column pair's, so the DMA staging
// and the first radix-16 pass are unchanged -- and split after the transform with realsplit_padded (item k carries
// the modes k and k + N, as the warp-specialised HR kernel's items); the inverse stages x of both modes at their real
// positions k and k + N and splits again into the spatial values x[k], x[k + N].  lamx of the modes k + N: the
// periodic symbol is even, lam(k + N) = lam(2N - k - N) = lam(N - k) (k >= 1; lam(N) = -4/dx^2), so LDS keeps only
// the first N of the host's values and reads mode k + N's from position N - k -- the host's value itself (forming it
// as -4/dx^2 - lam(k) cancels: 40 % off for the lowest modes).  The split twiddles W_2N^k come from two 64-entry
// tables (W^(k mod 64) W^(64 (k / 64))).
#pragma once
#include <type_traits>
#include "kernels_xt_batch.hpp"

namespace pdhg {

// Reads of the DMA-staged buffer S in inline asm (with their own lgkmcnt wait): the compiler cannot tell that
// the DMA has landed (it is retired by the counted vmcnt above) and would put a vmcnt(0) before every read of
// S it can see, which also waits for the batch's stores.
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
// v[r] = S-line element at a + r * 256 float2 (r < 16)
__device__ __forceinline__ void s_read16(unsigned a, float2 (&v)[16]) {
  typedef unsigned long long u64;
  u64 w[16];
  asm volatile(
      "ds_read_b64 %0, %16\n\tds_read_b64 %1, %16 offset:2048\n\tds_read_b64 %2, %16 offset:4096\n\t"
      "ds_read_b64 %3, %16 offset:6144\n\tds_read_b64 %4, %16 offset:8192\n\tds_read_b64 %5, %16 offset:10240\n\t"
      "ds_read_b64 %6, %16 offset:12288\n\tds_read_b64 %7, %16 offset:14336\n\tds_read_b64 %8, %16 offset:16384\n\t"
      "ds_read_b64 %9, %16 offset:18432\n\tds_read_b64 %10, %16 offset:20480\n\tds_read_b64 %11, %16 offset:22528\n\t"
      "ds_read_b64 %12, %16 offset:24576\n\tds_read_b64 %13, %16 offset:26624\n\t"
      "ds_read_b64 %14, %16 offset:28672\n\tds_read_b64 %15, %16 offset:30720\n\ts_waitcnt lgkmcnt(0)"
      : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3]), "=&v"(w[4]), "=&v"(w[5]), "=&v"(w[6]), "=&v"(w[7]),
        "=&v"(w[8]), "=&v"(w[9]), "=&v"(w[10]), "=&v"(w[11]), "=&v"(w[12]), "=&v"(w[13]), "=&v"(w[14]), "=&v"(w[15])
      : "v"(a)
      : "memory");
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = __builtin_bit_cast(float2, w[r]);
}
// the thread's 4 items (2t, 2t+1, 2(t+1024), 2(t+1024)+1) of both staged rows; a = &S[2t]
__device__ __forceinline__ void s_read_items(unsigned a, float2 (&v)[2][4]) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  f4 w[4];
  asm volatile(
      "ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:16384\n\tds_read_b128 %2, %4 offset:32768\n\t"
      "ds_read_b128 %3, %4 offset:49152\n\ts_waitcnt lgkmcnt(0)"
      : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3])
      : "v"(a)
      : "memory");
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      v[r][2 * h] = make_float2(w[2 * r + h].x, w[2 * r + h].y);
      v[r][2 * h + 1] = make_float2(w[2 * r + h].z, w[2 * r + h].w);
    }
}

template <int N, bool HR = false>
__global__ void __launch_bounds__(1024) k_precond_xt_dma_2d(KP<float> p, const float2* __restrict__ twx) {
  using C = float2;
  constexpr int NT = 1024, RB = 2, NL = 1;
  constexpr int NI = N * NL, IT = NI / NT;
  constexpr int B = 2 * NL;   // reals per item in a row (HR: x[2m], x[2m+1] of the one column)
  constexpr int LINE = Pad<N>::LINE;
  static_assert(N == 4096 && IT == 4, "one 4096-point line per block");
  if (p.ctrl->done) return;
  // three separate LDS objects: the compiler then knows the DMA writes only S and does not wait for it
  // (vmcnt(0)) before every access of A or of the twiddles
  __shared__ __align__(16) C A[RB * LINE];   // RB padded lines
  __shared__ __align__(16) C S[RB * NI];     // RB rows, lane-linear (float2 item i of row r at S[r * NI + i])
  __shared__ __align__(16) C twl[TwLds<N>::SIZE];
  __shared__ float lxs[N];                   // lamx per item: dd is recomputed per row (8 VGPRs fewer)
  __shared__ C rsw[HR ? 128 : 1];            // HR: W_2N^j and W_2N^(64 j), j < 64
  fill_twlds<C, N>(twl, twx, HR ? 2 : 1);    // HR: twx holds W_2N
  for (int i = threadIdx.x; i < N; i += NT) lxs[i] = p.lamx[i];
  if constexpr (HR)
    for (int i = threadIdx.x; i < 128; i += NT) rsw[i] = twx[i < 64 ? i : 64 * (i - 64)];
  __syncthreads();   // lxs (read by the converged-pivot rows below)
  const int T = p.T, tid = threadIdx.x;
  // the wave index in an SGPR and the lane from mbcnt: the laundered thread index costs no VGPR between uses
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int b = blockIdx.x + p.b0;
  constexpr int M = N * B;
  float* wb = p.work + (size_t)b * M;
  const size_t kstride = (size_t)p.nb * M;
  const float inv_ae = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, 1.f / p.ae)));
  const float ly0 = p.lamy[HR ? b : b * B], ly1 = p.lamy[HR ? b : b * B + 1], Cc = p.C;
  // HR: lam(N) (mode N of the 2N-point column, item 0's second mode): the host's value, a uniform load (SGPR)
  const float lam_n = HR ? p.lamx[N] : 0.f;
  auto lx_hi = [&](int item) { return item == 0 ? lam_n : lxs[N - item]; };   // HR: lam(item + N)
  auto dd_of = [&](int item) {
    const float lx = lxs[item];
    if constexpr (HR) return make_float2((Cc - lx - ly0) * inv_ae, (Cc - lx_hi(item) - ly0) * inv_ae);
    else return make_float2((Cc - lx - ly0) * inv_ae, (Cc - lx - ly1) * inv_ae);
    (void)ly1;
  };
  // the item's pair of modes from a transformed line: Hartley pair of the two packed columns, or (HR) the real
  // split of the one column (modes k and k + N)
  auto unpack2 = [&](const C* line, int k, float& h0, float& h1) {
    if constexpr (HR) realsplit_padded<C, float>(line, N, k, cmul(rsw[k & 63], rsw[64 + (k >> 6)]), h0, h1);
    else hartley_padded<C, float>(line, N, k, h0, h1);
  };
  // the thread index is laundered once per batch (tl), so the unrolled loops' LDS / global addresses are
  // recomputed there instead of being hoisted out of the row loops into registers (which spills)
  int tl = tid;
  auto launder = [&]() {
    if constexpr (HR) {   // the lane id itself from asm: else the compiler keeps wave*64 + lane live (spilled: HR is
      int l;              // at 128 VGPRs) as the one input of every launder
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
      tl = wave * 64 + l;
    } else {
      tl = wave * 64 + (int)__lane_id();
    }
    asm volatile("" : "+v"(tl));
  };
  auto item_of = [&](int i) { return 2 * (tl + (i >> 1) * NT) + (i & 1); };
  auto st_pair = [&](C* dst, int j, C a, C b2) {
    reinterpret_cast<float4*>(dst)[tl + j * NT] = make_float4(a.x, a.y, b2.x, b2.y);
  };
  auto row_ptr = [&](int k) { return reinterpret_cast<C*>(wb + (size_t)k * kstride); };
  // rows k_first + dir*r (r < RB), clamped into [0, T), HBM -> S: 2 x 16 KiB per row, 1 KiB per wave-instruction
  auto issue_rows = [&](int k_first, int dir) {
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const float4* src = reinterpret_cast<const float4*>(row_ptr(min(max(k_first + dir * r, 0), T - 1)));
#pragma unroll
      for (int h = 0; h < NI / 2 / NT; ++h)
        __builtin_amdgcn_global_load_lds(src + h * NT + tl,
                                         (__attribute__((address_space(3))) void*)(S + r * NI + 2 * (h * NT + wave * 64)),
                                         16, 0, 0);
    }
  };
  C c1[IT], c2[IT], c3[IT];     // theta (backward),  h | e^-th once converged (forward) | E | e^-th (backward),  b' | x
  // Converged pivots (kernels_xt_f64.hpp): g_k = e^-th E_{k+1}/E_{k+2} is e^-th to within 2^-26 once th (k+1) > 9
  // in every lane of the wave; kf[i] = the first such global row for item i (wave-uniform, SGPRs).  From it on the
  // forward step multiplies by e^-th (no reciprocal) and the backward step needs no expm1 / exp / reciprocal.
  int kf[IT];
  launder();
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const float2 dd = dd_of(item_of(i));
    const float dl0 = 0.5f * dd.x, dl1 = 0.5f * dd.y;
    float tm = fminf(log1pf(dl0 + sqrtf(dl0 * (dl0 + 2.f))), log1pf(dl1 + sqrtf(dl1 * (dl1 + 2.f))));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) tm = fminf(tm, __shfl_xor(tm, o, kWave));
    const float q = 9.f / fmaxf(tm, 1e-20f);
    kf[i] = __builtin_amdgcn_readfirstlane(q < 1e9f ? (int)q : 1000000000);
  }
  auto eth = [](float d) { return 1.f / (1.f + 0.5f * d + sqrtf(d * (1.f + 0.25f * d))); };   // e^-th

  // Waits.  A batch with both rows stored ("full") issues exactly 4 stores after the DMA of the next rows,
  // so vmcnt(4) retires that DMA; an edge batch waits vmcnt(0).  The waits are builtins, so the compiler's
  // own tracking sees that the DMA has landed and adds no vmcnt(0) before the reads of S (it would also wait
  // for this batch's stores).
  auto wait_dma = [&](bool full) {
    if (full) __builtin_amdgcn_s_waitcnt(0x0F74);   // vmcnt(4) (expcnt, lgkmcnt: no wait)
    else __builtin_amdgcn_s_waitcnt(0x0F70);        // vmcnt(0)
  };

  if (p.xt_phase != 2) {
    // ---------------- forward ----------------
    // s = dd + h_{k-1},  g_k = 1/(1+s),  h_k = s g_k,  b'_k = (rhs/ae + b'_{k-1}) g_k;
    // last (Neumann) row of the window: u_{T-1} = ae (dd + h_{T-2})
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const float2 d = dd_of(item_of(i));   // (HR: modes k and k + N)
      c2[i] = make_float2(h_entry(d.x, p.j0), h_entry(d.y, p.j0));
      c3[i] = make_float2(0.f, 0.f);
    }
    constexpr int nR = N / 16;
    static_assert(RB * nR == NT / 2, "first pass: one butterfly per thread for half the block");
    C v[16];
    // first radix-16 pass, read half: S (unpadded, line r = row r).  512 butterflies: the upper half of the
    // block repeats the lower half's reads (no divergent register state across the barrier), then idles.
    auto pass1_read = [&]() {
      launder();
      const int bt = tl & (NT / 2 - 1);
      const int l = bt / nR, j = bt - l * nR;
      s_read16(lds_addr(S + l * NI + j), v);
    };
    auto pass1_write = [&]() {
      const int bt = tl & (NT / 2 - 1);
      const int l = bt / nR, j = bt - l * nR;
      if (tl < NT / 2) {   // the upper half only loaded (no divergent state across the barrier)
        dft_any<C, 16>(v);
        C* d = A + l * LINE + pix(j * 16);
#pragma unroll
        for (int r = 0; r < 16; ++r) d[r] = v[r];
      }
    };
    // the two elimination steps of rows k0, k0+1 (FULL: both rows exist and are stored)
    auto thomas_fwd = [&](int k0, auto full_tag) {
      constexpr bool FULL = decltype(full_tag)::value;
      launder();
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const int k = k0 + r;
        if (!FULL && k >= T) break;
        C* dst = row_ptr(k);
        const int kg = p.j0 + k;   // global row
        if (FULL || k < T - 1 || !p.last_slab) {
#pragma unroll
          for (int i = 0; i < IT; ++i) {
            float ha, hb;
            unpack2(A + r * LINE, item_of(i), ha, hb);
            if (kg >= kf[i]) {   // converged: g = e^-th (in c2 from row kf on: h is no longer needed)
              if (kg == max(kf[i], p.j0)) {   // the first converged row of this sweep (a slab may start past kf)
                const float2 dd = dd_of(item_of(i));
                c2[i] = make_float2(eth(dd.x), eth(dd.y));
              }
              c3[i] = make_float2((ha * inv_ae + c3[i].x) * c2[i].x, (hb * inv_ae + c3[i].y) * c2[i].y);
            } else {
              const float2 dd = dd_of(item_of(i));
              const float s0 = dd.x + c2[i].x, s1 = dd.y + c2[i].y;
              const float g0 = rcp_fast(1.f + s0), g1 = rcp_fast(1.f + s1);
              c3[i] = make_float2((ha * inv_ae + c3[i].x) * g0, (hb * inv_ae + c3[i].y) * g1);
              c2[i] = make_float2(s0 * g0, s1 * g1);
            }
          }
#pragma unroll
          for (int j = 0; j < IT / 2; ++j) st_pair(dst, j, c3[2 * j], c3[2 * j + 1]);
        } else {
#pragma unroll
          for (int i = 0; i < IT; ++i) {
            float ha, hb;
            unpack2(A + r * LINE, item_of(i), ha, hb);
            const float2 dd = dd_of(item_of(i));
            if (max(kf[i], p.j0) < kg) {   // converged on an earlier row: dd + h = (1 - g) / g
              const float2 g = c2[i];
              c3[i] = make_float2((ha * inv_ae + c3[i].x) * g.x / (1.f - g.x), (hb * inv_ae + c3[i].y) * g.y / (1.f - g.y));
            } else {
              c3[i] = make_float2((ha * inv_ae + c3[i].x) / (dd.x + c2[i].x), (hb * inv_ae + c3[i].y) / (dd.y + c2[i].y));
            }
          }
          if (p.slab) {   // re-read (after the carry fix-up) by the backward sweep
#pragma unroll
            for (int j = 0; j < IT / 2; ++j) st_pair(dst, j, c3[2 * j], c3[2 * j + 1]);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    auto full_fwd = [&](int k0) { return k0 + 1 < T - 1 || (k0 + 1 < T && !p.last_slab); };
    issue_rows(0, 1);
    wait_dma(false);
    lds_sync();
    pass1_read();
    for (int k0 = 0;; k0 += RB) {
      lds_sync();                  // S read by every wave: free for the next rows
      issue_rows(k0 + RB, 1);      // clamped past the end (landed, never read)
      pass1_write();
      lds_sync();
      batch_pass<C, N, RB * NL, NT, 16, 16>(A, twl, tl);
      batch_pass<C, N, RB * NL, NT, 256, 16>(A, twl, tl);
      const bool full = full_fwd(k0);
      if (full) thomas_fwd(k0, std::true_type{});
      else thomas_fwd(k0, std::false_type{});
      wait_dma(full);
      lds_sync();                  // rows k0+2, k0+3 in S; this batch's A reads done
      if (k0 + RB >= T) break;
      pass1_read();
    }
  }
  if (p.xt_phase == 1) return;   // forward sweep only (t-slab: the carry fix-up runs in between)

  // ---------------- backward ----------------
  // x_k = b'_k + g_k x_{k+1},  g_k = e^-th E_{k+1}/E_{k+2},  E_m = expm1(-2 th m),  cosh th = 1 + dd/2
  lds_sync();   // lxs (xt_phase 2 skips the forward's barriers)
  launder();
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const float2 dd = dd_of(item_of(i));
    const float dl0 = 0.5f * dd.x, dl1 = 0.5f * dd.y;
    c1[i] = make_float2(fmaxf(log1pf(dl0 + sqrtf(dl0 * (dl0 + 2.f))), 1e-20f),
                        fmaxf(log1pf(dl1 + sqrtf(dl1 * (dl1 + 2.f))), 1e-20f));
    // E_{k+2} for the first substituted row: k = T-2 (single context) or T-1 (slab, from the right carry);
    // e^-th instead when that row is already converged
    const float e0 = (float)(p.j0 + T + (p.slab ? 1 : 0));
    if (p.j0 + T - (p.slab ? 1 : 2) >= kf[i]) c2[i] = make_float2(__expf(-c1[i].x), __expf(-c1[i].y));
    else c2[i] = make_float2(expm1f(-2.f * c1[i].x * e0), expm1f(-2.f * c1[i].y * e0));
    if (p.slab)
      c3[i] = p.carry_y ? reinterpret_cast<const C*>(p.carry_y + (size_t)b * M)[item_of(i)] : make_float2(0.f, 0.f);
  }
  // substitution steps of rows kt, kt-1 (b' from S), x staged in A
  auto thomas_bwd = [&](int kt) {
    launder();
#pragma unroll
    for (int i = 0; i < IT; ++i) {   // theta opaque per batch: exp(-theta) is recomputed, not held (spilled)
      asm volatile("" : "+v"(c1[i].x));
      asm volatile("" : "+v"(c1[i].y));
    }
    C bpv[RB][IT];
    s_read_items(lds_addr(S + 2 * tl), bpv);
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int k = kt - r;
      if (k < 0) break;
      if ((k < T - 1 || p.slab) && !(p.dbg & 4)) {
        const int kg = p.j0 + k;
        const float kk1 = (float)(kg + 1);   // global row index + 1
#pragma unroll
        for (int i = 0; i < IT; ++i) {
          const C bp = bpv[r][i];
          if (kg >= kf[i]) {   // converged: g = e^-th (c2)
            c3[i] = make_float2(bp.x + c2[i].x * c3[i].x, bp.y + c2[i].y * c3[i].y);
            continue;
          }
          if (kg + 1 == kf[i])   // first unconverged row below the converged ones: E_{k+2} from theta
            c2[i] = make_float2(expm1f(-2.f * c1[i].x * (kk1 + 1.f)), expm1f(-2.f * c1[i].y * (kk1 + 1.f)));
          // theta >= 1e-20 (clamped above): the closed form tends to (k+1)/(k+2) as theta -> 0
          const float2 E1 = expm1_neg2(-2.f * c1[i].x * kk1, -2.f * c1[i].y * kk1);
          const float g0 = __expf(-c1[i].x) * E1.x * rcp_fast(c2[i].x);
          const float g1 = __expf(-c1[i].y) * E1.y * rcp_fast(c2[i].y);
          c3[i] = make_float2(bp.x + g0 * c3[i].x, bp.y + g1 * c3[i].y);
          c2[i] = E1;
        }
      }
      if constexpr (HR) {   // modes k and k + N -> their real positions (float f at element f/2, part f%2)
        float* Af = reinterpret_cast<float*>(A + r * LINE);
#pragma unroll
        for (int i = 0; i < IT; ++i) {
          const int f0 = item_of(i), f1 = item_of(i) + N;
          Af[2 * pix(f0 >> 1) + (f0 & 1)] = c3[i].x;
          Af[2 * pix(f1 >> 1) + (f1 & 1)] = c3[i].y;
        }
      } else {
#pragma unroll
        for (int i = 0; i < IT; ++i) A[r * LINE + pix(item_of(i))] = c3[i];
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto store_bwd = [&](int kt, auto full_tag) {   // inverse-transformed rows kt, kt-1 (FULL: both exist)
    constexpr bool FULL = decltype(full_tag)::value;
    launder();
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int k = kt - r;
      if (!FULL && k < 0) break;
      C* wk = row_ptr(k);
      if constexpr (HR) {   // spatial x[k], x[k + N] of the real column: items 2m, 2m+1 -> float2 at 2m and 2m + N
        float* wf = reinterpret_cast<float*>(wk);
#pragma unroll
        for (int j = 0; j < IT / 2; ++j) {   // pair by pair (fewer values live: the kernel is at 128 VGPRs)
          float a0, b0, a1, b1;
          unpack2(A + r * LINE, item_of(2 * j), a0, b0);
          unpack2(A + r * LINE, item_of(2 * j + 1), a1, b1);
          const int m2 = 2 * (tl + j * NT);
          *reinterpret_cast<float2*>(wf + m2) = make_float2(a0, a1);
          *reinterpret_cast<float2*>(wf + m2 + N) = make_float2(b0, b1);
        }
      } else {
        C o[IT];
#pragma unroll
        for (int i = 0; i < IT; ++i) {
          float ha, hb;
          unpack2(A + r * LINE, item_of(i), ha, hb);
          o[i] = make_float2(ha, hb);
        }
#pragma unroll
        for (int j = 0; j < IT / 2; ++j) st_pair(wk, j, o[2 * j], o[2 * j + 1]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  issue_rows(T - 1, -1);
  wait_dma(false);
  lds_sync();
  for (int kt = T - 1;; kt -= RB) {
    thomas_bwd(kt);
    lds_sync();                    // S read, A staged
    issue_rows(kt - RB, -1);       // clamped past row 0 (landed, never read)
    if (!(p.dbg & 2)) batch_fft<C, N, RB * NL, NT, 1>(A, twl, tl);
    const bool full = kt - 1 >= 0;
    if (full) store_bwd(kt, std::true_type{});
    else store_bwd(kt, std::false_type{});
    wait_dma(full);
    lds_sync();                    // rows kt-2, kt-3 of b' in S; this batch's A reads done
    if (kt - RB < 0) break;
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);   // stores drained with the block (no DMA outstanding)
}

}  // namespace pdhg
