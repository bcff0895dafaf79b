// LDS-resident multi-line Stockham FFT for gfx950 + real Hartley unpack.
//
// The H1 preconditioner of the reference (utils/utils_precond.py:105-178) is an
// FFT in space, a tridiagonal solve in t per Fourier mode, and an inverse FFT.
// Because the spatial operator is a real symmetric circulant, the separable
// discrete Hartley transform (DHT) diagonalises it with the same symbol, so the
// whole preconditioner runs in REAL arithmetic with no half-spectrum padding:
// two real lines a, b are packed as z = a + i b, one complex FFT of z is
// taken, and   H_a(k) = (Re Z_k + Re Z_-k - Im Z_k + Im Z_-k) / 2,
//              H_b(k) = (Im Z_k + Im Z_-k - Re Z_-k + Re Z_k) / 2.
// The DHT is its own inverse up to 1/n, so the inverse pass is the same code.
#pragma once
#include "common.hpp"

namespace pdhg {

struct FFTPlan {
  int n;
  int npass;
  int pow2;             // n is a power of two (fast index math)
  int radix[kMaxPass];
};

// cos / sin of 2*pi*k/16
__device__ constexpr double kC16[16] = {1.0, 0.92387953251128674, 0.70710678118654752, 0.38268343236508977,
                                        0.0, -0.38268343236508977, -0.70710678118654752, -0.92387953251128674,
                                        -1.0, -0.92387953251128674, -0.70710678118654752, -0.38268343236508977,
                                        0.0, 0.38268343236508977, 0.70710678118654752, 0.92387953251128674};
__device__ constexpr double kS16[16] = {0.0, 0.38268343236508977, 0.70710678118654752, 0.92387953251128674,
                                        1.0, 0.92387953251128674, 0.70710678118654752, 0.38268343236508977,
                                        0.0, -0.38268343236508977, -0.70710678118654752, -0.92387953251128674,
                                        -1.0, -0.92387953251128674, -0.70710678118654752, -0.38268343236508977};

template <typename C>
__device__ __forceinline__ void dft2(C& a, C& b) {
  const C t = a;
  a = cadd(t, b);
  b = csub(t, b);
}
template <typename C>
__device__ __forceinline__ void dft4(C& v0, C& v1, C& v2, C& v3) {
  const C s02 = cadd(v0, v2), d02 = csub(v0, v2);
  const C s13 = cadd(v1, v3), d13 = cmul_mi(csub(v1, v3));
  v0 = cadd(s02, s13);
  v2 = csub(s02, s13);
  v1 = cadd(d02, d13);
  v3 = csub(d02, d13);
}
// multiply by W_16^m = exp(-2 pi i m / 16), m compile-time
template <typename C, int M>
__device__ __forceinline__ C tw16(C a) {
  using T = decltype(C::x);
  constexpr int m = M & 15;
  if constexpr (m == 0) return a;
  else if constexpr (m == 4) return cmul_mi(a);
  else if constexpr (m == 8) return cmk<C>(-a.x, -a.y);
  else if constexpr (m == 12) return cmk<C>(-a.y, a.x);
  else return cmul(a, cmk<C>((T)kC16[m], (T)(-kS16[m])));
}

// In-register forward DFT of size R in {2,3,4,8,16}, natural order in/out.
// R = R1*R2 split: n = n1 + R1 n2, k = R2 k1 + k2 (DFT_R2 over n2, twiddle W_R^{n1 k2}, DFT_R1 over n1).
template <typename C, int R>
__device__ __forceinline__ void dft_any(C* v) {
  if constexpr (R == 2) {
    dft2(v[0], v[1]);
  } else if constexpr (R == 3) {
    using T = decltype(C::x);
    const T h = (T)0.86602540378443865;  // sqrt(3)/2
    const C t1 = cadd(v[1], v[2]);
    const C t2 = cmk<C>(v[0].x - (T)0.5 * t1.x, v[0].y - (T)0.5 * t1.y);
    const C d = csub(v[1], v[2]);
    const C s = cmk<C>(h * d.y, -h * d.x);     // (b - c) * (-i sqrt(3)/2)
    v[0] = cadd(v[0], t1);
    v[1] = cadd(t2, s);
    v[2] = csub(t2, s);
  } else if constexpr (R == 4) {
    dft4(v[0], v[1], v[2], v[3]);
  } else if constexpr (R == 8) {
    // R1 = 2, R2 = 4
    dft4(v[0], v[2], v[4], v[6]);
    dft4(v[1], v[3], v[5], v[7]);
    v[3] = tw16<C, 2>(v[3]);
    v[5] = tw16<C, 4>(v[5]);
    v[7] = tw16<C, 6>(v[7]);
    // Y[n1][k2] sits at v[n1 + 2 k2]; X[4 k1 + k2] = DFT2 over n1
    C x[8];
#pragma unroll
    for (int k2 = 0; k2 < 4; ++k2) {
      C a = v[2 * k2], b = v[2 * k2 + 1];
      dft2(a, b);
      x[k2] = a;
      x[4 + k2] = b;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = x[i];
  } else if constexpr (R == 16) {
    // R1 = 4, R2 = 4: DFT4 over n2 of v[n1 + 4 n2] -> Y[n1][k2] stored back at v[n1 + 4 k2]
    dft4(v[0], v[4], v[8], v[12]);
    dft4(v[1], v[5], v[9], v[13]);
    dft4(v[2], v[6], v[10], v[14]);
    dft4(v[3], v[7], v[11], v[15]);
    v[5] = tw16<C, 1>(v[5]);
    v[9] = tw16<C, 2>(v[9]);
    v[13] = tw16<C, 3>(v[13]);
    v[6] = tw16<C, 2>(v[6]);
    v[10] = tw16<C, 4>(v[10]);
    v[14] = tw16<C, 6>(v[14]);
    v[7] = tw16<C, 3>(v[7]);
    v[11] = tw16<C, 6>(v[11]);
    v[15] = tw16<C, 9>(v[15]);
    // DFT4 over n1 for each k2: inputs v[4 k2 + n1], outputs X[4 k1 + k2]
    dft4(v[0], v[1], v[2], v[3]);
    dft4(v[4], v[5], v[6], v[7]);
    dft4(v[8], v[9], v[10], v[11]);
    dft4(v[12], v[13], v[14], v[15]);
    // now v[4 k2 + k1] = X[4 k1 + k2]: transpose the 4x4 index
    C x[16];
#pragma unroll
    for (int k2 = 0; k2 < 4; ++k2)
#pragma unroll
      for (int k1 = 0; k1 < 4; ++k1) x[4 * k1 + k2] = v[4 * k2 + k1];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = x[i];
  }
}

// One Stockham DIT pass of compile-time radix R on nl interleaved lines
// (element e of line l at index e*nl + l; nl a power of two).
template <typename C, int R>
__device__ __forceinline__ void stockham_pass(const C* __restrict__ src, C* __restrict__ dst, int n, int nl,
                                              int lnl, int Ls, int pow2, const C* __restrict__ tw) {
  const int nR = n / R;
  const int tws = n / (Ls * R);
  const int total = nR * nl;
#pragma unroll 1
  for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
    const int l = idx & (nl - 1);
    const int j = idx >> lnl;
    const int k = pow2 ? (j & (Ls - 1)) : (j % Ls);
    C v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = src[(size_t)(j + r * nR) * nl + l];
    if (k != 0) {
#pragma unroll
      for (int r = 1; r < R; ++r) v[r] = cmul(v[r], tw[r * k * tws]);
    }
    dft_any<C, R>(v);
    const int base = (j - k) * R + k;
#pragma unroll
    for (int r = 0; r < R; ++r) dst[(size_t)(base + r * Ls) * nl + l] = v[r];
  }
}

// Generic (any radix) pass: one output element per work item, O(R) reads.
template <typename C>
__device__ void stockham_pass_generic(const C* __restrict__ src, C* __restrict__ dst, int n, int nl, int lnl,
                                      int Ls, int R, const C* __restrict__ tw) {
  using T = decltype(C::x);
  const int nR = n / R;
  const int tws = n / (Ls * R);
  const int total = n * nl;
  for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
    const int l = idx & (nl - 1);
    const int q = idx >> lnl;
    const int k = q % Ls;
    const int s = (q / Ls) % R;
    const int j = (q / (Ls * R)) * Ls + k;
    T ax = 0, ay = 0;
    for (int qq = 0; qq < R; ++qq) {
      C v = src[(size_t)(j + qq * nR) * nl + l];
      if (k != 0 && qq != 0) v = cmul(v, tw[qq * k * tws]);
      const C w = tw[((qq * s) % R) * nR];
      ax += v.x * w.x - v.y * w.y;
      ay += v.x * w.y + v.y * w.x;
    }
    dst[(size_t)q * nl + l] = cmk<C>(ax, ay);
  }
}

// Full forward FFT of nl interleaved lines of length plan.n held in LDS buffer
// a; b is scratch of the same size.  All threads of the block take part; the
// call starts and ends with a barrier-complete state.  Returns the buffer that
// holds the result (natural order).
// GLB: a and b are global-memory scratch of this workgroup (lines longer than LDS holds); the
// passes are then separated by full barriers (stores drained), which orders them within the
// workgroup because all its waves share one CU's vector L1.
template <typename C, bool GLB = false>
__device__ C* lds_fft(C* a, C* b, int nl, const FFTPlan& pl, const C* __restrict__ tw) {
  int lnl = 0;
  while ((1 << lnl) < nl) ++lnl;
  int Ls = 1;
  C* src = a;
  C* dst = b;
  for (int p = 0; p < pl.npass; ++p) {
    const int R = pl.radix[p];
    switch (R) {
      case 16: stockham_pass<C, 16>(src, dst, pl.n, nl, lnl, Ls, pl.pow2, tw); break;
      case 8: stockham_pass<C, 8>(src, dst, pl.n, nl, lnl, Ls, pl.pow2, tw); break;
      case 4: stockham_pass<C, 4>(src, dst, pl.n, nl, lnl, Ls, pl.pow2, tw); break;
      case 2: stockham_pass<C, 2>(src, dst, pl.n, nl, lnl, Ls, pl.pow2, tw); break;
      case 3: stockham_pass<C, 3>(src, dst, pl.n, nl, lnl, Ls, pl.pow2, tw); break;
      default: stockham_pass_generic<C>(src, dst, pl.n, nl, lnl, Ls, R, tw); break;
    }
    if constexpr (GLB)
      __syncthreads();
    else
      lds_sync();
    C* t = src;
    src = dst;
    dst = t;
    Ls *= R;
  }
  return src;
}

// ---------------- compile-time-size FFT (hot sizes) ----------------
// N (power of two) and NL (lines) are template constants, so every LDS stride is an
// immediate offset and the radix schedule (16,16,..., then 8/4/2) unrolls statically.
template <int N>
struct Pow2Sched {
  static constexpr int lead = (N >= 16) ? 16 : N;
};

template <typename C, int N, int NL, int LS, int R>
__device__ __forceinline__ void fixed_pass(const C* __restrict__ src, C* __restrict__ dst, const C* __restrict__ tw) {
  constexpr int nR = N / R;
  constexpr int tws = N / (LS * R);
  constexpr int total = nR * NL;
  constexpr int lnl = (NL == 1) ? 0 : (NL == 2) ? 1 : (NL == 4) ? 2 : (NL == 8) ? 3 : 4;
#pragma unroll 1
  for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
    const int l = idx & (NL - 1);
    const int j = idx >> lnl;
    const int k = j & (LS - 1);
    C v[R];
    const C* s = src + (size_t)j * NL + l;
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = s[r * nR * NL];
    if (LS > 1 && k != 0) {
#pragma unroll
      for (int r = 1; r < R; ++r) v[r] = cmul(v[r], tw[r * k * tws]);
    }
    dft_any<C, R>(v);
    C* d = dst + (size_t)((j - k) * R + k) * NL + l;
#pragma unroll
    for (int r = 0; r < R; ++r) d[r * LS * NL] = v[r];
  }
}

template <typename C, int N, int NL, int LS>
__device__ __forceinline__ C* fixed_passes(C* src, C* dst, const C* __restrict__ tw) {
  if constexpr (LS >= N) {
    return src;
  } else {
    constexpr int rem = N / LS;
    constexpr int R = (rem >= 16) ? 16 : rem;
    fixed_pass<C, N, NL, LS, R>(src, dst, tw);
    lds_sync();
    return fixed_passes<C, N, NL, LS * R>(dst, src, tw);
  }
}

template <typename C, int N, int NL>
__device__ __forceinline__ C* lds_fft_fixed(C* a, C* b, const C* __restrict__ tw) {
  return fixed_passes<C, N, NL, 1>(a, b, tw);
}

// ---------------- in-place multi-line FFT (register-staged, one LDS buffer) ----------------
// Line-major with one pad element per 16: element e of line l lives at a[l*PADN(N) + pix(e)],
// pix(e) = e + e/16.  The first Stockham pass (LS = 1) writes 16 consecutive elements per lane;
// unpadded that is a 128-B lane stride (16-way bank conflict), padded it is 136 B (conflict-free).
// All other strides are multiples of 16 elements, so every offset stays a compile-time constant.
template <int N>
struct Pad {
  static constexpr int LINE = N + N / 16;
};
__device__ __forceinline__ int pix(int e) { return e + (e >> 4); }

// twiddles W^{r k} (W = exp(-2 pi i / (LS R))) for r = 1..R-1 from three table loads (W^k, W^4k,
// W^8k) and at most three complex products each.
template <typename C, int R>
__device__ __forceinline__ void twiddles_from3(C* w, const C* __restrict__ tw, int kt) {
  const C w1 = tw[kt];
  if constexpr (R == 2) {
    w[1] = w1;
  } else {
    w[1] = w1;
    w[2] = cmul(w1, w1);
    w[3] = cmul(w[2], w1);
    if constexpr (R > 4) {
      const C w4 = tw[4 * kt];
      w[4] = w4;
      w[5] = cmul(w4, w1);
      w[6] = cmul(w4, w[2]);
      w[7] = cmul(w4, w[3]);
      if constexpr (R > 8) {
        const C w8 = tw[8 * kt];
        w[8] = w8;
#pragma unroll
        for (int r = 1; r < 8; ++r) w[8 + r] = cmul(w8, w[r]);
      }
    }
  }
}

// LDS twiddle seeds: a kernel that runs many transforms keeps (W^k, W^4k, W^8k) for every k of each
// twiddled pass in a small LDS table (TwLds<N>::SIZE complex; 816 for N = 4096), so the passes read
// their seeds at LDS latency instead of from L2; the 15 per-butterfly twiddles are rebuilt with <= 3
// complex products (as twiddles_from3).  Pass LS = 16 at offset 0, LS = 256 at 48, LS = 4096 at 816.
template <int N>
struct TwLds {
  static constexpr int SIZE = 3 * ((N > 16 ? 16 : 0) + (N > 256 ? 256 : 0) + (N > 4096 ? 4096 : 0));
};
__host__ __device__ constexpr int twlds_off(int LS) { return LS >= 4096 ? 816 : LS >= 256 ? 48 : 0; }
// complex entries of TwLds<n> (host side: LDS sizing of the kernels that keep the table)
__host__ __device__ constexpr int twlds_size(int n) {
  return 3 * ((n > 16 ? 16 : 0) + (n > 256 ? 256 : 0) + (n > 4096 ? 4096 : 0));
}

// GLS: passes with LS >= GLS read their seeds from the global table tw (W_N) instead of twl -- the same values
// fill_twlds copies, so the transform is bitwise the same; only the LS < GLS segments of TwLds need LDS.
template <typename C, int N, int NL, int NT, int LS, int R, bool REG, int LINE = Pad<N>::LINE, int GLS = (1 << 30)>
__device__ __forceinline__ void inplace_pass(C* __restrict__ a, const C* __restrict__ tw, const C* twl) {
  constexpr int nR = N / R;
  constexpr int tws = N / (LS * R);
  constexpr int total = nR * NL;
  constexpr int PER = (total + NT - 1) / NT;
  static_assert(nR % 16 == 0 && (LS == 1 || LS % 16 == 0) && (LS > 1 || R == 16), "padded schedule");
  C v[PER][R];
  int base[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int idx = threadIdx.x + q * NT;
    base[q] = -1;
    if (total % NT == 0 || idx < total) {
      const int l = idx / nR;          // nR is a power of two: shift
      const int j = idx - l * nR;
      const int k = j & (LS - 1);
      const C* s = a + l * LINE + pix(j);
#pragma unroll
      for (int r = 0; r < R; ++r) v[q][r] = s[r * (nR + nR / 16)];
      if (LS > 1 && k != 0) {
        if constexpr (REG && R == 16 && sizeof(C) == 16) {
          // fp64: W^r = (W^4k)^(r>>2 part) (W^k)^(r&3) applied row by row of the 4 x 4 split, so at most the three
          // low powers and one high factor are live (the full w[16] table is 60 VGPRs next to 64 of values)
          const C* t3 = twl + twlds_off(LS) + 3 * k;
          auto sd = [&](int m) -> C {   // seed m of k: W^(k tws), W^(4 k tws), W^(8 k tws)
            if constexpr (LS >= GLS) return tw[((m == 0 ? 1 : m == 1 ? 4 : 8) * k * tws) & (N - 1)];
            else return t3[m];
          };
          const C w1 = sd(0), w2 = cmul(w1, w1), w3 = cmul(w2, w1);
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            C H;
            if (h == 1) H = sd(1);
            else if (h == 2) H = sd(2);
            else if (h == 3) H = cmul(sd(1), sd(2));
            if (h > 0) v[q][4 * h] = cmul(v[q][4 * h], H);
            v[q][4 * h + 1] = cmul(v[q][4 * h + 1], h > 0 ? cmul(H, w1) : w1);
            v[q][4 * h + 2] = cmul(v[q][4 * h + 2], h > 0 ? cmul(H, w2) : w2);
            v[q][4 * h + 3] = cmul(v[q][4 * h + 3], h > 0 ? cmul(H, w3) : w3);
          }
          base[q] = l * LINE + pix((j - k) * R + k);
          continue;
        }
        C w[R];
        if constexpr (REG) {
          const C* t3 = twl + twlds_off(LS) + 3 * k;
          auto sd = [&](int m) -> C {
            if constexpr (LS >= GLS) return tw[((m == 0 ? 1 : m == 1 ? 4 : 8) * k * tws) & (N - 1)];
            else return t3[m];
          };
          const C s0 = sd(0);
          w[1] = s0;
          if constexpr (R > 2) {
            w[2] = cmul(s0, s0);
            w[3] = cmul(w[2], s0);
          }
          if constexpr (R > 4) {
            const C s1 = sd(1);
            w[4] = s1;
            w[5] = cmul(s1, s0);
            w[6] = cmul(s1, w[2]);
            w[7] = cmul(s1, w[3]);
          }
          if constexpr (R > 8) {
            const C s2 = sd(2);
            w[8] = s2;
#pragma unroll
            for (int r = 1; r < 8; ++r) w[8 + r] = cmul(s2, w[r]);
          }
        } else {
          twiddles_from3<C, R>(w, tw, k * tws);
        }
#pragma unroll
        for (int r = 1; r < R; ++r) v[q][r] = cmul(v[q][r], w[r]);
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

template <typename C, int N, int NL, int NT, int LS, bool REG, int LINE = Pad<N>::LINE, int GLS = (1 << 30)>
__device__ __forceinline__ void inplace_passes(C* a, const C* __restrict__ tw, const C* twl) {
  if constexpr (LS < N) {
    constexpr int rem = N / LS;
    constexpr int R = (rem >= 16) ? 16 : rem;
    inplace_pass<C, N, NL, NT, LS, R, REG, LINE, GLS>(a, tw, twl);
    inplace_passes<C, N, NL, NT, LS * R, REG, LINE, GLS>(a, tw, twl);
  }
}

// Forward FFT in place of NL padded line-major lines (element e of line l at a[l*LINE + pix(e)]).
template <typename C, int N, int NL, int NT, int LINE = Pad<N>::LINE>
__device__ __forceinline__ void lds_fft_inplace(C* a, const C* __restrict__ tw) {
  inplace_passes<C, N, NL, NT, 1, false, LINE>(a, tw, nullptr);
}

// Same transform with the twiddle seeds read from an LDS table filled by fill_twlds.
template <typename C, int N, int NL, int NT, int LINE = Pad<N>::LINE>
__device__ __forceinline__ void lds_fft_inplace_tl(C* a, const C* twl) {
  inplace_passes<C, N, NL, NT, 1, true, LINE>(a, nullptr, twl);
}

// The same with only the LS = 16 pass's 48 seeds in LDS (twl) and the later passes' seeds read from the global
// table tw (W_N): bitwise the same transform in 768 B of seed LDS instead of TwLds<N>::SIZE * 16.
template <typename C, int N, int NL, int NT, int LINE = Pad<N>::LINE>
__device__ __forceinline__ void lds_fft_inplace_tl16(C* a, const C* twl, const C* __restrict__ tw) {
  inplace_passes<C, N, NL, NT, 1, true, LINE, 256>(a, tw, twl);
}


// Fill the TwLds<N> table from the global twiddle table (W_N^m at tw[m]); caller syncs before use.
template <typename C, int N>
__device__ __forceinline__ void fill_twlds(C* twl, const C* __restrict__ tw, int tw_stride = 1,
                                           int cnt = TwLds<N>::SIZE) {   // cnt = 48: the LS = 16 segment only
  for (int i = threadIdx.x; i < cnt; i += blockDim.x) {
    const int LS = i >= 816 ? 4096 : i >= 48 ? 256 : 16;
    const int e = i - twlds_off(LS);
    const int k = e / 3, m = e - 3 * k;
    const int R = (N / LS >= 16) ? 16 : N / LS;
    const int tws = N / (LS * R);
    const int mult = (m == 0) ? 1 : (m == 1) ? 4 : 8;
    twl[i] = tw[(size_t)tw_stride * ((mult * k * tws) & (N - 1))];   // tw holds W_{N*tw_stride}
  }
}

// ---------------- split passes for warp-specialised kernels ----------------
// Pass P (LS = 16^P) of the padded in-place schedule executed by a group of NTF threads, split at
// its barrier into a read half (loads + twiddles into registers) and a write half (DFT + stores),
// so another wave group can run between the barriers.  Twiddle seeds from the TwLds table.
template <int N, int NL, int NTF, int P>
struct SplitPass {
  static constexpr int LS = (P == 0) ? 1 : (P == 1) ? 16 : (P == 2) ? 256 : 4096;
  static constexpr int R = (N / LS >= 16) ? 16 : N / LS;
  static constexpr int nR = N / R;
  static constexpr int total = nR * NL;
  static constexpr int PER = (total + NTF - 1) / NTF;
  static_assert(nR % 16 == 0 && (LS == 1 || LS % 16 == 0) && (LS > 1 || R == 16), "padded schedule");
};

// v: flat register array of at least PER*R complex (element (q, r) at q*R + r); callers may alias it
// with other per-wave state (a warp-specialised kernel shares one array between its roles).
template <typename C, int N, int NL, int NTF, int P, int NV>
__device__ __forceinline__ void split_read(const C* __restrict__ a, const C* twl, int t, C (&v)[NV],
                                           int (&base)[SplitPass<N, NL, NTF, P>::PER]) {
  using SP = SplitPass<N, NL, NTF, P>;
  constexpr int R = SP::R, nR = SP::nR, LS = SP::LS, LINE = Pad<N>::LINE;
  static_assert(SP::PER * R <= NV, "register array too small");
#pragma unroll
  for (int q = 0; q < SP::PER; ++q) {
    const int idx = t + q * NTF;
    base[q] = -1;
    if (SP::total % NTF == 0 || idx < SP::total) {
      const int l = idx / nR;
      const int j = idx - l * nR;
      const int k = j & (LS - 1);
      const C* s = a + l * LINE + pix(j);
#pragma unroll
      for (int r = 0; r < R; ++r) v[q * R + r] = s[r * (nR + nR / 16)];
      if (LS > 1 && k != 0) {
        const C* t3 = twl + twlds_off(LS) + 3 * k;
        C w[R];
        w[1] = t3[0];
        if constexpr (R > 2) {
          w[2] = cmul(t3[0], t3[0]);
          w[3] = cmul(w[2], t3[0]);
        }
        if constexpr (R > 4) {
          w[4] = t3[1];
          w[5] = cmul(t3[1], t3[0]);
          w[6] = cmul(t3[1], w[2]);
          w[7] = cmul(t3[1], w[3]);
        }
        if constexpr (R > 8) {
          w[8] = t3[2];
#pragma unroll
          for (int r = 1; r < 8; ++r) w[8 + r] = cmul(t3[2], w[r]);
        }
#pragma unroll
        for (int r = 1; r < R; ++r) v[q * R + r] = cmul(v[q * R + r], w[r]);
      }
      base[q] = l * LINE + pix((j - k) * R + k);
    }
  }
}

template <typename C, int N, int NL, int NTF, int P, int NV>
__device__ __forceinline__ void split_write(C* __restrict__ a, C (&v)[NV],
                                            const int (&base)[SplitPass<N, NL, NTF, P>::PER]) {
  using SP = SplitPass<N, NL, NTF, P>;
  constexpr int R = SP::R, LS = SP::LS;
  static_assert(SP::PER * R <= NV, "register array too small");
#pragma unroll
  for (int q = 0; q < SP::PER; ++q) {
    if (base[q] >= 0) {
      C u[R];
#pragma unroll
      for (int r = 0; r < R; ++r) u[r] = v[q * R + r];
      dft_any<C, R>(u);
      C* d = a + base[q];
#pragma unroll
      for (int r = 0; r < R; ++r) d[(LS == 1) ? r : r * (LS + LS / 16)] = u[r];
    }
  }
}

// DHT of ONE real line of length 2M from the M-point complex FFT Z of z[m] = x[2m] + i x[2m+1]:
// E = (Z_k + conj Z_{M-k})/2, O = (Z_k - conj Z_{M-k})/(2i), X_k = E + W^k O, X_{k+M} = E - W^k O
// (W = e^{-2 pi i/(2M)}), H = Re X - Im X.  Returns H_k and H_{k+M}.  Z padded (pix).
template <typename C, typename T>
__device__ __forceinline__ void realsplit_padded(const C* Z, int M, int k, C w, T& h0, T& h1) {
  const int km = (k == 0) ? 0 : M - k;
  const C z = Z[pix(k)];
  const C c = Z[pix(km)];
  const T ex = (T)0.5 * (z.x + c.x), ey = (T)0.5 * (z.y - c.y);    // E
  const T ox = (T)0.5 * (z.y + c.y), oy = (T)-0.5 * (z.x - c.x);   // O = (Z - conj C) / 2i
  const T wox = w.x * ox - w.y * oy, woy = w.x * oy + w.y * ox;    // W O
  h0 = (ex + wox) - (ey + woy);
  h1 = (ex - wox) - (ey - woy);
}

// Hartley unpack from a padded line (see hartley_pair).
template <typename C, typename T>
__device__ __forceinline__ void hartley_padded(const C* Z, int n, int k, T& ha, T& hb) {
  const int km = (k == 0) ? 0 : n - k;
  const C z = Z[pix(k)];
  const C w = Z[pix(km)];
  ha = (T)0.5 * ((z.x + w.x) - (z.y - w.y));
  hb = (T)0.5 * ((z.y + w.y) - (w.x - z.x));
}

// FFT policies used as kernel template arguments.  kPadded: the line lives in LDS in the padded in-place layout
// (element e at pix(e)) instead of linearly.
struct FFTRt {              // any n (mixed radix, runtime plan), nl interleaved lines
  static constexpr bool kPadded = false;
  FFTPlan pl;
  int nl;
  template <typename C>
  __device__ __forceinline__ C* run(C* a, C* b, const C* __restrict__ tw) const { return lds_fft<C>(a, b, nl, pl, tw); }
  template <typename C>
  __device__ __forceinline__ C* buffer(C* lds, C*, int) const { return lds; }
  __device__ __forceinline__ int n() const { return pl.n; }
  __device__ __forceinline__ int lines() const { return nl; }
};
struct FFTGlb {             // any n, line buffers in global scratch (slot per workgroup): lines beyond LDS
  static constexpr bool kPadded = false;
  FFTPlan pl;
  int nl;
  template <typename C>
  __device__ __forceinline__ C* run(C* a, C* b, const C* __restrict__ tw) const {
    return lds_fft<C, true>(a, b, nl, pl, tw);
  }
  template <typename C>
  __device__ __forceinline__ C* buffer(C*, C* g, int slot) const { return g + (size_t)slot * 2 * pl.n * nl; }
  __device__ __forceinline__ int n() const { return pl.n; }
  __device__ __forceinline__ int lines() const { return nl; }
};

template <int N, int NL>
struct FFTFx {              // compile-time power-of-two n, NL lines
  static constexpr bool kPadded = false;
  template <typename C>
  __device__ __forceinline__ C* buffer(C* lds, C*, int) const { return lds; }
  template <typename C>
  __device__ __forceinline__ C* run(C* a, C* b, const C* __restrict__ tw) const {
    return lds_fft_fixed<C, N, NL>(a, b, tw);
  }
  __device__ __forceinline__ int n() const { return N; }
  __device__ __forceinline__ int lines() const { return NL; }
};

// compile-time power-of-two N, ONE line transformed in place in the padded layout with NT threads (global twiddle
// table): rows whose Stockham ping-pong (2 lines) does not fit LDS -- fp64 ny = 8192 (C4's y extent), 136 KiB
template <int N, int NT>
struct FFTIp {
  static constexpr bool kPadded = true;
  template <typename C>
  __device__ __forceinline__ C* buffer(C* lds, C*, int) const { return lds; }
  template <typename C>
  __device__ __forceinline__ C* run(C* a, C*, const C* __restrict__ tw) const {
    lds_fft_inplace<C, N, 1, NT>(a, tw);
    return a;
  }
  __device__ __forceinline__ int n() const { return N; }
  __device__ __forceinline__ int lines() const { return 1; }
};
// position of element e of a one-line buffer under policy F, and the Hartley pair of its transform
template <class F>
__device__ __forceinline__ int fpos(int e) { return F::kPadded ? pix(e) : e; }

// Hartley unpack of line l at frequency k from the FFT Z of z = a + i b.
// DCT-II (scipy norm=None: y_k = 2 sum x_n cos(pi k (2n+1) / 2n)) of two real columns a, b that were
// packed as z = v_a + i v_b in Makhoul order (v[m] = x[2m], v[n-1-m] = x[2m+1]) and FFT'd into Z:
// V_a = (Z_k + conj Z_{n-k})/2, V_b = (Z_k - conj Z_{n-k})/(2i), y = 2 Re(w_k V), w_k = e^{-i pi k/(2n)}.
template <typename C, typename T>
__device__ __forceinline__ void dct_pair(const C* Z, int n, int nl, int k, int l, C w, T& ya, T& yb) {
  const int km = (k == 0) ? 0 : n - k;
  const C z = Z[(size_t)k * nl + l];
  const C c = Z[(size_t)km * nl + l];
  const T ax = (T)0.5 * (z.x + c.x), ay = (T)0.5 * (z.y - c.y);     // V_a
  const T bx = (T)0.5 * (z.y + c.y), by = (T)-0.5 * (z.x - c.x);    // V_b
  ya = (T)2 * (w.x * ax - w.y * ay);
  yb = (T)2 * (w.x * bx - w.y * by);
}
// Makhoul position of sample x in the packed DCT sequence (and its inverse map)
__device__ __forceinline__ int dct_perm(int x, int n) { return (x & 1) ? n - 1 - (x >> 1) : (x >> 1); }

template <typename C, typename T>
__device__ __forceinline__ void hartley_pair(const C* Z, int n, int nl, int k, int l, T& ha, T& hb) {
  const int km = (k == 0) ? 0 : n - k;
  const C z = Z[(size_t)k * nl + l];
  const C w = Z[(size_t)km * nl + l];
  ha = (T)0.5 * ((z.x + w.x) - (z.y - w.y));
  hb = (T)0.5 * ((z.y + w.y) - (w.x - z.x));
}
// the Hartley pair of a one-line buffer under policy F (linear or padded)
template <class F, typename C, typename T>
__device__ __forceinline__ void hartley_line(const C* Z, int n, int k, T& ha, T& hb) {
  if constexpr (F::kPadded) hartley_padded<C, T>(Z, n, k, ha, hb);
  else hartley_pair<C, T>(Z, n, 1, k, 0, ha, hb);
}

}  // namespace pdhg
