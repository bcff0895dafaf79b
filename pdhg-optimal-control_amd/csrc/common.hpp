// Common device-side types and helpers for the MI355X PDHG kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pdhg {

// raw bit vectors for the buffer load / store builtins
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

constexpr int kWave = 64;          // CDNA wavefront width
constexpr int kMaxPass = 24;       // max FFT passes in a plan
constexpr int kNumSums = 16;       // doubles of partial sums per workgroup

template <typename R> struct Cplx;
template <> struct Cplx<float> { using type = float2; };
template <> struct Cplx<double> { using type = double2; };
template <typename R> using cplx = typename Cplx<R>::type;

template <typename C> __device__ __forceinline__ C cmk(decltype(C::x) a, decltype(C::x) b) { C c; c.x = a; c.y = b; return c; }
template <typename C> __device__ __forceinline__ C cadd(C a, C b) { return cmk<C>(a.x + b.x, a.y + b.y); }
template <typename C> __device__ __forceinline__ C csub(C a, C b) { return cmk<C>(a.x - b.x, a.y - b.y); }
template <typename C> __device__ __forceinline__ C cmul(C a, C b) {
  return cmk<C>(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
// multiply by -i
template <typename C> __device__ __forceinline__ C cmul_mi(C a) { return cmk<C>(a.y, -a.x); }

// NaN-propagating max/min (jnp.maximum / jnp.minimum semantics; fmax would drop the NaN)
template <typename R> __device__ __forceinline__ R nmax(R a, R b) { return (a != a) ? a : ((b != b) ? b : (a > b ? a : b)); }
template <typename R> __device__ __forceinline__ R nmin(R a, R b) { return (a != a) ? a : ((b != b) ? b : (a < b ? a : b)); }
// v_rcp_f32 (1 ulp) for the Thomas pivots of the fp32 sweeps: the recurrences are contractive, so the ulp does
// not accumulate, and a correctly rounded 1/x (__frcp_rn) costs ~10 instructions (div_scale / fmas / fixup)
__device__ __forceinline__ float rcp_fast(float x) { return __builtin_amdgcn_rcpf(x); }
// jnp.minimum(hi, jnp.maximum(lo, x)) for constant bounds: the hardware min / max (which drop a NaN operand)
// and one NaN select, instead of two NaN-propagating selects each
template <typename R> __device__ __forceinline__ R nclamp(R x, R lo, R hi) {
  const R c = fmin(hi, fmax(lo, x));
  return (x != x) ? x : c;
}

// Device control block: loop control that never round-trips through the host.
constexpr int kHaltTail = 3;   // Ctrl::done: a speculative one-sub-iteration iteration stopped for the host (iterate())
struct Ctrl {
  int done;          // 0 running, 1 converged, 2 NaN, kHaltTail: halted before the rest of the dual loop
  int iters;         // outer iterations executed since the last reset
  int inner_done;    // dual loop of the current outer iteration has exited early
  int inner_count;   // dual sub-iterations executed in the current outer iteration
  int inner_total;   // dual sub-iterations executed since the last reset
  int cur;           // which rho/alp buffer set holds the state (0/1)
  int primal_valid;  // primal sums of the current outer iteration are valid
  int nan_seen;      // a NaN appeared in phi' or rho' (recorded even when the NaN stop is off)
  int first_nan;     // iteration (1-based, since the last reset) at which nan_seen was first set; 0: none
  int kstar;         // chunked dual loop (k_dual_multi_2d): the exit sub-iteration count k*
  int kstar_found;   // ... fixed by a chunk's finalize (reset by k_finalize_outer)
  int kstored;       // ... sub-iterations of the state the second buffer set holds after the last chunk
  int fold_ticket;   // k_fold_finalize_dual: workgroups done with their fold row (0 between launches)
  double err1, err2, err_inner;
  double s_dphi, s_phi_old, s_phi_new;   // finalized primal sums
  double row0_sq;                        // sum phi_0^2 of the fixed row 0 (written by set_state / init_state)
  double dual_sums[kNumSums];            // finalized sums of the last dual sub-iteration
  double outer_sums[kNumSums];           // finalized outer (initial vs final) dual sums
};

// Workgroup barrier that waits only for this wave's LDS operations (lgkmcnt), not for its
// outstanding global loads/stores: __syncthreads() emits s_waitcnt vmcnt(0) before s_barrier,
// which would drain register prefetches and pending stores at every FFT pass.
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Per-launch reductions: one row of kNumSums doubles per workgroup, reduced in
// a fixed order by a single-workgroup finalize kernel (deterministic, no atomics).
template <int NS>
__device__ __forceinline__ void block_reduce_store(double (&v)[NS], double* __restrict__ partials, int row) {
  __shared__ double red[16][NS > 0 ? NS : 1];
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x >> 6;
  const int nw = (blockDim.x + kWave - 1) >> 6;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    double x = v[s];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, kWave);
    v[s] = x;
  }
  if (lane == 0) {
#pragma unroll
    for (int s = 0; s < NS; ++s) red[wid][s] = v[s];
  }
  __syncthreads();
  if (threadIdx.x < NS) {
    double acc = 0.0;
    for (int w = 0; w < nw; ++w) acc += red[w][threadIdx.x];
    partials[(size_t)row * kNumSums + threadIdx.x] = acc;
  }
  __syncthreads();
}

// Cross-lane neighbour values over the whole 64-lane wave (GFX9 DPP wave shifts).
// lane_from_prev(v): lane i receives v of lane i-1 (lane 0 receives `edge`);
// lane_from_next(v): lane i receives v of lane i+1 (lane 63 receives `edge`).
__device__ __forceinline__ float lane_from_prev(float v, float edge) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, edge), __builtin_bit_cast(int, v),
                                                               0x138 /* wave_shr:1 */, 0xF, 0xF, false));
}
__device__ __forceinline__ float lane_from_next(float v, float edge) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, edge), __builtin_bit_cast(int, v),
                                                               0x130 /* wave_shl:1 */, 0xF, 0xF, false));
}

// XCD-aware block index remap: hardware deals consecutive workgroups round-robin
// over the 8 XCDs; remap so each XCD walks a contiguous range of logical blocks
// (neighbouring tiles share that XCD's L2).  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int b, int nblocks) {
  const int per = nblocks >> 3;            // blocks per XCD in the full part
  const int full = per << 3;
  if (b >= full) return b;                 // tail keeps identity mapping
  return (b & 7) * per + (b >> 3);
}

}  // namespace pdhg
