// Host side of libpdhg: context, FFT plans, launch sequencing, C ABI (include/pdhg.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/pdhg.h"
#include "kernels_1d.hpp"
#include "kernels_2d.hpp"
#include "kernels_2d_fast.hpp"
#include "kernels_dual_lds.hpp"
#include "kernels_dual_multi.hpp"
#include "kernels_common.hpp"
#include "kernels_xslab.hpp"
#include "kernels_xt_batch.hpp"
#include "kernels_xt_dma.hpp"
#include "kernels_thomas_chunk.hpp"
#include "kernels_fs_wide.hpp"
#include "kernels_fs16.hpp"
#include "kernels_xt_f64.hpp"

using namespace pdhg;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                           \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess) return fail(PDHG_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
  } while (0)
// stream-ordered host -> device copy inside Impl (Impl::h2d)
#define H2D(d, s, n)                        \
  do {                                      \
    const int rc_h2d_ = h2d((d), (s), (n)); \
    if (rc_h2d_) return rc_h2d_;            \
  } while (0)

constexpr size_t kLdsBytes = 160 * 1024;

FFTPlan make_plan(int n, bool& ok) {
  FFTPlan pl{};
  pl.n = n;
  pl.pow2 = (n > 0) && ((n & (n - 1)) == 0);
  int m = n, np = 0;
  ok = true;
  auto push = [&](int r) {
    if (np >= kMaxPass) { ok = false; return; }
    pl.radix[np++] = r;
  };
  for (int r : {16, 8, 4, 2})
    while (m % r == 0 && m > 1) { push(r); m /= r; }
  while (m % 3 == 0) { push(3); m /= 3; }
  for (int f = 5; m > 1; f += 2)
    while (m % f == 0) { push(f); m /= f; }
  pl.npass = np;
  return pl;
}

template <typename R>
std::vector<cplx<R>> twiddles(int n) {
  std::vector<cplx<R>> t(n);
  for (int k = 0; k < n; ++k) {
    const double a = -2.0 * M_PI * (double)k / (double)n;
    t[k].x = (R)std::cos(a);
    t[k].y = (R)std::sin(a);
  }
  return t;
}

struct ProfEntry {
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
  size_t used = 0;
};

struct ImplBase {
  int device = 0;   // every entry point selects it before touching the context (dispatch)
  virtual ~ImplBase() {}
};

// handle tags: a pdhg_ctx* and a pdhg_multi* both start with one; an entry point rejects the other kind
constexpr uint32_t kCtxMagic = 0x50444843u;    // "PDHC"
constexpr uint32_t kMultiMagic = 0x5044484du;  // "PDHM"

template <typename R>
struct Impl : ImplBase {
  using C = cplx<R>;
  using Real = R;
  pdhg_problem pb{};
  hipStream_t stream = nullptr;
  KP<R> kp{};
  FFTPlan plx{}, ply{};
  C* twx = nullptr;
  C* twy = nullptr;
  std::vector<void*> allocs;
  // PDHG_ALLOC: "contig" / "none" override the default (contiguous planes for fp32 2-D contexts only)
  int alloc_mode = [] {
    const char* e = getenv("PDHG_ALLOC");
    return !e ? 0 : !strcmp(e, "contig") ? 1 : !strcmp(e, "none") ? -1 : 0;
  }();
  int n_contig_fail = 0;   // contiguous requests that fell back to hipMalloc
  size_t dev_bytes = 0;
  int na = 0, n_dead = 0;
  bool two_sets = false;
  double row0_sq = 0.0;
  // launch geometry
  int NT2 = 512;
  int gx1 = 0, gx4 = 0, g4 = 1, gx5 = 0, g5 = 1, g_outer = 1;
  int head_xrun = 4;   // x rows per workgroup of the head form's chunk passes (PDHG_HEAD_XRUN)
  int nt_row = 256;   // threads of the generic 2-D row kernels (k_res_fwdy_2d, k_invy_update_2d)
  int rows_var = 0;                       // row-kernel shape variant (see with_fast_rows)
  // fp64 fused residual threads at ny = 4096 (PDHG_RES64_NT=1024: GPT = 1, 128 VGPRs + 108 B of spills; interleaved
  // A/B at C3 fp64, round 5: 17.1 vs 15.5 ms, so 512 stays)
  int res64_nt = 512;
  int half_nt = 3;                        // ny = 4096 row kernels with 512 threads (bit 0 residual, bit 1 update)
  int upd_pf = 4;                         // update kernel (512 threads): old-phi row pairs in flight (1..4)
  bool fast_dual = false;                 // fp32 time-marching float4 dual kernel (k_dual_fast_2d)
  // rho_alp_iters > 1 loops that exit after one sub-iteration (most of C2's marching iterations): no outer-sum
  // pass, the sub-iteration-0 sums are the outer ones (env PDHG_K1_OUTER=0: always the pass)
  bool k1_outer = true;
  // dual sub-iterations with a folded partial table: fold + finalize in one launch (k_fold_finalize_dual; env
  // PDHG_FOLD_FIN=0: two launches)
  bool fold_fin = false;
  bool dual_head = false;    // ... below 2^25 points: sub-iteration 0 alone, the rest in chunks (kernels_dual_multi.hpp)
  bool spec_ok = false;      // iterate() may use the speculative one-sub-iteration schedule (head form, PDHG_SPEC)
  bool fin_merge = true;     // ... with its dual and outer finalizes in one launch (PDHG_FIN_MERGE=0: two)
  bool outer_merged = false; // launch_dual merged this iteration's outer finalize: launch_outer skips it
  bool spec = false;         // ... and uses it now (launch_dual / launch_outer / the captured graph)
  long long spec_iters = 0, spec_halts = 0;   // iterations enqueued speculatively / halts (path_info, tests)
  bool dual_multi = false;   // rho_alp_iters > 1: the dual loop in chunks of sub-iterations (kernels_dual_multi.hpp)
  static constexpr int kMultiSub = 5;     // sub-iterations one chunk pass runs
  int NTd = 256, gxd = 0, gyd = 0, gzd = 0, jchunk_d = 1;
  int dual_rx = 0;   // > 0: k_dual_lds_2d with dual_rx x rows per workgroup (x neighbours through LDS)
  int dual_one = 1;   // row-per-thread dual with one time row per workgroup: k_dual_fast_2d<.., ONE> (no prefetch)
  int dual_ypl = 4;  // y per lane of k_dual_lds_2d (fp64: 4 or 2)
  // fused residual: the dual sweep also forms the next primal's residual rows (k_dual_lds_2d FR), the
  // residual kernel only completes the tile-edge terms and transforms (k_res_fwdy_fused_2d)
  bool fuse_res = false;
  int gz_1d = 1, jchunk_1d = 1;   // 1-D fused residual (k_dual_1d_fr): time chunks of the dual sweep
  bool res_valid = false;   // p.res / p.ey hold the residual of the current (rho, alp)
  int n_cu = 256;           // compute units (persistent grids)
  size_t lds_res = 0, lds_xt = 0;
  // fast row kernels (fp32, power-of-two ny): RW rows per workgroup, NTf threads
  bool fast_rows = false;
  bool glb_line = false;          // 1-D line FFTs over global scratch (nx beyond LDS)
  bool ip_rows = false;           // fp64 ny = 8192: generic row kernels on one padded in-place line (FFTIp)
  bool fourstep = false;          // fp32 1-D nx = 65536: four-step DHT over 16 + 9 workgroups per row pair
  bool t1_xt = true;              // T = 1 windows: carry-free x transform (k_precond_x_t1_2d; env PDHG_T1_XT=0 off)
  C* tw256 = nullptr;             // W_256 table of the four-step stages
  bool half_real = false;         // 2-D nx = 8192: one real column per x-transform block
  int nt1d = 256;                 // 1-D residual / update block size (1024 on the global-scratch path)
  bool fast_xt = false;
  bool ws_xt = false;             // warp-specialised variant (k_precond_xt_ws_2d)            // fp32 power-of-two nx: k_precond_xt_fast_2d
  bool batch_xt = false;          // row-batched variant (k_precond_xt_batch_2d: 4 rows per transform, 1024 threads)
  size_t lds_batch_xt = 0;
  int xt_rpre = 0;
  bool xt_pair = false;           // batched x transform as 2 rows x 512 threads, two workgroups per CU
  bool xt_dma = false;            // x transform with the rows staged HBM -> LDS by DMA (k_precond_xt_dma_2d)
  bool xt_dma_hr = false;         // ... its half-real form at nx = 8192 (C4)
  bool t1_xt64 = false;           // fp64 T = 1 windows: k_precond_x_t1_2d<..., double> (shares PDHG_T1_XT)
  // fp64 unfused residual's threads at ny = 2048: 256 on one-row windows (two 4-wave workgroups per CU, 225 VGPRs;
  // C2's T = 1 residual 54 -> 47 us), 512 otherwise (C2's T = 100 unfused residual 4.66 vs 4.94 ms at 256)
  int res64_nt2048 = 512;
  int upd_t1 = 0;                 // fp64 ny = 2048 update on one-row windows: 256 threads + G16 seeds (2: PF 2, 1: PF 4)
  bool t1_g16 = true;             // ... with the later passes' twiddle seeds from global memory (PDHG_T1_G16=0: all in LDS)
  bool f64_xt = false;            // fp64 nx = 4096: in-place line + register carries (k_precond_xt_f64_2d)
  int xt64_var = 0;               // nx = 2048 shape of it (threads, b' in registers or LDS)
  bool thomas_chunk = false;      // 1-D: t-solve in chunks of 32 rows (k_thomas_chunk_1d)
  bool fs_wide = true;            // four-step DHT with 64-column / 32-row tiles (k_fs1w_1d / k_fs2w_1d)
  int f16_group = 16;             // rows n1 per load group of k_f16a_fwd_1d (PDHG_F16_GROUP: 4, 8, 16; 16 measured best)
  bool fs16 = false;              // 16 x 4096 split with a chunk-major spectrum (kernels_fs16.hpp)
  size_t lds_fast_xt = 0;
  int RWf = 8, NTf = 1024, g_fast_upd = 1;
  size_t lds_fast = 0, lds_fast_tw = 0;
  bool res64 = false;      // fp64 residual and update through the fast row kernels (4-row groups)
  bool upd8192 = false;    // fp64 ny = 8192, half-real x: update through the fast row kernel on 2-row tasks
  bool tc_spec = false;    // fp64 C3: residual spectrum in task order (KP::rspec)
  bool to_c4 = false;      // C4 (half-real x blocks): fused residual in task order + k_res_fwdy_fused_transpose_2d
  size_t lds_res64 = 0, lds_upd64 = 0;
  size_t partial_rows = 0;
  static constexpr int kFoldRows = 64;   // rows of the first fold level (k_fold_partials) after the table
  double* fold_out = nullptr;
  double* prim_partials = nullptr;   // the update's partial rows when the speculative finalize merges the primal's
  int prim_merged_rows = 0;          // > 0: launch_primal left its finalize to k_finalize_dual_outer (rows to reduce)
  bool primal_done = false;
  int stop_conv = 1, stop_nan = 1;   // reference stop rules (utils_pdhg_solver.py:74-80)
  // profiling
  bool prof = false;
  std::map<std::string, ProfEntry> prof_ev;
  int* h_done = nullptr;   // pinned
  bool own_stream = true;
  // t-slab decomposition (multi-GPU): this context owns unknown rows [slab_j0, slab_j0 + T) of slab_Tg
  bool slab = false;
  int slab_j0 = 0, slab_Tg = 0;
  size_t Mspec = 0;          // spectral plane (work row) size
  R* halo_rho = nullptr;     // rho row j0+T from the next slab
  R* carry_y = nullptr;      // backward right carry (spectral plane)
  R* dsbuf = nullptr;        // [D, S1] exchange planes of this slab (2 x Mspec)
  int* long_pos = nullptr;   // neighbour exchange: per mode, index in the long-range list or -1
  int* long_idx = nullptr;   // the long-range modes (long_K of them)
  int long_K = -1;           // -1: not classified yet
  // x-slab decomposition (multi-GPU for T = 1 marching windows): this context owns global x rows
  // [xs_x0, xs_x0 + xs_nloc) of xs_nxg; its spatial arrays hold nx = xs_nloc + 16 rows (kernels_xslab.hpp)
  bool xslab = false;
  int xs_rank = 0, xs_P = 1, xs_nxg = 0, xs_nloc = 0, xs_x0 = 0, xs_nbs = 0;
  R* colwork = nullptr;      // [T][nbs][nxg][B]: this rank's column blocks, whole x lines
  const R* lamy_base = nullptr;
  std::vector<double> xs_local;   // x coordinates of the nx local rows (ghost / padding rows wrap periodically)

  ~Impl() override {
    if (stream) hipStreamSynchronize(stream);
    drop_graph();
    for (void* p : allocs) hipFree(p);
    for (auto& kv : prof_ev)
      for (auto& e : kv.second.ev) {
        hipEventDestroy(e.first);
        hipEventDestroy(e.second);
      }
    if (h_done) hipHostFree(h_done);
    if (stream && own_stream) hipStreamDestroy(stream);
  }

  template <typename T>
  int alloc(T** p, size_t n) {
    void* q = nullptr;
    const size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
    // Large arrays of fp32 2-D contexts physically contiguous: with the default allocator the physical
    // placement of C3's 13 GB planes differs from context to context, and so did the dual / update times
    // (dual 30.3 - 35.4 ms across contexts, stable to 0.05 ms within one); contiguous planes ran 29.5 - 30.5.
    // The same placement made fp64 C3's generic residual 71 -> 91 ms and fp32 C1's update 0.12 -> 0.14 ms,
    // and C2 was neutral (interleaved A/B), hence fp32 2-D only.  Falls back to
    // hipMalloc (counted: path_info "contig_fail").
    const bool contig = alloc_mode > 0 || (alloc_mode == 0 && sizeof(R) == 4 && pb.ndim == 2);
    hipError_t e = hipErrorOutOfMemory;
    if (bytes >= ((size_t)64 << 20) && contig) {
      e = hipExtMallocWithFlags(&q, bytes, hipDeviceMallocContiguous);
      if (e != hipSuccess) {
        (void)hipGetLastError();
        n_contig_fail++;
      }
    }
    if (e != hipSuccess) e = hipMalloc(&q, bytes);
    if (e != hipSuccess) return fail(PDHG_ERR_NOMEM, "hipMalloc(%zu bytes) failed: %s", bytes, hipGetErrorString(e));
    allocs.push_back(q);
    dev_bytes += bytes;
    *p = static_cast<T*>(q);
    return PDHG_OK;
  }

  // Host -> device copies on the context's stream (stream-ordered): the stream is non-blocking, so a copy on the
  // legacy null stream (hipMemcpy / hipMemset) has no ordering guarantee with the kernels enqueued on it
  int h2d(void* dst, const void* src, size_t bytes) {
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    return PDHG_OK;
  }
  size_t plane() const { return (size_t)pb.nx * (size_t)pb.ny; }

  int setup() {
    const int nx = pb.nx, ny = pb.ny, T = pb.T;
    const int nxg = xslab ? xs_nxg : nx;   // length of the x transform (global nx for an x-slab)
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    HIP_TRY(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device));
    HIP_TRY(hipHostMalloc((void**)&h_done, sizeof(int), hipHostMallocDefault));
    const bool is2d = pb.ndim == 2;
    na = (pb.ndim == 1 || pb.egno == 3) ? 2 : 4;
    n_dead = (pb.ndim == 2 && pb.egno == 3) ? 2 : 0;
    two_sets = pb.rho_alp_iters > 1;
    bool ok1 = true, ok2 = true;
    plx = make_plan(nxg, ok1);
    if (is2d) ply = make_plan(ny, ok2);
    if (!ok1 || !ok2) return fail(PDHG_ERR_UNSUPPORTED, "FFT plan too deep for nx=%d ny=%d", nxg, ny);

    KP<R>& p = kp;
    p.egno = pb.egno;
    p.ndim = pb.ndim;
    p.bcx = pb.bc_x;
    p.bcy = pb.bc_y;
    p.nx = nx;
    p.ny = ny;
    p.T = T;
    p.na = na;
    p.inv_dx = (R)(1.0 / pb.dx);
    p.inv_dy = (R)(is2d ? 1.0 / pb.dy : 0.0);
    p.inv_dt = (R)(1.0 / pb.dt);
    p.inv_dx2 = (R)(1.0 / (pb.dx * pb.dx));
    p.inv_dy2 = (R)(is2d ? 1.0 / (pb.dy * pb.dy) : 0.0);
    p.epsl = (R)pb.epsl;
    p.c_over_dt = (R)(pb.c_on_rho / pb.dt);
    p.C = (R)pb.C;
    p.inv_n = (R)(1.0 / ((double)nxg * (double)ny));
    // t-Laplacian off-diagonal: Ct/dt^2 in 1-D (utils_precond.py:128-131); 2-D ignores Ct (:164-168)
    p.ae = (R)((is2d ? 1.0 : pb.Ct) / (pb.dt * pb.dt));

    const size_t csz = sizeof(C);
    if (is2d) {
      // spectral block width B: contiguous [nx][B] slabs; the x-transform workgroup holds
      // M = nx*B modes with 5*M*sizeof(R) bytes of LDS (FFT ping-pong + Thomas carries)
      const size_t cap = (sizeof(R) == 4) ? 8192 : 4096;
      int B = 16;
      while (B > 2 && (size_t)nxg * B > cap) B >>= 1;
      int nyp = 2;
      while (nyp < ny) nyp <<= 1;
      if (B > nyp) B = nyp;
      // fp64 nx = 512 / 1024 with T > 1: one column pair per block (B = 2) for the fp64 x kernel below (the generic
      // kernel would take B = 8 / 4 with its carries in global memory); T = 1 keeps the one-row kernel's B
      // (a t-slab takes the window's row count, so every slab of one window gets the same layout: a 1-row slab of a
      // longer window must not keep B = 8 / 4 while its neighbours exchange B = 2 carry planes)
      const bool f64_small = sizeof(R) == 8 && pb.bc_x == 0 && (slab ? slab_Tg : T) > 1 && (nxg == 1024 || nxg == 512) &&
                             ny % 2 == 0 && [] { const char* e = getenv("PDHG_XT64"); return !e || atoi(e) != 0; }();
      if (f64_small) B = 2;
      // fp32 nx = 8192 (C4): one real column per block, packed into a 4096-point FFT (half_real)
      // fp64 nx = 8192 (C4's grid in the reference's precision): the same half-real split in k_precond_xt_f64_2d<HR>
      half_real = nxg == 8192 && pb.bc_x == 0 && (sizeof(R) == 4 || !xslab);
      if (half_real) B = 1;
      // fp64 nx = 4096 (C3's grid in the reference's precision): k_precond_xt_f64_2d keeps the carries in
      // registers, so the column pair (B = 2) fits LDS although 5 M reals would not
      // (t-slab phases too: kernels_xt_f64.hpp)
      // fp64 nx = 2048 (C2's grid): the same kernel with b' in registers (BPR) instead of the generic runtime-radix
      // kernel's global carries (10.97 ms at C2, 0.15 of the HBM roofline, round 4)
      f64_xt = sizeof(R) == 8 && pb.bc_x == 0 &&
               (((nxg == 4096 || nxg == 2048) && B == 2) || (nxg == 8192 && half_real) || f64_small);
      if (const char* e = getenv("PDHG_XT64")) f64_xt = f64_xt && atoi(e) != 0;   // A/B: 0 = generic kernel
      if (const char* e = getenv("PDHG_XT64_VAR")) xt64_var = atoi(e);              // A/B: nx = 2048 shapes
      // fp64 one-row windows at a power-of-two nx: the carry-free transform needs only the padded lines
      t1_xt64 = sizeof(R) == 8 && T == 1 && pb.bc_x == 0 && !half_real && !slab && plx.pow2 &&
                nxg >= 512 && nxg <= 4096 && nxg * (B / 2) == (nxg == 4096 ? 4096 : 2048);
      if (const char* e = getenv("PDHG_T1_G16")) t1_g16 = atoi(e) != 0;   // A/B: the T = 1 x kernel's seed table
      res64_nt2048 = T == 1 ? 256 : 512;
      upd_t1 = T == 1 ? 2 : 0;   // steady marching iteration 0.2196 (512 threads) / 0.2150 (PF 4) / 0.2131 ms (PF 2)
      if (const char* e = getenv("PDHG_UPD_T1")) upd_t1 = T == 1 ? atoi(e) : 0;   // A/B: 0 = 512-thread update
      if (const char* e = getenv("PDHG_RES64_NT2048")) res64_nt2048 = atoi(e) == 256 ? 256 : 512;   // A/B
      if (!half_real && !f64_xt && (size_t)nxg * B > cap)
        return fail(PDHG_ERR_UNSUPPORTED, "nx=%d too large for the x-transform slab (max %zu in this precision)", nxg,
                    cap / 2);
      p.half_real = half_real ? 1 : 0;
      p.B = B;
      p.lB = 0;
      while ((1 << p.lB) < B) ++p.lB;
      p.nb = (ny + B - 1) / B;
      p.rows_per_wg = 2;
      lds_res = 2 * (size_t)ny * csz;
      const int nmodes = nxg * B;
      lds_xt = (size_t)5 * nmodes * sizeof(R);
      // fp64 ny = 8192 (C4's y extent in the reference's precision): the generic row kernels transform the row pair
      // in place in one padded line (FFTIp, 136 KiB) instead of a Stockham ping-pong of two (256 KiB)
      ip_rows = sizeof(R) == 8 && ny == 8192 && lds_res > kLdsBytes && !xslab;
      if (ip_rows) lds_res = (size_t)Pad<8192>::LINE * csz;
      // ... and the update through the fast row kernel on 2-row tasks when the x blocks are half-real (B = 1)
      upd8192 = ip_rows && half_real && nx % 2 == 0;
      if (const char* e = getenv("PDHG_UPD8192")) upd8192 = upd8192 && atoi(e) != 0;   // A/B: 0 = generic kernel
      if (upd8192) g_fast_upd = std::min((nx / 2) * T, 2048);
      if (lds_res > kLdsBytes) return fail(PDHG_ERR_UNSUPPORTED, "ny=%d exceeds the LDS row transform", ny);
      {   // generic row kernels: when the LDS admits few workgroups per CU (fp64 ny = 4096: one), wider
          // workgroups keep >= 16 waves per CU in flight for the residual's scattered loads
        const int wg = (int)std::max<size_t>(1, kLdsBytes / std::max<size_t>(lds_res, 1));
        nt_row = std::min(1024, 256 * std::max(1, 4 / wg));
      }
      NT2 = std::min(512, ((nmodes + 63) / 64) * 64);
      gx1 = ((nx + 1) / 2) * T;                      // row-pair tasks (flat grid)
      gx4 = (int)std::min<long long>((long long)gx1, 4096);
      g4 = 1;
      gx5 = (ny + 255) / 256;
      g5 = std::max(1, std::min(T * nx, 8192 / std::max(1, gx5)));
      if (const char* e = getenv("PDHG_DBG")) p.dbg = atoi(e);   // timing experiments only
      // tuning: k_dual_lds_2d step sync through neighbour counts instead of the block barrier.  Bitwise the same
      // results; measured (round 4, interleaved A/B at C3): fp32 dual 31.16 -> 31.85 ms, fp64 60.39 -> 60.39 ms,
      // so the barrier is not what bounds the sweep and the default stays the barrier
      if (const char* e = getenv("PDHG_DUAL_NBSYNC")) p.nbsync = atoi(e) != 0;
      if (const char* e = getenv("PDHG_T1_XT")) t1_xt = atoi(e) != 0;   // tuning override
      if (const char* e = getenv("PDHG_K1_OUTER")) k1_outer = atoi(e) != 0;   // tuning override
      if (const char* e = getenv("PDHG_FOLD_FIN")) fold_fin = atoi(e) != 0;   // tuning override
      // short windows (the reference's T = 1 marching default): few time rows per workgroup leave little to
      // pipeline over t, so occupancy decides.  Measured on C3's grid (bench --config c3w1/c3w4/c3w8): the
      // single-role x-transform kernel beats the warp-specialised one up to T = 8 at least (T = 1: 0.18 vs
      // 0.24 ms, T = 8: 0.79 vs 0.84 ms); the row-per-thread dual (146 VGPRs, 3 waves/SIMD) without the
      // fused residual beats the fused 8-row sweep (200 VGPRs, 2 waves/SIMD) at T = 1 (0.31 vs 0.41 ms),
      // ties at T = 4 and loses from T = 8 on.
      int short_t_xt = 16, short_t_dual = 3;
      if (const char* e = getenv("PDHG_SHORT_T_XT")) short_t_xt = atoi(e);   // tuning overrides (0: never)
      if (const char* e = getenv("PDHG_SHORT_T")) short_t_dual = atoi(e);
      const bool short_win = T < short_t_xt, short_dual = T < short_t_dual;
      if (half_real && sizeof(R) == 4) {
        fast_xt = true;
        ws_xt = true;
        // the LDS-DMA staged x transform on half-real blocks (k_precond_xt_dma_2d<4096, true>) for windows of >= 4
        // rows: c4w50 x transform 28.4 ms with the warp-specialised kernel (round 4, 1.9 TB/s)
        xt_dma_hr = T >= 4;
        if (const char* e = getenv("PDHG_XT_DMA_HR")) xt_dma_hr = atoi(e) != 0;   // A/B: 0 = warp-specialised
        lds_fast_xt = (size_t)(2 * (4096 + 4096 / 16) + 816 + 4096) * sizeof(C);   // + split twiddles
      } else if (sizeof(R) == 4 && plx.pow2 && nxg * (B / 2) == 4096 && nxg >= 512 && pb.bc_x == 0) {
        fast_xt = true;
        ws_xt = (nxg == 4096) && !short_win;   // the other widths spill registers in the warp-specialised form
        if (const char* e = getenv("PDHG_XT_WS")) ws_xt = atoi(e) != 0;   // tuning override
        // row-batched x transform (k_precond_xt_batch_2d): 4 rows per transform, 1024 threads.  Measured at C3
        // (nx = 4096, T = 200): 16.2 -> 14.5 ms against the warp-specialised kernel; at C2 (nx = 2048,
        // T = 100) 2.07 -> 1.82 ms against the single-role one.  nx = 1024 / 512 spill in it: not selected.
        batch_xt = (nxg == 4096 || nxg == 2048) && T >= 4;
        if (const char* e = getenv("PDHG_XT_BATCH")) batch_xt = atoi(e) != 0;   // tuning override
        if (const char* e = getenv("PDHG_XT_RPRE")) xt_rpre = atoi(e);           // tuning: rows prefetched across the FFT
        if (const char* e = getenv("PDHG_XT_PAIR")) xt_pair = atoi(e) != 0;      // tuning: 2 rows x 512 threads
        // LDS-DMA staged rows (k_precond_xt_dma_2d) at nx = 4096: C3 14.24 -> 13.52 ms
        xt_dma = nxg == 4096;
        if (const char* e = getenv("PDHG_XT_DMA")) xt_dma = atoi(e) != 0 && nxg == 4096;   // tuning override
        lds_batch_xt = (size_t)(4 * (4096 + 4096 / 16) + twlds_size(nxg)) * sizeof(C);
        // padded FFT buffer + theta, E, b' (float2 per item) + twiddle seeds (TwLds<nx>)
        lds_fast_xt = ws_xt ? (size_t)(2 * (4096 + 4096 / 16) + 816) * sizeof(C)
                            : (size_t)(4096 + 4096 / 16 + 3 * 4096 + 816) * sizeof(C);
      }
      // fp64: the row-per-thread time-marching dual (k_dual_fast_2d<EGNO, double>) instead of the generic
      // per-point kernel, which re-reads every phi_bar neighbour (fp64 C3: 248 GB fetched for 161 GB of reads).
      // Measured at fp64 C3 (same box, profiles/r04_ab_dual64_*.json): 52.7 vs 59.3 ms per dual, 6.61 vs 6.44
      // it/s.  PDHG_DUAL64=0 keeps the generic kernel.  The LDS-row and fused variants are fp32.
      const bool dual64_ok = sizeof(R) == 8 && ny % 256 == 0;
      bool dual64 = dual64_ok;
      if (const char* e = getenv("PDHG_DUAL64")) dual64 = dual64_ok && atoi(e) != 0;
      if ((sizeof(R) == 4 || dual64) && ny % 256 == 0) {
        fast_dual = true;
        // x rows through LDS (k_dual_lds_2d) for the fused-residual sweep; a context created for
        // rho_alp_iters > 1 (no fused residual) sweeps row-per-thread: measured at C3 with rho_alp_iters = 10,
        // k_dual_fast_2d 25.7 ms per sub-iteration against 38.1 for k_dual_lds_2d (2 waves per SIMD)
        // fp64 (k_dual_lds_2d<EGNO, 8, false, double>, 230 VGPRs, no spill): the phi_bar x neighbours through LDS
        // instead of the row-per-thread kernel's 1.25x re-reads from L2 (fp64 C3: 200 GB fetched for 161 GB of reads)
        dual_rx = (nx % 8 == 0 && !short_dual && !two_sets) ? 8 : 0;
        if (const char* e = getenv("PDHG_DUAL_RX")) {   // tuning override: 0 = row-per-thread kernel
          const int v = atoi(e);
          if (v == 0 || (((sizeof(R) == 4 && (v == 4 || v == 16)) || v == 8) && nx % v == 0)) dual_rx = v;
        }
        if (const char* e = getenv("PDHG_DUAL_YPL"))   // tuning: fp64 LDS dual with 2 y per lane
          if (sizeof(R) == 8 && dual_rx == 8 && atoi(e) == 2) dual_ypl = 2;
        if (const char* e = getenv("PDHG_DUAL_ONE")) dual_one = atoi(e);   // A/B: 0 marching form, 2 (fp64) 4 waves/SIMD
        NTd = dual_rx ? dual_rx * 64 : std::min(256, ny / 4);
        gxd = dual_rx ? nx / dual_rx : nx;
        gyd = dual_rx ? ny / (64 * dual_ypl) : (ny / 4 + NTd - 1) / NTd;
        const int nJ0 = std::max(1, std::min(T, (2048 + gxd * gyd - 1) / (gxd * gyd)));
        jchunk_d = (T + nJ0 - 1) / nJ0;
        gzd = (T + jchunk_d - 1) / jchunk_d;
      }
      if (const char* e = getenv("PDHG_ROWS_VAR")) rows_var = atoi(e);   // tuning override
      if (const char* e = getenv("PDHG_HALF_NT")) half_nt = atoi(e);     // tuning: 1 fused residual, 2 update
      if (const char* e = getenv("PDHG_RES64_NT")) res64_nt = atoi(e) == 1024 ? 1024 : 512;   // tuning
      if (const char* e = getenv("PDHG_UPD_PF")) upd_pf = atoi(e);       // tuning: update prefetch depth
      if (sizeof(R) == 4 && ply.pow2 && ny >= 256 && ny <= 8192) {
        RWf = (ny == 8192) ? 4 : 8;
        NTf = std::min(1024, ny / 4);
        if (rows_var == 1 && (ny == 4096 || ny == 2048)) {   // 4 rows / block, 2 blocks per CU
          RWf = 4;
          NTf = ny / 8;
        }
        if (nx % RWf == 0 && (RWf * B) % 4 == 0) {
          fast_rows = true;
          // residual task tiles of 8 time rows x 4 row groups (rows past the last whole tile run untiled)
          p.tile_j = ((nx / RWf) % 4 == 0) ? 8 : 1;
          if (const char* e = getenv("PDHG_TILE_J")) {   // tuning override
            const int v = atoi(e);
            if (v >= 1 && (v == 1 || (nx / RWf) % 4 == 0)) p.tile_j = v;
          }
          lds_fast = (size_t)(RWf / 2) * (ny + ny / 16) * sizeof(C);
          // + the twiddle-seed table of the persistent kernels (fused residual, update; ny <= 4096)
          lds_fast_tw = lds_fast + (ny <= 4096 ? (size_t)twlds_size(ny) * sizeof(C) : 0);
          g_fast_upd = std::min((nx / RWf) * T, 2048);
        }
      }
      // fp64 residual: the fast row kernel on 4-row groups (2 complex lines of 4096 doubles = 136 KiB of LDS),
      // rows read once per group over the sliding 3-row window, instead of the generic row-pair kernel's
      // per-point neighbour re-reads (fp64 C3: 204 GB moved against 80.5 GB algorithmic)
      if (sizeof(R) == 8 && ply.pow2 && (ny == 2048 || ny == 4096) && nx % 4 == 0) {
        res64 = true;
        if (const char* e = getenv("PDHG_RES64")) res64 = atoi(e) != 0;   // tuning override
        if (res64) {
          p.tile_j = ((nx / 4) % 4 == 0) ? 8 : 1;
          lds_res64 = (size_t)2 * (ny + ny / 16) * sizeof(C);
          // the update through the fast row kernel too: + the twiddle-seed table (152 KiB at ny = 4096)
          lds_upd64 = lds_res64 + (size_t)twlds_size(ny) * sizeof(C);
          g_fast_upd = std::min((nx / 4) * T, 2048);
        }
      }
      // fp64 C3 shape: the residual spectrum handed to the x transform in task order (p.rspec; one contiguous run per
      // 4-row task instead of 64-B chunks of the blocked layout), the x kernel's forward sweep reading it
      // Interleaved A/B (round 5): C3's T = 200 118.8 -> 118.3 ms; its 25-row slab share (8 GPUs) 16.05 -> 16.35 ms
      // (the x kernel's 64-B reads cost relatively more on short windows), so windows of >= 100 rows only
      // (never on one-row windows: the T = 1 x kernel reads the blocked work buffer)
      const bool tc_ok = sizeof(R) == 8 && res64 && ny == 4096 && f64_xt && !half_real && nxg == 4096 && B == 2 &&
                         !xslab && T > 1 && !t1_xt64;
      tc_spec = tc_ok && T >= 100;
      if (const char* e = getenv("PDHG_TC_SPEC")) tc_spec = tc_ok && atoi(e) != 0;   // A/B: 0 blocked, 1 task order
      // fused residual: fp32 fast kernels with 8-row tiles on both sides, rho_alp_iters = 1 (in place),
      // periodic bc, egno 1/2, single context; each dual workgroup must march the whole window (the
      // residual row j needs rho'_{j+1}), so only grids with enough (x, y) tiles to fill the chip
      // (PDHG_FUSE_RES=1 forces it for any eligible size, =0 turns it off)
      // fp64: the sweep k_dual_lds_2d<.., double, YPL = 2> (128-column strips, 211 VGPRs) and the residual in
      // half-tile tasks of 4 rows (k_res_fwdy_fused_2d<.., 4, 512, double>, the lines + twiddles fill the LDS)
      // fp32 ny = 8192 (C4's y extent): the 4-row fast kernels, so the residual runs half-tile tasks as in fp64
      // fp64 ny = 8192 (C4): the row pairs of the generic kernels (ip_rows) for the unfused residual and the update,
      // the fused residual on quarter-tile tasks (one line of 8192 complex doubles)
      const bool fr_rows = sizeof(R) == 4 ? (fast_rows && (RWf == 8 || (RWf == 4 && ny == 8192)))
                                          : ((res64 && (ny == 4096 || ny == 2048)) || (ip_rows && ny == 8192));
      if (fast_dual && dual_rx == 8 && fr_rows && pb.bc_x == 0 && pb.bc_y == 0 && pb.egno != 3 && !two_sets &&
          !xslab) {
        // fp32 ny = 8192 (4-row half-tile tasks, 16-B chunks of the B = 1 spectrum): round 4 measured it neutral
        // (residual 31.2 -> 25.9 ms, dual 26.7 -> 31.3); with the XCD-ordered tasks (round 5, interleaved A/B at
        // c4w50) the fused residual runs 22.9 ms against 30.3 unfused, step 88.25 -> 85.64 ms: on by default
        fuse_res = gxd * gyd >= 1024;
        if (const char* e = getenv("PDHG_FUSE_RES")) fuse_res = atoi(e) != 0;
        if (fuse_res) {
          if (sizeof(R) == 8) {
            dual_ypl = 2;
            gyd = ny / 128;
          }
          jchunk_d = T;
          gzd = 1;
        }
      }
      // C4 (ny = 8192 with half-real x blocks, B = 1): the fused residual's task-order spectrum + a transpose into the
      // blocked layout instead of 16-B chunk stores (fp64 RW = 2 / fp32 RW = 4 tasks: 16-B elements)
      to_c4 = fuse_res && half_real && B == 1 && ny == 8192 && !xslab &&
              (sizeof(R) == 8 ? ip_rows : (fast_rows && RWf == 4)) && (nx % (sizeof(R) == 8 ? 64 : 128)) == 0;
      if (const char* e = getenv("PDHG_C4_TO")) to_c4 = to_c4 && atoi(e) != 0;   // A/B: 0 = blocked 16-B chunks
    } else {
      p.B = 1;
      p.lB = 0;
      p.nb = 1;
      p.rows_per_wg = 2;
      lds_res = 2 * (size_t)nx * csz;
      gx1 = (T + 1) / 2;
      gx4 = std::min(gx1, 2048);
      if (lds_res > kLdsBytes) {   // lines beyond LDS (C1: nx = 65536): Stockham passes over global scratch
        glb_line = true;
        lds_res = 0;
        nt1d = 1024;
        // fp32 nx = 65536 (C1): four-step DHT over 16 + 9 workgroups of 1024 threads per row pair instead of
        // one workgroup per pair (T = 400 gave 200 workgroups for 256 CUs): 1.41 -> 1.12 ms per iteration
        // fp64 nx = 65536: the same 16 x 4096 split (kernels_fs16.hpp on complex doubles) instead of the
        // generic Stockham passes over global scratch (fp64 C1: 3.9x the algorithmic bytes)
        fourstep = nx == 65536;
        if (const char* e = getenv("PDHG_FOURSTEP")) fourstep = fourstep && atoi(e) != 0;   // tuning override
        if (const char* e = getenv("PDHG_FS_WIDE")) fs_wide = atoi(e) != 0;                 // tuning override
        fs16 = fourstep;
        if (const char* e = getenv("PDHG_FS16")) fs16 = fs16 && atoi(e) != 0;               // tuning override
        if (sizeof(R) == 8 && !fs16) fourstep = false;   // the other four-step forms are fp32
        if (const char* e = getenv("PDHG_F16_GROUP")) f16_group = atoi(e);                   // tuning override
      }
      g4 = 1;
      gx5 = (nx + 255) / 256;
      g5 = std::max(1, std::min(T, 8192 / std::max(1, gx5)));
      // chunked t-solve: one wave per 32-row chunk of 64 modes (T <= 512, Ct != 0)
      thomas_chunk = pb.Ct != 0.0 && T <= 16 * 32;
      // fused 1-D residual (C1's 16 x 4096 path, rho_alp_iters = 1, periodic x): the dual sweep forms the residual
      // rows (k_dual_1d_fr), stage A reads them (k_f16a_fwd_fused_1d); 8 time chunks of the sweep
      fuse_res = fs16 && pb.bc_x == 0 && !two_sets && pb.egno != 3 && nx % 256 == 0;
      if (const char* e = getenv("PDHG_FUSE_RES1D")) fuse_res = fuse_res && atoi(e) != 0;   // A/B: 0 = unfused
      gz_1d = 8;
      if (const char* e = getenv("PDHG_FR1D_CHUNKS")) gz_1d = std::max(1, std::min(32, atoi(e)));   // tuning
      gz_1d = std::min(gz_1d, T);
      jchunk_1d = (T + gz_1d - 1) / gz_1d;
      gz_1d = (T + jchunk_1d - 1) / jchunk_1d;
      if (const char* e = getenv("PDHG_THOMAS_CHUNK")) thomas_chunk = thomas_chunk && atoi(e) != 0;   // override
    }
    g_outer = 2048;
    if (const char* e = getenv("PDHG_G_OUTER")) g_outer = std::max(64, std::min(4096, atoi(e)));   // tuning override
    if (const char* e = getenv("PDHG_HEAD_XRUN")) head_xrun = std::max(1, atoi(e));               // tuning override
    // rho_alp_iters > 1 on the row-per-thread dual grid, single contexts: the dual loop in chunk passes of
    // kMultiSub sub-iterations in registers (+ a final pass when the exit falls inside a chunk)
    // Only where a pass is bandwidth-bound: C2's T = 1 marching windows (4 M points, the loop exiting after a few
    // sub-iterations) ran 30.5 s with the chunks against 22.9 s per sub-iteration (launch-bound: the chunk computes
    // 5 sub-iterations and the final pass re-runs k*), C2's T = 100 window 22.1 vs 10.5 it/s and C3 5.80 vs
    // 3.00 it/s (round 4, fp64 / fp32, rho_alp_iters = 10)
    const bool multi_ok = is2d && two_sets && fast_dual && dual_rx == 0 && !slab && !xslab &&
                          pb.rho_alp_iters <= kDualMultiMax;
    dual_multi = multi_ok && (double)T * nx * ny >= (double)(1 << 25);
    if (const char* e = getenv("PDHG_DUAL_MULTI")) dual_multi = multi_ok && atoi(e) != 0;   // A/B, tests
    // below that: the head form (sub-iteration 0 per-sub-iteration, the rest in chunks).  C2's marching windows exit
    // after sub-iteration 0 in nearly every outer iteration, where 18 returning launches cost ~0.2 ms
    dual_head = multi_ok && !dual_multi;
    if (const char* e = getenv("PDHG_DUAL_HEAD")) dual_head = multi_ok && !dual_multi && atoi(e) != 0;   // A/B, tests
    // the speculative schedule of iterate() needs the head form's one-sub-iteration shortcuts (k1_outer) and the
    // two-launch fold / finalize (the halt flag is set by k_finalize_dual)
    spec_ok = dual_head && k1_outer && !fold_fin;
    if (const char* e = getenv("PDHG_SPEC")) spec_ok = spec_ok && atoi(e) != 0;   // A/B, tests
    if (const char* e = getenv("PDHG_FIN_MERGE")) fin_merge = atoi(e) != 0;        // A/B, tests
    partial_rows = std::max<size_t>({(size_t)gx4 * g4, (size_t)gx5 * g5, (size_t)g_outer, (size_t)g_fast_upd,
                                     (size_t)gxd * gyd * (gzd + 1), fourstep ? (size_t)9 * ((T + 1) / 2) : 1, 1,
                                     (dual_multi || dual_head) ? (size_t)kMultiSub * gxd * gyd * gzd : (size_t)1});
    p.slab = slab ? 1 : 0;
    p.j0 = slab ? slab_j0 : 0;
    p.Tg = slab ? slab_Tg : T;
    p.last_slab = (p.j0 + T == p.Tg) ? 1 : 0;
    p.xt_phase = 0;
    p.row_base = 0;
    p.row_cnt = T;
    p.xl0 = xslab ? 8 : 0;
    p.xl1 = xslab ? 8 + xs_nloc : nx;
    if (xslab) {
      // the row kernels that skip the ghost / padding rows: fp32 fast rows (ny in [256, 8192]), fp64 4-row kernels
      if (!(is2d && (sizeof(R) == 4 ? fast_rows : res64) && fast_dual && (pb.bc_x == 0 || pb.bc_x == 1) &&
            pb.bc_y == 0))
        return fail(PDHG_ERR_UNSUPPORTED, "x-slab decomposition needs ndim 2, bc (0,0) or (1,0) and a power-of-two ny "
                                          "in [256, 8192] (fp32) or ny = 2048 / 4096 (fp64) (fast row and dual kernels)");
      if (p.nb % xs_P) return fail(PDHG_ERR_UNSUPPORTED, "%d column blocks do not split over %d ranks", p.nb, xs_P);
      xs_nbs = p.nb / xs_P;
    }
    // t-slab phases: the fast DHT x kernels (power-of-two nx 512 - 8192), the fp64 x kernel (nx = 4096, and 8192
    // half-real) or the generic runtime-radix kernel (any nx, the DCT of egno 3's bc (1, 0)).  fp32 needs the
    // fast row kernels; fp64 splits the residual's halo row off with the 4-row kernels (ny 2048 / 4096) and runs
    // the generic row kernels over the whole slab after the halo otherwise
    if (slab && !(is2d && (fast_rows || sizeof(R) == 8)))
      return fail(PDHG_ERR_UNSUPPORTED, "t-slab decomposition needs ndim 2 and, in fp32, a power-of-two ny in "
                                        "[256, 8192] (fast row kernels)");

    // ---- device buffers ----
    const size_t npl = plane();
    int rc;
    if ((rc = alloc(&p.phi, (size_t)(T + 1) * npl))) return rc;
    if ((rc = alloc(&p.phibar, (size_t)(T + 1) * npl))) return rc;
    const size_t nwork = is2d ? (size_t)T * p.nb * nx * p.B : (size_t)T * nx;
    if ((rc = alloc(&p.work, nwork))) return rc;
    for (int s = 0; s < (two_sets ? 2 : 1); ++s) {
      if ((rc = alloc(&p.rho[s], (size_t)T * npl))) return rc;
      for (int a = 0; a < na; ++a)
        if ((rc = alloc(&p.alp[s][a], (size_t)T * npl))) return rc;
    }
    if (!two_sets) {
      p.rho[1] = p.rho[0];
      for (int a = 0; a < 4; ++a) p.alp[1][a] = p.alp[0][a];
    }
    for (int a = na; a < 4; ++a) p.alp[0][a] = p.alp[1][a] = nullptr;
    // rows: the kernels' partials, the fold's rows, and the update's partials of a speculative iteration (kept for the
    // merged finalize: the dual reuses the first region)
    if ((rc = alloc(&p.partials, (2 * partial_rows + kFoldRows) * kNumSums))) return rc;
    fold_out = p.partials + partial_rows * kNumSums;
    prim_partials = fold_out + kFoldRows * kNumSums;
    if ((rc = alloc(&p.ctrl, 1))) return rc;
    if (glb_line) {   // 2 lines of nx complex per concurrent workgroup (gx1 >= gx4)
      C* g = nullptr;
      if ((rc = alloc(&g, (size_t)gx1 * 2 * nx))) return rc;
      p.gscr = g;
    }
    p.res = p.ex = p.ey = nullptr;
    p.rspec = nullptr;
    if (fuse_res && is2d) {
      if ((rc = alloc(&p.res, (size_t)T * npl))) return rc;
      if ((rc = alloc(&p.ex, (size_t)T * (nx / 8) * 2 * ny))) return rc;
      if ((rc = alloc(&p.ey, (size_t)T * nx * (ny / (64 * dual_ypl)) * 2))) return rc;
    } else if (fuse_res) {   // 1-D: residual rows + the wave-edge terms [2][T][nx/64]
      if ((rc = alloc(&p.res, (size_t)T * npl))) return rc;
      if ((rc = alloc(&p.ex, (size_t)2 * T * (nx / 64)))) return rc;
    }
    // the task-order spectrum reuses the fused residual's R plane: a task's spectrum run [x0 rows, all ky] is exactly
    // the region its R rows occupy, and the residual kernel holds those rows in registers before it stores the run
    if (tc_spec) {
      if (fuse_res) p.rspec = p.res;
      else if ((rc = alloc(&p.rspec, nwork))) return rc;
    }
    if (xslab && (rc = alloc(&colwork, (size_t)T * xs_nbs * nxg * p.B))) return rc;
    if (slab) {
      Mspec = (size_t)p.nb * nx * p.B;
      if ((rc = alloc(&halo_rho, npl))) return rc;
      if ((rc = alloc(&carry_y, Mspec))) return rc;
      if ((rc = alloc(&dsbuf, 2 * Mspec))) return rc;
      HIP_TRY(hipMemsetAsync(halo_rho, 0, npl * sizeof(R), stream));
      HIP_TRY(hipMemsetAsync(carry_y, 0, Mspec * sizeof(R), stream));
      p.rho_halo = p.last_slab ? nullptr : halo_rho;
      p.carry_y = carry_y;
    }
    HIP_TRY(hipMemsetAsync(p.ctrl, 0, sizeof(Ctrl), stream));

    // ---- coefficient / symbol tables (host fp64 -> R) ----
    std::vector<R> ax(nx), ay(std::max(ny, 1)), lamx(nxg), d0(nxg);
    for (int i = 0; i < nx; ++i) {
      const double x = pb.xs[i];
      ax[i] = (R)(pb.egno == 3 ? x : (x - 1.0) * (x - 1.0) + 0.1);   // set_fns.py:145 / :117-118 / :98
    }
    if (is2d)
      for (int i = 0; i < ny; ++i) {
        const double y = pb.ys[i];
        ay[i] = (R)((y - 1.0) * (y - 1.0) + 0.1);
      }
    // Laplacian symbol = FFT of the periodic stencil (utils_precond.py:42-71), real part.
    // bc (1,0) (egno 3): fv = fft_y(dct_x(lap)) = DCT-II(x stencil)[kx] + 2 cos(pi kx/2nx) * lam_y[ky]
    // -- the reference transforms the periodic stencil array with the DCT, and DCT-II(e_0) = 2 cos(.)
    const bool dct_x = is2d && pb.bc_x == 1;
    std::vector<R> cx(nxg, (R)1);
    std::vector<C> dctw;
    for (int k = 0; k < nxg; ++k) {
      double l = -2.0 * (1.0 - std::cos(2.0 * M_PI * k / nxg)) / (pb.dx * pb.dx);
      if (dct_x) {
        auto c2 = [&](int n) { return 2.0 * std::cos(M_PI * k * (2.0 * n + 1.0) / (2.0 * nxg)); };
        l = (-2.0 * c2(0) + c2(1) + c2(nxg - 1)) / (pb.dx * pb.dx);
        cx[k] = (R)c2(0);
      }
      lamx[k] = (R)l;
      d0[k] = (R)std::pow(pb.C - l, pb.pow_);   // 1-D thomas_b = (C - fv)^pow, :125-126
    }
    if (fs16) {   // chunk-major spectrum of kernels_fs16.hpp: mode k1 + 16 k2 at position 4096 k1 + k2
      std::vector<R> d0p(nxg);
      for (int k1 = 0; k1 < 16; ++k1)
        for (int k2 = 0; k2 < kF16N2; ++k2) d0p[(size_t)k1 * kF16N2 + k2] = d0[k1 + 16 * k2];
      d0.swap(d0p);
    }
    if (dct_x) {
      dctw.resize(nxg);
      for (int k = 0; k < nxg; ++k) {
        dctw[k].x = (R)std::cos(-M_PI * k / (2.0 * nxg));
        dctw[k].y = (R)std::sin(-M_PI * k / (2.0 * nxg));
      }
    }
    R *d_ax, *d_ay, *d_lamx, *d_lamy, *d_d0;
    if ((rc = alloc(&d_ax, nx))) return rc;
    if ((rc = alloc(&d_ay, std::max(ny, 1)))) return rc;
    if ((rc = alloc(&d_lamx, nxg))) return rc;
    if ((rc = alloc(&d_d0, nxg))) return rc;
    H2D(d_ax, ax.data(), nx * sizeof(R));
    H2D(d_ay, ay.data(), ay.size() * sizeof(R));
    H2D(d_lamx, lamx.data(), nxg * sizeof(R));
    H2D(d_d0, d0.data(), nxg * sizeof(R));
    const int nyp = is2d ? p.nb * p.B : 1;
    std::vector<R> lamy(nyp, (R)0);
    if (is2d)
      for (int k = 0; k < ny; ++k) lamy[k] = (R)(-2.0 * (1.0 - std::cos(2.0 * M_PI * k / ny)) / (pb.dy * pb.dy));
    if ((rc = alloc(&d_lamy, nyp))) return rc;
    H2D(d_lamy, lamy.data(), nyp * sizeof(R));
    {
      R* d_cx;
      if ((rc = alloc(&d_cx, nxg))) return rc;
      H2D(d_cx, cx.data(), nxg * sizeof(R));
      p.cx = d_cx;
      p.dctw = nullptr;
      if (dct_x) {
        C* d_w;
        if ((rc = alloc(&d_w, nxg))) return rc;
        H2D(d_w, dctw.data(), nxg * sizeof(C));
        p.dctw = d_w;
      }
    }
    p.ax = d_ax;
    p.ay = d_ay;
    p.lamx = d_lamx;
    p.lamy = d_lamy;
    lamy_base = d_lamy;
    p.d0_1d = d_d0;
    {
      auto t = twiddles<R>(nxg);
      if ((rc = alloc(&twx, nxg))) return rc;
      H2D(twx, t.data(), nxg * sizeof(C));
    }
    if (fourstep) {
      auto t = twiddles<R>(256);
      if ((rc = alloc(&tw256, 256))) return rc;
      H2D(tw256, t.data(), 256 * sizeof(C));
    }
    if (is2d) {
      auto t = twiddles<R>(ny);
      if ((rc = alloc(&twy, ny))) return rc;
      H2D(twy, t.data(), ny * sizeof(C));
    }
    return set_lds_attrs();
  }

  std::vector<const void*> lds_done;
  template <typename K>
  int ensure_lds(K kern, size_t bytes) {
    const void* f = reinterpret_cast<const void*>(kern);
    for (const void* q : lds_done)
      if (q == f) return PDHG_OK;
    HIP_TRY(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    lds_done.push_back(f);
    return PDHG_OK;
  }
  int set_lds_attrs() { return PDHG_OK; }

  // FFT policy dispatch: compile-time sizes for the hot power-of-two lengths (fp32),
  // runtime mixed-radix plan otherwise.
  template <typename Fn>
  int with_line_fft(const FFTPlan& pl, Fn&& fn) {
    if (glb_line) return fn(FFTGlb{pl, 1});   // 1-D lines beyond LDS
    if constexpr (sizeof(R) == 8) {
      if (ip_rows && &pl == &ply) return fn(FFTIp<8192, 1024>{});   // the row kernels' 1024 threads (nt_row)
    }
    if constexpr (sizeof(R) == 4) {
      if (pl.pow2) {
        switch (pl.n) {
          case 256: return fn(FFTFx<256, 1>{});
          case 512: return fn(FFTFx<512, 1>{});
          case 1024: return fn(FFTFx<1024, 1>{});
          case 2048: return fn(FFTFx<2048, 1>{});
          case 4096: return fn(FFTFx<4096, 1>{});
          case 8192: return fn(FFTFx<8192, 1>{});
          default: break;
        }
      }
    }
    return fn(FFTRt{pl, 1});
  }
  // fast row-kernel dispatch on ny (compile-time N, RW, NT)
  template <typename Fn>
  int with_fast_rows(Fn&& fn) {
    if constexpr (sizeof(R) == 4) {
      switch (pb.ny) {
        case 256: return fn(std::integral_constant<int, 256>{}, std::integral_constant<int, 8>{},
                            std::integral_constant<int, 64>{});
        case 512: return fn(std::integral_constant<int, 512>{}, std::integral_constant<int, 8>{},
                            std::integral_constant<int, 128>{});
        case 1024: return fn(std::integral_constant<int, 1024>{}, std::integral_constant<int, 8>{},
                             std::integral_constant<int, 256>{});
        case 2048:
          if (rows_var == 1)
            return fn(std::integral_constant<int, 2048>{}, std::integral_constant<int, 4>{},
                      std::integral_constant<int, 256>{});
          return fn(std::integral_constant<int, 2048>{}, std::integral_constant<int, 8>{},
                    std::integral_constant<int, 512>{});
        case 4096:
          if (rows_var == 1)
            return fn(std::integral_constant<int, 4096>{}, std::integral_constant<int, 4>{},
                      std::integral_constant<int, 512>{});
          return fn(std::integral_constant<int, 4096>{}, std::integral_constant<int, 8>{},
                    std::integral_constant<int, 1024>{});
        case 8192: return fn(std::integral_constant<int, 8192>{}, std::integral_constant<int, 4>{},
                             std::integral_constant<int, 1024>{});
        default: break;
      }
    }
    return fail(PDHG_ERR_UNSUPPORTED, "no fast row kernel for ny=%d", pb.ny);
  }

  template <typename Fn>
  int with_xt_fft(Fn&& fn) {
    const int nl = kp.B / 2;
    if constexpr (sizeof(R) == 4) {
      if (plx.pow2) {
        const int n = plx.n;
        if (n == 4096 && nl == 1) return fn(FFTFx<4096, 1>{});
        if (n == 2048 && nl == 2) return fn(FFTFx<2048, 2>{});
        if (n == 1024 && nl == 4) return fn(FFTFx<1024, 4>{});
        if (n == 512 && nl == 8) return fn(FFTFx<512, 8>{});
        if (n == 256 && nl == 8) return fn(FFTFx<256, 8>{});
      }
    }
    return fn(FFTRt{plx, nl});
  }

  // ---------------- profiling ----------------
  struct ProfScope {
    Impl* im;
    ProfEntry* e = nullptr;
    ProfScope(Impl* i, const char* cls) : im(i) {
      if (!im->prof) return;
      e = &im->prof_ev[cls];
      if (e->used == e->ev.size()) {
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        e->ev.push_back({a, b});
      }
      hipEventRecord(e->ev[e->used].first, im->stream);
    }
    ~ProfScope() {
      if (!e) return;
      hipEventRecord(e->ev[e->used].second, im->stream);
      e->used++;
    }
  };

  // the fused residual kernel over time rows [lo, hi) (launch_residual's fused branch)
  int launch_fused_residual(KP<R> p, int lo, int hi) {
    int rc = PDHG_OK;
    if constexpr (sizeof(R) == 8) {
      auto go = [&](auto Nc) {
        constexpr int N_ = decltype(Nc)::value;
        const dim3 g(std::min((pb.nx / 4) * (hi - lo), n_cu));   // persistent, one workgroup per CU (LDS)
        int r2;
        if constexpr (N_ == 4096) {
          if (res64_nt == 1024) {   // A/B: 16 waves per CU (GPT = 1)
            if (pb.egno == 1) {
              if ((r2 = ensure_lds(k_res_fwdy_fused_2d<1, N_, 4, 1024, double>, lds_upd64))) return r2;
              hipLaunchKernelGGL((k_res_fwdy_fused_2d<1, N_, 4, 1024, double>), g, dim3(1024), lds_upd64, stream, p, twy);
            } else {
              if ((r2 = ensure_lds(k_res_fwdy_fused_2d<2, N_, 4, 1024, double>, lds_upd64))) return r2;
              hipLaunchKernelGGL((k_res_fwdy_fused_2d<2, N_, 4, 1024, double>), g, dim3(1024), lds_upd64, stream, p, twy);
            }
            return (int)PDHG_OK;
          }
        }
        if (pb.egno == 1) {
          if ((r2 = ensure_lds(k_res_fwdy_fused_2d<1, N_, 4, 512, double>, lds_upd64))) return r2;
          hipLaunchKernelGGL((k_res_fwdy_fused_2d<1, N_, 4, 512, double>), g, dim3(512), lds_upd64, stream, p, twy);
        } else {
          if ((r2 = ensure_lds(k_res_fwdy_fused_2d<2, N_, 4, 512, double>, lds_upd64))) return r2;
          hipLaunchKernelGGL((k_res_fwdy_fused_2d<2, N_, 4, 512, double>), g, dim3(512), lds_upd64, stream, p, twy);
        }
        return (int)PDHG_OK;
      };
      if (pb.ny == 8192) {   // quarter-tile tasks: one padded line of 8192 complex doubles (+ the strip-edge terms)
        const dim3 g(std::min((pb.nx / 2) * (hi - lo), n_cu));
        const size_t lds = (size_t)Pad<8192>::LINE * sizeof(C);
        if (pb.egno == 1) {
          if ((rc = ensure_lds(k_res_fwdy_fused_2d<1, 8192, 2, 512, double>, lds))) return rc;
          hipLaunchKernelGGL((k_res_fwdy_fused_2d<1, 8192, 2, 512, double>), g, dim3(512), lds, stream, p, twy);
        } else {
          if ((rc = ensure_lds(k_res_fwdy_fused_2d<2, 8192, 2, 512, double>, lds))) return rc;
          hipLaunchKernelGGL((k_res_fwdy_fused_2d<2, 8192, 2, 512, double>), g, dim3(512), lds, stream, p, twy);
        }
      } else {
        rc = pb.ny == 4096 ? go(std::integral_constant<int, 4096>{}) : go(std::integral_constant<int, 2048>{});
      }
      if (rc) return rc;
      HIP_TRY(hipGetLastError());
      return PDHG_OK;
    }
    rc = with_fast_rows([&](auto Nc, auto RWc, auto NTc) {
      constexpr int N_ = decltype(Nc)::value, RW_ = decltype(RWc)::value, NT_ = decltype(NTc)::value;
      int r2;
      if constexpr (sizeof(R) == 4 && (RW_ == 8 || (RW_ == 4 && N_ == 8192)) && N_ % 256 == 0 &&
                    (N_ / 4) % NT_ == 0) {
        const dim3 g(std::min((pb.nx / RW_) * (hi - lo), n_cu));   // persistent, one workgroup per CU (LDS)
        auto go = [&](auto ntc) {
          constexpr int NTF = decltype(ntc)::value;
          int r3;
          if (pb.egno == 1) {
            if ((r3 = ensure_lds(k_res_fwdy_fused_2d<1, N_, RW_, NTF>, lds_fast_tw))) return r3;
            hipLaunchKernelGGL((k_res_fwdy_fused_2d<1, N_, RW_, NTF>), g, dim3(NTF), lds_fast_tw, stream, p, twy);
          } else {
            if ((r3 = ensure_lds(k_res_fwdy_fused_2d<2, N_, RW_, NTF>, lds_fast_tw))) return r3;
            hipLaunchKernelGGL((k_res_fwdy_fused_2d<2, N_, RW_, NTF>), g, dim3(NTF), lds_fast_tw, stream, p, twy);
          }
          return (int)PDHG_OK;
        };
        if constexpr (NT_ == 1024) {
          if (half_nt & 1) return go(std::integral_constant<int, 512>{});
        }
        return go(std::integral_constant<int, NT_>{});
      }
      return fail(PDHG_ERR_STATE, "fused residual without 8-row fast kernels (ny=%d)", pb.ny);
    });
    if (rc) return rc;
    HIP_TRY(hipGetLastError());
    return PDHG_OK;
  }

  // C4's task-order residual spectrum (p.rspec) of time rows [lo, hi) into the blocked layout of `work`
  int launch_spec_to_blocked(const KP<R>& p, int lo, int hi) {
    const int RWt = sizeof(R) == 8 ? 2 : 4, XQ = pb.nx / RWt, NK = p.nb;   // 16-B elements: RWt reals
    if (XQ % 32 || NK % 64) return fail(PDHG_ERR_STATE, "task-order transpose needs nx/%d %% 32 == 0", RWt);
    KP<R> q = p;
    q.row_base = lo;
    hipLaunchKernelGGL(k_res_fwdy_fused_transpose_2d<R>, dim3(NK / 64, XQ / 32, hi - lo), dim3(256), 0, stream, q,
                       XQ, NK);
    HIP_TRY(hipGetLastError());
    return PDHG_OK;
  }

  // residual + forward y transform over time rows [lo, hi) (2-D).  The generic kernels only run the
  // whole window (lo = 0, hi = T).
  int launch_residual(KP<R> p, int lo, int hi) {
    if (hi <= lo) return PDHG_OK;
    int rc = PDHG_OK;
    if (fuse_res && res_valid && (slab || (lo == 0 && hi == pb.T))) {
      ProfScope ps(this, "residual");
      // C4 (half-real x blocks, B = 1): the fused residual stores its spectrum in task order over the R rows it was
      // formed from (full 128-B lines instead of 16-B chunks of the blocked layout), and k_spec_to_blocked_2d
      // transposes it into the x kernel's blocked layout
      if (to_c4) p.rspec = p.res;
      // the task-order spectrum is stored over the R rows it was formed from (p.rspec == p.res): once the launch
      // that ends the window has run, R is gone until the next fused dual sweep forms it again
      if (p.rspec != nullptr && p.rspec == p.res && hi == pb.T) res_valid = false;
      p.row_base = lo;
      p.row_cnt = hi - lo;
      if ((rc = launch_fused_residual(p, lo, hi))) return rc;
      HIP_TRY(hipGetLastError());
      if (to_c4) return launch_spec_to_blocked(p, lo, hi);
      return PDHG_OK;
    }
    if constexpr (sizeof(R) == 8) {
      if (res64) {
        ProfScope ps(this, "residual");
        p.row_base = lo;
        p.row_cnt = hi - lo;
        auto go = [&](auto Nc, auto NTc) {
          // 1024 threads cap the fp64 rows at 128 VGPRs (spills); ny = 2048 A/B: 256 threads (2 workgroups per CU)
          constexpr int N_ = decltype(Nc)::value, NT_ = decltype(NTc)::value;
          const dim3 g((pb.nx / 4) * (hi - lo));
          int r2;
          switch (pb.egno) {
            case 1:
              if ((r2 = ensure_lds(k_res_fwdy_fast_2d<1, N_, 4, NT_, double>, lds_res64))) return r2;
              hipLaunchKernelGGL((k_res_fwdy_fast_2d<1, N_, 4, NT_, double>), g, dim3(NT_), lds_res64, stream, p, twy);
              break;
            case 2:
              if ((r2 = ensure_lds(k_res_fwdy_fast_2d<2, N_, 4, NT_, double>, lds_res64))) return r2;
              hipLaunchKernelGGL((k_res_fwdy_fast_2d<2, N_, 4, NT_, double>), g, dim3(NT_), lds_res64, stream, p, twy);
              break;
            default:
              if ((r2 = ensure_lds(k_res_fwdy_fast_2d<3, N_, 4, NT_, double>, lds_res64))) return r2;
              hipLaunchKernelGGL((k_res_fwdy_fast_2d<3, N_, 4, NT_, double>), g, dim3(NT_), lds_res64, stream, p, twy);
              break;
          }
          return (int)PDHG_OK;
        };
        using I = std::integral_constant<int, 512>;
        rc = pb.ny == 4096 ? go(std::integral_constant<int, 4096>{}, I{})
             : res64_nt2048 == 256 ? go(std::integral_constant<int, 2048>{}, std::integral_constant<int, 256>{})
                                   : go(std::integral_constant<int, 2048>{}, I{});
        if (rc) return rc;
        HIP_TRY(hipGetLastError());
        return PDHG_OK;
      }
    }
    if (fast_rows) {
      ProfScope ps(this, "residual");
      p.row_base = lo;
      p.row_cnt = hi - lo;
      rc = with_fast_rows([&](auto Nc, auto RWc, auto NTc) {
        constexpr int N_ = decltype(Nc)::value, RW_ = decltype(RWc)::value, NT_ = decltype(NTc)::value;
        const dim3 g((pb.nx / RW_) * (hi - lo));
        int r2;
        if constexpr (sizeof(R) == 4) {
          switch (pb.egno) {
            case 1:
              if ((r2 = ensure_lds(k_res_fwdy_fast_2d<1, N_, RW_, NT_>, lds_fast))) return r2;
              hipLaunchKernelGGL((k_res_fwdy_fast_2d<1, N_, RW_, NT_>), g, dim3(NT_), lds_fast, stream, p, twy);
              break;
            case 2:
              if ((r2 = ensure_lds(k_res_fwdy_fast_2d<2, N_, RW_, NT_>, lds_fast))) return r2;
              hipLaunchKernelGGL((k_res_fwdy_fast_2d<2, N_, RW_, NT_>), g, dim3(NT_), lds_fast, stream, p, twy);
              break;
            default:
              if ((r2 = ensure_lds(k_res_fwdy_fast_2d<3, N_, RW_, NT_>, lds_fast))) return r2;
              hipLaunchKernelGGL((k_res_fwdy_fast_2d<3, N_, RW_, NT_>), g, dim3(NT_), lds_fast, stream, p, twy);
              break;
          }
        }
        return (int)PDHG_OK;
      });
    } else {
      if (lo != 0 || hi != pb.T) return fail(PDHG_ERR_UNSUPPORTED, "row-range residual needs the fast row kernels");
      ProfScope ps(this, "residual");
      dim3 g(gx1);
      rc = with_line_fft(ply, [&](auto f) {
        using F = decltype(f);
        auto go = [&](auto ntb) {
          constexpr int NTB = decltype(ntb)::value;
          int r2;
          switch (pb.egno) {
            case 1:
              if ((r2 = ensure_lds(k_res_fwdy_2d<R, 1, F, NTB>, lds_res))) return r2;
              hipLaunchKernelGGL((k_res_fwdy_2d<R, 1, F, NTB>), g, dim3(nt_row), lds_res, stream, p, f, twy);
              break;
            case 2:
              if ((r2 = ensure_lds(k_res_fwdy_2d<R, 2, F, NTB>, lds_res))) return r2;
              hipLaunchKernelGGL((k_res_fwdy_2d<R, 2, F, NTB>), g, dim3(nt_row), lds_res, stream, p, f, twy);
              break;
            default:
              if ((r2 = ensure_lds(k_res_fwdy_2d<R, 3, F, NTB>, lds_res))) return r2;
              hipLaunchKernelGGL((k_res_fwdy_2d<R, 3, F, NTB>), g, dim3(nt_row), lds_res, stream, p, f, twy);
              break;
          }
          return (int)PDHG_OK;
        };
        return nt_row <= 256 ? go(std::integral_constant<int, 256>{}) : go(std::integral_constant<int, 1024>{});
      });
    }
    if (rc) return rc;
    HIP_TRY(hipGetLastError());
    return PDHG_OK;
  }

  // ---------------- launches ----------------
  void launch_thomas_1d(const KP<R>& p) {
    if (thomas_chunk) {
      if constexpr (sizeof(R) == 4) {   // one 32-row chunk per wave
        const int P = (pb.T + 31) / 32;
        hipLaunchKernelGGL((k_thomas_chunk_1d<32, 1, R>), dim3((pb.nx + 63) / 64), dim3(64 * P), 0, stream, p);
      } else {                           // one 16-row chunk per half-wave (32 modes per workgroup)
        const int P = (pb.T + 15) / 16;
        hipLaunchKernelGGL((k_thomas_chunk_1d<16, 2, R>), dim3((pb.nx + 31) / 32), dim3(64 * ((P + 1) / 2)), 0, stream,
                           p);
      }
      return;
    }
    hipLaunchKernelGGL((k_thomas_1d<R>), dim3((pb.nx + 255) / 256), dim3(256), 0, stream, p);
  }

  // x transform + Thomas in t + inverse x transform of the spectral blocks in p.work (p.nx-point lines,
  // p.nb blocks); p.xt_phase selects the sweeps (t-slab)
  int launch_precond(const KP<R>& p, int nblk = -1) {   // nblk: blocks [p.b0, p.b0 + nblk) (default: all)
    int rc = PDHG_OK;
    if (nblk < 0) nblk = p.nb - p.b0;
    if constexpr (sizeof(R) == 4) {
      // one-row window: no t carries (k_precond_x_t1_2d), two workgroups per CU
      if (fast_xt && !half_real && p.T == 1 && !p.slab && p.xt_phase == 0 && t1_xt) {
        ProfScope ps(this, "precond");
        const size_t lds = (size_t)((p.B / 2) * (p.nx + p.nx / 16) + twlds_size(p.nx)) * sizeof(C);
        auto go = [&](auto kern) -> int {
          int r2;
          if ((r2 = ensure_lds(kern, lds))) return r2;
          hipLaunchKernelGGL(kern, dim3(nblk), dim3(512), lds, stream, p, twx);
          return (int)PDHG_OK;
        };
        switch (p.nx) {
          case 4096: rc = go(k_precond_x_t1_2d<4096, 1, 512>); break;
          case 2048: rc = go(k_precond_x_t1_2d<2048, 2, 512>); break;
          case 1024: rc = go(k_precond_x_t1_2d<1024, 4, 512>); break;
          case 512: rc = go(k_precond_x_t1_2d<512, 8, 512>); break;
          default: rc = fail(PDHG_ERR_UNSUPPORTED, "no one-row x kernel for nx=%d", p.nx);
        }
        if (rc) return rc;
        HIP_TRY(hipGetLastError());
        return PDHG_OK;
      }
    }
    if constexpr (sizeof(R) == 8) {
      // fp64 one-row window (the reference's marching default in its own precision): the carry-free x transform.
      // Measured (C2 marching, nx = 2048, B = 2): the generic kernel took
      // 156 us per launch, this one 28 us (67 MB read + 67 MB written: 4.8 TB/s)
      if (t1_xt64 && p.T == 1 && !p.slab && p.xt_phase == 0 && t1_xt) {
        ProfScope ps(this, "precond");
        // G16 (nx = 2048 / 4096, t1_g16): only the first twiddled pass's 48 seeds in LDS, so 4 (nx = 2048, 256
        // threads) or 2 (nx = 4096, 512 threads) workgroups fit a CU instead of 3 / 1
        const bool g16 = t1_g16 && (p.nx == 2048 || p.nx == 4096);
        const size_t lds = (size_t)((p.B / 2) * (p.nx + p.nx / 16) + (g16 ? 48 : twlds_size(p.nx))) * sizeof(C);
        auto go = [&](auto kern, int nt) -> int {
          int r2;
          if ((r2 = ensure_lds(kern, lds))) return r2;
          hipLaunchKernelGGL(kern, dim3(nblk), dim3(nt), lds, stream, p, twx);
          return (int)PDHG_OK;
        };
        switch (p.nx) {
          case 4096:
            rc = g16 ? go(k_precond_x_t1_2d<4096, 1, 512, double, true>, 512)
                     : go(k_precond_x_t1_2d<4096, 1, 512, double>, 512);
            break;
          case 2048:   // 512 threads: 28.06 vs 27.64 us (3 workgroups per CU by LDS)
            rc = g16 ? go(k_precond_x_t1_2d<2048, 1, 256, double, true>, 256)
                     : go(k_precond_x_t1_2d<2048, 1, 256, double>, 256);
            break;
          case 1024: rc = go(k_precond_x_t1_2d<1024, 2, 512, double>, 512); break;
          case 512: rc = go(k_precond_x_t1_2d<512, 4, 512, double>, 512); break;
          default: rc = fail(PDHG_ERR_UNSUPPORTED, "no fp64 one-row x kernel for nx=%d", p.nx);
        }
        if (rc) return rc;
        HIP_TRY(hipGetLastError());
        return PDHG_OK;
      }
      if (f64_xt) {
        ProfScope ps(this, "precond");
        if (half_real) {   // nx = 8192: one real column per block + the split-twiddle tables
          const size_t lds = (size_t)(Pad<4096>::LINE + TwLds<4096>::SIZE + 4096 + 128) * sizeof(C);
          if ((rc = ensure_lds(k_precond_xt_f64_2d<4096, 512, true>, lds))) return rc;
          hipLaunchKernelGGL((k_precond_xt_f64_2d<4096, 512, true>), dim3(nblk), dim3(512), lds, stream, p, twx);
          HIP_TRY(hipGetLastError());
          return PDHG_OK;
        }
        if (p.nx == 1024 || p.nx == 512) {   // b' in registers, 4 items per thread
          const size_t lds = (size_t)((p.nx == 1024 ? Pad<1024>::LINE + TwLds<1024>::SIZE : Pad<512>::LINE +
                                       TwLds<512>::SIZE)) * sizeof(C);
          auto go = [&](auto kern, int nt) -> int {
            int r2;
            if ((r2 = ensure_lds(kern, lds))) return r2;
            hipLaunchKernelGGL(kern, dim3(nblk), dim3(nt), lds, stream, p, twx);
            return (int)PDHG_OK;
          };
          rc = p.nx == 1024 ? go(k_precond_xt_f64_2d<1024, 256, false, true>, 256)
                            : go(k_precond_xt_f64_2d<512, 128, false, true>, 128);
          if (rc) return rc;
          HIP_TRY(hipGetLastError());
          return PDHG_OK;
        }
        if (p.nx == 2048) {   // b' in registers (IT = 4 at 512 threads; PDHG_XT64_VAR: A/B of the shapes)
          const int var = xt64_var;
          auto go = [&](auto kern, int nt, bool bpr) -> int {
            const size_t lds = (size_t)(Pad<2048>::LINE + TwLds<2048>::SIZE + (bpr ? 0 : 2048)) * sizeof(C);
            int r2;
            if ((r2 = ensure_lds(kern, lds))) return r2;
            hipLaunchKernelGGL(kern, dim3(nblk), dim3(nt), lds, stream, p, twx);
            return (int)PDHG_OK;
          };
          if (var == 1) rc = go(k_precond_xt_f64_2d<2048, 256, false, false>, 256, false);
          else if (var == 2) rc = go(k_precond_xt_f64_2d<2048, 256, false, true>, 256, true);
          else if (var == 3) rc = go(k_precond_xt_f64_2d<2048, 1024, false, true>, 1024, true);
          else rc = go(k_precond_xt_f64_2d<2048, 512, false, true>, 512, true);
          if (rc) return rc;
          HIP_TRY(hipGetLastError());
          return PDHG_OK;
        }
        const size_t lds = (size_t)(Pad<4096>::LINE + TwLds<4096>::SIZE + 4096) * sizeof(C);
        if (p.rspec) {   // task-order residual spectrum in (tc_spec; b' / x rows in `work` as always)
          if ((rc = ensure_lds(k_precond_xt_f64_2d<4096, 512, false, false, true>, lds))) return rc;
          hipLaunchKernelGGL((k_precond_xt_f64_2d<4096, 512, false, false, true>), dim3(nblk), dim3(512), lds, stream, p,
                             twx);
        } else {
          if ((rc = ensure_lds(k_precond_xt_f64_2d<4096, 512>, lds))) return rc;
          hipLaunchKernelGGL((k_precond_xt_f64_2d<4096, 512>), dim3(nblk), dim3(512), lds, stream, p, twx);
        }
        HIP_TRY(hipGetLastError());
        return PDHG_OK;
      }
    }
    if (fast_xt) {
      ProfScope ps(this, "precond");
      rc = PDHG_OK;
      if constexpr (sizeof(R) == 4) {
        const dim3 g(nblk);
        auto go = [&](auto kern) -> int {
          int r2;
          if ((r2 = ensure_lds(kern, lds_fast_xt))) return r2;
          hipLaunchKernelGGL(kern, g, dim3(512), lds_fast_xt, stream, p, twx);
          return (int)PDHG_OK;
        };
        if (batch_xt) {
          auto gob = [&](auto kern) -> int {
            int r2;
            if ((r2 = ensure_lds(kern, lds_batch_xt))) return r2;
            hipLaunchKernelGGL(kern, g, dim3(1024), lds_batch_xt, stream, p, twx);
            return (int)PDHG_OK;
          };
          auto gob2 = [&](auto kern) -> int {   // RB = 2 rows, 512 threads: two workgroups per CU
            int r2;
            const size_t lds = (size_t)(2 * (4096 + 4096 / 16) + twlds_size(p.nx)) * sizeof(C);
            if ((r2 = ensure_lds(kern, lds))) return r2;
            hipLaunchKernelGGL(kern, g, dim3(512), lds, stream, p, twx);
            return (int)PDHG_OK;
          };
          switch (p.nx) {
            case 4096:
              if (xt_dma) {   // static LDS (kernels_xt_dma.hpp)
                hipLaunchKernelGGL(k_precond_xt_dma_2d<4096>, g, dim3(1024), 0, stream, p, twx);
              } else if (xt_pair) rc = gob2(k_precond_xt_batch_2d<4096, 1, 2, 0, 512>);
              else if (xt_rpre == 2) rc = gob(k_precond_xt_batch_2d<4096, 1, 4, 2>);
              else rc = gob(k_precond_xt_batch_2d<4096, 1>);
              break;
            case 2048: rc = gob(k_precond_xt_batch_2d<2048, 2>); break;
            case 1024: rc = gob(k_precond_xt_batch_2d<1024, 4>); break;
            case 512: rc = gob(k_precond_xt_batch_2d<512, 8>); break;
            default: rc = fail(PDHG_ERR_UNSUPPORTED, "no batched x kernel for nx=%d", p.nx);
          }
        } else if (half_real && xt_dma_hr) {   // static LDS (kernels_xt_dma.hpp, HR)
          hipLaunchKernelGGL((k_precond_xt_dma_2d<4096, true>), g, dim3(1024), 0, stream, p, twx);
        } else if (ws_xt) {
          switch (p.nx) {
            case 8192: rc = go(k_precond_xt_ws_2d<4096, 1, true>); break;
            case 4096: rc = go(k_precond_xt_ws_2d<4096, 1>); break;
            case 2048: rc = go(k_precond_xt_ws_2d<2048, 2>); break;
            case 1024: rc = go(k_precond_xt_ws_2d<1024, 4>); break;
            case 512: rc = go(k_precond_xt_ws_2d<512, 8>); break;
            default: rc = fail(PDHG_ERR_UNSUPPORTED, "no fast x kernel for nx=%d", p.nx);
          }
        } else switch (p.nx) {
          case 4096: rc = go(k_precond_xt_fast_2d<4096, 1, 512>); break;
          case 2048: rc = go(k_precond_xt_fast_2d<2048, 2, 512>); break;
          case 1024: rc = go(k_precond_xt_fast_2d<1024, 4, 512>); break;
          case 512: rc = go(k_precond_xt_fast_2d<512, 8, 512>); break;
          default: rc = fail(PDHG_ERR_UNSUPPORTED, "no fast x kernel for nx=%d", p.nx);
        }
      }
      if (rc) return rc;
    } else {
      ProfScope ps(this, "precond");
      dim3 g(nblk);
      rc = with_xt_fft([&](auto f) {
        using F = decltype(f);
        int r2;
        if ((r2 = ensure_lds(k_precond_xt_2d<R, F>, lds_xt))) return r2;
        hipLaunchKernelGGL((k_precond_xt_2d<R, F>), g, dim3(NT2), lds_xt, stream, p, f, twx);
        return (int)PDHG_OK;
      });
      if (rc) return rc;
    }
    return PDHG_OK;
  }

  // stages: 1 residual (+ forward y transform), 2 x transform + Thomas (sweeps per xt_phase: 0 both,
  // 1 forward, 2 backward), 4 inverse transforms + phi/phi_bar update + primal sums.  sums_out != null
  // (t-slab mode): the primal sums go to that vector (all-reduced by the caller) instead of ctrl.
  int launch_primal(R tau, int stages = 7, int xt_phase = 0, double* sums_out = nullptr) {
    KP<R> p = kp;
    p.tau = tau;
    p.xt_phase = xt_phase;
    const int T = pb.T;
    if (pb.ndim == 2) {
      int rc = PDHG_OK;
      if (stages & 1)
        if ((rc = launch_residual(p, 0, T))) return rc;
      if ((stages & 2) && (rc = launch_precond(p))) return rc;
      if (!(stages & 4)) {
        HIP_TRY(hipGetLastError());
        return PDHG_OK;
      }
      int upd_rows = gx4 * g4;
      bool upd_done = false;
      // speculative schedule: the update's sums go to their own rows and k_finalize_dual_outer reduces them (the
      // same rows in the same order as k_finalize_primal), one launch fewer
      const bool prim_merge = spec && fin_merge && !dual_multi && !sums_out;
      if (prim_merge) p.partials = prim_partials;
      if constexpr (sizeof(R) == 8) {
        if (res64) {
          ProfScope ps(this, "update");
          upd_rows = g_fast_upd;
          auto go = [&](auto kern) {
            int r3;
            if ((r3 = ensure_lds(kern, lds_upd64))) return r3;
            hipLaunchKernelGGL(kern, dim3(g_fast_upd), dim3(512), lds_upd64, stream, p, twy);
            return (int)PDHG_OK;
          };
          if (pb.ny == 2048 && upd_t1 > 0) {   // one-row windows: 256 threads, two workgroups per CU (G16 seeds)
            const size_t lds = lds_res64 + (size_t)48 * sizeof(C);
            auto go2 = [&](auto kern) {
              int r3;
              if ((r3 = ensure_lds(kern, lds))) return r3;
              hipLaunchKernelGGL(kern, dim3(g_fast_upd), dim3(256), lds, stream, p, twy);
              return (int)PDHG_OK;
            };
            rc = upd_t1 == 2 ? go2(k_invy_update_fast_2d<2048, 4, 256, 2, double, true>)
                             : go2(k_invy_update_fast_2d<2048, 4, 256, 4, double, true>);
          } else {
            rc = pb.ny == 4096 ? go(k_invy_update_fast_2d<4096, 4, 512, 4, double>)
                               : go(k_invy_update_fast_2d<2048, 4, 512, 4, double>);
          }
          if (rc) return rc;
          upd_done = true;
        } else if (upd8192) {   // fp64 ny = 8192, half-real x blocks: 2-row tasks on one padded line
          ProfScope ps(this, "update");
          upd_rows = g_fast_upd;
          const size_t lds = (size_t)Pad<8192>::LINE * sizeof(C);
          if ((rc = ensure_lds(k_invy_update_fast_2d<8192, 2, 512, 2, double>, lds))) return rc;
          hipLaunchKernelGGL((k_invy_update_fast_2d<8192, 2, 512, 2, double>), dim3(g_fast_upd), dim3(512), lds, stream,
                             p, twy);
          upd_done = true;
        }
      }
      if (upd_done) {
      } else if (fast_rows) {
        ProfScope ps(this, "update");
        upd_rows = g_fast_upd;
        rc = with_fast_rows([&](auto Nc, auto RWc, auto NTc) {
          constexpr int N_ = decltype(Nc)::value, RW_ = decltype(RWc)::value, NT_ = decltype(NTc)::value;
          int r2;
          if constexpr (sizeof(R) == 4) {
            if constexpr (NT_ == 1024 && RW_ == 8) {
              if (half_nt & 2) {
                auto go = [&](auto kern) {
                  int r3;
                  if ((r3 = ensure_lds(kern, lds_fast_tw))) return r3;
                  hipLaunchKernelGGL(kern, dim3(g_fast_upd), dim3(512), lds_fast_tw, stream, p, twy);
                  return (int)PDHG_OK;
                };
                switch (upd_pf) {
                  case 2: return go(k_invy_update_fast_2d<N_, RW_, 512, 2>);
                  case 3: return go(k_invy_update_fast_2d<N_, RW_, 512, 3>);
                  case 4: return go(k_invy_update_fast_2d<N_, RW_, 512, 4>);
                  default: return go(k_invy_update_fast_2d<N_, RW_, 512, 1>);
                }
              }
            }
            if ((r2 = ensure_lds(k_invy_update_fast_2d<N_, RW_, NT_>, lds_fast_tw))) return r2;
            hipLaunchKernelGGL((k_invy_update_fast_2d<N_, RW_, NT_>), dim3(g_fast_upd), dim3(NT_), lds_fast_tw, stream,
                               p, twy);
          }
          return (int)PDHG_OK;
        });
        if (rc) return rc;
      } else {
        ProfScope ps(this, "update");
        rc = with_line_fft(ply, [&](auto f) {
          using F = decltype(f);
          int r2;
          auto go = [&](auto kern) {
            int r3;
            if ((r3 = ensure_lds(kern, lds_res))) return r3;
            hipLaunchKernelGGL(kern, dim3(gx4), dim3(nt_row), lds_res, stream, p, f, twy);
            return (int)PDHG_OK;
          };
          (void)r2;
          return nt_row <= 256 ? go(k_invy_update_2d<R, F, 256>) : go(k_invy_update_2d<R, F, 1024>);
        });
        if (rc) return rc;
      }
      if (sums_out)
        hipLaunchKernelGGL(k_reduce_vec, dim3(1), dim3(1024), 0, stream, p.partials, upd_rows, 3,
                           kp.j0 == 0 ? row0_sq : 0.0, sums_out);
      else if (prim_merge)
        prim_merged_rows = upd_rows;
      else
        hipLaunchKernelGGL(k_finalize_primal, dim3(1), dim3(1024), 0, stream, p.partials, upd_rows, 1, p.ctrl);
    } else {
      int rc;
      if (fourstep) return launch_fourstep_1d(p);
      {
        ProfScope ps(this, "residual");
        rc = with_line_fft(plx, [&](auto f) {
          using F = decltype(f);
          int r2;
          if (pb.egno == 1) {
            if ((r2 = ensure_lds(k_res_fwdx_1d<R, 1, F>, lds_res))) return r2;
            hipLaunchKernelGGL((k_res_fwdx_1d<R, 1, F>), dim3(gx1), dim3(nt1d), lds_res, stream, p, f, twx);
          } else {
            if ((r2 = ensure_lds(k_res_fwdx_1d<R, 2, F>, lds_res))) return r2;
            hipLaunchKernelGGL((k_res_fwdx_1d<R, 2, F>), dim3(gx1), dim3(nt1d), lds_res, stream, p, f, twx);
          }
          return (int)PDHG_OK;
        });
        if (rc) return rc;
      }
      {
        ProfScope ps(this, "precond");
        launch_thomas_1d(p);
      }
      {
        ProfScope ps(this, "update");
        rc = with_line_fft(plx, [&](auto f) {
          using F = decltype(f);
          int r2;
          if ((r2 = ensure_lds(k_invx_update_1d<R, F>, lds_res))) return r2;
          hipLaunchKernelGGL((k_invx_update_1d<R, F>), dim3(gx4), dim3(nt1d), lds_res, stream, p, f, twx);
          return (int)PDHG_OK;
        });
        if (rc) return rc;
      }
      hipLaunchKernelGGL(k_finalize_primal, dim3(1), dim3(1024), 0, stream, p.partials, gx4, 1, p.ctrl);
    }
    HIP_TRY(hipGetLastError());
    return PDHG_OK;
  }

  // 1-D primal with the four-step DHT (nx = 65536, fp32): residual + DHT, Thomas, inverse DHT + update
  int launch_fourstep_1d(const KP<R>& p) {
    if (fs16) return launch_fs16_1d(p);
    if constexpr (sizeof(R) == 4) {
      if (fs_wide) return launch_fourstep_wide_1d(p);
      constexpr int kFsNT = 1024;   // 16 waves: the load / unpack loops keep more rows in flight
      const int npairs = (pb.T + 1) / 2;
      const size_t lds1 = (size_t)2 * 256 * 16 * sizeof(C), lds2 = 2 * lds1;
      float2* Y = reinterpret_cast<float2*>(p.gscr);
      int rc;
      {
        ProfScope ps(this, "residual");
        if (pb.egno == 1) {
          if ((rc = ensure_lds(k_fs1_1d<0, 1>, lds1))) return rc;
          hipLaunchKernelGGL((k_fs1_1d<0, 1>), dim3(16, npairs), dim3(kFsNT), lds1, stream, p, tw256, twx, Y);
        } else {
          if ((rc = ensure_lds(k_fs1_1d<0, 2>, lds1))) return rc;
          hipLaunchKernelGGL((k_fs1_1d<0, 2>), dim3(16, npairs), dim3(kFsNT), lds1, stream, p, tw256, twx, Y);
        }
        if ((rc = ensure_lds(k_fs2_1d<0>, lds2))) return rc;
        hipLaunchKernelGGL((k_fs2_1d<0>), dim3(9, npairs), dim3(kFsNT), lds2, stream, p, tw256, Y);
      }
      {
        ProfScope ps(this, "precond");
        launch_thomas_1d(p);
      }
      {
        ProfScope ps(this, "update");
        if ((rc = ensure_lds(k_fs1_1d<1, 1>, lds1))) return rc;
        hipLaunchKernelGGL((k_fs1_1d<1, 1>), dim3(16, npairs), dim3(kFsNT), lds1, stream, p, tw256, twx, Y);
        if ((rc = ensure_lds(k_fs2_1d<1>, lds2))) return rc;
        hipLaunchKernelGGL((k_fs2_1d<1>), dim3(9, npairs), dim3(kFsNT), lds2, stream, p, tw256, Y);
      }
      hipLaunchKernelGGL(k_finalize_primal, dim3(1), dim3(1024), 0, stream, p.partials, 9 * npairs, 1, p.ctrl);
      HIP_TRY(hipGetLastError());
    }
    return PDHG_OK;
  }

  // the same with the wide-tile stages (kernels_fs_wide.hpp): 4 + 5 workgroups per row pair
  int launch_fourstep_wide_1d(const KP<R>& p) {
    if constexpr (sizeof(R) == 4) {
      const int npairs = (pb.T + 1) / 2;
      const size_t lds = (size_t)(64 * kFwLine + twlds_size(256)) * sizeof(C);
      float2* Y = reinterpret_cast<float2*>(p.gscr);
      int rc;
      {
        ProfScope ps(this, "residual");
        if (pb.egno == 1) {
          if ((rc = ensure_lds(k_fs1w_1d<0, 1>, lds))) return rc;
          hipLaunchKernelGGL((k_fs1w_1d<0, 1>), dim3(4, npairs), dim3(1024), lds, stream, p, tw256, twx, Y);
        } else {
          if ((rc = ensure_lds(k_fs1w_1d<0, 2>, lds))) return rc;
          hipLaunchKernelGGL((k_fs1w_1d<0, 2>), dim3(4, npairs), dim3(1024), lds, stream, p, tw256, twx, Y);
        }
        if ((rc = ensure_lds(k_fs2w_1d<0>, lds))) return rc;
        hipLaunchKernelGGL((k_fs2w_1d<0>), dim3(5, npairs), dim3(1024), lds, stream, p, tw256, Y);
      }
      {
        ProfScope ps(this, "precond");
        launch_thomas_1d(p);
      }
      {
        ProfScope ps(this, "update");
        if ((rc = ensure_lds(k_fs1w_1d<1, 1>, lds))) return rc;
        hipLaunchKernelGGL((k_fs1w_1d<1, 1>), dim3(4, npairs), dim3(1024), lds, stream, p, tw256, twx, Y);
        if ((rc = ensure_lds(k_fs2w_1d<1>, lds))) return rc;
        hipLaunchKernelGGL((k_fs2w_1d<1>), dim3(5, npairs), dim3(1024), lds, stream, p, tw256, Y);
      }
      hipLaunchKernelGGL(k_finalize_primal, dim3(1), dim3(1024), 0, stream, p.partials, 5 * npairs, 1, p.ctrl);
      HIP_TRY(hipGetLastError());
    }
    return PDHG_OK;
  }

  // the same as 16 x 4096 with a chunk-major spectrum (kernels_fs16.hpp): 16 + 8 workgroups per row pair
  // forward, 8 + 8 inverse
  int launch_fs16_1d(const KP<R>& p) {
    {
      const int npairs = (pb.T + 1) / 2;
      const size_t ldsb = (size_t)(2 * kF16Line + twlds_size(kF16N2)) * sizeof(C);
      C* Y = reinterpret_cast<C*>(p.gscr);
      int rc;
      {
        ProfScope ps(this, "residual");
        const dim3 ga(kF16N2 / 256, npairs);
        auto fwd = [&](auto eg) {
          constexpr int E = decltype(eg)::value;
          if (f16_group == 4) hipLaunchKernelGGL((k_f16a_fwd_1d<E, 4, R>), ga, dim3(256), 0, stream, p, twx, Y);
          else if (f16_group == 8) hipLaunchKernelGGL((k_f16a_fwd_1d<E, 8, R>), ga, dim3(256), 0, stream, p, twx, Y);
          else hipLaunchKernelGGL((k_f16a_fwd_1d<E, 16, R>), ga, dim3(256), 0, stream, p, twx, Y);
        };
        if (fuse_res && res_valid)   // the residual rows the last dual sweep formed (k_dual_1d_fr)
          hipLaunchKernelGGL((k_f16a_fwd_fused_1d<R>), ga, dim3(256), 0, stream, p, twx, Y, jchunk_1d);
        else if (pb.egno == 1) fwd(std::integral_constant<int, 1>{});
        else fwd(std::integral_constant<int, 2>{});
        if ((rc = ensure_lds(k_f16b_fwd_1d<R>, ldsb))) return rc;
        hipLaunchKernelGGL(k_f16b_fwd_1d<R>, dim3(8, npairs), dim3(512), ldsb, stream, p, twx, Y);
      }
      {
        ProfScope ps(this, "precond");
        launch_thomas_1d(p);
      }
      {
        ProfScope ps(this, "update");
        if ((rc = ensure_lds(k_f16b_inv_1d<R>, ldsb))) return rc;
        hipLaunchKernelGGL(k_f16b_inv_1d<R>, dim3(8, npairs), dim3(512), ldsb, stream, p, twx, Y);
        hipLaunchKernelGGL(k_f16a_inv_1d<R>, dim3(kF16N2 / 2 / 256, npairs), dim3(256), 0, stream, p, twx, Y);
      }
      hipLaunchKernelGGL(k_finalize_primal, dim3(1), dim3(1024), 0, stream, p.partials, 8 * npairs, 1, p.ctrl);
      HIP_TRY(hipGetLastError());
    }
    return PDHG_OK;
  }

  // fast dual over time rows [lo, hi); its partials start at block row zbase.  Returns the z extent.
  template <int EGNO>
  void launch_dual_fast_e(const KP<R>& p, int lo, int hi, int gz, int zbase) {
    if constexpr (std::is_same<R, float>::value) {
      const dim3 g(gxd, gyd, gz);
      if constexpr (EGNO != 3) {
        if (fuse_res && p.inplace && gz == 1 && (slab || (lo == 0 && hi == pb.T))) {
          hipLaunchKernelGGL((k_dual_lds_2d<EGNO, 8, true>), g, dim3(NTd), 0, stream, p, jchunk_d, lo, hi, zbase);
          res_valid = true;
          return;
        }
      }
      res_valid = false;
      switch (dual_rx) {
        case 4: hipLaunchKernelGGL((k_dual_lds_2d<EGNO, 4>), g, dim3(NTd), 0, stream, p, jchunk_d, lo, hi, zbase); break;
        case 8: hipLaunchKernelGGL((k_dual_lds_2d<EGNO, 8>), g, dim3(NTd), 0, stream, p, jchunk_d, lo, hi, zbase); break;
        case 16: hipLaunchKernelGGL((k_dual_lds_2d<EGNO, 16>), g, dim3(NTd), 0, stream, p, jchunk_d, lo, hi, zbase); break;
        default:
          if (jchunk_d == 1 && dual_one)
            hipLaunchKernelGGL((k_dual_fast_2d<EGNO, float, 1>), g, dim3(NTd), 0, stream, p, jchunk_d, lo, hi, zbase);
          else
            hipLaunchKernelGGL((k_dual_fast_2d<EGNO>), g, dim3(NTd), 0, stream, p, jchunk_d, lo, hi, zbase);
      }
    } else {
      const dim3 g(gxd, gyd, gz);
      if constexpr (EGNO != 3) {
        if (fuse_res && p.inplace && gz == 1 && (slab || (lo == 0 && hi == pb.T))) {
          hipLaunchKernelGGL((k_dual_lds_2d<EGNO, 8, true, double, 2>), g, dim3(NTd), 0, stream, p, jchunk_d, lo, hi,
                             zbase);
          res_valid = true;
          return;
        }
      }
      res_valid = false;
      if (dual_rx == 8 && dual_ypl == 2)
        hipLaunchKernelGGL((k_dual_lds_2d<EGNO, 8, false, double, 2>), g, dim3(NTd), 0, stream, p, jchunk_d, lo, hi, zbase);
      else if (dual_rx == 8)
        hipLaunchKernelGGL((k_dual_lds_2d<EGNO, 8, false, double>), g, dim3(NTd), 0, stream, p, jchunk_d, lo, hi, zbase);
      else if (jchunk_d == 1 && dual_one == 2)
        hipLaunchKernelGGL((k_dual_fast_2d<EGNO, double, 2>), g, dim3(NTd), 0, stream, p, jchunk_d, lo, hi, zbase);
      else if (jchunk_d == 1 && dual_one)
        hipLaunchKernelGGL((k_dual_fast_2d<EGNO, double, 1>), g, dim3(NTd), 0, stream, p, jchunk_d, lo, hi, zbase);
      else
        hipLaunchKernelGGL((k_dual_fast_2d<EGNO, double>), g, dim3(NTd), 0, stream, p, jchunk_d, lo, hi, zbase);
    }
  }
  int launch_dual_fast(const KP<R>& p, int lo = 0, int hi = -1, int zbase = 0) {
    if (hi < 0) hi = pb.T;
    if (hi <= lo) return 0;
    const int gz = (hi - lo + jchunk_d - 1) / jchunk_d;
    if (pb.egno == 1) launch_dual_fast_e<1>(p, lo, hi, gz, zbase);
    else if (pb.egno == 2) launch_dual_fast_e<2>(p, lo, hi, gz, zbase);
    else launch_dual_fast_e<3>(p, lo, hi, gz, zbase);
    return gz;
  }

  // the dual loop in chunks of kMultiSub sub-iterations + a final pass when the exit falls inside a chunk
  // (kernels_dual_multi.hpp); k in [2, kDualMultiMax]
  template <int EGNO>
  void launch_dual_multi_e(const KP<R>& p, int k, double eps, int slo0 = 0) {   // slo0 = 1: head form
    // head form: runs of 4 x rows per workgroup (its passes mostly return at once; fewer workgroups to retire)
    const int xrun = (slo0 > 0 && pb.nx % head_xrun == 0) ? head_xrun : 1;
    const int gx = (pb.nx + xrun - 1) / xrun;
    const dim3 g(gx, gyd, gzd);
    const int rows = gx * gyd * gzd;
    constexpr int NS = kMultiSub;
    for (int slo = slo0; slo < k; slo += NS) {
      hipLaunchKernelGGL((k_dual_multi_2d<EGNO, R, NS, false>), g, dim3(NTd), 0, stream, p, slo, k, rows, jchunk_d, 0,
                         pb.T, 0, xrun);
      hipLaunchKernelGGL(k_finalize_dual_multi, dim3(1), dim3(1024), 0, stream, p.partials, rows,
                         std::min(NS, k - slo), slo, k, na, n_dead, eps, p.ctrl);
    }
    hipLaunchKernelGGL((k_dual_multi_2d<EGNO, R, NS, true>), g, dim3(NTd), 0, stream, p, 0, k, rows, jchunk_d, 0, pb.T,
                       0, xrun);
  }

  int launch_dual(R sigma, double eps, int k) {
    KP<R> p = kp;
    p.sigma = sigma;
    p.inplace = (k <= 1) ? 1 : 0;
    if (!p.inplace && !two_sets)
      return fail(PDHG_ERR_STATE, "rho_alp_iters=%d needs a context created with rho_alp_iters > 1", k);
    if (dual_multi && k > 1 && k <= kDualMultiMax) {
      ProfScope ps(this, "dual");
      if (pb.egno == 1) launch_dual_multi_e<1>(p, k, eps);
      else if (pb.egno == 2) launch_dual_multi_e<2>(p, k, eps);
      else launch_dual_multi_e<3>(p, k, eps);
      HIP_TRY(hipGetLastError());
      return PDHG_OK;
    }
    // head form: sub-iteration 0 below, then the chunks from sub-iteration 1
    const bool head = dual_head && k > 1 && k <= kDualMultiMax;
    for (int s = 0; s < (head ? 1 : k); ++s) {
      p.sub = s;
      {
        ProfScope ps(this, "dual");
        dim3 g(gx5, g5);
        if (pb.ndim == 2 && fast_dual) {
          launch_dual_fast(p);
        } else if (pb.ndim == 2) {
          switch (pb.egno) {
            case 1: hipLaunchKernelGGL((k_dual_2d<R, 1>), g, dim3(256), 0, stream, p); break;
            case 2: hipLaunchKernelGGL((k_dual_2d<R, 2>), g, dim3(256), 0, stream, p); break;
            default: hipLaunchKernelGGL((k_dual_2d<R, 3>), g, dim3(256), 0, stream, p); break;
          }
        } else if (fuse_res && p.inplace) {   // the sweep also forms the next residual (k_dual_1d_fr)
          const dim3 gf(pb.nx / 256, gz_1d);
          if (pb.egno == 1)
            hipLaunchKernelGGL((k_dual_1d_fr<R, 1>), gf, dim3(256), 0, stream, p, jchunk_1d);
          else
            hipLaunchKernelGGL((k_dual_1d_fr<R, 2>), gf, dim3(256), 0, stream, p, jchunk_1d);
          res_valid = true;
        } else {
          res_valid = false;
          if (pb.egno == 1)
            hipLaunchKernelGGL((k_dual_1d<R, 1>), g, dim3(256), 0, stream, p);
          else
            hipLaunchKernelGGL((k_dual_1d<R, 2>), g, dim3(256), 0, stream, p);
        }
      }
      const int nrows_d = (pb.ndim == 2 && fast_dual) ? gxd * gyd * gzd
                                                      : (pb.ndim == 1 && fuse_res && p.inplace) ? (pb.nx / 256) * gz_1d
                                                                                                : gx5 * g5;
      const double* rows = p.partials;
      int nrows = nrows_d;
      if (nrows_d > 2 * kFoldRows * 16) {   // one workgroup reading ~1 MiB of rows took 45-65 us at C1 / C3
        const int chunk = (nrows_d + kFoldRows - 1) / kFoldRows;
        if (fold_fin) {   // fold + finalize in one launch (the last workgroup finalizes)
          hipLaunchKernelGGL(k_fold_finalize_dual, dim3(kFoldRows), dim3(1024), 0, stream, p.partials, nrows_d, chunk,
                             fold_out, na, n_dead, eps, s, p.ctrl);
          continue;
        }
        hipLaunchKernelGGL(k_fold_partials, dim3(kFoldRows), dim3(1024), 0, stream, p.partials, nrows_d, 3 + 3 * na,
                           chunk, fold_out, p.ctrl);
        rows = fold_out;
        nrows = kFoldRows;
      }
      if (head && spec && s == 0 && k > 1 && k1_outer && !dual_multi && fin_merge) {
        // the speculative iteration's dual and outer finalizes in one launch; launch_outer then launches nothing
        hipLaunchKernelGGL(k_finalize_dual_outer, dim3(1), dim3(1024), 0, stream, prim_partials, prim_merged_rows,
                           rows, nrows, na, n_dead, eps, 1, stop_conv, stop_nan, p.ctrl);
        prim_merged_rows = 0;
        outer_merged = true;
      } else {
        hipLaunchKernelGGL(k_finalize_dual, dim3(1), dim3(1024), 0, stream, rows, nrows, na, n_dead, eps, s, p.ctrl,
                           (head && spec) ? 1 : 0);
      }
    }
    if (head && !spec) return launch_dual_tail(sigma, eps, k);   // spec: only when sub-iteration 0 did not exit
    HIP_TRY(hipGetLastError());
    return PDHG_OK;
  }
  // the head form's rest of the dual loop: chunk passes from sub-iteration 1 (+ their finalizes, the final pass)
  int launch_dual_tail(R sigma, double eps, int k) {
    KP<R> p = kp;
    p.sigma = sigma;
    p.inplace = 0;
    {
      ProfScope ps(this, "dual");
      if (pb.egno == 1) launch_dual_multi_e<1>(p, k, eps, 1);
      else if (pb.egno == 2) launch_dual_multi_e<2>(p, k, eps, 1);
      else launch_dual_multi_e<3>(p, k, eps, 1);
    }
    HIP_TRY(hipGetLastError());
    return PDHG_OK;
  }

  int launch_outer(double eps, int k) {
    if (outer_merged) {   // k_finalize_dual_outer ran it (speculative schedule)
      outer_merged = false;
      return PDHG_OK;
    }
    KP<R> p = kp;
    int rows = 0;
    // the chunked dual loop keeps no sub-iteration-0 outer sums (its tables hold 2 + 2 na sums), so only the
    // per-sub-iteration kernels skip the outer pass after a one-sub-iteration loop
    const int k1_skip = (k1_outer && !dual_multi) ? 1 : 0;
    if (k > 1) {
      // spec: the iteration reaches here only after a one-sub-iteration loop, whose outer-sum pass returns at once
      if (!spec)
        hipLaunchKernelGGL((k_outer_sums<R>), dim3(g_outer), dim3(256), 0, stream, p, (size_t)pb.T * plane(), k1_skip);
      rows = g_outer;
    }
    hipLaunchKernelGGL(k_finalize_outer, dim3(1), dim3(1024), 0, stream, p.partials, rows, na, eps, k > 1 ? 1 : 0,
                       stop_conv, stop_nan, p.ctrl, k > 1 ? k1_skip : 0);
    HIP_TRY(hipGetLastError());
    return PDHG_OK;
  }

  int reset_ctrl() {
    // zero everything except `cur` (which buffer set holds the state)
    Ctrl h{};
    int cur = 0;
    HIP_TRY(hipMemcpyAsync(&cur, &kp.ctrl->cur, sizeof(int), hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    h.cur = cur;
    h.row0_sq = row0_sq;
    HIP_TRY(hipMemcpyAsync(kp.ctrl, &h, sizeof(Ctrl), hipMemcpyHostToDevice, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    return PDHG_OK;
  }

  int read_ctrl(Ctrl& h) {
    HIP_TRY(hipMemcpyAsync(&h, kp.ctrl, sizeof(Ctrl), hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    return PDHG_OK;
  }

  // ---------------- iteration chunks replayed from a HIP graph ----------------
  // The launch chain of `window` outer iterations (primal, <= k dual sub-iterations, outer tests: 8-12
  // kernels each) is captured once per (tau, sigma, eps, k) and replayed with one hipGraphLaunch, so the
  // host issues one call per window instead of ~10 per iteration -- the marching default's T = 1 windows
  // and small grids are launch-bound (utils_pdhg_solver.py:166-212 runs up to N_maxiter iterations per
  // window).  The device-side stop flags (Ctrl) make the kernels after convergence no-ops, exactly as in the
  // eager loop, so a replayed chunk needs no host decision.  Captured only with the fused residual valid
  // (or not in use) so every captured primal is the steady-state one; off while profiling (per-launch
  // events) and with PDHG_GRAPH=0.
  hipGraphExec_t gexec = nullptr;
  double g_tau = 0, g_sigma = 0, g_eps = 0;
  int g_k = 0, g_window = 0, g_stop = -1, g_spec = -1;
  bool use_graph = true;
  bool warm = false;   // one eager iteration ran (kernel attributes set outside any capture)
  void drop_graph() {
    if (gexec) hipGraphExecDestroy(gexec);
    gexec = nullptr;
  }
  int launch_iteration(double tau, double sigma, double eps, int k) {
    int rc;
    if ((rc = launch_primal((R)tau))) return rc;
    if ((rc = launch_dual((R)sigma, eps, k))) return rc;
    return launch_outer(eps, k);
  }
  int ensure_graph(double tau, double sigma, double eps, int k, int window) {
    const int stop = stop_conv * 2 + stop_nan;   // kernel arguments of k_finalize_outer
    if (gexec && g_tau == tau && g_sigma == sigma && g_eps == eps && g_k == k && g_window == window && g_stop == stop &&
        g_spec == (int)spec)
      return PDHG_OK;
    drop_graph();
    hipGraph_t g = nullptr;
    HIP_TRY(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
    int rc = PDHG_OK;
    for (int i = 0; i < window && rc == PDHG_OK; ++i) rc = launch_iteration(tau, sigma, eps, k);
    hipError_t e = hipStreamEndCapture(stream, &g);
    if (rc) {
      if (g) hipGraphDestroy(g);
      return rc;
    }
    HIP_TRY(e);
    e = hipGraphInstantiate(&gexec, g, nullptr, nullptr, 0);
    hipGraphDestroy(g);
    if (e != hipSuccess) {
      gexec = nullptr;
      return fail(PDHG_ERR_HIP, "hipGraphInstantiate failed: %s", hipGetErrorString(e));
    }
    g_tau = tau;
    g_sigma = sigma;
    g_eps = eps;
    g_k = k;
    g_window = window;
    g_stop = stop;
    g_spec = (int)spec;
    return PDHG_OK;
  }

  // A speculative iteration halted after sub-iteration 0 (done = kHaltTail): wait for the no-op launches behind it,
  // re-arm, and run the rest of its dual loop and its outer tests (launch_dual's tail + launch_outer of the full
  // schedule).  h: the control block after it (iters counts the completed iterations, the halted one included).
  int finish_halted(double sigma, double eps, int k, Ctrl& h) {
    int rc;
    HIP_TRY(hipStreamSynchronize(stream));
    int zero = 0;
    HIP_TRY(hipMemcpyAsync(&kp.ctrl->done, &zero, sizeof(int), hipMemcpyHostToDevice, stream));
    spec = false;
    if ((rc = launch_dual_tail((R)sigma, eps, k))) return rc;
    if ((rc = launch_outer(eps, k))) return rc;
    return read_ctrl(h);   // synchronizes (zero stays valid until the copy ran)
  }

  int iterate(int n, double tau, double sigma, double eps, int k, pdhg_stats* st) {
    int rc;
    if ((rc = reset_ctrl())) return rc;
    const int window = 8;   // host runs at most 2*window iterations ahead of the device
    std::vector<hipEvent_t> evs;
    if (const char* e = getenv("PDHG_GRAPH")) use_graph = atoi(e) != 0;
    // Speculative one-sub-iteration schedule (the head form, rho_alp_iters > 1): C2's T = 1 marching windows exit the
    // dual loop after sub-iteration 0 in nearly every iteration, and the rest of the loop (chunk passes, finalizes,
    // final pass, outer-sum pass: 6 launches) then only returns at once.  After a window of iterations that all ran
    // one sub-iteration, the host enqueues iterations without those launches; an iteration whose loop does not exit
    // after sub-iteration 0 halts (done = kHaltTail, every later kernel returns), and the host runs the rest of its
    // loop and its outer tests -- the launches the full schedule would have made, in the same order -- then goes on
    // with the full schedule for a few windows.  Same kernels on the same data: the states are the full schedule's
    // bit for bit.  PDHG_SPEC=0 keeps the full schedule.
    const bool spec_able = spec_ok && dual_head && k > 1 && k <= kDualMultiMax;
    // PDHG_SPEC_FORCE=1 (tests): speculate from the first iteration and again right after every halt, so the halt /
    // finish path runs as often as the loop needs more than one sub-iteration
    const bool spec_force = spec_able && [] { const char* e = getenv("PDHG_SPEC_FORCE"); return e && atoi(e) != 0; }();
    spec = spec_force;
    struct SpecOff {   // every return path leaves the full schedule for the drop-in update_* calls
      bool& s;
      ~SpecOff() { s = false; }
    } spec_off{spec};
    int cool = 0;
    long long last_iters = 0, last_inner = 0;
    auto drain_events = [&]() {
      for (auto e : evs) hipEventDestroy(e);
      evs.clear();
    };
    for (int i = 0; i < n;) {
      // a whole window from the graph when one fits and the state allows it; otherwise one eager iteration
      const bool steady = !fuse_res || res_valid;
      if (use_graph && warm && !prof && steady && i % window == 0 && n - i >= window) {
        if ((rc = ensure_graph(tau, sigma, eps, k, window))) return rc;
        HIP_TRY(hipGraphLaunch(gexec, stream));
        i += window;
        if (spec) spec_iters += window;
      } else {
        if ((rc = launch_iteration(tau, sigma, eps, k))) return rc;
        warm = true;
        ++i;
        if (spec) ++spec_iters;
      }
      const bool check = i % window == 0 && i < n;
      if (!check) continue;
      hipEvent_t e;
      HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      HIP_TRY(hipEventRecord(e, stream));
      evs.push_back(e);
      if (evs.size() < 2) continue;
      HIP_TRY(hipEventSynchronize(evs[evs.size() - 2]));
      Ctrl h;
      HIP_TRY(hipMemcpy(&h, kp.ctrl, sizeof(Ctrl), hipMemcpyDeviceToHost));
      if (h.done == kHaltTail) {
        ++spec_halts;
        if ((rc = finish_halted(sigma, eps, k, h))) return rc;
        drain_events();
        i = h.iters;              // the halted iteration is complete; the ones enqueued after it were no-ops
        spec = spec_force;
        cool = spec_force ? 0 : 4;   // windows on the full schedule before speculating again
        last_iters = h.iters;
        last_inner = h.inner_total;
        if (h.done) break;
        continue;
      }
      if (h.done) break;
      if (spec_able) {   // the checked window's iterations all ran one sub-iteration: speculate from here on
        const long long d_it = h.iters - last_iters, d_in = h.inner_total - last_inner;
        if (cool > 0) --cool;
        else if (!spec && d_it > 0 && d_in == d_it) spec = true;
        last_iters = h.iters;
        last_inner = h.inner_total;
      }
    }
    drain_events();
    Ctrl h;
    if ((rc = read_ctrl(h))) return rc;
    while (h.done == kHaltTail) {   // a halt in the last windows: finish it and run what is left
      ++spec_halts;
      if ((rc = finish_halted(sigma, eps, k, h))) return rc;
      spec = false;
      for (int i = h.iters; i < n && !h.done; ++i) {
        if ((rc = launch_iteration(tau, sigma, eps, k))) return rc;
        if ((i + 1) % window == 0 && (rc = read_ctrl(h))) return rc;
      }
      if ((rc = read_ctrl(h))) return rc;
    }
    spec = false;
    if (st) {
      st->iters_run = h.iters;
      st->status = h.done;
      st->inner_last = h.inner_count;
      st->inner_total = h.inner_total;
      st->err1 = h.err1;
      st->err2 = h.err2;
      st->err_inner = h.err_inner;
      st->rho_min = NAN;
      st->rho_max = NAN;
      st->nan_seen = h.nan_seen;
      st->first_nan_iter = h.first_nan;
    }
    primal_done = false;
    return PDHG_OK;
  }

  // ---------------- t-slab phases (multi-GPU; the caller moves planes between slabs) ----------------
  // One outer iteration of a slab (include/pdhg.h): slab_residual(rows without the rho halo) ||
  // [rho halo] -> slab_residual(the halo row) -> slab_forward -> [allgather D, S1] -> slab_fixup ->
  // slab_backward -> [allreduce sums] -> slab_primal_finalize -> slab_dual(rows without the phi_bar
  // halo) || [phi_bar halo] -> slab_dual(the halo row + sums) -> [allreduce] -> slab_dual_finalize ->
  // ... -> slab_outer -> [allreduce] -> slab_outer_finalize.  With one slab this is iterate().
  int need_slab() const { return slab ? PDHG_OK : fail(PDHG_ERR_STATE, "not a t-slab context"); }
  int slab_G(R* out) {   // [G, S2] (iteration-invariant)
    hipLaunchKernelGGL((k_slab_sums<R>), dim3((unsigned)((Mspec + 255) / 256)), dim3(256), 0, stream, kp, 0, out,
                       (size_t)0, Mspec);
    HIP_TRY(hipGetLastError());
    return PDHG_OK;
  }
  // residual rows: parts bit 0 = the rows that do not read the rho halo, bit 1 = the row that does
  // (the last row, unless this is the window's last slab)
  int slab_residual(int parts) {
    const bool rows = fast_rows || res64;   // row-range residual kernels (else the whole slab after the halo)
    const int T = pb.T, split = (rows && !kp.last_slab) ? T - 1 : (rows ? T : 0);
    int rc;
    if ((parts & 1) && (rc = launch_residual(kp, 0, split))) return rc;
    if ((parts & 2) && (rc = launch_residual(kp, split, T))) return rc;
    return PDHG_OK;
  }
  int slab_forward(R tau) { return slab_forward_part(tau, 0, 1); }
  // part `part` of `nparts` of the column blocks: blocks [b0, b1), spectral modes [m0, m1)
  void part_range(int part, int nparts, int& b0, int& b1, size_t& m0, size_t& m1) const {
    b0 = (int)((long long)kp.nb * part / nparts);
    b1 = (int)((long long)kp.nb * (part + 1) / nparts);
    const size_t Mb = (size_t)pb.nx * kp.B;
    m0 = b0 * Mb;
    m1 = b1 * Mb;
  }
  // zero-carry forward sweep + [D, S1] of one part of the column blocks (after both residual parts)
  int slab_forward_part(R tau, int part, int nparts) {
    int b0, b1;
    size_t m0, m1;
    part_range(part, nparts, b0, b1, m0, m1);
    if (b1 <= b0) return PDHG_OK;
    KP<R> p = kp;
    p.tau = tau;
    p.xt_phase = 1;
    p.b0 = b0;
    int rc = launch_precond(p, b1 - b0);
    if (rc) return rc;
    hipLaunchKernelGGL((k_slab_sums<R>), dim3((unsigned)((m1 - m0 + 255) / 256)), dim3(256), 0, stream, kp, 1, dsbuf,
                       m0, m1);
    HIP_TRY(hipGetLastError());
    return PDHG_OK;
  }
  int slab_carry_out_part(void* dst, int part, int nparts) {   // [D, S1] modes [m0, m1) into dst (2 planes)
    int b0, b1;
    size_t m0, m1;
    part_range(part, nparts, b0, b1, m0, m1);
    if (m1 <= m0) return PDHG_OK;
    R* d = static_cast<R*>(dst);
    HIP_TRY(hipMemcpyAsync(d + m0, dsbuf + m0, (m1 - m0) * sizeof(R), hipMemcpyDeviceToDevice, stream));
    HIP_TRY(hipMemcpyAsync(d + Mspec + m0, dsbuf + Mspec + m0, (m1 - m0) * sizeof(R), hipMemcpyDeviceToDevice, stream));
    return PDHG_OK;
  }
  int slab_backward_part(R tau, int part, int nparts) {   // carry-corrected backward sweep of one part
    int b0, b1;
    size_t m0, m1;
    part_range(part, nparts, b0, b1, m0, m1);
    if (b1 <= b0) return PDHG_OK;
    KP<R> p = kp;
    p.tau = tau;
    p.xt_phase = 2;
    p.b0 = b0;
    return launch_precond(p, b1 - b0);
  }
  int slab_update(R tau, double* sums) { return launch_primal(tau, 4, 0, sums); }   // after every part
  // classify the modes once from everybody's [G, S2]: long-range where some slab's gain G >= delta
  int slab_long_modes(const R* allGS, int nranks, double delta, int* K_out) {
    R* gmax = nullptr;
    HIP_TRY(hipMalloc(&gmax, Mspec * sizeof(R)));
    hipLaunchKernelGGL((k_slab_gmax<R>), dim3((unsigned)((Mspec + 255) / 256)), dim3(256), 0, stream, allGS, Mspec,
                       nranks, gmax);
    std::vector<R> h(Mspec);
    hipError_t e = hipMemcpyAsync(h.data(), gmax, Mspec * sizeof(R), hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    hipFree(gmax);
    HIP_TRY(e);
    std::vector<int> pos(Mspec), idx;
    for (size_t m = 0; m < Mspec; ++m) {
      const bool lng = !((double)h[m] < delta);   // NaN counts as long (exact path)
      pos[m] = lng ? (int)idx.size() : -1;
      if (lng) idx.push_back((int)m);
    }
    int rc;
    if (!long_pos && (rc = alloc(&long_pos, Mspec))) return rc;
    if (long_idx) {   // re-classification: drop the old list
      hipFree(long_idx);
      allocs.erase(std::find(allocs.begin(), allocs.end(), (void*)long_idx));
      long_idx = nullptr;
    }
    if (!idx.empty() && (rc = alloc(&long_idx, idx.size()))) return rc;
    HIP_TRY(hipMemcpyAsync(long_pos, pos.data(), Mspec * sizeof(int), hipMemcpyHostToDevice, stream));
    if (!idx.empty())
      HIP_TRY(hipMemcpyAsync(long_idx, idx.data(), idx.size() * sizeof(int), hipMemcpyHostToDevice, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    long_K = (int)idx.size();
    *K_out = long_K;
    return PDHG_OK;
  }
  int slab_fixup_nb(const R* D_left, const R* S1_right, const R* allLong, const R* allGS, int rank, int nranks,
                    int part = 0, int nparts = 1) {
    if (long_K < 0) return fail(PDHG_ERR_STATE, "pdhg_slab_long_modes has not been called");
    int b0, b1;
    size_t m0, m1;
    part_range(part, nparts, b0, b1, m0, m1);
    if (m1 <= m0) return PDHG_OK;
    hipLaunchKernelGGL((k_slab_fix_nb<R>), dim3((unsigned)((m1 - m0 + 255) / 256)), dim3(256), 0, stream, kp, dsbuf,
                       D_left, S1_right, allLong, long_pos, long_K, allGS, rank, nranks, carry_y, m0, m1);
    HIP_TRY(hipGetLastError());
    return PDHG_OK;
  }
  int slab_fixup(const R* allDS, const R* allGS, int rank, int nranks) {
    hipLaunchKernelGGL((k_slab_fix<R>), dim3((unsigned)((Mspec + 255) / 256)), dim3(256), 0, stream, kp, allDS,
                       allGS, rank, nranks, carry_y);
    HIP_TRY(hipGetLastError());
    return PDHG_OK;
  }
  int slab_backward(R tau, double* sums) { return launch_primal(tau, 2 | 4, 2, sums); }
  int slab_primal_finalize(const double* sums) {
    hipLaunchKernelGGL(k_finalize_primal, dim3(1), dim3(1024), 0, stream, sums, 1, 0, kp.ctrl);
    HIP_TRY(hipGetLastError());
    return PDHG_OK;
  }
  // dual rows: parts bit 0 = the rows that do not read the phi_bar halo, bit 1 = the row that does
  // (row 0, unless this is the window's first slab) followed by the sum reduction into `sums`
  int slab_dual(R sigma, int k, int sub, double* sums, int parts) {
    KP<R> p = kp;
    p.sigma = sigma;
    p.inplace = (k <= 1) ? 1 : 0;
    p.sub = sub;
    if (!p.inplace && !two_sets)
      return fail(PDHG_ERR_STATE, "rho_alp_iters=%d needs a context created with rho_alp_iters > 1", k);
    const int T = pb.T, split = fast_dual ? (kp.j0 > 0 ? 1 : 0) : T;   // halo rows [0, split)
    const int gz_in = fast_dual ? (T - split + jchunk_d - 1) / jchunk_d : 0;
    if ((parts & 1) && fast_dual) {
      ProfScope ps(this, "dual");
      launch_dual_fast(p, split, T, 0);
    }
    if (!(parts & 2)) {
      HIP_TRY(hipGetLastError());
      return PDHG_OK;
    }
    int nrows_d;
    if (fast_dual) {
      if (split > 0) {
        ProfScope ps(this, "dual");
        launch_dual_fast(p, 0, split, gz_in);
      }
      nrows_d = gxd * gyd * (gz_in + (split > 0 ? 1 : 0));
    } else {
      ProfScope ps(this, "dual");
      dim3 g(gx5, g5);
      switch (pb.egno) {
        case 1: hipLaunchKernelGGL((k_dual_2d<R, 1>), g, dim3(256), 0, stream, p); break;
        case 2: hipLaunchKernelGGL((k_dual_2d<R, 2>), g, dim3(256), 0, stream, p); break;
        default: hipLaunchKernelGGL((k_dual_2d<R, 3>), g, dim3(256), 0, stream, p); break;
      }
      nrows_d = gx5 * g5;
    }
    hipLaunchKernelGGL(k_reduce_vec, dim3(1), dim3(1024), 0, stream, p.partials, nrows_d, 3 + 3 * na, 0.0, sums);
    HIP_TRY(hipGetLastError());
    return PDHG_OK;
  }
  int slab_dual_finalize(double eps, int sub, const double* sums) {
    hipLaunchKernelGGL(k_finalize_dual, dim3(1), dim3(1024), 0, stream, sums, 1, na, n_dead, eps, sub, kp.ctrl);
    HIP_TRY(hipGetLastError());
    return PDHG_OK;
  }
  int slab_outer(int k, double* sums) {
    if (k > 1) {
      hipLaunchKernelGGL((k_outer_sums<R>), dim3(g_outer), dim3(256), 0, stream, kp, (size_t)pb.T * plane(), 0);
      hipLaunchKernelGGL(k_reduce_vec, dim3(1), dim3(1024), 0, stream, kp.partials, g_outer, kNumSums, 0.0, sums);
    }
    HIP_TRY(hipGetLastError());
    return PDHG_OK;
  }
  int slab_outer_finalize(double eps, int k, const double* sums) {
    hipLaunchKernelGGL(k_finalize_outer, dim3(1), dim3(1024), 0, stream, sums, k > 1 ? 1 : 0, na, eps, k > 1 ? 1 : 0,
                       stop_conv, stop_nan, kp.ctrl);
    HIP_TRY(hipGetLastError());
    return PDHG_OK;
  }
  // planes out: 0 rho row 0 (current set), 1 phi_bar row T, 2 [D, S1] (2 spectral planes),
  // 3 [D, S1] of the long-range modes (2 x long_K)
  int slab_plane_out(int which, void* dst) {
    const size_t npl = plane();
    switch (which) {
      case 0:
        hipLaunchKernelGGL((k_copy_cur_rho<R>), dim3(1024), dim3(256), 0, stream, kp, (R*)dst, npl);
        break;
      case 1: HIP_TRY(hipMemcpyAsync(dst, kp.phibar + (size_t)pb.T * npl, npl * sizeof(R), hipMemcpyDeviceToDevice, stream)); break;
      case 2: HIP_TRY(hipMemcpyAsync(dst, dsbuf, 2 * Mspec * sizeof(R), hipMemcpyDeviceToDevice, stream)); break;
      case 3:
        if (long_K < 0) return fail(PDHG_ERR_STATE, "pdhg_slab_long_modes has not been called");
        if (long_K > 0)
          hipLaunchKernelGGL((k_slab_gather_long<R>), dim3((unsigned)((long_K + 255) / 256)), dim3(256), 0, stream,
                             dsbuf, Mspec, long_idx, long_K, (R*)dst);
        break;
      default: return fail(PDHG_ERR_ARG, "unknown plane %d", which);
    }
    HIP_TRY(hipGetLastError());
    return PDHG_OK;
  }
  // planes in: 0 rho halo (next slab's rho row 0), 1 phi_bar row 0 (previous slab's phi_bar row T)
  int slab_plane_in(int which, const void* src) {
    const size_t npl = plane();
    switch (which) {
      case 0: HIP_TRY(hipMemcpyAsync(halo_rho, src, npl * sizeof(R), hipMemcpyDeviceToDevice, stream)); break;
      case 1: HIP_TRY(hipMemcpyAsync(kp.phibar, src, npl * sizeof(R), hipMemcpyDeviceToDevice, stream)); break;
      default: return fail(PDHG_ERR_ARG, "unknown plane %d", which);
    }
    return PDHG_OK;
  }
  int set_stream(hipStream_t s) {
    HIP_TRY(hipStreamSynchronize(stream));
    if (own_stream) HIP_TRY(hipStreamDestroy(stream));
    stream = s;
    own_stream = false;
    return PDHG_OK;
  }
  // ---------------- x-slab phases (multi-GPU for T = 1 windows; the caller moves data between ranks) ------------
  // One outer iteration (include/pdhg.h): halo_out(0) -> [allgather] -> halo_in(0) -> residual ->
  // wire(0) -> [all-to-all] -> wire(1) -> precond -> wire(2) -> [all-to-all] -> wire(3) -> update(sums) ->
  // halo_out(1) -> [allgather] || [allreduce sums] -> primal_finalize -> halo_in(1) -> dual ... as a t-slab.
  int need_xslab() const { return xslab ? PDHG_OK : fail(PDHG_ERR_STATE, "not an x-slab context"); }
  KP<R> col_params() const {   // the x transform of this rank's column blocks (whole x lines)
    KP<R> q = kp;
    q.nx = xs_nxg;
    q.nb = xs_nbs;
    q.work = colwork;
    q.lamy = lamy_base + (size_t)xs_rank * xs_nbs * kp.B;
    q.xt_phase = 0;
    q.xl0 = 0;
    q.xl1 = xs_nxg;
    return q;
  }
  size_t xs_chunk() const { return (size_t)pb.T * xs_nbs * xs_nloc * kp.B; }   // wire floats per rank pair
  size_t xs_halo_elems(int which) const { return (size_t)2 * (which == 0 ? 1 + na : 1) * pb.T * pb.ny; }
  int xs_wire(int stage, void* buf) {
    // 0: rows -> wire (after the residual), 1: wire -> cols, 2: cols -> wire (after the precond), 3: wire -> rows
    const size_t L = (size_t)xs_nloc * kp.B;
    const size_t total4 = xs_chunk() * xs_P / 4;
    const unsigned g = (unsigned)std::max<size_t>(1, std::min<size_t>((total4 + 255) / 256, 8192));
    R* S = static_cast<R*>(buf);
    if (stage == 0 || stage == 3)
      hipLaunchKernelGGL((k_xs_rows_wire<R>), dim3(g), dim3(256), 0, stream, kp.work, S, stage == 0 ? 0 : 1, xs_P,
                         pb.T, kp.nb, xs_nbs, pb.nx, kp.xl0, kp.B, L);
    else if (stage == 1 || stage == 2)
      hipLaunchKernelGGL((k_xs_cols_wire<R>), dim3(g), dim3(256), 0, stream, colwork, S, stage == 2 ? 0 : 1, xs_P,
                         pb.T, xs_nbs, xs_nxg, xs_nloc, kp.B, L);
    else
      return fail(PDHG_ERR_ARG, "unknown wire stage %d", stage);
    HIP_TRY(hipGetLastError());
    return PDHG_OK;
  }
  int xs_halo_out(int which, void* dst) {
    if (which != 0 && which != 1) return fail(PDHG_ERR_ARG, "unknown halo %d", which);
    const unsigned g = (unsigned)std::max<size_t>(1, std::min<size_t>((xs_halo_elems(which) + 255) / 256, 4096));
    hipLaunchKernelGGL((k_xs_halo_out<R>), dim3(g), dim3(256), 0, stream, kp, which, static_cast<R*>(dst));
    HIP_TRY(hipGetLastError());
    return PDHG_OK;
  }
  int xs_halo_in(int which, const void* left, const void* right) {
    if (which != 0 && which != 1) return fail(PDHG_ERR_ARG, "unknown halo %d", which);
    const unsigned g = (unsigned)std::max<size_t>(1, std::min<size_t>((xs_halo_elems(which) + 255) / 256, 4096));
    // Neumann x edges (bc_x 1): the first slab's left ghost and the last slab's right ghost replicate the slab's own
    // edge row instead of the ring neighbour's
    const int own_l = (pb.bc_x == 1 && xs_x0 == 0) ? 1 : 0, own_r = (pb.bc_x == 1 && xs_x0 + xs_nloc == xs_nxg) ? 1 : 0;
    hipLaunchKernelGGL((k_xs_halo_in<R>), dim3(g), dim3(256), 0, stream, kp, which, static_cast<const R*>(left),
                       static_cast<const R*>(right), own_l, own_r);
    HIP_TRY(hipGetLastError());
    if (which == 0) res_valid = false;
    return PDHG_OK;
  }
  int xs_residual() { return launch_residual(kp, 0, pb.T); }
  int xs_precond() { return launch_precond(col_params()); }
  int xs_update(R tau, double* sums) { return launch_primal(tau, 4, 0, sums); }

  int slab_status(pdhg_stats* st) {
    Ctrl h;
    int rc;
    if ((rc = read_ctrl(h))) return rc;
    st->iters_run = h.iters;
    st->status = h.done;
    st->inner_last = h.inner_count;
    st->inner_total = h.inner_total;
    st->err1 = h.err1;
    st->err2 = h.err2;
    st->err_inner = h.err_inner;
    st->rho_min = NAN;
    st->rho_max = NAN;
    st->nan_seen = h.nan_seen;
    st->first_nan_iter = h.first_nan;
    return PDHG_OK;
  }

  // ---------------- state ----------------
  bool live(int a, int comp, int n_ctrl) const {   // which (array, component) is stored
    if (pb.ndim == 1 || pb.egno == 3) return a < 2 && comp == 0;
    (void)n_ctrl;
    return (a < 2) ? comp == 0 : comp == 1;
  }
  int n_ctrl() const { return (pb.ndim == 1 || pb.egno == 3) ? 1 : 2; }
  int n_alp_ref() const { return pb.ndim == 1 ? 2 : 4; }

  void compute_row0_sq(const std::vector<R>& row0) {
    double s = 0.0;   // live rows only (x-slab: [xl0, xl1) of the padded local rows)
    const size_t ny = pb.ny;
    for (size_t i = (size_t)kp.xl0 * ny; i < (size_t)kp.xl1 * ny; ++i) s += (double)row0[i] * (double)row0[i];
    row0_sq = s;
  }

  int set_state(const double* phi, const double* rho, const double* alp) {
    res_valid = false;
    const size_t npl = plane();
    const int T = pb.T;
    // the parts given overwrite the CURRENT buffer set (two sets when rho_alp_iters > 1), so a part passed as null
    // keeps the device's values -- window marching re-seeds phi alone when rho / alp are already resident
    int cur = 0;
    HIP_TRY(hipMemcpyAsync(&cur, &kp.ctrl->cur, sizeof(int), hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    const size_t nphi = (size_t)(T + 1) * npl;
    std::unique_ptr<R[]> buf(new R[nphi]);   // not value-initialised: filled before every copy out of it
    // fp64 planes straight from the caller's arrays (same layout); fp32 through a narrowing copy
    auto src_of = [&](const double* p, size_t cnt) -> const R* {
      if constexpr (sizeof(R) == 8) {
        (void)cnt;
        return p;
      } else {
        for (size_t i = 0; i < cnt; ++i) buf[i] = (R)p[i];
        return buf.get();
      }
    };
    if (phi) {
      const R* src = src_of(phi, nphi);
      H2D(kp.phi, src, nphi * sizeof(R));
      H2D(kp.phibar, src, nphi * sizeof(R));
      compute_row0_sq(std::vector<R>(src, src + npl));
    }
    const size_t n = (size_t)T * npl;
    if (rho) H2D(kp.rho[cur], src_of(rho, n), n * sizeof(R));
    if (alp) {
      const int nc = n_ctrl(), nar = n_alp_ref();
      for (int a = 0; a < nar; ++a)
        for (int c = 0; c < nc; ++c)
          if (!live(a, c, nc))
            for (size_t i = 0; i < n; ++i)
              if (alp[((size_t)a * n + i) * nc + c] != 0.0)
                return fail(PDHG_ERR_UNSUPPORTED,
                            "alp[%d][...][%d] is a dead control component (identically zero in the reference "
                            "examples) but holds non-zero values; only live components are stored", a, c);
      for (int a = 0; a < nar; ++a)
        for (int c = 0; c < nc; ++c) {
          if (!live(a, c, nc)) continue;
          for (size_t i = 0; i < n; ++i) buf[i] = (R)alp[((size_t)a * n + i) * nc + c];
          H2D(kp.alp[cur][a], buf.get(), n * sizeof(R));
        }
    }
    Ctrl h{};
    h.cur = cur;
    h.row0_sq = row0_sq;
    H2D(kp.ctrl, &h, sizeof(Ctrl));
    primal_done = false;
    return PDHG_OK;
  }

  int set_phi_bar(const double* pbar) {
    const size_t n = (size_t)(pb.T + 1) * plane();
    std::vector<R> buf(n);
    for (size_t i = 0; i < n; ++i) buf[i] = (R)pbar[i];
    H2D(kp.phibar, buf.data(), n * sizeof(R));
    return PDHG_OK;
  }

  int get_phi_bar(double* pbar) {
    HIP_TRY(hipStreamSynchronize(stream));
    const size_t n = (size_t)(pb.T + 1) * plane();
    std::vector<R> buf(n);
    HIP_TRY(hipMemcpy(buf.data(), kp.phibar, n * sizeof(R), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < n; ++i) pbar[i] = (double)buf[i];
    return PDHG_OK;
  }

  int get_state(double* phi, double* rho, double* alp) {
    HIP_TRY(hipStreamSynchronize(stream));
    Ctrl h;
    int rc;
    if ((rc = read_ctrl(h))) return rc;
    const int cur = h.cur;
    const size_t npl = plane();
    const int T = pb.T;
    const size_t nphi = (size_t)(T + 1) * npl;
    std::unique_ptr<R[]> buf(new R[nphi]);   // not value-initialised: every element read is copied in first
    const size_t n = (size_t)T * npl;
    // fp64 planes straight into the caller's arrays (same layout); fp32 through the buffer and a widening copy
    auto plane_out = [&](double* dst, const R* src, size_t cnt) -> int {
      if constexpr (sizeof(R) == 8) {
        HIP_TRY(hipMemcpy(dst, src, cnt * sizeof(R), hipMemcpyDeviceToHost));
      } else {
        HIP_TRY(hipMemcpy(buf.get(), src, cnt * sizeof(R), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < cnt; ++i) dst[i] = (double)buf[i];
      }
      return PDHG_OK;
    };
    if (phi && (rc = plane_out(phi, kp.phi, nphi))) return rc;
    if (rho && (rc = plane_out(rho, kp.rho[cur], n))) return rc;
    if (alp) {
      const int nc = n_ctrl(), nar = n_alp_ref();
      std::memset(alp, 0, sizeof(double) * n * nc * nar);
      for (int a = 0; a < nar; ++a)
        for (int c = 0; c < nc; ++c) {
          if (!live(a, c, nc)) continue;
          HIP_TRY(hipMemcpy(buf.get(), kp.alp[cur][a], n * sizeof(R), hipMemcpyDeviceToHost));
          for (size_t i = 0; i < n; ++i) alp[((size_t)a * n + i) * nc + c] = (double)buf[i];
        }
    }
    return PDHG_OK;
  }

  // rows [row0, row0 + nrows) of phi / phi_bar ([T+1]) and rho / alp ([T]) in the reference layouts
  int get_rows(int row0, int nrows, double* phi, double* pbar, double* rho, double* alp) {
    const int T = pb.T;
    if (row0 < 0 || nrows < 1 || row0 + nrows > T + 1 || ((rho || alp) && row0 + nrows > T))
      return fail(PDHG_ERR_ARG, "rows [%d, %d) outside phi [0, %d) / rho, alp [0, %d)", row0, row0 + nrows, T + 1, T);
    HIP_TRY(hipStreamSynchronize(stream));
    Ctrl h;
    int rc;
    if ((rc = read_ctrl(h))) return rc;
    const size_t npl = plane(), n = (size_t)nrows * npl, off = (size_t)row0 * npl;
    std::unique_ptr<R[]> buf(sizeof(R) == 8 && !alp ? nullptr : new R[n]);
    auto rows_out = [&](double* dst, const R* src) -> int {
      if constexpr (sizeof(R) == 8) {
        HIP_TRY(hipMemcpy(dst, src + off, n * sizeof(R), hipMemcpyDeviceToHost));
      } else {
        HIP_TRY(hipMemcpy(buf.get(), src + off, n * sizeof(R), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < n; ++i) dst[i] = (double)buf[i];
      }
      return PDHG_OK;
    };
    if (phi && (rc = rows_out(phi, kp.phi))) return rc;
    if (pbar && (rc = rows_out(pbar, kp.phibar))) return rc;
    if (rho && (rc = rows_out(rho, kp.rho[h.cur]))) return rc;
    if (alp) {
      const int nc = n_ctrl(), nar = n_alp_ref();
      std::memset(alp, 0, sizeof(double) * n * nc * nar);
      for (int a = 0; a < nar; ++a)
        for (int c = 0; c < nc; ++c) {
          if (!live(a, c, nc)) continue;
          HIP_TRY(hipMemcpy(buf.get(), kp.alp[h.cur][a] + off, n * sizeof(R), hipMemcpyDeviceToHost));
          for (size_t i = 0; i < n; ++i) alp[((size_t)a * n + i) * nc + c] = (double)buf[i];
        }
    }
    return PDHG_OK;
  }

  int init_state(const double* g) {
    res_valid = false;
    const size_t npl = plane();
    const int T = pb.T;
    std::vector<R> row(npl);
    for (size_t i = 0; i < npl; ++i) row[i] = (R)g[i];
    compute_row0_sq(row);
    R* d_row;
    int rc;
    HIP_TRY(hipMalloc((void**)&d_row, npl * sizeof(R)));
    H2D(d_row, row.data(), npl * sizeof(R));
    const int grid = 4096;
    hipLaunchKernelGGL((k_bcast_rows<R>), dim3(grid), dim3(256), 0, stream, kp.phi, d_row, npl, T + 1);
    hipLaunchKernelGGL((k_bcast_rows<R>), dim3(grid), dim3(256), 0, stream, kp.phibar, d_row, npl, T + 1);
    hipLaunchKernelGGL((k_fill<R>), dim3(grid), dim3(256), 0, stream, kp.rho[0], (size_t)T * npl, (R)pb.c_on_rho);
    for (int a = 0; a < na; ++a)
      hipLaunchKernelGGL((k_fill<R>), dim3(grid), dim3(256), 0, stream, kp.alp[0][a], (size_t)T * npl, (R)0);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(stream));
    hipFree(d_row);
    Ctrl h{};
    h.row0_sq = row0_sq;
    H2D(kp.ctrl, &h, sizeof(Ctrl));
    (void)rc;
    primal_done = false;
    return PDHG_OK;
  }

  int update_primal(double tau) {
    int rc;
    if ((rc = reset_ctrl())) return rc;
    if ((rc = launch_primal((R)tau))) return rc;
    HIP_TRY(hipStreamSynchronize(stream));
    primal_done = true;
    return PDHG_OK;
  }

  int update_dual(double sigma, double eps, int k, int* inner_used) {
    int rc;
    Ctrl h;
    if ((rc = read_ctrl(h))) return rc;
    h.done = 0;
    h.inner_done = 0;
    h.inner_count = 0;
    h.kstar_found = 0;
    H2D(kp.ctrl, &h, sizeof(Ctrl));
    if ((rc = launch_dual((R)sigma, eps, k))) return rc;
    if (primal_done) {
      if ((rc = launch_outer(eps, k))) return rc;
    } else if (k > 1) {
      // no primal in this pairing: still move the state to the current buffer set
      hipLaunchKernelGGL(k_finalize_outer, dim3(1), dim3(1024), 0, stream, kp.partials, 0, na, -1.0, 1, 0, 0, kp.ctrl);
    }
    if ((rc = read_ctrl(h))) return rc;
    if (inner_used) *inner_used = h.inner_count;
    primal_done = false;
    return PDHG_OK;
  }

  int errors(double* e1, double* e2) {
    Ctrl h;
    int rc;
    if ((rc = read_ctrl(h))) return rc;
    if (e1) *e1 = h.err1;
    if (e2) *e2 = h.err2;
    return PDHG_OK;
  }

  double algorithmic_bytes(int k, const std::string& cls) const {
    const double N = (double)pb.T * (double)(kp.xl1 - kp.xl0) * (double)pb.ny;   // live rows (x-slab)
    const double S = (double)sizeof(R);
    const bool d2 = pb.ndim == 2;
    const double nr = 1.0 + na;   // rho + live alp arrays
    if (cls == "iteration") {
      // 2-D 4N(14 + 11k + 5[k>1]), 1-D 4N(12 + 7k + 3[k>1]); generalised to S and na
      if (d2) return S * N * (14.0 + 11.0 * k + 5.0 * (k > 1));
      return S * N * (12.0 + 7.0 * k + 3.0 * (k > 1));
    }
    // fused residual: the dual also writes the residual rows (+1), the tile-edge row terms (2 rows per 8)
    // and the strip-edge column terms (2 per 256); the residual kernel reads them and writes the spectrum
    const double edge = !fuse_res ? 0.0 : d2 ? 2.0 / 8.0 + 2.0 / (64.0 * dual_ypl) : 2.0 / 64.0;   // 1-D: per wave
    if (cls == "dual") return S * N * (1.0 + 2.0 * nr + (fuse_res ? 1.0 + edge : 0.0));
    if (cls == "residual") return S * N * (fuse_res ? 2.0 + edge : nr + 1.0);
    if (cls == "precond") return S * N * (d2 ? 4.0 : 2.0);   // 2-D: x-DHT+Thomas fwd (2N) + bwd+x-DHT (2N)
    if (cls == "update") return S * N * 4.0;                 // read U, phi; write phi, phi_bar
    return -1.0;
  }
};

struct CtxBox {
  uint32_t magic = kCtxMagic;
  int precision;
  std::unique_ptr<ImplBase> impl;
};

// the context behind a handle, with its device made current (a thread may drive contexts on several GPUs:
// every kernel launch, allocation and hipFuncSetAttribute of the call then lands on the context's device)
CtxBox* ctx_box(pdhg_ctx* ctx) {
  if (!ctx) return nullptr;
  CtxBox* b = reinterpret_cast<CtxBox*>(ctx);
  if (b->magic != kCtxMagic || !b->impl) return nullptr;
  if (hipSetDevice(b->impl->device) != hipSuccess) return nullptr;
  return b;
}

template <typename F>
int dispatch(pdhg_ctx* ctx, F&& f) {
  CtxBox* b = ctx_box(ctx);
  if (!b) return fail(PDHG_ERR_ARG, "null or foreign context handle");
  if (b->precision == 8) return f(*static_cast<Impl<double>*>(b->impl.get()));
  return f(*static_cast<Impl<float>*>(b->impl.get()));
}

// phases shared by the t-slab and x-slab contexts (begin, finalizers, dual, outer, status)
template <typename F>
int phase_dispatch(pdhg_ctx* ctx, F&& f) {
  return dispatch(ctx, [&](auto& im) {
    if (!im.slab && !im.xslab) return fail(PDHG_ERR_STATE, "not a t-slab / x-slab context");
    return f(im);
  });
}

template <typename F>
int xslab_dispatch(pdhg_ctx* ctx, F&& f) {
  return dispatch(ctx, [&](auto& im) {
    int rc = im.need_xslab();
    return rc ? rc : f(im);
  });
}

// t-slab contexts are fp32 or fp64 (the reference's arithmetic); planes crossing this ABI are in the context's
// precision (RealOf)
template <typename F>
int slab_dispatch(pdhg_ctx* ctx, F&& f) {
  return dispatch(ctx, [&](auto& im) {
    int rc = im.need_slab();
    return rc ? rc : f(im);
  });
}
template <typename I>
using RealOf = typename std::remove_reference<I>::type::Real;

// the multi-device context (pdhg_multi.hpp): the done flag of a slab's control block, read by a synchronous
// copy that does not wait for the slab's stream (the caller synchronised on an event recorded after the
// iteration it wants), and the device a slab computes on
int slab_done_flag(pdhg_ctx* ctx, int* done) {
  return slab_dispatch(ctx, [&](auto& im) {
    HIP_TRY(hipMemcpy(im.h_done, &im.kp.ctrl->done, sizeof(int), hipMemcpyDeviceToHost));
    *done = *im.h_done;
    return (int)PDHG_OK;
  });
}
int slab_device(pdhg_ctx* ctx, int* device) {
  return slab_dispatch(ctx, [&](auto& im) {
    int d = -1;
    HIP_TRY(hipGetDevice(&d));
    *device = d;
    return (int)PDHG_OK;
  });
}

}  // namespace

extern "C" {

const char* pdhg_last_error(void) { return g_err.c_str(); }
#ifndef PDHG_BUILD_ID
#define PDHG_BUILD_ID "unknown"
#endif
__attribute__((used)) static const char kBuildTag[] = "PDHG_BUILD_ID=" PDHG_BUILD_ID;   // read by build()
const char* pdhg_build_id(void) { return kBuildTag + 14; }
int pdhg_abi_version(void) { return PDHG_ABI_VERSION; }

int pdhg_device_count(int* count) {
  if (!count) return fail(PDHG_ERR_ARG, "null count");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  *count = (e == hipSuccess) ? n : 0;
  return PDHG_OK;
}

int pdhg_create(const pdhg_problem* prob, int device, pdhg_ctx** out) {
  if (!prob || !out) return fail(PDHG_ERR_ARG, "null argument");
  *out = nullptr;
  const pdhg_problem& p = *prob;
  if (p.ndim != 1 && p.ndim != 2) return fail(PDHG_ERR_ARG, "ndim %d not implemented", p.ndim);
  if (p.egno < 1 || p.egno > 3) return fail(PDHG_ERR_ARG, "egno %d not implemented", p.egno);
  if (p.egno == 3 && p.ndim != 2) return fail(PDHG_ERR_ARG, "egno 3 requires ndim 2 (set_fns.py:96)");
  if (p.nx < 3 || (p.ndim == 2 && p.ny < 3)) return fail(PDHG_ERR_ARG, "grid must be at least 3 points per axis");
  if (p.ndim == 1 && p.ny != 1) return fail(PDHG_ERR_ARG, "ndim 1 requires ny == 1");
  if (p.T < 1) return fail(PDHG_ERR_ARG, "T must be >= 1");
  if (!(p.dx > 0) || !(p.dt > 0) || (p.ndim == 2 && !(p.dy > 0))) return fail(PDHG_ERR_ARG, "grid spacings must be > 0");
  if (!p.xs || (p.ndim == 2 && !p.ys)) return fail(PDHG_ERR_ARG, "grid coordinates required");
  if (p.precision != 4 && p.precision != 8) return fail(PDHG_ERR_ARG, "precision must be 4 or 8");
  if (p.rho_alp_iters < 1) return fail(PDHG_ERR_ARG, "rho_alp_iters must be >= 1");
  // preconditioner boundary conditions (utils_precond.py:121-124, :157-163)
  if (p.ndim == 1 && p.bc_x != 0) return fail(PDHG_ERR_UNSUPPORTED, "H1_precond_1d supports bc=0 only");
  if (p.ndim == 2 && !((p.bc_x == 0 || p.bc_x == 1) && p.bc_y == 0))
    return fail(PDHG_ERR_UNSUPPORTED, "bc (%d,%d): H1_precond_2d supports (0,0) and (1,0) only "
                                      "(utils_precond.py:157-163)", p.bc_x, p.bc_y);
  if (p.ndim == 1 && p.Ct < 0) return fail(PDHG_ERR_ARG, "Ct must be >= 0");
  if (p.C < 0) return fail(PDHG_ERR_ARG, "C must be >= 0");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(PDHG_ERR_HIP, "no HIP device available");
  if (device < 0 || device >= ndev) return fail(PDHG_ERR_ARG, "device %d out of range (%d devices)", device, ndev);
  auto box = std::make_unique<CtxBox>();
  box->precision = p.precision;
  int rc;
  if (p.precision == 8) {
    auto im = std::make_unique<Impl<double>>();
    im->pb = p;
    im->device = device;
    rc = im->setup();
    box->impl = std::move(im);
  } else {
    auto im = std::make_unique<Impl<float>>();
    im->pb = p;
    im->device = device;
    rc = im->setup();
    box->impl = std::move(im);
  }
  if (rc) return rc;
  *out = reinterpret_cast<pdhg_ctx*>(box.release());
  return PDHG_OK;
}

int pdhg_destroy(pdhg_ctx* ctx) {
  if (!ctx) return PDHG_OK;
  CtxBox* b = ctx_box(ctx);
  if (!b) return fail(PDHG_ERR_ARG, "foreign context handle");
  b->magic = 0;
  delete b;
  return PDHG_OK;
}

int pdhg_set_state(pdhg_ctx* ctx, const double* phi, const double* rho, const double* alp) {
  return dispatch(ctx, [&](auto& im) { return im.set_state(phi, rho, alp); });
}
int pdhg_get_state(pdhg_ctx* ctx, double* phi, double* rho, double* alp) {
  return dispatch(ctx, [&](auto& im) { return im.get_state(phi, rho, alp); });
}
int pdhg_get_phi_bar(pdhg_ctx* ctx, double* phi_bar) {
  if (!phi_bar) return fail(PDHG_ERR_ARG, "null phi_bar");
  return dispatch(ctx, [&](auto& im) { return im.get_phi_bar(phi_bar); });
}
int pdhg_set_phi_bar(pdhg_ctx* ctx, const double* phi_bar) {
  if (!phi_bar) return fail(PDHG_ERR_ARG, "null phi_bar");
  return dispatch(ctx, [&](auto& im) { return im.set_phi_bar(phi_bar); });
}
int pdhg_get_rows(pdhg_ctx* ctx, int row0, int nrows, double* phi, double* phi_bar, double* rho, double* alp) {
  return dispatch(ctx, [&](auto& im) { return im.get_rows(row0, nrows, phi, phi_bar, rho, alp); });
}
int pdhg_init_state(pdhg_ctx* ctx, const double* g) {
  if (!g) return fail(PDHG_ERR_ARG, "null g");
  return dispatch(ctx, [&](auto& im) { return im.init_state(g); });
}
int pdhg_update_primal(pdhg_ctx* ctx, double tau) {
  return dispatch(ctx, [&](auto& im) { return im.update_primal(tau); });
}
int pdhg_update_dual(pdhg_ctx* ctx, double sigma, double eps, int rho_alp_iters, int* inner_used) {
  if (rho_alp_iters < 1) return fail(PDHG_ERR_ARG, "rho_alp_iters must be >= 1");
  return dispatch(ctx, [&](auto& im) { return im.update_dual(sigma, eps, rho_alp_iters, inner_used); });
}
int pdhg_errors(pdhg_ctx* ctx, double* err1, double* err2) {
  return dispatch(ctx, [&](auto& im) { return im.errors(err1, err2); });
}
int pdhg_inner_error(pdhg_ctx* ctx, double* err) {
  if (!err) return fail(PDHG_ERR_ARG, "null err");
  return dispatch(ctx, [&](auto& im) {
    Ctrl h;
    int rc = im.read_ctrl(h);
    if (rc) return rc;
    *err = h.err_inner;
    return (int)PDHG_OK;
  });
}
int pdhg_iterate(pdhg_ctx* ctx, int n_iters, double tau, double sigma, double eps, int rho_alp_iters,
                 pdhg_stats* out) {
  if (n_iters < 0 || rho_alp_iters < 1) return fail(PDHG_ERR_ARG, "bad iteration counts");
  return dispatch(ctx, [&](auto& im) { return im.iterate(n_iters, tau, sigma, eps, rho_alp_iters, out); });
}
int pdhg_set_stop_rules(pdhg_ctx* ctx, int stop_on_converge, int stop_on_nan) {
  return dispatch(ctx, [&](auto& im) {
    im.stop_conv = stop_on_converge ? 1 : 0;
    im.stop_nan = stop_on_nan ? 1 : 0;
    return (int)PDHG_OK;
  });
}
int pdhg_synchronize(pdhg_ctx* ctx) {
  return dispatch(ctx, [&](auto& im) {
    HIP_TRY(hipStreamSynchronize(im.stream));
    return (int)PDHG_OK;
  });
}
int pdhg_device_bytes(pdhg_ctx* ctx, unsigned long long* bytes) {
  if (!bytes) return fail(PDHG_ERR_ARG, "null bytes");
  return dispatch(ctx, [&](auto& im) {
    *bytes = im.dev_bytes;
    return (int)PDHG_OK;
  });
}
int pdhg_path_info(pdhg_ctx* ctx, const char* key, int* value) {
  if (!key || !value) return fail(PDHG_ERR_ARG, "null argument");
  return dispatch(ctx, [&](auto& im) {
    const std::string k(key);
    if (k == "fused_residual") *value = im.fuse_res ? 1 : 0;
    else if (k == "fast_rows") *value = im.fast_rows ? 1 : 0;
    else if (k == "contig_fail") *value = im.n_contig_fail;
    else if (k == "res64") *value = im.res64 ? 1 : 0;
    else if (k == "dual_multi") *value = im.dual_multi ? 1 : 0;   // rho_alp_iters > 1: chunked dual passes
    else if (k == "dual_head") *value = im.dual_head ? 1 : 0;   // ... sub-iteration 0 alone, then the chunks
    else if (k == "spec") *value = im.spec_ok ? 1 : 0;   // iterate(): speculative one-sub-iteration schedule allowed
    else if (k == "spec_iters") *value = (int)std::min<long long>(im.spec_iters, INT_MAX);   // ... iterations run so
    else if (k == "spec_halts") *value = (int)std::min<long long>(im.spec_halts, INT_MAX);   // ... and halts (cumulative)
    else if (k == "dual64") *value = (sizeof(typename std::remove_reference<decltype(im)>::type::Real) == 8 && im.fast_dual) ? 1 : 0;
    else if (k == "fast_dual") *value = im.fast_dual ? im.dual_rx : -1;
    else if (k == "dual_ypl") *value = im.fast_dual && im.dual_rx ? im.dual_ypl : 0;
    else if (k == "res64_nt") *value = im.res64 ? (im.pb.ny == 2048 ? im.res64_nt2048 : 512) : 0;
    else if (k == "upd_t1") *value = (im.res64 && im.pb.ny == 2048) ? im.upd_t1 : 0;
    else if (k == "t1_g16") *value = (im.t1_xt64 && im.t1_xt && im.t1_g16 && (im.pb.nx == 2048 || im.pb.nx == 4096)) ? 1 : 0;
    else if (k == "dual_one") *value = (im.fast_dual && !im.dual_rx && im.jchunk_d == 1 && im.dual_one) ? 1 : 0;
    else if (k == "fast_xt")
      *value = im.fast_xt ? (im.half_real && im.xt_dma_hr ? 5 : im.batch_xt && !im.half_real
                                                                    ? (im.xt_dma && im.pb.nx == 4096 ? 4 : 3)
                                                                    : im.ws_xt ? 2 : 1) : 0;
    else if (k == "half_real") *value = im.half_real ? 1 : 0;
    else if (k == "fourstep") *value = im.fourstep ? 1 : 0;
    else if (k == "glb_line") *value = im.glb_line ? 1 : 0;
    else if (k == "ip_rows") *value = im.ip_rows ? 1 : 0;   // fp64 ny = 8192 row pairs in one padded line
    else if (k == "upd8192") *value = im.upd8192 ? 1 : 0;   // fp64 ny = 8192: 2-row fast update
    else if (k == "tc_spec") *value = im.tc_spec ? 1 : 0;   // fp64 C3: task-order residual spectrum
    else if (k == "to_c4") *value = im.to_c4 ? 1 : 0;       // C4: task-order residual spectrum + transpose
    else if (k == "thomas_chunk") *value = im.thomas_chunk ? 1 : 0;
    else if (k == "fs_wide") *value = (im.fourstep && im.fs_wide && !im.fs16) ? 1 : 0;
    else if (k == "fs16") *value = im.fs16 ? 1 : 0;
    else if (k == "rows_rw") *value = im.fast_rows ? im.RWf : 0;   // rows per fast row-kernel workgroup
    // threads of the fast row kernels as launched (ny = 4096: 512 instead of 1024 per half_nt)
    else if (k == "row_threads") *value = im.nt_row;
    else if (k == "res_threads") *value = im.fast_rows ? ((im.NTf == 1024 && (im.half_nt & 1) && im.fuse_res) ? 512
                                                                                                      : im.NTf) : 0;
    else if (k == "upd_threads") *value = im.fast_rows ? ((im.NTf == 1024 && im.RWf == 8 && (im.half_nt & 2))
                                                              ? 512 : im.NTf) : 0;
    else if (k == "f64_xt") *value = im.f64_xt ? 1 : 0;   // fp64 nx = 4096 x transform (kernels_xt_f64.hpp)
    else if (k == "t1_xt64") *value = (im.t1_xt64 && im.t1_xt) ? 1 : 0;   // fp64 T = 1: carry-free x transform
    else if (k == "graph") *value = im.use_graph ? 1 : 0;   // iteration windows replayed from a HIP graph
    else if (k == "graph_window") *value = im.gexec ? im.g_window : 0;   // 0: no graph captured yet
    else return fail(PDHG_ERR_ARG, "unknown path key %s", key);
    return (int)PDHG_OK;
  });
}
int pdhg_profile_enable(pdhg_ctx* ctx, int enable) {
  return dispatch(ctx, [&](auto& im) {
    HIP_TRY(hipStreamSynchronize(im.stream));
    im.prof = enable != 0;
    for (auto& kv : im.prof_ev) kv.second.used = 0;
    return (int)PDHG_OK;
  });
}
int pdhg_profile_query(pdhg_ctx* ctx, const char* cls, double* total_ms, int* launches) {
  if (!cls || !total_ms || !launches) return fail(PDHG_ERR_ARG, "null argument");
  return dispatch(ctx, [&](auto& im) {
    HIP_TRY(hipStreamSynchronize(im.stream));
    *total_ms = 0.0;
    *launches = 0;
    auto it = im.prof_ev.find(cls);
    if (it == im.prof_ev.end()) return (int)PDHG_OK;
    for (size_t i = 0; i < it->second.used; ++i) {
      float ms = 0.f;
      HIP_TRY(hipEventElapsedTime(&ms, it->second.ev[i].first, it->second.ev[i].second));
      *total_ms += ms;
    }
    *launches = (int)it->second.used;
    return (int)PDHG_OK;
  });
}
int pdhg_algorithmic_bytes(pdhg_ctx* ctx, int k, const char* cls, double* bytes) {
  if (!cls || !bytes) return fail(PDHG_ERR_ARG, "null argument");
  return dispatch(ctx, [&](auto& im) {
    *bytes = im.algorithmic_bytes(k, cls);
    return *bytes < 0 ? fail(PDHG_ERR_ARG, "unknown kernel class %s", cls) : (int)PDHG_OK;
  });
}

/* ---------------- t-slab decomposition ---------------- */
int pdhg_create_slab(const pdhg_problem* prob, int j0, int T_total, int device, pdhg_ctx** out) {
  if (!prob || !out) return fail(PDHG_ERR_ARG, "null argument");
  *out = nullptr;
  if (j0 < 0 || prob->T < 1 || j0 + prob->T > T_total)
    return fail(PDHG_ERR_ARG, "slab rows [%d, %d) outside the window of %d rows", j0, j0 + prob->T, T_total);
  if (prob->ndim != 2) return fail(PDHG_ERR_UNSUPPORTED, "t-slab decomposition is 2-D only");
  // validate the rest exactly like pdhg_create, then rebuild as a slab (fp32, or fp64 = the reference's arithmetic,
  // jaxsrc/update_fns_in_pdhg.py:10)
  pdhg_ctx* probe = nullptr;
  pdhg_problem q = *prob;
  q.T = 1;
  int rc = pdhg_create(&q, device, &probe);
  if (rc) return rc;
  pdhg_destroy(probe);
  auto box = std::make_unique<CtxBox>();
  box->precision = prob->precision;
  auto build = [&](auto tag) {
    using Rt = decltype(tag);
    auto im = std::make_unique<Impl<Rt>>();
    im->pb = *prob;
    im->device = device;
    im->slab = true;
    im->slab_j0 = j0;
    im->slab_Tg = T_total;
    const int r = im->setup();
    box->impl = std::move(im);
    return r;
  };
  rc = prob->precision == 8 ? build(0.0) : build(0.f);
  if (rc) return rc;
  *out = reinterpret_cast<pdhg_ctx*>(box.release());
  return PDHG_OK;
}

int pdhg_set_stream(pdhg_ctx* ctx, void* hip_stream) {   // null = the device's default stream
  return dispatch(ctx, [&](auto& im) { return im.set_stream(static_cast<hipStream_t>(hip_stream)); });
}
int pdhg_slab_begin(pdhg_ctx* ctx) {
  return phase_dispatch(ctx, [&](auto& im) { return im.reset_ctrl(); });
}
int pdhg_slab_carry_gain(pdhg_ctx* ctx, void* GS_out) {
  if (!GS_out) return fail(PDHG_ERR_ARG, "null plane");
  return slab_dispatch(ctx, [&](auto& im) { return im.slab_G(static_cast<RealOf<decltype(im)>*>(GS_out)); });
}
int pdhg_slab_residual(pdhg_ctx* ctx, int parts) {
  return slab_dispatch(ctx, [&](auto& im) { return im.slab_residual(parts); });
}
int pdhg_slab_forward(pdhg_ctx* ctx, double tau) {
  return slab_dispatch(ctx, [&](auto& im) { return im.slab_forward((RealOf<decltype(im)>)tau); });
}
int pdhg_slab_fixup(pdhg_ctx* ctx, const void* all_DS, const void* all_GS, int rank, int nranks) {
  if (!all_DS || !all_GS) return fail(PDHG_ERR_ARG, "null carry planes");
  if (rank < 0 || rank >= nranks) return fail(PDHG_ERR_ARG, "rank %d of %d", rank, nranks);
  return slab_dispatch(ctx, [&](auto& im) {
    return im.slab_fixup(static_cast<const RealOf<decltype(im)>*>(all_DS), static_cast<const RealOf<decltype(im)>*>(all_GS), rank, nranks);
  });
}
int pdhg_slab_long_modes(pdhg_ctx* ctx, const void* all_GS, int nranks, double delta, int* K) {
  if (!all_GS || !K || nranks < 1) return fail(PDHG_ERR_ARG, "null plane / count or nranks < 1");
  return slab_dispatch(ctx, [&](auto& im) {
    return im.slab_long_modes(static_cast<const RealOf<decltype(im)>*>(all_GS), nranks, delta, K);
  });
}
int pdhg_slab_fixup_nb(pdhg_ctx* ctx, const void* D_left, const void* S1_right, const void* all_long,
                       const void* all_GS, int rank, int nranks) {
  if (!D_left || !S1_right || !all_GS || rank < 0 || rank >= nranks)
    return fail(PDHG_ERR_ARG, "null plane or rank %d outside [0, %d)", rank, nranks);
  return slab_dispatch(ctx, [&](auto& im) {
    return im.slab_fixup_nb(static_cast<const RealOf<decltype(im)>*>(D_left), static_cast<const RealOf<decltype(im)>*>(S1_right),
                            static_cast<const RealOf<decltype(im)>*>(all_long), static_cast<const RealOf<decltype(im)>*>(all_GS), rank, nranks);
  });
}
int pdhg_slab_backward(pdhg_ctx* ctx, double tau, double* sums) {
  if (!sums) return fail(PDHG_ERR_ARG, "null sums");
  return slab_dispatch(ctx, [&](auto& im) { return im.slab_backward((RealOf<decltype(im)>)tau, sums); });
}
int pdhg_slab_primal_finalize(pdhg_ctx* ctx, const double* sums) {
  if (!sums) return fail(PDHG_ERR_ARG, "null sums");
  return phase_dispatch(ctx, [&](auto& im) { return im.slab_primal_finalize(sums); });
}
int pdhg_slab_dual(pdhg_ctx* ctx, double sigma, int rho_alp_iters, int sub, double* sums, int parts) {
  if (!sums) return fail(PDHG_ERR_ARG, "null sums");
  return phase_dispatch(ctx, [&](auto& im) { return im.slab_dual((RealOf<decltype(im)>)sigma, rho_alp_iters, sub, sums, parts); });
}
int pdhg_slab_dual_finalize(pdhg_ctx* ctx, double eps, int sub, const double* sums) {
  if (!sums) return fail(PDHG_ERR_ARG, "null sums");
  return phase_dispatch(ctx, [&](auto& im) { return im.slab_dual_finalize(eps, sub, sums); });
}
int pdhg_slab_outer(pdhg_ctx* ctx, int rho_alp_iters, double* sums) {
  if (!sums) return fail(PDHG_ERR_ARG, "null sums");
  return phase_dispatch(ctx, [&](auto& im) { return im.slab_outer(rho_alp_iters, sums); });
}
int pdhg_slab_outer_finalize(pdhg_ctx* ctx, double eps, int rho_alp_iters, const double* sums) {
  if (!sums) return fail(PDHG_ERR_ARG, "null sums");
  return phase_dispatch(ctx, [&](auto& im) { return im.slab_outer_finalize(eps, rho_alp_iters, sums); });
}
int pdhg_slab_plane_out(pdhg_ctx* ctx, int which, void* dst) {
  if (!dst) return fail(PDHG_ERR_ARG, "null plane");
  return slab_dispatch(ctx, [&](auto& im) { return im.slab_plane_out(which, dst); });
}
int pdhg_slab_plane_in(pdhg_ctx* ctx, int which, const void* src) {
  if (!src) return fail(PDHG_ERR_ARG, "null plane");
  return slab_dispatch(ctx, [&](auto& im) { return im.slab_plane_in(which, src); });
}
int pdhg_slab_status(pdhg_ctx* ctx, pdhg_stats* st) {
  if (!st) return fail(PDHG_ERR_ARG, "null stats");
  return phase_dispatch(ctx, [&](auto& im) { return im.slab_status(st); });
}
int pdhg_slab_plane_size(pdhg_ctx* ctx, unsigned long long* spatial, unsigned long long* spectral) {
  if (!spatial || !spectral) return fail(PDHG_ERR_ARG, "null argument");
  return slab_dispatch(ctx, [&](auto& im) {
    *spatial = im.plane();
    *spectral = im.Mspec;
    return (int)PDHG_OK;
  });
}

/* ---------------- x-slab decomposition ---------------- */
int pdhg_create_xslab(const pdhg_problem* prob, int rank, int nranks, int device, pdhg_ctx** out) {
  if (!prob || !out) return fail(PDHG_ERR_ARG, "null argument");
  *out = nullptr;
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(PDHG_ERR_ARG, "rank %d of %d", rank, nranks);
  if (prob->ndim != 2) return fail(PDHG_ERR_UNSUPPORTED, "x-slab decomposition is 2-D only");
  // bc (0,0), or egno 3's (1,0): Neumann x edges -- the first / last slab's outer ghost row replicates its own edge
  // row (nb_index bc 1), the transposed x lines take the DCT of the generic x kernel
  if (prob->bc_y != 0 || (prob->bc_x != 0 && prob->bc_x != 1))
    return fail(PDHG_ERR_UNSUPPORTED, "x-slab decomposition needs bc (0,0) or (1,0)");
  if (prob->nx % nranks || (prob->nx / nranks) % 8)
    return fail(PDHG_ERR_UNSUPPORTED, "nx=%d must split into %d slabs of a multiple of 8 rows", prob->nx, nranks);
  // validate the rest exactly like pdhg_create (one row of the global grid), then build the slab
  pdhg_ctx* probe = nullptr;
  pdhg_problem q = *prob;
  q.T = 1;
  int rc = pdhg_create(&q, device, &probe);
  if (rc) return rc;
  pdhg_destroy(probe);
  const int nloc = prob->nx / nranks, nxl = nloc + 16, x0 = rank * nloc;
  auto box = std::make_unique<CtxBox>();
  box->precision = prob->precision;
  // fp32, or fp64 = the reference's arithmetic (jaxsrc/update_fns_in_pdhg.py:10): the x-slab kernels, the fp64 row
  // kernels (ny = 2048 / 4096) and the fp64 duals honour the live-row bounds; the column blocks go through the
  // generic x kernel
  auto build = [&](auto tag) {
    using Rt = decltype(tag);
    auto im = std::make_unique<Impl<Rt>>();
    im->xslab = true;
    im->xs_rank = rank;
    im->xs_P = nranks;
    im->xs_nxg = prob->nx;
    im->xs_nloc = nloc;
    im->xs_x0 = x0;
    im->xs_local.resize(nxl);
    for (int i = 0; i < nxl; ++i) {   // local row i = global row x0 - 8 + i (periodic; clamped at Neumann edges)
      const int gi = x0 - 8 + i;
      const int g = prob->bc_x == 1 ? std::min(std::max(gi, 0), prob->nx - 1) : ((gi % prob->nx) + prob->nx) % prob->nx;
      im->xs_local[i] = prob->xs[g];
    }
    im->pb = *prob;
    im->pb.nx = nxl;
    im->pb.xs = im->xs_local.data();
    im->device = device;
    const int r = im->setup();
    box->impl = std::move(im);
    return r;
  };
  rc = prob->precision == 8 ? build(0.0) : build(0.f);
  if (rc) return rc;
  *out = reinterpret_cast<pdhg_ctx*>(box.release());
  return PDHG_OK;
}
int pdhg_xslab_layout(pdhg_ctx* ctx, int* x0, int* nloc, int* nx_local, int* xl0) {
  if (!x0 || !nloc || !nx_local || !xl0) return fail(PDHG_ERR_ARG, "null argument");
  return xslab_dispatch(ctx, [&](auto& im) {
    *x0 = im.xs_x0;
    *nloc = im.xs_nloc;
    *nx_local = im.pb.nx;
    *xl0 = im.kp.xl0;
    return (int)PDHG_OK;
  });
}
int pdhg_xslab_sizes(pdhg_ctx* ctx, unsigned long long* wire, unsigned long long* halo_state,
                     unsigned long long* halo_phibar) {
  if (!wire || !halo_state || !halo_phibar) return fail(PDHG_ERR_ARG, "null argument");
  return xslab_dispatch(ctx, [&](auto& im) {
    *wire = im.xs_chunk() * im.xs_P;
    *halo_state = im.xs_halo_elems(0);
    *halo_phibar = im.xs_halo_elems(1);
    return (int)PDHG_OK;
  });
}
int pdhg_xslab_halo_out(pdhg_ctx* ctx, int which, void* dst) {
  if (!dst) return fail(PDHG_ERR_ARG, "null buffer");
  return xslab_dispatch(ctx, [&](auto& im) { return im.xs_halo_out(which, dst); });
}
int pdhg_xslab_halo_in(pdhg_ctx* ctx, int which, const void* from_left, const void* from_right) {
  if (!from_left || !from_right) return fail(PDHG_ERR_ARG, "null buffer");
  return xslab_dispatch(ctx, [&](auto& im) { return im.xs_halo_in(which, from_left, from_right); });
}
int pdhg_xslab_residual(pdhg_ctx* ctx) {
  return xslab_dispatch(ctx, [&](auto& im) { return im.xs_residual(); });
}
int pdhg_xslab_wire(pdhg_ctx* ctx, int stage, void* buf) {
  if (!buf) return fail(PDHG_ERR_ARG, "null buffer");
  return xslab_dispatch(ctx, [&](auto& im) { return im.xs_wire(stage, buf); });
}
int pdhg_xslab_precond(pdhg_ctx* ctx) {
  return xslab_dispatch(ctx, [&](auto& im) { return im.xs_precond(); });
}
int pdhg_xslab_update(pdhg_ctx* ctx, double tau, double* sums) {
  if (!sums) return fail(PDHG_ERR_ARG, "null sums");
  return xslab_dispatch(ctx, [&](auto& im) { return im.xs_update((RealOf<decltype(im)>)tau, sums); });
}

int pdhg_slab_part_modes(pdhg_ctx* ctx, int part, int nparts, unsigned long long* m0, unsigned long long* m1) {
  if (!m0 || !m1 || nparts < 1 || part < 0 || part >= nparts) return fail(PDHG_ERR_ARG, "part %d of %d", part, nparts);
  return slab_dispatch(ctx, [&](auto& im) {
    int b0, b1;
    size_t a, b;
    im.part_range(part, nparts, b0, b1, a, b);
    *m0 = a;
    *m1 = b;
    return (int)PDHG_OK;
  });
}
int pdhg_slab_forward_part(pdhg_ctx* ctx, double tau, int part, int nparts) {
  if (nparts < 1 || part < 0 || part >= nparts) return fail(PDHG_ERR_ARG, "part %d of %d", part, nparts);
  return slab_dispatch(ctx, [&](auto& im) { return im.slab_forward_part((RealOf<decltype(im)>)tau, part, nparts); });
}
int pdhg_slab_carry_out_part(pdhg_ctx* ctx, void* dst, int part, int nparts) {
  if (!dst || nparts < 1 || part < 0 || part >= nparts) return fail(PDHG_ERR_ARG, "null plane or part %d of %d", part, nparts);
  return slab_dispatch(ctx, [&](auto& im) { return im.slab_carry_out_part(dst, part, nparts); });
}
int pdhg_slab_fixup_nb_part(pdhg_ctx* ctx, const void* D_left, const void* S1_right, const void* all_long,
                            const void* all_GS, int rank, int nranks, int part, int nparts) {
  if (!D_left || !S1_right || !all_GS || rank < 0 || rank >= nranks || nparts < 1 || part < 0 || part >= nparts)
    return fail(PDHG_ERR_ARG, "null plane, rank %d of %d or part %d of %d", rank, nranks, part, nparts);
  return slab_dispatch(ctx, [&](auto& im) {
    return im.slab_fixup_nb(static_cast<const RealOf<decltype(im)>*>(D_left), static_cast<const RealOf<decltype(im)>*>(S1_right),
                            static_cast<const RealOf<decltype(im)>*>(all_long), static_cast<const RealOf<decltype(im)>*>(all_GS), rank, nranks,
                            part, nparts);
  });
}
int pdhg_slab_backward_part(pdhg_ctx* ctx, double tau, int part, int nparts) {
  if (nparts < 1 || part < 0 || part >= nparts) return fail(PDHG_ERR_ARG, "part %d of %d", part, nparts);
  return slab_dispatch(ctx, [&](auto& im) { return im.slab_backward_part((RealOf<decltype(im)>)tau, part, nparts); });
}
int pdhg_slab_update(pdhg_ctx* ctx, double tau, double* sums) {
  if (!sums) return fail(PDHG_ERR_ARG, "null sums");
  return slab_dispatch(ctx, [&](auto& im) { return im.slab_update((RealOf<decltype(im)>)tau, sums); });
}

}  // extern "C"

#include "pdhg_multi.hpp"   // multi-device context over the t-slab entry points above
