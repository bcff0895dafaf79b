// Kernel parameter block (passed by value) and problem-plugin device functions.
#pragma once
#include "common.hpp"
#include "fft_lds.hpp"

namespace pdhg {

template <typename R>
struct KP {
  int egno, ndim, bcx, bcy;
  int nx, ny, T;
  int B, lB, nb;           // spectral block width (power of two), log2(B), number of column blocks
  int rows_per_wg;         // rows handled by one residual / inverse-y workgroup (even)
  int na;                  // live control arrays stored (2 or 4)
  int inplace;             // dual updates rho/alp in place (rho_alp_iters == 1)
  int sub;                 // dual sub-iteration index of this launch
  int dbg;                 // timing experiments only (env PDHG_DBG); 0 in production
  int nbsync;              // k_dual_lds_2d: neighbour-flag sync between the row waves instead of a block barrier
  int tile_j;              // residual task tiling: TJ time rows x 4 row groups per tile (1 = off)
  int row_base, row_cnt;   // fast residual launch: time rows [row_base, row_base + row_cnt)
  R inv_dx, inv_dy, inv_dt, inv_dx2, inv_dy2;
  R epsl, c_over_dt;
  R ae;                    // Ct/dt^2 (1-D) or 1/dt^2 (2-D): off-diagonal magnitude of the t-Laplacian
  R tau, sigma;
  R inv_n;                 // 1/(nx*ny): DHT normalisation
  const R* ax;             // f coefficient a(x) = (x-1)^2+0.1 (egno 1/2) or x coordinate (egno 3)  [nx]
  const R* ay;             // a(y) [ny]
  const R* lamx;           // symbol of the x Laplacian per mode (<= 0) [nx]
  const R* lamy;           // symbol of the y Laplacian per mode [nb*B], zero padded
  const R* d0_1d;          // 1-D: (C - lam)^pow per mode [nx]
  R C;
  R* phi;                  // [T+1][nx][ny]
  R* phibar;               // [T+1][nx][ny]
  R* work;                 // spectral work buffer
  // residual spectrum in task order (fp64 C3, tc_spec): the row kernels store each task's RW rows x all ky as one
  // contiguous run [T][nx/RW][N/B][RW][B] instead of RW*B-real chunks of the blocked layout; the x kernel's forward
  // sweep reads it and writes b' into `work` (blocked).  nullptr: the residual goes to `work` directly
  R* rspec;
  R* rho[2];               // [T][nx][ny]
  R* alp[2][4];            // live control components, each [T][nx][ny]
  double* partials;        // [blocks][kNumSums]
  Ctrl* ctrl;
  // t-slab decomposition (multi-GPU): this context owns unknown rows [j0, j0+T) of Tg.
  // slab == 0 -> j0 = 0, Tg = T, last_slab = 1 and no halos (single-context path).
  int slab, j0, Tg, last_slab;
  int xt_phase;            // x-transform/Thomas kernel: 0 both sweeps, 1 forward only, 2 backward only
  const R* rho_halo;       // rho row j0+T (first row of the next slab) [nx][ny]; null on the last slab
  const R* carry_y;        // backward right carry x_{j0+T} (spectral, work-row layout); null = zero
  void* gscr;              // per-workgroup global FFT scratch (1-D lines beyond LDS), 2 lines per slot
  int half_real;           // 2-D x-transform on one real column per block (nx = 8192, B = 1)
  // bc_x = 1 (egno 3, utils_precond.py:159-174): DCT-II along x instead of the DHT
  const R* cx;             // y-symbol factor per x mode: 2 cos(pi kx / 2nx) (DCT) or 1 [nx]
  const cplx<R>* dctw;     // e^{-i pi k / 2nx}, k < nx (DCT only)
  // fused residual (k_dual_lds_2d FR / k_res_fwdy_fused_2d): residual rows formed by the dual sweep
  R* res;                  // [T][nx][ny]
  R* ex;                   // [T][nx/8][2][ny]: tile-edge row terms (0: row x0 from x0-1, 1: row x0+7 from x0+8)
  R* ey;                   // [T][nx][ny/256][2]: strip-edge column terms (0: first column, 1: last column)
  // x-slab decomposition (pdhg_create_xslab): rows [xl0, xl1) are this rank's own rows; the others are
  // ghost / padding rows, which the dual neither stores nor sums (all rows otherwise: 0, nx)
  int xl0, xl1;
  // x transform on a column-block range (t-slab: the carry exchange of one part overlaps the other's sweep):
  // workgroup b handles block b0 + b
  int b0;
};

// neighbour index along an axis of length n with boundary condition bc
// (utils_diff_op.py:5-7): returns -1 when the value is a Dirichlet zero.
__device__ __forceinline__ int nb_index(int i, int n, int bc) {
  if (i >= 0 && i < n) return i;
  if (bc == 0) return (i < 0) ? i + n : i - n;       // periodic (jnp.roll)
  if (bc == 1) return (i < 0) ? 0 : n - 1;           // Neumann: one-sided difference 0 / mirrored Dxx
  return -1;                                         // Dirichlet: zero outside
}

template <typename R>
__device__ __forceinline__ R load_or_zero(const R* __restrict__ p, int idx) {
  return idx >= 0 ? p[idx] : (R)0;
}

// f1 = f(alp1)^+ , f2 = f(alp2)^- for the x (d=0) / y (d=1) controls,
// update_fns_in_pdhg.py:13-47 with f_fn of set_fns.py:96-160.
// egno 1/2: f = -a * alp ; egno 3: f_x = alp, f_y = x coordinate.
template <typename R>
__device__ __forceinline__ R fpos(R f) { return f * (R)(f >= (R)0 ? 1 : 0); }
template <typename R>
__device__ __forceinline__ R fneg(R f) { return f * (R)(f < (R)0 ? 1 : 0); }

// alpha prox (set_fns.py:63-95 base functions + masks :108-110, :132-138, :157-159).
// D = one-sided derivative of phi_bar, a = coefficient, p = (rho+1e-4)/sigma (param_inv, set_fns.py:127),
// q = prox_recip(rho, sigma, p): the one reciprocal a grid point's controls share (egno 2: 1/p; egno 1/3:
// 1/(1+p)), so a point costs one division (egno 2) instead of one per control plus param_inv's.
// right = true -> alp1 (mask f >= 0), false -> alp2 (mask f < 0).
template <typename R, int EGNO>
__device__ __forceinline__ R prox_recip(R rho, R sigma, R p) {
  if constexpr (EGNO == 2) return sigma / (rho + (R)1e-4);
  else return (R)1 / ((R)1 + p);
}
template <typename R, int EGNO>
__device__ __forceinline__ R alp_prox(R alp, R D, R a, R p, R q, bool right) {
  R n;
  R f;
  if constexpr (EGNO == 1) {
    n = (D * a + p * alp) * q;
    f = -(a * n);
  } else if constexpr (EGNO == 2) {
    n = D * a * q + alp;
    n = nclamp<R>(n, (R)-1, (R)1);
    f = -(a * n);
  } else {  // egno 3 x-controls: f = alp, coefficient -1 on D
    n = (-D + p * alp) * q;
    f = n;
  }
  const bool keep = right ? (f >= (R)0) : (f < (R)0);
  return n * (R)(keep ? 1 : 0);
}

template <typename R, int EGNO>
__device__ __forceinline__ R fval(R alp, R a) {
  if constexpr (EGNO == 3) return alp;
  else return -(a * alp);
}

template <typename R, int EGNO>
__device__ __forceinline__ R lag(R a2) {   // numerical L per component (set_fns.py:26-49)
  if constexpr (EGNO == 2) return (R)0 * a2;
  else return a2 / (R)2;
}

}  // namespace pdhg
