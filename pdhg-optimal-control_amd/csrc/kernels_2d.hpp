// 2-D PDHG kernels (ndim = 2).  One outer iteration:
//   k_res_fwdy_2d   continuity residual (update_fns_in_pdhg.py:83-96) + forward DHT along y
//   k_precond_xt_2d forward DHT along x + Thomas forward sweep in t + back substitution
//                   + inverse DHT along x   (utils_precond.py:142-178, Thomas :10-35)
//   k_invy_update_2d inverse DHT along y + phi' = phi + tau U, phi_bar = 2 phi' - phi, err1 sums
//                   (update_fns_in_pdhg.py:146, utils_pdhg_solver.py:55,58)
//   k_dual_2d       alpha prox, HJ residual, rho prox, err sums (update_fns_in_pdhg.py:150-165)
//
// Spectral work layout ("blocked"): work[k][b][x][c] with ky = b*B + c, so a
// column block is one contiguous [nx][B] slab (= B/2 interleaved complex lines
// for the x transform) and a row's block segment is B contiguous values.
#pragma once
#include "params.hpp"

namespace pdhg {

// ---- residual of the continuity equation at unknown row j (res row j+1) ----
template <typename R, int EGNO>
__device__ __forceinline__ R cont_residual_2d(const KP<R>& p, const R* __restrict__ rho, const R* const* alp, int j,
                                              int x, int y) {
  const int nx = p.nx, ny = p.ny;
  const size_t plane = (size_t)nx * ny;
  const R* rj = rho + (size_t)j * plane;
  const R* a1x = alp[0] + (size_t)j * plane;
  const R* a2x = alp[1] + (size_t)j * plane;
  const size_t c = (size_t)x * ny + y;
  const int xm = nb_index(x - 1, nx, p.bcx), xp = nb_index(x + 1, nx, p.bcx);
  const int ym = nb_index(y - 1, ny, p.bcy), yp = nb_index(y + 1, ny, p.bcy);
  const R eps = (R)1e-4;
  const R r0 = rj[c];
  const R rnext = (j + 1 < p.T) ? rho[(size_t)(j + 1) * plane + c] : p.last_slab ? (R)0 : p.rho_halo[c];
  // Dt_increasedim (utils_diff_op.py:193-206)
  R res = (rnext - r0) * p.inv_dt;
  if (p.epsl != (R)0) {   // Dxx/Dyy_increasedim (:241-253, :287-299)
    const R rxm = (xm >= 0) ? rj[(size_t)xm * ny + y] : (R)0;
    const R rxp = (xp >= 0) ? rj[(size_t)xp * ny + y] : (R)0;
    const R rym = (ym >= 0) ? rj[(size_t)x * ny + ym] : (R)0;
    const R ryp = (yp >= 0) ? rj[(size_t)x * ny + yp] : (R)0;
    res = res + p.epsl * ((rxp + rxm - (R)2 * r0) * p.inv_dx2);
    res = res + p.epsl * ((ryp + rym - (R)2 * r0) * p.inv_dy2);
  }
  // fluxes m = (rho + eps) f  (get_f_vals_2d, :29-47)
  const R axc = p.ax[x];
  const R ayc = p.ay[y];
  // Dx_left_increasedim(m1x): (m1x[x] - m1x[x-1]) / dx
  const R m1x_c = (r0 + eps) * fpos<R>(fval<R, EGNO>(a1x[c], axc));
  R m1x_m = (R)0;
  if (xm >= 0) {
    const size_t cm = (size_t)xm * ny + y;
    m1x_m = (rj[cm] + eps) * fpos<R>(fval<R, EGNO>(a1x[cm], p.ax[xm]));
  }
  // Dx_right_increasedim(m2x): (m2x[x+1] - m2x[x]) / dx
  const R m2x_c = (r0 + eps) * fneg<R>(fval<R, EGNO>(a2x[c], axc));
  R m2x_p = (R)0;
  if (xp >= 0) {
    const size_t cp = (size_t)xp * ny + y;
    m2x_p = (rj[cp] + eps) * fneg<R>(fval<R, EGNO>(a2x[cp], p.ax[xp]));
  }
  R m1y_c, m1y_m = (R)0, m2y_c, m2y_p = (R)0;
  if constexpr (EGNO == 3) {
    // f_y = x coordinate for both y controls (set_fns.py:98)
    const R f1 = fpos<R>(axc), f2 = fneg<R>(axc);
    m1y_c = (r0 + eps) * f1;
    if (ym >= 0) m1y_m = (rj[(size_t)x * ny + ym] + eps) * f1;
    m2y_c = (r0 + eps) * f2;
    if (yp >= 0) m2y_p = (rj[(size_t)x * ny + yp] + eps) * f2;
  } else {
    const R* a1y = alp[2] + (size_t)j * plane;
    const R* a2y = alp[3] + (size_t)j * plane;
    m1y_c = (r0 + eps) * fpos<R>(fval<R, EGNO>(a1y[c], ayc));
    if (ym >= 0) {
      const size_t cm = (size_t)x * ny + ym;
      m1y_m = (rj[cm] + eps) * fpos<R>(fval<R, EGNO>(a1y[cm], p.ay[ym]));
    }
    m2y_c = (r0 + eps) * fneg<R>(fval<R, EGNO>(a2y[c], ayc));
    if (yp >= 0) {
      const size_t cp = (size_t)x * ny + yp;
      m2y_p = (rj[cp] + eps) * fneg<R>(fval<R, EGNO>(a2y[cp], p.ay[yp]));
    }
  }
  const R div = (m1x_c - m1x_m) * p.inv_dx + (m2x_p - m2x_c) * p.inv_dx + (m1y_c - m1y_m) * p.inv_dy +
                (m2y_p - m2y_c) * p.inv_dy;
  res = res - div;
  if (j == p.T - 1 && p.last_slab) res = res + p.c_over_dt;   // update_fns_in_pdhg.py:95 (window's last row)
  return res;
}

// flat grid over (T x npairs) row-pair tasks; block nt_row (256..1024, by LDS occupancy); LDS 2 * ny complex.
// The XCD-aware remap puts consecutive row pairs on one XCD at the same time, so the
// 32/B row pairs that fill one 128-B line of the blocked layout merge in that XCD's L2.
// NTB: launch bound (256 for nt_row = 256, 1024 for the wider launches), so the 256-thread instantiations keep
// their full register budget
template <typename R, int EGNO, class F, int NTB>
__global__ void __launch_bounds__(NTB) k_res_fwdy_2d(KP<R> p, F ply, const cplx<R>* __restrict__ twy) {
  using C = cplx<R>;
  if (p.ctrl->done) return;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  C* A = reinterpret_cast<C*>(smem_raw);
  C* Bf = A + ply.n();
  const int cur = p.ctrl->cur;
  const R* rho = p.rho[cur];
  const R* alp[4] = {p.alp[cur][0], p.alp[cur][1], p.alp[cur][2], p.alp[cur][3]};
  const int nx = p.nx, ny = p.ny, B = p.B, nb = p.nb;
  const int npairs = (nx + 1) >> 1;
  const int task = xcd_remap(blockIdx.x, gridDim.x);
  const int j = task / npairs;
  const int x0 = 2 * (task - j * npairs);
  R* wk = p.work + (size_t)j * nb * nx * B;
  const bool has2 = (x0 + 1) < nx;
#pragma unroll 2
  for (int y = threadIdx.x; y < ny; y += blockDim.x) {
    const R r0 = cont_residual_2d<R, EGNO>(p, rho, alp, j, x0, y);
    const R r1 = has2 ? cont_residual_2d<R, EGNO>(p, rho, alp, j, x0 + 1, y) : (R)0;
    A[fpos<F>(y)] = cmk<C>(r0, r1);
  }
  __syncthreads();
  const C* Z = ply.template run<C>(A, Bf, twy);
  const int ncol = nb * B;
  for (int ky = threadIdx.x; ky < ncol; ky += blockDim.x) {
    R ha = (R)0, hb = (R)0;
    if (ky < ny) hartley_line<F, C, R>(Z, ny, ky, ha, hb);
    const int b = ky >> p.lB, c = ky & (B - 1);
    R* dst = wk + ((size_t)b * nx + x0) * B + c;
    dst[0] = ha;
    if (has2) dst[B] = hb;
  }
}

// grid: nb (one workgroup per column block); block NT <= 512 (NT >= M/16, M = nx*B modes per block).
// LDS: two FFT buffers of M/2 complex + per-mode Thomas carries theta, E, b' (3 M reals)
//      = 5 M * sizeof(R)  (M = 8192 fp32 / 4096 fp64 -> 160 KiB).
// Each workgroup owns its M modes for all t: forward (DHT_x, elimination) for k = 0..T-1,
// then backward (substitution, inverse DHT_x) for k = T-1..0.  b' of rows < T-1 goes through HBM.
// t-slab (p.slab; any transform, so egno 3's DCT slabs too): the pivots are the closed form at the GLOBAL row
// j0 + k, the forward sweep starts from a zero carry and stores every row (the Neumann end only on the last
// slab), xt_phase 1 stops after it, xt_phase 2 runs only the backward sweep from the right carry (carry_y) over
// the fixed-up rows -- the phases of k_precond_xt_fast_2d (oracle/slab_oracle.py).
template <typename R, class F>
__global__ void __launch_bounds__(512) k_precond_xt_2d(KP<R> p, F plx, const cplx<R>* __restrict__ twx) {
  using C = cplx<R>;
  constexpr int PF = (sizeof(R) == 4) ? 8 : 4;   // complex prefetch registers per thread (forward)
  constexpr int PB = 2 * PF;                       // real prefetch registers per thread (backward)
  if (p.ctrl->done) return;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  const int nx = p.nx, B = p.B, T = p.T, NT = blockDim.x, tid = threadIdx.x;
  const int nl = B >> 1;
  const int M = nx * B;
  const int NC = M >> 1;
  C* A = reinterpret_cast<C*>(smem_raw);
  C* Bf = A + NC;
  R* sth = reinterpret_cast<R*>(Bf + NC);
  R* sE = sth + M;
  R* sbp = sE + M;
  const int b = blockIdx.x + p.b0;
  R* wb = p.work + (size_t)b * M;
  const size_t kstride = (size_t)p.nb * M;
  const R ae = p.ae;
  const R inv_ae = (R)1 / ae;

  const bool dct = p.dctw != nullptr;   // bc_x = 1: DCT-II along x (egno 3)
  const int j0 = p.j0, Tg = p.Tg;       // global row of local row 0, window length (single context: 0, T)
  for (int pos = tid; pos < M; pos += NT) {
    const int kx = pos >> p.lB, c = pos & (B - 1);
    const R d0 = p.C - p.lamx[kx] - p.cx[kx] * p.lamy[b * B + c];
    const R delta = d0 / ((R)2 * ae);
    const R th = log1p(delta + sqrt(delta * (delta + (R)2)));   // cosh(th) = 1 + d0/(2 ae)
    sth[pos] = th;
    sE[pos] = expm1((R)-2 * th * (R)(j0 + 1));                   // E_{j0+1}, E_m = expm1(-2 th m)
    sbp[pos] = (R)0;
  }
  if (p.xt_phase != 2) {
  C pf[PF];
  {
    const C* s0 = reinterpret_cast<const C*>(wb);
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int e = tid + i * NT;
      if (e < NC) pf[i] = s0[e];
    }
  }
  // ---------------- forward: DHT_x + elimination, k = 0..T-1 ----------------
  for (int k = 0; k < T; ++k) {
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int e = tid + i * NT;
      if (e < NC) {
        if (dct) {   // sample x of line l -> Makhoul position
          const int xs = e / nl, l = e - xs * nl;
          A[(size_t)dct_perm(xs, nx) * nl + l] = pf[i];
        } else {
          A[e] = pf[i];
        }
      }
    }
    __syncthreads();
    if (k + 1 < T) {
      const C* sn = reinterpret_cast<const C*>(wb + (size_t)(k + 1) * kstride);
#pragma unroll
      for (int i = 0; i < PF; ++i) {
        const int e = tid + i * NT;
        if (e < NC) pf[i] = sn[e];
      }
    }
    const C* Z = plx.template run<C>(A, Bf, twx);
    R* dst = wb + (size_t)k * kstride;
#pragma unroll 1
    for (int pos = tid; pos < M; pos += NT) {
      const int kx = pos >> p.lB, c = pos & (B - 1);
      R ha, hb;
      if (dct)
        dct_pair<C, R>(Z, nx, nl, kx, c >> 1, p.dctw[kx], ha, hb);
      else
        hartley_pair<C, R>(Z, nx, nl, kx, c >> 1, ha, hb);
      const R h = (c & 1) ? hb : ha;
      const R th = sth[pos];
      const R prev = sbp[pos];
      const int kg = j0 + k;   // global row
      if (k < T - 1 || !p.last_slab) {
        // 1/u_k = e^-th E_{k+1} / (ae E_{k+2})   (closed form of the Thomas pivots)
        const R E2 = expm1((R)-2 * th * (R)(kg + 2));
        const R g = (th > (R)0) ? exp(-th) * sE[pos] / E2 : (R)(kg + 1) / (R)(kg + 2);
        const R v = (h * inv_ae + prev) * g;
        sE[pos] = E2;
        sbp[pos] = v;
        dst[pos] = v;
      } else {
        // Neumann last row: u_{Tg-1} = d0 + ae expm1(-th)(1 + e^{-th(2Tg-1)}) / E_Tg
        const R d0 = p.C - p.lamx[kx] - p.cx[kx] * p.lamy[b * B + c];
        R u;
        if (th > (R)0) {
          const R ET = expm1((R)-2 * th * (R)Tg);
          u = d0 + ae * expm1(-th) * ((R)1 + exp(-th * (R)(2 * Tg - 1))) / ET;
        } else {
          u = d0 + ae / (R)Tg;
        }
        sbp[pos] = (h + ae * prev) / u;
        if (p.slab) dst[pos] = sbp[pos];   // re-read (after the carry fix-up) by the backward sweep
      }
    }
    __syncthreads();
  }
  }   // xt_phase != 2
  if (p.xt_phase == 1) return;   // forward sweep only (t-slab: the carry fix-up runs in between)
  // ---------------- backward: substitution + inverse DHT_x, k = T-1..0 ----------------
  // x_k = b'_k + g_k x_{k+1},  g_k = ae/u_k = e^-th E_{k+1}/E_{k+2}
  // single context: from x_{T-1} (the forward's Neumann row, in LDS); t-slab: from the right carry x_{j0+T}
  // over every local row of the fixed-up b' in HBM
  R* Ar = reinterpret_cast<R*>(A);
  const int ks = p.slab ? T - 1 : T - 2;   // first substituted local row
  for (int pos = tid; pos < M; pos += NT) {
    sE[pos] = expm1((R)-2 * sth[pos] * (R)(j0 + ks + 2));   // E_{k+2} of row ks
    if (p.slab) sbp[pos] = p.carry_y ? p.carry_y[(size_t)b * M + pos] : (R)0;
  }
  __syncthreads();
  R pb[PB];
  if (ks >= 0) {
    const R* s0 = wb + (size_t)ks * kstride;
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      const int pos = tid + i * NT;
      if (pos < M) pb[i] = s0[pos];
    }
  }
  for (int k = T - 1; k >= 0; --k) {
    R* wk = wb + (size_t)k * kstride;
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      const int pos = tid + i * NT;
      if (pos < M) {
        R x = sbp[pos];
        if (k <= ks) {
          const R th = sth[pos];
          const int kg = j0 + k;
          const R E1 = expm1((R)-2 * th * (R)(kg + 1));
          const R g = (th > (R)0) ? exp(-th) * E1 / sE[pos] : (R)(kg + 1) / (R)(kg + 2);
          x = pb[i] + g * x;
          sE[pos] = E1;
          sbp[pos] = x;
        }
        Ar[pos] = x;
      }
    }
    if (k >= 1 && k - 1 <= ks) {
      const R* sn = wb + (size_t)(k - 1) * kstride;
#pragma unroll
      for (int i = 0; i < PB; ++i) {
        const int pos = tid + i * NT;
        if (pos < M) pb[i] = sn[pos];
      }
    }
    __syncthreads();
    const C* Z;
    if (dct) {
      // inverse DCT-II (scipy idct) via one forward FFT: V_k = 1/2 e^{i pi k/2n} (y_k - i y_{n-k}) per
      // column (y_n = 0), z = V_a + i V_b, v = IFFT(z) = conj(FFT(conj z)) (the 1/n sits in the update's
      // 1/(nx ny)); x[2m] = v[m], x[2m+1] = v[n-1-m]
      for (int e = tid; e < NC; e += NT) {
        const int kk = e / nl, l = e - kk * nl;
        const C ck = A[(size_t)kk * nl + l];                                    // (y_a[k], y_b[k])
        const C cr = (kk == 0) ? cmk<C>((R)0, (R)0) : A[(size_t)(nx - kk) * nl + l];
        const C w = p.dctw[kk];                                                 // conj -> e^{+i pi k/2n}
        const R vax = (R)0.5 * (w.x * ck.x - w.y * cr.x), vay = (R)0.5 * (-w.x * cr.x - w.y * ck.x);
        const R vbx = (R)0.5 * (w.x * ck.y - w.y * cr.y), vby = (R)0.5 * (-w.x * cr.y - w.y * ck.y);
        Bf[e] = cmk<C>(vax - vby, -(vay + vbx));                                // conj(V_a + i V_b)
      }
      __syncthreads();
      Z = plx.template run<C>(Bf, A, twx);
    } else {
      Z = plx.template run<C>(A, Bf, twx);
    }
    for (int e = tid; e < M; e += NT) {
      const int xx = e >> p.lB, c = e & (B - 1);
      R ha, hb;
      if (dct) {
        const C v = Z[(size_t)dct_perm(xx, nx) * nl + (c >> 1)];   // conj of the FFT output
        ha = v.x;
        hb = -v.y;
      } else {
        hartley_pair<C, R>(Z, nx, nl, xx, c >> 1, ha, hb);
      }
      wk[e] = (c & 1) ? hb : ha;
    }
    __syncthreads();
  }
}

// G workgroups striding over the (T x npairs) row-pair tasks (XCD-aware, as k_res_fwdy_2d);
// block nt_row (as k_res_fwdy_2d); LDS 2 * ny complex.
// sums: [0] sum (phi'-phi)^2, [1] sum phi^2 (old), [2] sum phi'^2 (NaN detector)
template <typename R, class F, int NTB>
__global__ void __launch_bounds__(NTB) k_invy_update_2d(KP<R> p, F ply, const cplx<R>* __restrict__ twy) {
  using C = cplx<R>;
  if (p.ctrl->done) return;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  C* A = reinterpret_cast<C*>(smem_raw);
  C* Bf = A + ply.n();
  const int nx = p.nx, ny = p.ny, B = p.B, nb = p.nb;
  const int npairs = (nx + 1) >> 1;
  const int ntask = npairs * p.T;
  const size_t plane = (size_t)nx * ny;
  const R scale = p.tau * p.inv_n;
  double s[3] = {0.0, 0.0, 0.0};
  for (int task = xcd_remap(blockIdx.x, gridDim.x); task < ntask; task += gridDim.x) {
    const int j = task / npairs;
    const int x0 = 2 * (task - j * npairs);
    const R* wk = p.work + (size_t)j * nb * nx * B;
    R* phi = p.phi + (size_t)(j + 1) * plane;
    R* pbar = p.phibar + (size_t)(j + 1) * plane;
    const bool has2 = (x0 + 1) < nx;
    for (int ky = threadIdx.x; ky < ny; ky += blockDim.x) {
      const int b = ky >> p.lB, c = ky & (B - 1);
      const R* srcp = wk + ((size_t)b * nx + x0) * B + c;
      A[fpos<F>(ky)] = cmk<C>(srcp[0], has2 ? srcp[B] : (R)0);
    }
    __syncthreads();
    const C* Z = ply.template run<C>(A, Bf, twy);
    for (int y = threadIdx.x; y < ny; y += blockDim.x) {
      R u0, u1;
      hartley_line<F, C, R>(Z, ny, y, u0, u1);
      for (int r = 0; r < 2; ++r) {
        if (r == 1 && !has2) break;
        const size_t idx = (size_t)(x0 + r) * ny + y;
        const R old = phi[idx];
        const R nw = old + scale * (r ? u1 : u0);
        phi[idx] = nw;
        pbar[idx] = (R)2 * nw - old;
        const double d = (double)nw - (double)old;
        s[0] += d * d;
        s[1] += (double)old * (double)old;
        s[2] += (double)nw * (double)nw;
      }
    }
    __syncthreads();
  }
  block_reduce_store<3>(s, p.partials, blockIdx.x);
}

// One grid point of the dual step (update_fns_in_pdhg.py:150-165): alpha prox from the one-sided
// differences of phi_bar at row j+1, HJ residual (:58-70), rho prox (update_rho_2d, :115-119).
// pc/pxm/pxp/pym/pyp: phi_bar row j+1 at (x, y) and its 4 neighbours (0 outside a Dirichlet edge);
// f0c: phi_bar row j at (x, y).
// The chunked dual loop (kernels_dual_multi.hpp) uses it split in two: the phi_bar part (dual_pre: the one-sided
// differences and the time / eps terms of the HJ residual) is the same for every sub-iteration of the dual loop,
// which keeps phi_bar fixed (update_fns_in_pdhg.py:167-180); dual_core is the per-sub-iteration rest.
template <typename R>
struct DualPre {
  R DxR, DxL, DyR, DyL, vec0;
};
template <typename R>
__device__ __forceinline__ DualPre<R> dual_pre(const KP<R>& p, R pc, R pxm, R pxp, R pym, R pyp, R f0c) {
  DualPre<R> d;
  d.DxR = (pxp - pc) * p.inv_dx;
  d.DxL = (pc - pxm) * p.inv_dx;
  d.DyR = (pyp - pc) * p.inv_dy;
  d.DyL = (pc - pym) * p.inv_dy;
  R vec = (pc - f0c) * p.inv_dt;
  if (p.epsl != (R)0) {
    vec = vec - p.epsl * ((pxp + pxm - (R)2 * pc) * p.inv_dx2);
    vec = vec - p.epsl * ((pyp + pym - (R)2 * pc) * p.inv_dy2);
  }
  d.vec0 = vec;
  return d;
}
template <typename R, int EGNO>
__device__ __forceinline__ R dual_core(const KP<R>& p, const DualPre<R>& d, R rho, const R* ao, R axc, R ayc, R* an,
                                       R* fo = nullptr) {
  const R pinv = (rho + (R)1e-4) / p.sigma;              // param_inv, set_fns.py:127 (unused for egno 2)
  const R q = prox_recip<R, EGNO>(rho, p.sigma, pinv);
  an[0] = alp_prox<R, EGNO>(ao[0], d.DxR, axc, pinv, q, true);
  an[1] = alp_prox<R, EGNO>(ao[1], d.DxL, axc, pinv, q, false);
  const R f1x = fpos<R>(fval<R, EGNO>(an[0], axc));
  const R f2x = fneg<R>(fval<R, EGNO>(an[1], axc));
  R f1y, f2y, L;
  if constexpr (EGNO == 3) {
    f1y = fpos<R>(axc);
    f2y = fneg<R>(axc);
    L = lag<R, EGNO>(an[0] * an[0]) + lag<R, EGNO>(an[1] * an[1]);
  } else {
    an[2] = alp_prox<R, EGNO>(ao[2], d.DyR, ayc, pinv, q, true);
    an[3] = alp_prox<R, EGNO>(ao[3], d.DyL, ayc, pinv, q, false);
    f1y = fpos<R>(fval<R, EGNO>(an[2], ayc));
    f2y = fneg<R>(fval<R, EGNO>(an[3], ayc));
    L = lag<R, EGNO>(an[0] * an[0]) + lag<R, EGNO>(an[1] * an[1]) + lag<R, EGNO>(an[2] * an[2]) +
        lag<R, EGNO>(an[3] * an[3]);
  }
  if (fo) {   // f1x, f2x, f1y, f2y of the new controls (the next residual's fluxes, :13-47)
    fo[0] = f1x;
    fo[1] = f2x;
    fo[2] = f1y;
    fo[3] = f2y;
  }
  R vec = d.vec0 - (d.DxR * f1x + d.DxL * f2x + d.DyR * f1y + d.DyL * f2y);
  vec = vec - L;
  return nmax<R>(rho + p.sigma * vec, (R)0);
}
// the per-sub-iteration kernels' form: one function, the phi_bar terms formed after the controls (the
// compiler's FMA contraction follows this order; the chunked loop's split form agrees to rounding)
template <typename R, int EGNO>
__device__ __forceinline__ R dual_point(const KP<R>& p, R pc, R pxm, R pxp, R pym, R pyp, R f0c, R rho, const R* ao,
                                        R axc, R ayc, R* an, R* fo = nullptr) {
  const R DxR = (pxp - pc) * p.inv_dx;
  const R DxL = (pc - pxm) * p.inv_dx;
  const R DyR = (pyp - pc) * p.inv_dy;
  const R DyL = (pc - pym) * p.inv_dy;
  const R pinv = (rho + (R)1e-4) / p.sigma;              // param_inv, set_fns.py:127 (unused for egno 2)
  const R q = prox_recip<R, EGNO>(rho, p.sigma, pinv);
  an[0] = alp_prox<R, EGNO>(ao[0], DxR, axc, pinv, q, true);
  an[1] = alp_prox<R, EGNO>(ao[1], DxL, axc, pinv, q, false);
  const R f1x = fpos<R>(fval<R, EGNO>(an[0], axc));
  const R f2x = fneg<R>(fval<R, EGNO>(an[1], axc));
  R f1y, f2y, L;
  if constexpr (EGNO == 3) {
    f1y = fpos<R>(axc);
    f2y = fneg<R>(axc);
    L = lag<R, EGNO>(an[0] * an[0]) + lag<R, EGNO>(an[1] * an[1]);
  } else {
    an[2] = alp_prox<R, EGNO>(ao[2], DyR, ayc, pinv, q, true);
    an[3] = alp_prox<R, EGNO>(ao[3], DyL, ayc, pinv, q, false);
    f1y = fpos<R>(fval<R, EGNO>(an[2], ayc));
    f2y = fneg<R>(fval<R, EGNO>(an[3], ayc));
    L = lag<R, EGNO>(an[0] * an[0]) + lag<R, EGNO>(an[1] * an[1]) + lag<R, EGNO>(an[2] * an[2]) +
        lag<R, EGNO>(an[3] * an[3]);
  }
  R vec = (pc - f0c) * p.inv_dt;
  if (p.epsl != (R)0) {
    vec = vec - p.epsl * ((pxp + pxm - (R)2 * pc) * p.inv_dx2);
    vec = vec - p.epsl * ((pyp + pym - (R)2 * pc) * p.inv_dy2);
  }
  if (fo) {   // f1x, f2x, f1y, f2y of the new controls (the next residual's fluxes, :13-47)
    fo[0] = f1x;
    fo[1] = f2x;
    fo[2] = f1y;
    fo[3] = f2y;
  }
  vec = vec - (DxR * f1x + DxL * f2x + DyR * f1y + DyL * f2y);
  vec = vec - L;
  return nmax<R>(rho + p.sigma * vec, (R)0);
}

// grid: (ceil(ny/256), G) where the G workgroup rows stride over the T*nx (j, x) rows; block 256
// sums: [0] sum (rho'-rho)^2 [1] sum rho'^2 [2] sum rho^2, then per live alpha array a:
//       [3+3a] sum (alp'-alp)^2 [4+3a] sum alp'^2 [5+3a] sum alp^2
template <typename R, int EGNO>
__global__ void __launch_bounds__(256) k_dual_2d(KP<R> p) {
  if (p.ctrl->done || p.ctrl->inner_done) return;
  const int cur = p.ctrl->cur;
  const int src_set = (p.inplace || p.sub == 0) ? cur : 1 - cur;
  const int dst_set = p.inplace ? cur : 1 - cur;
  const int nx = p.nx, ny = p.ny;
  const int y = blockIdx.x * blockDim.x + threadIdx.x;
  constexpr int NA = (EGNO == 3) ? 2 : 4;
  constexpr int NS = 3 + 3 * NA;
  double s[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) s[i] = 0.0;
  const size_t plane = (size_t)nx * ny;
  const int nrows = p.T * nx;
  const int ym = nb_index(y - 1, ny, p.bcy), yp = nb_index(y + 1, ny, p.bcy);
  const R ayc = (y < ny) ? p.ay[y] : (R)0;
  for (int row = blockIdx.y; row < nrows && y < ny; row += gridDim.y) {
    const int j = row / nx;
    const int x = row - j * nx;
    const size_t c = (size_t)x * ny + y;
    const R* f1 = p.phibar + (size_t)(j + 1) * plane;   // phi_bar row j+1
    const R* f0 = p.phibar + (size_t)j * plane;         // phi_bar row j
    const int xm = nb_index(x - 1, nx, p.bcx), xp = nb_index(x + 1, nx, p.bcx);
    const R pc = f1[c];
    const R pxm = (xm >= 0) ? f1[(size_t)xm * ny + y] : (R)0;
    const R pxp = (xp >= 0) ? f1[(size_t)xp * ny + y] : (R)0;
    const R pym = (ym >= 0) ? f1[(size_t)x * ny + ym] : (R)0;
    const R pyp = (yp >= 0) ? f1[(size_t)x * ny + yp] : (R)0;
    const size_t o = (size_t)j * plane + c;
    const R rho = p.rho[src_set][o];
    R an[4], ao[4];
#pragma unroll
    for (int a = 0; a < NA; ++a) ao[a] = p.alp[src_set][a][o];
    const R rn = dual_point<R, EGNO>(p, pc, pxm, pxp, pym, pyp, f0[c], rho, ao, p.ax[x], ayc, an);
    p.rho[dst_set][o] = rn;
    const double dr = (double)rn - (double)rho;
    s[0] += dr * dr;
    s[1] += (double)rn * (double)rn;
    s[2] += (double)rho * (double)rho;
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      p.alp[dst_set][a][o] = an[a];
      const double da = (double)an[a] - (double)ao[a];
      s[3 + 3 * a] += da * da;
      s[4 + 3 * a] += (double)an[a] * (double)an[a];
      s[5 + 3 * a] += (double)ao[a] * (double)ao[a];
    }
  }
  block_reduce_store<NS>(s, p.partials, blockIdx.y * gridDim.x + blockIdx.x);
}

}  // namespace pdhg
