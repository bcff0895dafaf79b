// The dual loop of rho_alp_iters > 1 (update_dual_alternative, update_fns_in_pdhg.py:167-180) in chunks of NSUB
// sub-iterations per pass instead of one pass per sub-iteration.
//
// With phi_bar fixed, a dual sub-iteration is pointwise in (rho, alp): the alpha prox reads phi_bar's one-sided
// differences and the point's own rho / alpha, the HJ residual phi_bar and the point's new alpha, the rho prox
// the point's rho (update_fns_in_pdhg.py:49-70, 99-165; set_fns.py:63-160).  Only the exit test couples the
// points: after sub-iteration s the loop stops when err_s = sum (drho)^2 / sum rho'^2 + sum_a sum (dalp)^2 /
// sum alp'^2 < eps (:162-164, 176).  So:
//   chunk pass (SLO)   every point runs sub-iterations SLO .. SLO + n - 1 in registers from the state after SLO
//                      (the start state for SLO = 0, else the previous chunk's stored one), accumulates the err
//                      sums of each, and stores the state after the chunk (second buffer set);
//   k_finalize_dual_multi  reduces the sums in a fixed order and finds k* = the first s + 1 with err_s < eps
//                      (or the loop's last), recording which state the buffer holds; later chunks see
//                      kstar_found and return at once;
//   final pass         only when the exit fell inside a chunk (k* != the stored state): every point re-runs its
//                      k* sub-iterations from the start state and stores that state.
// Without an early exit (k = 10: two chunks of 5) that is 2 reads + 2 writes of rho, alpha and 2 of phi_bar
// instead of 10 + 10; with one, at most one more read + write.  The phi_bar part of each point (dual_pre) is
// formed once per pass; every sub-iteration is dual_core, the per-sub-iteration kernels' arithmetic -- up to
// the compiler's FMA contraction, which differs once the phi_bar products (D * a(x)) are hoisted out of the
// sub-iteration loop: states agree to an ulp per sub-iteration, not bitwise (tests/test_gpu_dual_multi.py).
// Head form (the default below 2^25 points per window): sub-iteration 0 through the per-sub-iteration kernel and
// its finalize, then the chunks from SLO = 1 (they read the state sub-iteration 0 stored) -- a loop that exits after
// sub-iteration 0 then costs three returning launches instead of 2 (k - 1), and its state is the per-sub-iteration
// kernels' bit for bit.
// Layout as k_dual_fast_2d (a thread owns 4 consecutive y of one x row and marches over t; x neighbours of phi_bar
// from L2, y neighbours from the adjacent lanes); block 256; a workgroup takes a run of xrun consecutive x rows
// (grid x = ceil(nx / xrun)): the head form's chunk passes, which return at once after most loops, launch 4x fewer
// workgroups (a returning 4096-workgroup launch of this kernel took 12 us).
// The err sums of a sub-iteration are formed over a thread's 4 points in R (as the fused dual's) and accumulated
// in fp64 over its rows.
// Partials: table i (sub-iteration SLO + i) at partials + i * table_rows rows of kNumSums doubles; per row
// [0] sum (rho_s - rho_{s-1})^2 [1] sum rho_s^2, per live alpha a: [2+2a] sum (dalp)^2 [3+2a] sum alp_s^2.
#pragma once
#include "kernels_2d_fast.hpp"

namespace pdhg {

constexpr int kDualMultiMax = 10;   // rho_alp_iters handled in registers (the reference default)

template <int EGNO, typename R, int NSUB, bool FINAL>
__global__ void __launch_bounds__(256) k_dual_multi_2d(KP<R> p, int slo, int kmax, int table_rows, int jchunk,
                                                       int jbase, int jend, int zbase, int xrun) {
  using V = V4<R>;
  constexpr int NA = (EGNO == 3) ? 2 : 4;
  constexpr int SP = 2 + 2 * NA;
  constexpr int NIT = FINAL ? kDualMultiMax : NSUB;
  if (p.ctrl->done) return;
  // inner_done without kstar_found: the head form's sub-iteration 0 (a per-sub-iteration kernel) exited the loop
  if (!FINAL && slo > 0 && (p.ctrl->kstar_found || p.ctrl->inner_done)) return;
  if (FINAL && (!p.ctrl->kstar_found || p.ctrl->kstar == p.ctrl->kstored)) return;   // stored state is the exit one
  // sub-iterations this pass runs (uniform)
  const int nrun = FINAL ? p.ctrl->kstar : min(NSUB, kmax - slo);
  const int cur = p.ctrl->cur;
  const int nx = p.nx, ny = p.ny;
  const size_t plane = (size_t)nx * ny;
  const int xb = xcd_remap(blockIdx.x, gridDim.x);   // x rows [xb xrun, xb xrun + xrun): a run per workgroup
  const int y = 4 * (blockIdx.y * blockDim.x + threadIdx.x);
  const int j0 = jbase + blockIdx.z * jchunk;
  const int j1 = min(jend, j0 + jchunk);
  double sm[FINAL ? 1 : NSUB][SP];
#pragma unroll
  for (int i = 0; i < (FINAL ? 1 : NSUB); ++i)
#pragma unroll
    for (int k = 0; k < SP; ++k) sm[i][k] = 0.0;
#pragma unroll 1
  for (int x = xb * xrun; x < min(nx, xb * xrun + xrun); ++x) {
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
    const int src = (FINAL || slo == 0) ? cur : 1 - cur;   // the start state, or the previous chunk's
    const R* rs = p.rho[src];
    R* rd = p.rho[1 - cur];
    const R* as[NA];
    R* ad[NA];
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      as[a] = p.alp[src][a];
      ad[a] = p.alp[1 - cur][a];
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
    In nxt = load(j0);
#pragma unroll 1
    for (int j = j0; j < j1; ++j) {
      const In in = nxt;
      nxt = load(min(j + 1, j1 - 1));
      const V pm = zxm ? z4r<R>() : in.pm, pp = zxp ? z4r<R>() : in.pp, pc = in.pc;
      const R pyl = lane_from_prev(pc.w, zym ? (R)0 : in.el);
      const R pyr = lane_from_next(pc.x, zyp ? (R)0 : in.er);
      // the 4 points' phi_bar parts and states, then the sub-iterations over the 4 points together (4 independent
      // chains per sub-iteration); each sub-iteration's sums over the 4 points in R, then one fp64 add per sum
      DualPre<R> d[4];
      R rho[4], al[4][4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const R c = f4(pc, e);
        const R lft = e == 0 ? pyl : f4(pc, e - 1);
        const R rgt = e == 3 ? pyr : f4(pc, e + 1);
        d[e] = dual_pre<R>(p, c, f4(pm, e), f4(pp, e), lft, rgt, f4(f0, e));
        rho[e] = f4(in.rho, e);
#pragma unroll
        for (int a = 0; a < NA; ++a) al[e][a] = f4(in.al[a], e);
      }
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        if (it < nrun) {   // uniform
          R tf[SP];
#pragma unroll
          for (int k = 0; k < SP; ++k) tf[k] = (R)0;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            R an[4];
            const R rn = dual_core<R, EGNO>(p, d[e], rho[e], al[e], axc, f4(ay4, e), an);
            if constexpr (!FINAL) {
              const R dr = rn - rho[e];
              tf[0] = fmar(dr, dr, tf[0]);
              tf[1] = fmar(rn, rn, tf[1]);
#pragma unroll
              for (int a = 0; a < NA; ++a) {
                const R da = an[a] - al[e][a];
                tf[2 + 2 * a] = fmar(da, da, tf[2 + 2 * a]);
                tf[3 + 2 * a] = fmar(an[a], an[a], tf[3 + 2 * a]);
              }
            }
            rho[e] = rn;
#pragma unroll
            for (int a = 0; a < NA; ++a) al[e][a] = an[a];
          }
          if constexpr (!FINAL) {
#pragma unroll
            for (int k = 0; k < SP; ++k) sm[FINAL ? 0 : it][k] += (double)tf[k];
          }
        }
      }
      V rn4, an4[NA];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        f4set(rn4, e, rho[e]);
#pragma unroll
        for (int a = 0; a < NA; ++a) f4set(an4[a], e, al[e][a]);
      }
      const size_t o = (size_t)j * plane + rxc + y;
      st4(rd + o, rn4);
#pragma unroll
      for (int a = 0; a < NA; ++a) st4(ad[a] + o, an4[a]);
      f0 = pc;
    }
  }
  }   // x run
  if constexpr (!FINAL) {
    const int row = ((zbase + (int)blockIdx.z) * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
#pragma unroll
    for (int i = 0; i < NSUB; ++i) block_reduce_store<SP>(sm[i], p.partials + (size_t)i * table_rows * kNumSums, row);
  }
}

}  // namespace pdhg
