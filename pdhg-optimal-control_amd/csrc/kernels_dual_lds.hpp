// Dual sweep (update_fns_in_pdhg.py:150-165) with the x neighbours staged through LDS (fp32, and fp64 without
// the fused residual: R = double, 4 consecutive y per lane as dbl4).
//
// k_dual_fast_2d (kernels_2d_fast.hpp) gives every thread one x row and reads the x-1 / x+1 rows of
// phi_bar straight from global memory, relying on L2 for the reuse between workgroups; the measured
// fetch is ~1.25x the algorithmic read volume.  Here a workgroup = RX waves, wave r owns x row x0 + r
// and 256 consecutive y (4 per lane).  Each time step the waves store their phi_bar row j+1 strip
// (plus the halo rows x0-1 and x0+RX, loaded by the first and the last wave) into an LDS double
// buffer, so phi_bar is fetched (RX+2)/RX times per point.  One barrier per step; the next step's
// global loads are in flight during the current step's arithmetic, as in k_dual_fast_2d, and the
// march over t keeps phi_bar row j+1 as the next step's row j.
#pragma once
#include "kernels_2d_fast.hpp"

namespace pdhg {

//
// FR (fused residual, rho_alp_iters = 1, periodic bc, egno 1/2, one time chunk per workgroup): the sweep
// also forms the NEXT primal's continuity residual (update_fns_in_pdhg.py:72-96) from the rho', alp'
// it has just computed, so the residual kernel does not re-read rho and the four alp arrays.  Row j's
// fluxes m = (rho'+1e-4) f(alp') are exchanged between the waves through a second LDS double buffer
// (x neighbours) and the adjacent lanes (y neighbours); R_j needs rho'_{j+1}, so it is completed and
// stored one step later (R_{T-1} with rho_T = 0 and + c/dt after the loop).  Terms that need values
// outside the workgroup's 8 x 256 tile are left out of R; instead each sweep writes the terms its own
// edge rows / columns contribute to the neighbouring tiles (p.ex: eps rho'/dx^2 + m1x/dx of row x0+RX-1
// for the next tile's first row, eps rho'/dx^2 - m2x/dx of row x0 for the previous tile's last row;
// p.ey: likewise per strip-edge column with m1y / m2y), and k_res_fwdy_fused_2d adds them.
template <int EGNO, int RX, bool FR = false, typename R = float, int YPL = 4>
__global__ void __launch_bounds__(RX * 64, 2) k_dual_lds_2d(KP<R> p, int jchunk, int jbase, int jend,
                                                                     int zbase) {
  using V = VY<R, YPL>;   // YPL consecutive y per lane
  if (p.ctrl->done || p.ctrl->inner_done) return;
  constexpr int NA = (EGNO == 3) ? 2 : 4;
  constexpr int NS = 3 + 3 * NA;
  constexpr int YW = 64 * YPL;                    // y strip per workgroup (64 lanes x YPL)
  static_assert(!FR || EGNO != 3, "fused residual: egno 1/2 (four live controls)");
  static_assert(YPL == 4 || YPL == 2, "4 or 2 y per lane");
  __shared__ __align__(16) V strip[2][RX + 2][64];
  // FR: [buffer][row][rho', m1x, m2x][lane]
  __shared__ __align__(16) V flux[FR ? 2 : 1][FR ? RX : 1][3][64];
  // p.nbsync: steps staged per row wave.  A wave reads only its neighbours' strip rows and flux rows, so instead of a
  // block barrier per step it publishes its own count after staging and waits for the two neighbours' counts: waves
  // drift by up to a step against each other and the CU's loads are no longer issued in lock-step.  (The double
  // buffers stay safe: a neighbour that has staged step t has finished reading the buffer staged at step t-1.)
  __shared__ int nstaged[RX];
  const int cur = p.ctrl->cur;
  const int src_set = (p.inplace || p.sub == 0) ? cur : 1 - cur;
  const int dst_set = p.inplace ? cur : 1 - cur;
  const int nx = p.nx, ny = p.ny;
  const size_t plane = (size_t)nx * ny;
  const int lane = threadIdx.x & 63, r = threadIdx.x >> 6;
  const int x0 = xcd_remap(blockIdx.x, gridDim.x) * RX;
  const int x = x0 + r;
  const bool live = x >= p.xl0 && x < p.xl1;   // wave-uniform (x-slab ghost / padding rows: neither stored nor summed)
  const int y = blockIdx.y * YW + YPL * lane;
  const int j0 = jbase + blockIdx.z * jchunk;
  const int j1 = min(jend, j0 + jchunk);
  double s[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) s[i] = 0.0;
  // halo row of the group (wave-uniform): x0-1 for wave 0, x0+RX for wave RX-1; clamped and zeroed
  // at a Dirichlet edge, wrapped when periodic, clamped when Neumann (nb_index)
  const bool has_h = (r == 0) || (r == RX - 1);
  const int xh = (r == 0) ? nb_index(x0 - 1, nx, p.bcx) : nb_index(x0 + RX, nx, p.bcx);
  const bool zh = xh < 0;
  const size_t rxh = (size_t)(zh ? x : xh) * ny, rxc = (size_t)x * ny;
  const int hslot = (r == 0) ? 0 : RX + 1;
  const int yw0 = __builtin_amdgcn_readfirstlane(y);
  const int ywm = nb_index(yw0 - 1, ny, p.bcy), ywp = nb_index(yw0 + YPL * kWave, ny, p.bcy);
  const bool zym = ywm < 0, zyp = ywp < 0;
  const int ywmc = zym ? 0 : ywm, ywpc = zyp ? 0 : ywp;
  const V ay4 = ldy<YPL>(p.ay + y);
  const R axc = p.ax[x];
  const R* rs = p.rho[src_set];
  R* rd = p.rho[dst_set];
  const R* as[NA];
  R* ad[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    as[a] = p.alp[src_set][a];
    ad[a] = p.alp[dst_set][a];
  }
  struct In {
    V pc, ph, rho, al[NA];
    R el, er;
  };
  auto load = [&](int j) {
    In in;
    const R* f1 = p.phibar + (size_t)(j + 1) * plane;
    in.pc = ldy<YPL>(f1 + rxc + y);
    in.ph = has_h ? ldy<YPL>(f1 + rxh + y) : zy<R, YPL>();
    in.el = f1[rxc + ywmc];
    in.er = f1[rxc + ywpc];
    const size_t o = (size_t)j * plane + rxc + y;
    in.rho = ldy<YPL>(rs + o);
#pragma unroll
    for (int a = 0; a < NA; ++a) in.al[a] = ldy<YPL>(as[a] + o);
    return in;
  };
  auto stage = [&](const In& in, int buf) {
    strip[buf][r + 1][lane] = in.pc;
    if (has_h) strip[buf][hslot][lane] = zh ? zy<R, YPL>() : in.ph;
  };
  // FR state: the y part of row j-1's residual (eps*Dyy rho' and the y flux divergence), completed at
  // step j once rho'_j and the x neighbours' fluxes (LDS) are known
  R yeps[YPL], ydiv[YPL];
#pragma unroll
  for (int e = 0; e < YPL; ++e) yeps[e] = ydiv[e] = (R)0;
  const bool use_eps = p.epsl != (R)0;
  const int nstrip = ny / YW;
  // R_{jr} (row jr of the next residual) = (rho'_{jr+1} - rho'_{jr})/dt + eps*Lap rho' - div m, from the
  // flux buffer fb (row jr's values) and rnext = rho'_{jr+1} at this thread's 4 points.  The time difference
  // is added last (one fma), so a t-slab's last row -- stored without it (tdiff = false) and completed by
  // k_res_fwdy_fused_2d from the next slab's rho row 0 with the same fma -- rounds exactly as the row does
  // inside one window (with epsl > 0 the eps*Lap rho' terms are ~1e8 at dx = 2/8192, so any other order
  // differs by their ulp)
  auto finish_res = [&](int jr, int fb, const V& rnext, R cdt, bool tdiff = true) {
    const V rc = flux[fb][r][0][lane], m1c = flux[fb][r][1][lane], m2c = flux[fb][r][2][lane];
    const int rmi = r > 0 ? r - 1 : r, rpi = r < RX - 1 ? r + 1 : r;   // wave-uniform
    V rm = flux[fb][rmi][0][lane], m1m = flux[fb][rmi][1][lane];
    V rp = flux[fb][rpi][0][lane], m2p = flux[fb][rpi][2][lane];
    if (r == 0) rm = m1m = zy<R, YPL>();        // row x0-1: added by the residual kernel
    if (r == RX - 1) rp = m2p = zy<R, YPL>();   // row x0+RX: likewise
    V out;
#pragma unroll
    for (int e = 0; e < YPL; ++e) {
      const R r0 = f4(rc, e);
      R res = (R)0;
      if (use_eps) {
        res = p.epsl * ((f4(rp, e) + f4(rm, e) - (R)2 * r0) * p.inv_dx2);
        res = res + yeps[e];
      }
      const R div = (f4(m1c, e) - f4(m1m, e)) * p.inv_dx + (f4(m2p, e) - f4(m2c, e)) * p.inv_dx + ydiv[e];
      const R other = res - div + cdt;
      f4set(out, e, tdiff ? fmar(f4(rnext, e) - r0, p.inv_dt, other) : other);
    }
    sty<YPL>(p.res + (size_t)jr * plane + rxc + y, out);
  };
  const bool nbs = p.nbsync != 0;
  // neighbour sync after staging step t's rows (see nstaged): publish, then wait for waves r-1 and r+1
  auto step_sync = [&](int t) {
    if (!nbs) {
      __syncthreads();
      return;
    }
    // LDS only: the count is written once this wave's strip / flux writes have landed (lgkmcnt), and no wait
    // touches vmcnt, so the next rows' global loads stay in flight across the sync
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    typedef __attribute__((address_space(3))) volatile int lds_int;   // ds_read / ds_write (a generic pointer
    lds_int* cnt = (lds_int*)nstaged;                                  // would be flat: vmcnt-counted)
    if (lane == 0) cnt[r] = t;
    const int rl = r > 0 ? r - 1 : r, rr = r < RX - 1 ? r + 1 : r;
    while (min(cnt[rl], cnt[rr]) < t) __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");   // the neighbours' rows are read after their counts
  };
  if (threadIdx.x < RX) nstaged[threadIdx.x] = 0;
  if (j0 < j1) {
    V f0 = ldy<YPL>(p.phibar + (size_t)j0 * plane + rxc + y);   // phi_bar row j
    // Two register sets, A and B, alternate between the rows (no copies: a register copy of a row still in
    // flight would wait for it).  Step j computes from cur (row j), re-fills cur with row j+2 and stages oth
    // (row j+1, loaded one step earlier) into LDS: the loads of a row are in flight across a whole step,
    // and no wait ever covers a store.
    auto step = [&](int j, In& cur, const In& oth) {
      const int buf = (j - j0) & 1;
      const V pm = strip[buf][r][lane], pp = strip[buf][r + 2][lane], pc = cur.pc;
      const R pyl = lane_from_prev(f4(pc, YPL - 1), zym ? (R)0 : cur.el);
      const R pyr = lane_from_next(f4(pc, 0), zyp ? (R)0 : cur.er);
      V rn4, an4[NA];
      V m1x4, m2x4;
      R m1y[YPL], m2y[YPL];
      // this step's 4 points summed in fp32 (4 terms), then one fp64 add per sum: the fixed-order fp64
      // accumulation over t stays, with a quarter of the fp64 work
      // (fp64: straight into the fixed-order fp64 sums, s)
      R fsb[sizeof(R) == 4 ? NS : 1];
      double* const fs_d = s;
      auto fsr = [&](int i) -> R& { if constexpr (sizeof(R) == 4) return fsb[i]; else return fs_d[i]; };
      if constexpr (sizeof(R) == 4) {
#pragma unroll
        for (int i = 0; i < NS; ++i) fsb[i] = (R)0;
      }
#pragma unroll
      for (int e = 0; e < YPL; ++e) {
        const R c = f4(pc, e);
        const R lft = e == 0 ? pyl : f4(pc, e - 1);
        const R rgt = e == YPL - 1 ? pyr : f4(pc, e + 1);
        R ao[4], an[4], fo[4];
#pragma unroll
        for (int a = 0; a < NA; ++a) ao[a] = f4(cur.al[a], e);
        const R rho = f4(cur.rho, e);
        const R rn = dual_point<R, EGNO>(p, c, f4(pm, e), f4(pp, e), lft, rgt, f4(f0, e), rho, ao, axc,
                                                 f4(ay4, e), an, FR ? fo : nullptr);
        f4set(rn4, e, rn);
        if constexpr (FR) {   // fluxes (rho'+1e-4) f(alp') of row j (m1f / m2f of the residual kernel)
          const R rq = rn + (R)1e-4;
          f4set(m1x4, e, rq * fo[0]);
          f4set(m2x4, e, rq * fo[1]);
          m1y[e] = rq * fo[2];
          m2y[e] = rq * fo[3];
        }
#pragma unroll
        for (int a = 0; a < NA; ++a) f4set(an4[a], e, an[a]);
        if (sizeof(R) == 4 || live) {
          const R dr = rn - rho;
          fsr(0) = fmar(dr, dr, fsr(0));
          fsr(1) = fmar(rn, rn, fsr(1));
          fsr(2) = fmar(rho, rho, fsr(2));
#pragma unroll
          for (int a = 0; a < NA; ++a) {
            const R da = an[a] - ao[a];
            fsr(3 + 3 * a) = fmar(da, da, fsr(3 + 3 * a));
            fsr(4 + 3 * a) = fmar(an[a], an[a], fsr(4 + 3 * a));
            fsr(5 + 3 * a) = fmar(ao[a], ao[a], fsr(5 + 3 * a));
          }
        }
      }
      // cur is consumed: the row after next goes into its registers now, ahead of this step's stores, so the
      // wait for the next row's loads (at the staging below) counts these 7 loads and never this step's stores
      const V pcs = pc;
      cur = load(min(j + 2, j1 - 1));   // clamped: the last rows re-load row j1-1 (never used)
      if constexpr (sizeof(R) == 4) {
        if (live) {
#pragma unroll
          for (int i = 0; i < NS; ++i) s[i] += (double)fsb[i];
        }
      }
      const size_t o = (size_t)j * plane + rxc + y;
      if (live && !(p.dbg & 128)) {   // PDHG_DBG 128: no rho / alp stores (timing experiments only)
        sty<YPL>(rd + o, rn4);
#pragma unroll
        for (int a = 0; a < NA; ++a) sty<YPL>(ad[a] + o, an4[a]);
      }
      f0 = pcs;
      if constexpr (FR) if (!(p.dbg & 256)) {   // PDHG_DBG 256: no residual / edge terms (timing only)
        if (j > j0) finish_res(j - 1, buf ^ 1, rn4, (R)0);   // row j-1, with rho'_j
        flux[buf][r][0][lane] = rn4;
        flux[buf][r][1][lane] = m1x4;
        flux[buf][r][2][lane] = m2x4;
        // y part of row j: neighbours from the adjacent lanes; the strip's outer columns are left out
        // (0 here) and handed to the residual kernel through p.ey
        const R rym = lane_from_prev(f4(rn4, YPL - 1), (R)0), ryp = lane_from_next(f4(rn4, 0), (R)0);
        const R m1ym = lane_from_prev(m1y[YPL - 1], (R)0), m2yp = lane_from_next(m2y[0], (R)0);
#pragma unroll
        for (int e = 0; e < YPL; ++e) {
          const R r0 = f4(rn4, e);
          const R lo = e == 0 ? rym : f4(rn4, e - 1), hi = e == YPL - 1 ? ryp : f4(rn4, e + 1);
          const R m1l = e == 0 ? m1ym : m1y[e - 1], m2h = e == YPL - 1 ? m2yp : m2y[e + 1];
          yeps[e] = p.epsl * ((hi + lo - (R)2 * r0) * p.inv_dy2);
          ydiv[e] = (m1y[e] - m1l) * p.inv_dy + (m2h - m2y[e]) * p.inv_dy;
        }
        // the neighbouring strips' outer-column terms that need this strip's edge column: lane 0 feeds the
        // previous strip's last column (eps rho'/dy^2 - m2y/dy), lane 63 the next strip's first column
        // (eps rho'/dy^2 + m1y/dy); k_res_fwdy_fused_2d adds them (p.ey)
        if (lane == 0 || lane == kWave - 1) {
          const bool first = lane == 0;
          R c = first ? -m2y[0] * p.inv_dy : m1y[YPL - 1] * p.inv_dy;
          if (use_eps) c = c + p.epsl * ((first ? f4(rn4, 0) : f4(rn4, YPL - 1)) * p.inv_dy2);
          const int sy = first ? (blockIdx.y == 0 ? nstrip - 1 : blockIdx.y - 1)
                               : (blockIdx.y + 1 == nstrip ? 0 : blockIdx.y + 1);
          p.ey[(((size_t)j * nx + x) * nstrip + sy) * 2 + (first ? 1 : 0)] = c;
        }
        // likewise the neighbouring tiles' edge rows (wave-uniform): the last wave feeds row 0 of the next
        // tile (eps rho'/dx^2 + m1x/dx), wave 0 row RX-1 of the previous tile (eps rho'/dx^2 - m2x/dx) (p.ex)
        if (r == 0 || r == RX - 1) {
          const bool top = r == 0;
          const int ngx = nx / RX, tile = x0 / RX;
          const int tt = top ? (tile == 0 ? ngx - 1 : tile - 1) : (tile + 1 == ngx ? 0 : tile + 1);
          V c;
#pragma unroll
          for (int e = 0; e < YPL; ++e) {
            R v = top ? -f4(m2x4, e) * p.inv_dx : f4(m1x4, e) * p.inv_dx;
            if (use_eps) v = v + p.epsl * (f4(rn4, e) * p.inv_dx2);
            f4set(c, e, v);
          }
          sty<YPL>(p.ex + (((size_t)j * ngx + tt) * 2 + (top ? 1 : 0)) * ny + y, c);
        }
      }
      if (j + 1 < j1) {     // uniform over the workgroup
        stage(oth, buf ^ 1);
        step_sync(j + 1 - j0);
      }
    };
    In A = load(j0), B = load(min(j0 + 1, j1 - 1));
    stage(A, 0);
    __syncthreads();
#pragma unroll 1
    for (int j = j0; j < j1; j += 2) {
      step(j, A, B);
      if (j + 1 < j1) step(j + 1, B, A);
    }
    if constexpr (FR) {
      // the launch's last row: inside the window (t-slab halo launch of row 0) rho'_{j1} comes from memory;
      // at the window's end rho_T = 0 and + c/dt (update_fns_in_pdhg.py:80, 95); at a t-slab's end rho_T is
      // the next slab's row 0: the time difference is left to k_res_fwdy_fused_2d (halo)
      __syncthreads();
      const bool inner = j1 < p.T;
      const V rnx = inner ? ldy<YPL>(rd + (size_t)j1 * plane + rxc + y) : zy<R, YPL>();
      finish_res(j1 - 1, (j1 - 1 - j0) & 1, rnx, (!inner && p.last_slab) ? p.c_over_dt : (R)0,
                 inner || p.last_slab);
    }
  }
  block_reduce_store<NS>(s, p.partials, ((zbase + (int)blockIdx.z) * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x);
}

}  // namespace pdhg
