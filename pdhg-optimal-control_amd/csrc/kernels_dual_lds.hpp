// Dual sweep (update_fns_in_pdhg.py:150-165) with the x neighbours staged through LDS.
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

template <int EGNO, int RX>
__global__ void __launch_bounds__(RX * 64, 3) k_dual_lds_2d(KP<float> p, int jchunk, int jbase, int jend, int zbase) {
  if (p.ctrl->done || p.ctrl->inner_done) return;
  constexpr int NA = (EGNO == 3) ? 2 : 4;
  constexpr int NS = 3 + 3 * NA;
  constexpr int YW = 256;                         // y strip per workgroup (64 lanes x float4)
  __shared__ __align__(16) float4 strip[2][RX + 2][YW / 4];
  const int cur = p.ctrl->cur;
  const int src_set = (p.inplace || p.sub == 0) ? cur : 1 - cur;
  const int dst_set = p.inplace ? cur : 1 - cur;
  const int nx = p.nx, ny = p.ny;
  const size_t plane = (size_t)nx * ny;
  const int lane = threadIdx.x & 63, r = threadIdx.x >> 6;
  const int x0 = xcd_remap(blockIdx.x, gridDim.x) * RX;
  const int x = x0 + r;
  const int y = blockIdx.y * YW + 4 * lane;
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
  const int ywm = nb_index(yw0 - 1, ny, p.bcy), ywp = nb_index(yw0 + 4 * kWave, ny, p.bcy);
  const bool zym = ywm < 0, zyp = ywp < 0;
  const int ywmc = zym ? 0 : ywm, ywpc = zyp ? 0 : ywp;
  const float4 ay4 = ld4(p.ay + y);
  const float axc = p.ax[x];
  const float* rs = p.rho[src_set];
  float* rd = p.rho[dst_set];
  const float* as[NA];
  float* ad[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    as[a] = p.alp[src_set][a];
    ad[a] = p.alp[dst_set][a];
  }
  struct In {
    float4 pc, ph, rho, al[NA];
    float el, er;
  };
  auto load = [&](int j) {
    In in;
    const float* f1 = p.phibar + (size_t)(j + 1) * plane;
    in.pc = ld4(f1 + rxc + y);
    in.ph = has_h ? ld4(f1 + rxh + y) : z4();
    in.el = f1[rxc + ywmc];
    in.er = f1[rxc + ywpc];
    const size_t o = (size_t)j * plane + rxc + y;
    in.rho = ld4(rs + o);
#pragma unroll
    for (int a = 0; a < NA; ++a) in.al[a] = ld4(as[a] + o);
    return in;
  };
  auto stage = [&](const In& in, int buf) {
    strip[buf][r + 1][lane] = in.pc;
    if (has_h) strip[buf][hslot][lane] = zh ? z4() : in.ph;
  };
  if (j0 < j1) {
    float4 f0 = ld4(p.phibar + (size_t)j0 * plane + rxc + y);   // phi_bar row j
    In nxt = load(j0);
    stage(nxt, 0);
    __syncthreads();
#pragma unroll 1
    for (int j = j0; j < j1; ++j) {
      const int buf = (j - j0) & 1;
      const In in = nxt;
      if (j + 1 < j1) nxt = load(j + 1);
      const float4 pm = strip[buf][r][lane], pp = strip[buf][r + 2][lane], pc = in.pc;
      const float pyl = lane_from_prev(pc.w, zym ? 0.f : in.el);
      const float pyr = lane_from_next(pc.x, zyp ? 0.f : in.er);
      float4 rn4, an4[NA];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float c = f4(pc, e);
        const float lft = e == 0 ? pyl : f4(pc, e - 1);
        const float rgt = e == 3 ? pyr : f4(pc, e + 1);
        float ao[4], an[4];
#pragma unroll
        for (int a = 0; a < NA; ++a) ao[a] = f4(in.al[a], e);
        const float rho = f4(in.rho, e);
        const float rn = dual_point<float, EGNO>(p, c, f4(pm, e), f4(pp, e), lft, rgt, f4(f0, e), rho, ao, axc,
                                                 f4(ay4, e), an);
        f4set(rn4, e, rn);
        const double dr = (double)rn - (double)rho;
        s[0] += dr * dr;
        s[1] += (double)rn * (double)rn;
        s[2] += (double)rho * (double)rho;
#pragma unroll
        for (int a = 0; a < NA; ++a) {
          f4set(an4[a], e, an[a]);
          const double da = (double)an[a] - (double)ao[a];
          s[3 + 3 * a] += da * da;
          s[4 + 3 * a] += (double)an[a] * (double)an[a];
          s[5 + 3 * a] += (double)ao[a] * (double)ao[a];
        }
      }
      const size_t o = (size_t)j * plane + rxc + y;
      st4(rd + o, rn4);
#pragma unroll
      for (int a = 0; a < NA; ++a) st4(ad[a] + o, an4[a]);
      f0 = pc;
      if (j + 1 < j1) {     // uniform over the workgroup
        stage(nxt, buf ^ 1);
        __syncthreads();
      }
    }
  }
  block_reduce_store<NS>(s, p.partials, ((zbase + (int)blockIdx.z) * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x);
}

}  // namespace pdhg
