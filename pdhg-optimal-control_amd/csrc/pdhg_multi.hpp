// Multi-device context ("pdhg_create(const pdhg_problem*, const int* devices, int ndev, ...)
// ... one host thread drives all of its GPUs through streams").  Native counterpart of pdhg_amd/slab.py's
// SlabRunner: the window's T rows are split into ndev t-slabs (one pdhg_create_slab context per listed device,
// a device may repeat), and pdhg_multi_iterate runs the outer iteration of utils_pdhg_solver.py:51-88 with
// the slab choreography documented in include/pdhg.h (neighbour carry exchange), from this one thread:
//   * every slab computes on its own stream of its own device;
//   * planes move device to device with hipMemcpyPeerAsync (xGMI / SDMA; plain device copies when two slabs
//     share a GPU): rho halo up, phi_bar halo down, D to the next slab, S1 to the previous one, the
//     long-range modes to everybody;
//   * the 16-double sum vectors are gathered on slab 0's device, folded in slab order by k_multi_sum, and
//     copied back, so every slab takes the same stop decisions in its own control block;
//   * an exchange is bracketed by stream barriers (events): producers done -> copies -> consumers.
// Included by pdhg_api.hip after the C ABI (uses only the slab entry points).
#pragma once
#include <vector>

namespace pdhg {
__global__ void k_multi_sum(const double* __restrict__ in, int n, double* __restrict__ out) {
  const int s = threadIdx.x;   // one thread per sum, slabs in order (fixed-order, deterministic)
  if (s >= pdhg::kNumSums) return;
  double t = 0.0;
  for (int q = 0; q < n; ++q) t += in[(size_t)q * kNumSums + s];
  out[s] = t;
}
}  // namespace pdhg

struct pdhg_multi {
  int P = 0;
  std::vector<int> dev;
  std::vector<pdhg_ctx*> s;
  std::vector<hipStream_t> st;
  std::vector<hipEvent_t> ev;
  std::vector<int> j0, j1;
  pdhg_problem pb{};
  std::vector<double> xs, ys;
  size_t sp = 0, spec = 0;
  int K = 0;               // long-range modes
  int nar = 4, nc = 2;     // reference alp layout [nar][T][nx][ny][nc]
  struct Buf {
    float *rho_send = nullptr, *rho_recv = nullptr, *pb_send = nullptr, *pb_recv = nullptr;
    float *DS = nullptr, *GS = nullptr, *Dl = nullptr, *S1r = nullptr, *LONG = nullptr, *allLong = nullptr,
          *allGS = nullptr;
    double* sums = nullptr;
  };
  std::vector<Buf> b;
  double* gather = nullptr;   // slab 0's device: [P][16] sums, then the folded [16]
  std::vector<void*> allocs;  // (device, pointer) freed at destroy
  std::vector<int> alloc_dev;

  int on(int r) { return hipSetDevice(dev[r]) == hipSuccess ? 0 : -1; }
  template <typename T>
  int alloc(int r, T** p, size_t n) {
    if (on(r)) return fail(PDHG_ERR_HIP, "hipSetDevice(%d)", dev[r]);
    void* q = nullptr;
    if (hipMalloc(&q, std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess)
      return fail(PDHG_ERR_HIP, "hipMalloc of %zu bytes on device %d", n * sizeof(T), dev[r]);
    if (hipMemset(q, 0, std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) return fail(PDHG_ERR_HIP, "hipMemset");
    allocs.push_back(q);
    alloc_dev.push_back(dev[r]);
    *p = static_cast<T*>(q);
    return PDHG_OK;
  }
  // every stream waits for everything enqueued so far on every stream
  int barrier() {
    for (int r = 0; r < P; ++r) {
      if (on(r)) return fail(PDHG_ERR_HIP, "hipSetDevice");
      HIP_TRY(hipEventRecord(ev[r], st[r]));
    }
    for (int r = 0; r < P; ++r) {
      if (on(r)) return fail(PDHG_ERR_HIP, "hipSetDevice");
      for (int q = 0; q < P; ++q)
        if (q != r) HIP_TRY(hipStreamWaitEvent(st[r], ev[q], 0));
    }
    return PDHG_OK;
  }
  // copy on the destination slab's stream (call between barriers)
  int copy(int rd, void* dst, int rs, const void* src, size_t bytes) {
    if (on(rd)) return fail(PDHG_ERR_HIP, "hipSetDevice");
    if (dev[rd] == dev[rs]) HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st[rd]));
    else HIP_TRY(hipMemcpyPeerAsync(dst, dev[rd], src, dev[rs], bytes, st[rd]));
    return PDHG_OK;
  }
  int allreduce() {   // sums of every slab -> fixed-order fold on slab 0 -> back to every slab
    int rc;
    if ((rc = barrier())) return rc;
    for (int q = 0; q < P; ++q)
      if ((rc = copy(0, gather + (size_t)q * kNumSums, q, b[q].sums, kNumSums * sizeof(double)))) return rc;
    if (on(0)) return fail(PDHG_ERR_HIP, "hipSetDevice");
    hipLaunchKernelGGL(pdhg::k_multi_sum, dim3(1), dim3(64), 0, st[0], gather, P, gather + (size_t)P * kNumSums);
    HIP_TRY(hipGetLastError());
    if ((rc = barrier())) return rc;
    for (int q = 0; q < P; ++q)
      if ((rc = copy(q, b[q].sums, 0, gather + (size_t)P * kNumSums, kNumSums * sizeof(double)))) return rc;
    return barrier();
  }

  int setup(const pdhg_problem& prob, const int* devices, int ndev) {
    P = ndev;
    dev.assign(devices, devices + ndev);
    pb = prob;
    xs.assign(prob.xs, prob.xs + prob.nx);
    ys.assign(prob.ys, prob.ys + prob.ny);
    pb.xs = xs.data();
    pb.ys = ys.data();
    nc = prob.egno == 3 ? 1 : 2;
    const int T = prob.T;
    if (P < 1 || P > T) return fail(PDHG_ERR_ARG, "need 1 <= ndev <= T (ndev %d, T %d)", P, T);
    const int base = T / P, extra = T % P;
    for (int q = 0, j = 0; q < P; ++q) {   // pdhg_amd.slab.slab_bounds
      const int n = base + (q < extra ? 1 : 0);
      j0.push_back(j);
      j1.push_back(j + n);
      j += n;
    }
    // peer access where the runtime offers it (copies work either way)
    for (int r = 0; r < P; ++r)
      for (int q = 0; q < P; ++q) {
        if (dev[r] == dev[q]) continue;
        int ok = 0;
        if (hipDeviceCanAccessPeer(&ok, dev[r], dev[q]) == hipSuccess && ok) {
          hipSetDevice(dev[r]);
          hipError_t e = hipDeviceEnablePeerAccess(dev[q], 0);
          if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return fail(PDHG_ERR_HIP, "peer access");
          (void)hipGetLastError();
        }
      }
    s.assign(P, nullptr);
    st.assign(P, nullptr);
    ev.assign(P, nullptr);
    b.assign(P, Buf{});
    int rc;
    for (int r = 0; r < P; ++r) {
      pdhg_problem q = pb;
      q.T = j1[r] - j0[r];
      if ((rc = pdhg_create_slab(&q, j0[r], T, dev[r], &s[r]))) return rc;
      if (on(r)) return fail(PDHG_ERR_HIP, "hipSetDevice");
      HIP_TRY(hipStreamCreateWithFlags(&st[r], hipStreamNonBlocking));
      HIP_TRY(hipEventCreateWithFlags(&ev[r], hipEventDisableTiming));
      if ((rc = pdhg_set_stream(s[r], st[r]))) return rc;
    }
    unsigned long long a = 0, c = 0;
    if ((rc = pdhg_slab_plane_size(s[0], &a, &c))) return rc;
    sp = a;
    spec = c;
    for (int r = 0; r < P; ++r) {
      Buf& x = b[r];
      if ((rc = alloc(r, &x.rho_send, sp)) || (rc = alloc(r, &x.rho_recv, sp)) || (rc = alloc(r, &x.pb_send, sp)) ||
          (rc = alloc(r, &x.pb_recv, sp)) || (rc = alloc(r, &x.DS, 2 * spec)) || (rc = alloc(r, &x.GS, 2 * spec)) ||
          (rc = alloc(r, &x.Dl, spec)) || (rc = alloc(r, &x.S1r, spec)) || (rc = alloc(r, &x.allGS, 2 * spec * P)) ||
          (rc = alloc(r, &x.sums, (size_t)kNumSums)))
        return rc;
      if ((rc = pdhg_slab_carry_gain(s[r], x.GS))) return rc;
    }
    if ((rc = alloc(0, &gather, (size_t)(P + 1) * kNumSums))) return rc;
    // iteration-invariant gains of every slab to every slab, then the long-range classification
    if ((rc = barrier())) return rc;
    for (int r = 0; r < P; ++r)
      for (int q = 0; q < P; ++q)
        if ((rc = copy(r, b[r].allGS + (size_t)q * 2 * spec, q, b[q].GS, 2 * spec * sizeof(float)))) return rc;
    if ((rc = barrier())) return rc;
    for (int r = 0; r < P; ++r) {   // the classification reads the planes on the host side
      if (on(r)) return fail(PDHG_ERR_HIP, "hipSetDevice");
      HIP_TRY(hipStreamSynchronize(st[r]));
    }
    for (int r = 0; r < P; ++r) {
      int k = 0;
      if ((rc = pdhg_slab_long_modes(s[r], b[r].allGS, P, 9.094947017729282e-13 /* 2^-40 */, &k))) return rc;
      if (r == 0) K = k;
      else if (k != K) return fail(PDHG_ERR_STATE, "slabs disagree on the long-range modes (%d vs %d)", k, K);
    }
    for (int r = 0; r < P; ++r)
      if ((rc = alloc(r, &b[r].LONG, (size_t)std::max(1, 2 * K))) ||
          (rc = alloc(r, &b[r].allLong, (size_t)std::max(1, 2 * K) * P)))
        return rc;
    for (int r = 0; r < P; ++r) {
      if (on(r)) return fail(PDHG_ERR_HIP, "hipSetDevice");
      HIP_TRY(hipStreamSynchronize(st[r]));
    }
    return PDHG_OK;
  }

  ~pdhg_multi() {
    for (int r = 0; r < P; ++r)
      if (r < (int)st.size() && st[r]) {
        hipSetDevice(dev[r]);
        hipStreamSynchronize(st[r]);
      }
    for (auto* c : s) pdhg_destroy(c);
    for (size_t i = 0; i < allocs.size(); ++i) {
      hipSetDevice(alloc_dev[i]);
      hipFree(allocs[i]);
    }
    for (int r = 0; r < P; ++r) {
      if (r < (int)ev.size() && ev[r]) { hipSetDevice(dev[r]); hipEventDestroy(ev[r]); }
      if (r < (int)st.size() && st[r]) { hipSetDevice(dev[r]); hipStreamDestroy(st[r]); }
    }
  }

  // one outer iteration (include/pdhg.h t-slab choreography, neighbour exchange)
  int step(double tau, double sigma, double eps, int k) {
    int rc;
    const size_t pbytes = sp * sizeof(float), sbytes = spec * sizeof(float);
    for (int r = 0; r < P; ++r)
      if ((rc = pdhg_slab_plane_out(s[r], 0, b[r].rho_send))) return rc;
    if ((rc = barrier())) return rc;
    for (int r = 0; r + 1 < P; ++r)   // rho row 0 of slab r+1 -> slab r
      if ((rc = copy(r, b[r].rho_recv, r + 1, b[r + 1].rho_send, pbytes))) return rc;
    if ((rc = barrier())) return rc;
    for (int r = 0; r < P; ++r) {
      if (r + 1 < P && (rc = pdhg_slab_plane_in(s[r], 0, b[r].rho_recv))) return rc;
      if ((rc = pdhg_slab_residual(s[r], 3))) return rc;
      if ((rc = pdhg_slab_forward(s[r], tau))) return rc;
      if ((rc = pdhg_slab_plane_out(s[r], 2, b[r].DS))) return rc;
      if ((rc = pdhg_slab_plane_out(s[r], 3, b[r].LONG))) return rc;
    }
    if ((rc = barrier())) return rc;
    for (int r = 0; r < P; ++r) {
      if (r > 0 && (rc = copy(r, b[r].Dl, r - 1, b[r - 1].DS, sbytes))) return rc;              // D -> next
      if (r + 1 < P && (rc = copy(r, b[r].S1r, r + 1, b[r + 1].DS + spec, sbytes))) return rc;  // S1 -> previous
      for (int q = 0; q < P && K > 0; ++q)
        if ((rc = copy(r, b[r].allLong + (size_t)q * 2 * K, q, b[q].LONG, 2 * (size_t)K * sizeof(float)))) return rc;
    }
    if ((rc = barrier())) return rc;
    for (int r = 0; r < P; ++r) {
      if ((rc = pdhg_slab_fixup_nb(s[r], b[r].Dl, b[r].S1r, b[r].allLong, b[r].allGS, r, P))) return rc;
      if ((rc = pdhg_slab_backward(s[r], tau, b[r].sums))) return rc;
    }
    if ((rc = allreduce())) return rc;
    for (int r = 0; r < P; ++r) {
      if ((rc = pdhg_slab_primal_finalize(s[r], b[r].sums))) return rc;
      if ((rc = pdhg_slab_plane_out(s[r], 1, b[r].pb_send))) return rc;
    }
    if ((rc = barrier())) return rc;
    for (int r = 1; r < P; ++r)   // phi_bar row T of slab r-1 -> slab r
      if ((rc = copy(r, b[r].pb_recv, r - 1, b[r - 1].pb_send, pbytes))) return rc;
    if ((rc = barrier())) return rc;
    for (int sub = 0; sub < k; ++sub) {
      for (int r = 0; r < P; ++r) {
        if (sub == 0 && r > 0 && (rc = pdhg_slab_plane_in(s[r], 1, b[r].pb_recv))) return rc;
        if ((rc = pdhg_slab_dual(s[r], sigma, k, sub, b[r].sums, 3))) return rc;
      }
      if ((rc = allreduce())) return rc;
      for (int r = 0; r < P; ++r)
        if ((rc = pdhg_slab_dual_finalize(s[r], eps, sub, b[r].sums))) return rc;
    }
    for (int r = 0; r < P; ++r)
      if ((rc = pdhg_slab_outer(s[r], k, b[r].sums))) return rc;
    if (k > 1 && (rc = allreduce())) return rc;
    for (int r = 0; r < P; ++r)
      if ((rc = pdhg_slab_outer_finalize(s[r], eps, k, b[r].sums))) return rc;
    return PDHG_OK;
  }

  int iterate(int n, double tau, double sigma, double eps, int k, pdhg_stats* out) {
    int rc;
    for (int r = 0; r < P; ++r)
      if ((rc = pdhg_slab_begin(s[r]))) return rc;
    for (int it = 0; it < n; ++it) {
      if ((rc = step(tau, sigma, eps, k))) return rc;
      if ((it + 1) % 8 == 0 && it + 1 < n) {   // the device loop control, read every 8 iterations
        pdhg_stats h{};
        if ((rc = pdhg_slab_status(s[0], &h))) return rc;
        if (h.status) break;
      }
    }
    pdhg_stats h{};
    if ((rc = pdhg_slab_status(s[0], &h))) return rc;
    if (out) *out = h;
    return PDHG_OK;
  }

  // reference layouts, whole window: phi [T+1][nx][ny], rho [T][nx][ny], alp [nar][T][nx][ny][nc]
  int state(bool set, double* phi, double* rho, double* alp) {
    const size_t npl = (size_t)pb.nx * pb.ny;
    const int T = pb.T;
    int rc;
    for (int r = 0; r < P; ++r) {   // the state copies are synchronous (null stream): drain the slab streams
      if (on(r)) return fail(PDHG_ERR_HIP, "hipSetDevice");
      HIP_TRY(hipStreamSynchronize(st[r]));
    }
    for (int r = 0; r < P; ++r) {
      const int Tr = j1[r] - j0[r];
      std::vector<double> ph(phi ? (size_t)(Tr + 1) * npl : 0), rh(rho ? (size_t)Tr * npl : 0),
          al(alp ? (size_t)nar * Tr * npl * nc : 0);
      if (set) {
        if (phi) std::copy(phi + (size_t)j0[r] * npl, phi + (size_t)(j1[r] + 1) * npl, ph.begin());
        if (rho) std::copy(rho + (size_t)j0[r] * npl, rho + (size_t)j1[r] * npl, rh.begin());
        if (alp)
          for (int a = 0; a < nar; ++a)
            std::copy(alp + ((size_t)a * T + j0[r]) * npl * nc, alp + ((size_t)a * T + j1[r]) * npl * nc,
                      al.begin() + (size_t)a * Tr * npl * nc);
        if ((rc = pdhg_set_state(s[r], phi ? ph.data() : nullptr, rho ? rh.data() : nullptr,
                                 alp ? al.data() : nullptr)))
          return rc;
      } else {
        if ((rc = pdhg_get_state(s[r], phi ? ph.data() : nullptr, rho ? rh.data() : nullptr,
                                 alp ? al.data() : nullptr)))
          return rc;
        // phi rows j0..j1 of slab r; row j0 is slab r-1's last row too (the same values: row 0 of a slab is
        // refreshed from the previous slab only through phi_bar, so take each slab's own rows 1..Tr)
        if (phi) {
          const int from = (r == 0) ? 0 : 1;
          std::copy(ph.begin() + (size_t)from * npl, ph.end(), phi + (size_t)(j0[r] + from) * npl);
        }
        if (rho) std::copy(rh.begin(), rh.end(), rho + (size_t)j0[r] * npl);
        if (alp)
          for (int a = 0; a < nar; ++a)
            std::copy(al.begin() + (size_t)a * Tr * npl * nc, al.begin() + (size_t)(a + 1) * Tr * npl * nc,
                      alp + ((size_t)a * T + j0[r]) * npl * nc);
      }
    }
    return PDHG_OK;
  }
};

extern "C" {

int pdhg_create_multi(const pdhg_problem* prob, const int* devices, int ndev, pdhg_multi** out) {
  if (!prob || !devices || !out || ndev < 1) return fail(PDHG_ERR_ARG, "null argument or ndev < 1");
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(PDHG_ERR_HIP, "no HIP device available");
  for (int r = 0; r < ndev; ++r)
    if (devices[r] < 0 || devices[r] >= n) return fail(PDHG_ERR_ARG, "device %d out of range (%d)", devices[r], n);
  auto m = std::make_unique<pdhg_multi>();
  int rc = m->setup(*prob, devices, ndev);
  if (rc) return rc;
  *out = m.release();
  return PDHG_OK;
}
int pdhg_multi_destroy(pdhg_multi* m) {
  delete m;
  return PDHG_OK;
}
int pdhg_multi_set_state(pdhg_multi* m, const double* phi, const double* rho, const double* alp) {
  if (!m) return fail(PDHG_ERR_ARG, "null context");
  return m->state(true, const_cast<double*>(phi), const_cast<double*>(rho), const_cast<double*>(alp));
}
int pdhg_multi_get_state(pdhg_multi* m, double* phi, double* rho, double* alp) {
  if (!m) return fail(PDHG_ERR_ARG, "null context");
  return m->state(false, phi, rho, alp);
}
int pdhg_multi_iterate(pdhg_multi* m, int n_iters, double tau, double sigma, double eps, int rho_alp_iters,
                       pdhg_stats* out) {
  if (!m) return fail(PDHG_ERR_ARG, "null context");
  if (n_iters < 0 || rho_alp_iters < 1) return fail(PDHG_ERR_ARG, "bad iteration counts");
  return m->iterate(n_iters, tau, sigma, eps, rho_alp_iters, out);
}
int pdhg_multi_set_stop_rules(pdhg_multi* m, int stop_on_converge, int stop_on_nan) {
  if (!m) return fail(PDHG_ERR_ARG, "null context");
  for (auto* c : m->s) {
    int rc = pdhg_set_stop_rules(c, stop_on_converge, stop_on_nan);
    if (rc) return rc;
  }
  return PDHG_OK;
}
int pdhg_multi_synchronize(pdhg_multi* m) {
  if (!m) return fail(PDHG_ERR_ARG, "null context");
  for (int r = 0; r < m->P; ++r) {
    if (m->on(r)) return fail(PDHG_ERR_HIP, "hipSetDevice");
    HIP_TRY(hipStreamSynchronize(m->st[r]));
  }
  return PDHG_OK;
}
int pdhg_multi_info(pdhg_multi* m, const char* key, int* value) {
  if (!m || !key || !value) return fail(PDHG_ERR_ARG, "null argument");
  const std::string k(key);
  if (k == "ndev") *value = m->P;
  else if (k == "long_modes") *value = m->K;
  else if (k.rfind("rows:", 0) == 0) {
    const int r = atoi(k.c_str() + 5);
    if (r < 0 || r >= m->P) return fail(PDHG_ERR_ARG, "slab %d of %d", r, m->P);
    *value = m->j1[r] - m->j0[r];
  } else return fail(PDHG_ERR_ARG, "unknown key '%s'", key);
  return PDHG_OK;
}

}  // extern "C"
