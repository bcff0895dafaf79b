// Multi-device context ("pdhg_create(const pdhg_problem*, const int* devices, int ndev, ...)
// ... one host thread drives all of its GPUs through streams").  Native counterpart of pdhg_amd/slab.py's
// SlabRunner: the window's T rows are split into ndev t-slabs (one pdhg_create_slab context per listed device,
// a device may repeat), and pdhg_multi_iterate runs the outer iteration of utils_pdhg_solver.py:51-88 with
// the slab choreography documented in include/pdhg.h (neighbour carry exchange), from this one thread:
//   * slab r computes on its main stream st[r] and receives planes on its side stream ss[r] (both on dev[r]);
//   * a plane moves device to device with hipMemcpyPeerAsync (xGMI / SDMA; a plain device copy when two slabs
//     share a GPU) on the RECEIVER's side stream, after an event its producer recorded; the receiver's main
//     stream waits for the side stream's event only where the plane is consumed.  So the rho halo travels
//     while the residual rows that do not read it compute, the phi_bar halo while the primal sums are
//     reduced and the dual rows that do not read it run, and the column-block part q's carry planes while
//     part q+1 sweeps forward (SlabRunner's schedule, pdhg_amd/slab.py);
//   * waits are per neighbour (rho halo: r+1 -> r, phi_bar halo: r-1 -> r, D: r-1 -> r, S1: r+1 -> r), never
//     all-to-all; only the long-range carry modes (few, pdhg_slab_long_modes) and the sums need every slab;
//   * the 16-double sum vectors (opt-in, PDHG_MULTI_PEER_FOLD=1; default: the gather fold below): with peer
//     access between every pair of devices (xGMI), every slab's main
//     stream waits for every slab's contribution event and one 64-thread kernel on its own device folds the P
//     vectors in slab order straight from their owners' memory (peer pointers) -- the same order on every
//     device, so every slab takes bitwise the same stop decisions in its own control block, with no copies
//     and no device waiting for another's fold.  Contributions alternate between two buffers per slab: slab q
//     rewrites a buffer two allreduces later, after its own fold of the allreduce in between, which waited for
//     every slab's next contribution, recorded after that slab's fold of this one.  Without peer access the
//     vectors are gathered on slab 0's device, folded there (k_multi_sum) and copied back.
// Reuse of an exchange buffer is safe without extra events: every plane a receiver consumes is consumed
// before that receiver's next sums contribution, and every producer overwrites its send buffer only after
// the following sums fold, which waited for every slab's contribution.
// Included by pdhg_api.hip after the C ABI (uses the slab entry points and, for the lagged done read, the
// slab context's control block).
#pragma once
#include <vector>

namespace pdhg {
constexpr int kMultiMaxPeerFold = 16;
struct SumPtrs {
  const double* p[kMultiMaxPeerFold];
};
// fixed-order fold of P contribution vectors read in place (local or peer device memory)
__global__ void k_multi_fold(SumPtrs in, int n, double* __restrict__ out) {
  const int s = threadIdx.x;
  if (s >= pdhg::kNumSums) return;
  double t = 0.0;
  for (int q = 0; q < n; ++q) t += in.p[q][s];
  out[s] = t;
}
// same-device plane copy as a kernel (PDHG_MULTI_KCOPY=1; diagnostic against the runtime's D2D copy engine)
__global__ void k_multi_copy(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}
__global__ void k_multi_sum(const double* __restrict__ in, int n, double* __restrict__ out) {
  const int s = threadIdx.x;   // one thread per sum, slabs in order (fixed-order, deterministic)
  if (s >= pdhg::kNumSums) return;
  double t = 0.0;
  for (int q = 0; q < n; ++q) t += in[(size_t)q * kNumSums + s];
  out[s] = t;
}
}  // namespace pdhg

struct pdhg_multi {
  uint32_t magic = kMultiMagic;
  int P = 0;
  int parts = 2;           // column-block parts of the carry exchange
  std::vector<int> dev;
  std::vector<pdhg_ctx*> s;
  std::vector<hipStream_t> st, ss;
  std::vector<int> j0, j1;
  pdhg_problem pb{};
  std::vector<double> xs, ys;
  size_t sp = 0, spec = 0;
  int K = 0;               // long-range modes
  int nar = 4, nc = 2;     // reference alp layout [nar][T][nx][ny][nc]
  size_t es = 4;           // bytes per plane element: 4 (fp32 slabs) or 8 (fp64, the reference's arithmetic)
  struct Buf {
    // planes in the slabs' precision (es bytes per element): byte pointers, element offsets scaled by es
    char *rho_send = nullptr, *rho_recv = nullptr, *pb_send = nullptr, *pb_recv = nullptr;
    char *DS = nullptr, *GS = nullptr, *Dl = nullptr, *S1r = nullptr, *LONG = nullptr, *allLong = nullptr,
         *allGS = nullptr;
    double* sums = nullptr;      // the folded vector this slab's finalize kernels read
    double* contrib = nullptr;   // peer fold: [2][16] contributions, alternating per allreduce
    // events: producer side (main stream) and receiver side (side stream)
    hipEvent_t rho = nullptr, rho_in = nullptr, longp = nullptr, long_in = nullptr, pb = nullptr, pb_in = nullptr,
               sum = nullptr;
    std::vector<hipEvent_t> ds, carry_in;   // per part
  };
  std::vector<Buf> b;
  double* gather = nullptr;   // slab 0's device: [P][16] sums, then the folded [16] (no peer access)
  hipEvent_t folded = nullptr;
  bool peer_fold = false;     // every pair of devices has peer access: per-device folds of the contributions
  bool kcopy = false;         // same-device plane copies as a kernel (PDHG_MULTI_KCOPY=1)
  int sync_mask = 0;          // diagnostic: full barrier at these step() marks (PDHG_MULTI_SYNC, bit i = mark i)
  bool one_stream = false;    // diagnostic: planes received on the main stream (PDHG_MULTI_ONESTREAM=1)
  // step fence (diagnostic, PDHG_MULTI_STEP_FENCE=1): every stream of every slab starts an outer iteration only
  // after every slab's main stream finished the previous one (events, no host sync)
  bool step_fence = false;
  std::vector<hipEvent_t> step_end;   // per slab, recorded on its main stream at the end of step()
  unsigned round = 0;         // allreduces so far (peer fold: which contribution buffer)
  bool stepped = false;       // step_end holds a recorded event
  std::vector<void*> allocs;  // (device, pointer) freed at destroy
  std::vector<int> alloc_dev;
  std::vector<hipEvent_t> all_events;   // (created on the device of the slab that records them)
  std::vector<int> event_dev;
  // per-phase timing on slab 0's main stream (waits included): marks between the phases of step()
  bool prof = false;
  static constexpr int kMarks = 8;
  std::vector<std::vector<hipEvent_t>> marks;   // [step][kMarks]
  size_t marks_used = 0;

  int on(int r) { return hipSetDevice(dev[r]) == hipSuccess ? 0 : -1; }
  template <typename T>
  int alloc(int r, T** p, size_t n) {
    if (on(r)) return fail(PDHG_ERR_HIP, "hipSetDevice(%d)", dev[r]);
    void* q = nullptr;
    if (hipMalloc(&q, std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess)
      return fail(PDHG_ERR_HIP, "hipMalloc of %zu bytes on device %d", n * sizeof(T), dev[r]);
    // zeroed on the slab's main stream: st / ss are non-blocking streams, which a legacy-stream hipMemset is not
    // ordered with (a plane a slab never receives -- slab 0's D_left, the last slab's S1_right -- must read zero);
    // setup() drains st / ss (full_barrier) before any exchange
    if (hipMemsetAsync(q, 0, std::max<size_t>(n, 1) * sizeof(T), st[r]) != hipSuccess)
      return fail(PDHG_ERR_HIP, "hipMemsetAsync");
    allocs.push_back(q);
    alloc_dev.push_back(dev[r]);
    *p = static_cast<T*>(q);
    return PDHG_OK;
  }
  int event(int r, hipEvent_t* e, bool timing = false) {
    if (on(r)) return fail(PDHG_ERR_HIP, "hipSetDevice(%d)", dev[r]);
    HIP_TRY(hipEventCreateWithFlags(e, timing ? hipEventDefault : hipEventDisableTiming));
    all_events.push_back(*e);
    event_dev.push_back(dev[r]);
    return PDHG_OK;
  }
  int rec(hipEvent_t e, int r, hipStream_t s_) {
    if (on(r)) return fail(PDHG_ERR_HIP, "hipSetDevice");
    HIP_TRY(hipEventRecord(e, s_));
    return PDHG_OK;
  }
  int wait(int r, hipStream_t s_, hipEvent_t e) {
    if (on(r)) return fail(PDHG_ERR_HIP, "hipSetDevice");
    HIP_TRY(hipStreamWaitEvent(s_, e, 0));
    return PDHG_OK;
  }
  // copy on stream s_ of slab rd (the receiver)
  int copy(int rd, hipStream_t s_, void* dst, int rs, const void* src, size_t bytes) {
    if (on(rd)) return fail(PDHG_ERR_HIP, "hipSetDevice");
    if (dev[rd] == dev[rs] && kcopy && bytes % 16 == 0 && ((uintptr_t)dst | (uintptr_t)src) % 16 == 0) {
      const size_t n16 = bytes / 16;
      hipLaunchKernelGGL(pdhg::k_multi_copy, dim3((unsigned)std::min<size_t>((n16 + 255) / 256, 4096)), dim3(256), 0, s_,
                         static_cast<const uint4*>(src), static_cast<uint4*>(dst), n16);
      HIP_TRY(hipGetLastError());
    } else if (dev[rd] == dev[rs]) HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s_));
    else HIP_TRY(hipMemcpyPeerAsync(dst, dev[rd], src, dev[rs], bytes, s_));
    return PDHG_OK;
  }
  // every main stream waits for everything enqueued so far on every main and side stream (setup only)
  int full_barrier() {
    for (int r = 0; r < P; ++r) {
      if (on(r)) return fail(PDHG_ERR_HIP, "hipSetDevice");
      HIP_TRY(hipStreamSynchronize(ss[r]));
      HIP_TRY(hipStreamSynchronize(st[r]));
    }
    return PDHG_OK;
  }
  int mark(int i) {
    if (sync_mask & (1 << i)) {   // diagnostic (PDHG_MULTI_SYNC): drain every stream at this phase boundary
      int rc = full_barrier();
      if (rc) return rc;
    }
    if (!prof) return PDHG_OK;
    if (i == 0) {
      if (marks_used == marks.size()) {
        marks.emplace_back(kMarks, nullptr);
        for (int m = 0; m < kMarks; ++m) {
          int rc = event(0, &marks.back()[m], true);
          if (rc) return rc;
        }
      }
      ++marks_used;
    }
    return rec(marks[marks_used - 1][i], 0, st[0]);
  }
  // where slab r writes its contribution to the next allreduce
  double* cs(int r) { return peer_fold ? b[r].contrib + (size_t)(round & 1) * kNumSums : b[r].sums; }
  // sums of every slab -> fixed-order fold -> every slab (b[r].sums)
  int allreduce() {
    int rc;
    if (peer_fold) {
      SumPtrs ptrs{};
      for (int q = 0; q < P; ++q) ptrs.p[q] = cs(q);
      for (int q = 0; q < P; ++q)
        if ((rc = rec(b[q].sum, q, st[q]))) return rc;
      for (int r = 0; r < P; ++r) {
        for (int q = 0; q < P; ++q)
          if (q != r && (rc = wait(r, st[r], b[q].sum))) return rc;
        hipLaunchKernelGGL(pdhg::k_multi_fold, dim3(1), dim3(64), 0, st[r], ptrs, P, b[r].sums);
        HIP_TRY(hipGetLastError());
      }
      ++round;
      return PDHG_OK;
    }
    for (int q = 0; q < P; ++q)
      if ((rc = rec(b[q].sum, q, st[q]))) return rc;
    for (int q = 1; q < P; ++q)
      if ((rc = wait(0, st[0], b[q].sum))) return rc;
    for (int q = 0; q < P; ++q)
      if ((rc = copy(0, st[0], gather + (size_t)q * kNumSums, q, b[q].sums, kNumSums * sizeof(double)))) return rc;
    if (on(0)) return fail(PDHG_ERR_HIP, "hipSetDevice");
    hipLaunchKernelGGL(pdhg::k_multi_sum, dim3(1), dim3(64), 0, st[0], gather, P, gather + (size_t)P * kNumSums);
    HIP_TRY(hipGetLastError());
    if ((rc = rec(folded, 0, st[0]))) return rc;
    for (int q = 0; q < P; ++q) {
      if (q > 0 && (rc = wait(q, st[q], folded))) return rc;
      if ((rc = copy(q, st[q], b[q].sums, 0, gather + (size_t)P * kNumSums, kNumSums * sizeof(double)))) return rc;
    }
    return PDHG_OK;
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
    es = prob.precision == 8 ? 8 : 4;
    const int T = prob.T;
    if (P < 1 || P > T) return fail(PDHG_ERR_ARG, "need 1 <= ndev <= T (ndev %d, T %d)", P, T);
    if (const char* e = getenv("PDHG_MULTI_PARTS")) parts = std::max(1, atoi(e));   // tuning override
    if (const char* e = getenv("PDHG_MULTI_KCOPY")) kcopy = atoi(e) != 0;            // diagnostic
    if (const char* e = getenv("PDHG_MULTI_SYNC")) sync_mask = (int)strtol(e, nullptr, 0);   // diagnostic
    if (const char* e = getenv("PDHG_MULTI_ONESTREAM")) one_stream = atoi(e) != 0;          // diagnostic
    if (const char* e = getenv("PDHG_MULTI_STEP_FENCE")) step_fence = atoi(e) != 0;
    const int base = T / P, extra = T % P;
    for (int q = 0, j = 0; q < P; ++q) {   // pdhg_amd.slab.slab_bounds
      const int n = base + (q < extra ? 1 : 0);
      j0.push_back(j);
      j1.push_back(j + n);
      j += n;
    }
    // peer access where the runtime offers it (copies work either way).  The per-device peer fold of the sums
    // (plain loads of another device's buffers, cross-device event order for the alternating contribution
    // buffers) is opt-in, PDHG_MULTI_PEER_FOLD=1, until a run on two real devices has shown it bitwise equal to
    // the gather fold; the default is the gather -> fold -> scatter chain on slab 0's device
    peer_fold = false;
    if (const char* e = getenv("PDHG_MULTI_PEER_FOLD")) peer_fold = P <= pdhg::kMultiMaxPeerFold && atoi(e) != 0;
    for (int r = 0; r < P; ++r)
      for (int q = 0; q < P; ++q) {
        if (dev[r] == dev[q]) continue;
        int ok = 0;
        if (hipDeviceCanAccessPeer(&ok, dev[r], dev[q]) == hipSuccess && ok) {
          hipSetDevice(dev[r]);
          hipError_t e = hipDeviceEnablePeerAccess(dev[q], 0);
          if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return fail(PDHG_ERR_HIP, "peer access");
          (void)hipGetLastError();
        } else {
          peer_fold = false;
        }
      }
    s.assign(P, nullptr);
    st.assign(P, nullptr);
    ss.assign(P, nullptr);
    b.assign(P, Buf{});
    int rc;
    for (int r = 0; r < P; ++r) {
      pdhg_problem q = pb;
      q.T = j1[r] - j0[r];
      if ((rc = pdhg_create_slab(&q, j0[r], T, dev[r], &s[r]))) return rc;
      if (on(r)) return fail(PDHG_ERR_HIP, "hipSetDevice");
      HIP_TRY(hipStreamCreateWithFlags(&st[r], hipStreamNonBlocking));
      if (one_stream) ss[r] = st[r];   // diagnostic (PDHG_MULTI_ONESTREAM=1): receives on the main stream
      else HIP_TRY(hipStreamCreateWithFlags(&ss[r], hipStreamNonBlocking));
      if ((rc = pdhg_set_stream(s[r], st[r]))) return rc;
      Buf& x = b[r];
      for (hipEvent_t* e : {&x.rho, &x.rho_in, &x.longp, &x.long_in, &x.pb, &x.pb_in, &x.sum})
        if ((rc = event(r, e))) return rc;
      x.ds.assign(parts, nullptr);
      x.carry_in.assign(parts, nullptr);
      for (int q = 0; q < parts; ++q)
        if ((rc = event(r, &x.ds[q])) || (rc = event(r, &x.carry_in[q]))) return rc;
    }
    if ((rc = event(0, &folded))) return rc;
    step_end.assign(P, nullptr);
    for (int r = 0; r < P; ++r)
      if ((rc = event(r, &step_end[r]))) return rc;
    unsigned long long a = 0, c = 0;
    if ((rc = pdhg_slab_plane_size(s[0], &a, &c))) return rc;
    sp = a;
    spec = c;
    for (int r = 0; r < P; ++r) {
      Buf& x = b[r];
      if ((rc = alloc(r, &x.rho_send, sp * es)) || (rc = alloc(r, &x.rho_recv, sp * es)) ||
          (rc = alloc(r, &x.pb_send, sp * es)) || (rc = alloc(r, &x.pb_recv, sp * es)) ||
          (rc = alloc(r, &x.DS, 2 * spec * es)) || (rc = alloc(r, &x.GS, 2 * spec * es)) ||
          (rc = alloc(r, &x.Dl, spec * es)) || (rc = alloc(r, &x.S1r, spec * es)) ||
          (rc = alloc(r, &x.allGS, 2 * spec * P * es)) ||
          (rc = alloc(r, &x.sums, (size_t)kNumSums)) || (rc = alloc(r, &x.contrib, (size_t)2 * kNumSums)))
        return rc;
      if ((rc = pdhg_slab_carry_gain(s[r], x.GS))) return rc;
    }
    if ((rc = alloc(0, &gather, (size_t)(P + 1) * kNumSums))) return rc;
    // iteration-invariant gains of every slab to every slab, then the long-range classification
    if ((rc = full_barrier())) return rc;
    for (int r = 0; r < P; ++r)
      for (int q = 0; q < P; ++q)
        if ((rc = copy(r, st[r], b[r].allGS + (size_t)q * 2 * spec * es, q, b[q].GS, 2 * spec * es))) return rc;
    if ((rc = full_barrier())) return rc;
    for (int r = 0; r < P; ++r) {
      int k = 0;
      if ((rc = pdhg_slab_long_modes(s[r], b[r].allGS, P, 9.094947017729282e-13 /* 2^-40 */, &k))) return rc;
      if (r == 0) K = k;
      else if (k != K) return fail(PDHG_ERR_STATE, "slabs disagree on the long-range modes (%d vs %d)", k, K);
    }
    for (int r = 0; r < P; ++r)
      if ((rc = alloc(r, &b[r].LONG, (size_t)std::max(1, 2 * K) * es)) ||
          (rc = alloc(r, &b[r].allLong, (size_t)std::max(1, 2 * K) * P * es)))
        return rc;
    return full_barrier();
  }

  ~pdhg_multi() {
    for (int r = 0; r < P; ++r) {
      if (r < (int)st.size() && st[r]) { hipSetDevice(dev[r]); hipStreamSynchronize(st[r]); }
      if (r < (int)ss.size() && ss[r]) { hipSetDevice(dev[r]); hipStreamSynchronize(ss[r]); }
    }
    for (auto* c : s) pdhg_destroy(c);
    for (size_t i = 0; i < allocs.size(); ++i) {
      hipSetDevice(alloc_dev[i]);
      hipFree(allocs[i]);
    }
    for (size_t i = 0; i < all_events.size(); ++i) {
      hipSetDevice(event_dev[i]);
      hipEventDestroy(all_events[i]);
    }
    for (int r = 0; r < P; ++r) {
      if (r < (int)st.size() && st[r]) { hipSetDevice(dev[r]); hipStreamDestroy(st[r]); }
      if (r < (int)ss.size() && ss[r] && ss[r] != st[r]) { hipSetDevice(dev[r]); hipStreamDestroy(ss[r]); }
    }
    magic = 0;
  }

  // one outer iteration (include/pdhg.h t-slab choreography, neighbour exchange in `parts` column-block parts)
  int step(double tau, double sigma, double eps, int k) {
    int rc;
    const size_t pbytes = sp * es;
    if (step_fence && stepped) {   // the previous step's end on every slab's main stream, for every stream
      for (int r = 0; r < P; ++r)
        for (int q = 0; q < P; ++q) {
          if (q != r && (rc = wait(r, st[r], step_end[q]))) return rc;
          if (ss[r] != st[r] && (rc = wait(r, ss[r], step_end[q]))) return rc;
        }
    }
    if ((rc = mark(0))) return rc;
    // rho halo (row 0 of slab r+1 -> slab r) on the receiver's side stream || the residual rows without it
    for (int r = 0; r < P; ++r)
      if ((rc = pdhg_slab_plane_out(s[r], 0, b[r].rho_send)) || (rc = rec(b[r].rho, r, st[r]))) return rc;
    for (int r = 0; r + 1 < P; ++r)
      if ((rc = wait(r, ss[r], b[r + 1].rho)) ||
          (rc = copy(r, ss[r], b[r].rho_recv, r + 1, b[r + 1].rho_send, pbytes)) || (rc = rec(b[r].rho_in, r, ss[r])))
        return rc;
    for (int r = 0; r < P; ++r)
      if ((rc = pdhg_slab_residual(s[r], 1))) return rc;
    for (int r = 0; r < P; ++r) {
      if (r + 1 < P && ((rc = wait(r, st[r], b[r].rho_in)) || (rc = pdhg_slab_plane_in(s[r], 0, b[r].rho_recv))))
        return rc;
      if ((rc = pdhg_slab_residual(s[r], 2))) return rc;
    }
    if ((rc = mark(1))) return rc;
    // zero-carry forward sweeps part by part; part q's D (to r+1) and S1 (to r-1) travel during part q+1
    for (int q = 0; q < parts; ++q) {
      unsigned long long m0 = 0, m1 = 0;
      if ((rc = pdhg_slab_part_modes(s[0], q, parts, &m0, &m1))) return rc;
      const size_t off = m0 * es, n = (m1 - m0) * es;   // bytes
      for (int r = 0; r < P; ++r)
        if ((rc = pdhg_slab_forward_part(s[r], tau, q, parts)) || (rc = pdhg_slab_carry_out_part(s[r], b[r].DS, q, parts)) ||
            (rc = rec(b[r].ds[q], r, st[r])))
          return rc;
      for (int r = 0; r < P; ++r) {
        if (r > 0 && ((rc = wait(r, ss[r], b[r - 1].ds[q])) ||
                      (rc = copy(r, ss[r], b[r].Dl + off, r - 1, b[r - 1].DS + off, n))))
          return rc;
        if (r + 1 < P && ((rc = wait(r, ss[r], b[r + 1].ds[q])) ||
                          (rc = copy(r, ss[r], b[r].S1r + off, r + 1, b[r + 1].DS + spec * es + off, n))))
          return rc;
        if ((rc = rec(b[r].carry_in[q], r, ss[r]))) return rc;
      }
    }
    // the long-range modes go to every slab
    if (K > 0) {
      for (int r = 0; r < P; ++r)
        if ((rc = pdhg_slab_plane_out(s[r], 3, b[r].LONG)) || (rc = rec(b[r].longp, r, st[r]))) return rc;
      for (int r = 0; r < P; ++r) {
        for (int q = 0; q < P; ++q)
          if ((rc = wait(r, ss[r], b[q].longp)) ||
              (rc = copy(r, ss[r], b[r].allLong + (size_t)q * 2 * K * es, q, b[q].LONG, 2 * (size_t)K * es)))
            return rc;
        if ((rc = rec(b[r].long_in, r, ss[r]))) return rc;
      }
    }
    if ((rc = mark(2))) return rc;
    // carry fix-ups and backward sweeps part by part, then the inverse y transform + update (primal sums)
    for (int q = 0; q < parts; ++q)
      for (int r = 0; r < P; ++r) {
        if ((rc = wait(r, st[r], b[r].carry_in[q]))) return rc;
        if (q == 0 && K > 0 && (rc = wait(r, st[r], b[r].long_in))) return rc;
        if ((rc = pdhg_slab_fixup_nb_part(s[r], b[r].Dl, b[r].S1r, b[r].allLong, b[r].allGS, r, P, q, parts)) ||
            (rc = pdhg_slab_backward_part(s[r], tau, q, parts)))
          return rc;
      }
    for (int r = 0; r < P; ++r)
      if ((rc = pdhg_slab_update(s[r], tau, cs(r)))) return rc;
    if ((rc = mark(3))) return rc;
    // phi_bar halo (row T of slab r-1 -> row 0 of slab r) || the primal sums and the interior dual rows
    for (int r = 0; r < P; ++r)
      if ((rc = pdhg_slab_plane_out(s[r], 1, b[r].pb_send)) || (rc = rec(b[r].pb, r, st[r]))) return rc;
    for (int r = 1; r < P; ++r)
      if ((rc = wait(r, ss[r], b[r - 1].pb)) || (rc = copy(r, ss[r], b[r].pb_recv, r - 1, b[r - 1].pb_send, pbytes)) ||
          (rc = rec(b[r].pb_in, r, ss[r])))
        return rc;
    if ((rc = allreduce())) return rc;
    for (int r = 0; r < P; ++r)
      if ((rc = pdhg_slab_primal_finalize(s[r], b[r].sums))) return rc;
    if ((rc = mark(4))) return rc;
    for (int sub = 0; sub < k; ++sub) {
      for (int r = 0; r < P; ++r)
        if ((rc = pdhg_slab_dual(s[r], sigma, k, sub, cs(r), sub == 0 ? 1 : 3))) return rc;
      if (sub == 0)
        for (int r = 0; r < P; ++r) {
          if (r > 0 && ((rc = wait(r, st[r], b[r].pb_in)) || (rc = pdhg_slab_plane_in(s[r], 1, b[r].pb_recv))))
            return rc;
          if ((rc = pdhg_slab_dual(s[r], sigma, k, sub, cs(r), 2))) return rc;
        }
      if ((rc = allreduce())) return rc;
      for (int r = 0; r < P; ++r)
        if ((rc = pdhg_slab_dual_finalize(s[r], eps, sub, b[r].sums))) return rc;
    }
    if ((rc = mark(5))) return rc;
    for (int r = 0; r < P; ++r)
      if ((rc = pdhg_slab_outer(s[r], k, cs(r)))) return rc;
    if (k > 1 && (rc = allreduce())) return rc;
    for (int r = 0; r < P; ++r)
      if ((rc = pdhg_slab_outer_finalize(s[r], eps, k, b[r].sums))) return rc;
    for (int r = 0; r < P; ++r)
      if ((rc = rec(step_end[r], r, st[r]))) return rc;
    stepped = true;
    return mark(6);
  }

  int iterate(int n, double tau, double sigma, double eps, int k, pdhg_stats* out) {
    int rc;
    for (int r = 0; r < P; ++r)
      if ((rc = pdhg_slab_begin(s[r]))) return rc;
    // the device loop control of Impl::iterate: at most two windows of 8 iterations ahead of the device,
    // the done flag of the window before the last one read without draining the pipeline
    const int window = 8;
    std::vector<hipEvent_t> evs;
    int ret = PDHG_OK;
    for (int it = 0; it < n && ret == PDHG_OK; ++it) {
      if ((ret = step(tau, sigma, eps, k))) break;
      if ((it + 1) % window == 0 && it + 1 < n) {
        hipEvent_t e;
        if ((ret = event(0, &e))) break;
        if ((ret = rec(e, 0, st[0]))) break;
        evs.push_back(e);
        if (evs.size() >= 2) {
          int done = 0;
          if (hipEventSynchronize(evs[evs.size() - 2]) != hipSuccess) { ret = fail(PDHG_ERR_HIP, "event sync"); break; }
          if ((ret = slab_done_flag(s[0], &done))) break;
          if (done) break;
        }
      }
    }
    for (auto e : evs) {   // drop the window events (created through event(): remove from the pool)
      for (size_t i = 0; i < all_events.size(); ++i)
        if (all_events[i] == e) {
          hipSetDevice(event_dev[i]);
          hipEventSynchronize(e);
          hipEventDestroy(e);
          all_events.erase(all_events.begin() + i);
          event_dev.erase(event_dev.begin() + i);
          break;
        }
    }
    if (ret) return ret;
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
    if ((rc = full_barrier())) return rc;   // the state copies are synchronous: drain the slab streams
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

  // total ms between marks [m0, m1) over the recorded steps
  int phase_ms(int m0, int m1, double* ms, int* n) {
    *ms = 0.0;
    *n = 0;
    if (on(0)) return fail(PDHG_ERR_HIP, "hipSetDevice");
    HIP_TRY(hipStreamSynchronize(st[0]));
    for (size_t i = 0; i < marks_used; ++i) {
      float t = 0.f;
      HIP_TRY(hipEventElapsedTime(&t, marks[i][m0], marks[i][m1]));
      *ms += t;
      ++*n;
    }
    return PDHG_OK;
  }
};

namespace {
pdhg_multi* multi_handle(pdhg_multi* m) { return (m && m->magic == kMultiMagic) ? m : nullptr; }
}  // namespace

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
  if (!m) return PDHG_OK;
  if (!multi_handle(m)) return fail(PDHG_ERR_ARG, "not a multi-device context");
  delete m;
  return PDHG_OK;
}
#define MULTI_GET(m)                                                                       \
  do {                                                                                     \
    if (!multi_handle(m)) return fail(PDHG_ERR_ARG, "null or foreign multi-device handle"); \
  } while (0)
int pdhg_multi_set_state(pdhg_multi* m, const double* phi, const double* rho, const double* alp) {
  MULTI_GET(m);
  return m->state(true, const_cast<double*>(phi), const_cast<double*>(rho), const_cast<double*>(alp));
}
int pdhg_multi_init_state(pdhg_multi* m, const double* g) {
  MULTI_GET(m);
  if (!g) return fail(PDHG_ERR_ARG, "null g");
  int rc = m->full_barrier();
  for (int r = 0; r < m->P && !rc; ++r) rc = pdhg_init_state(m->s[r], g);   // utils_pdhg_solver.py:123-137
  return rc;
}
int pdhg_multi_get_state(pdhg_multi* m, double* phi, double* rho, double* alp) {
  MULTI_GET(m);
  return m->state(false, phi, rho, alp);
}
int pdhg_multi_iterate(pdhg_multi* m, int n_iters, double tau, double sigma, double eps, int rho_alp_iters,
                       pdhg_stats* out) {
  MULTI_GET(m);
  if (n_iters < 0 || rho_alp_iters < 1) return fail(PDHG_ERR_ARG, "bad iteration counts");
  return m->iterate(n_iters, tau, sigma, eps, rho_alp_iters, out);
}
int pdhg_multi_set_stop_rules(pdhg_multi* m, int stop_on_converge, int stop_on_nan) {
  MULTI_GET(m);
  for (auto* c : m->s) {
    int rc = pdhg_set_stop_rules(c, stop_on_converge, stop_on_nan);
    if (rc) return rc;
  }
  return PDHG_OK;
}
int pdhg_multi_synchronize(pdhg_multi* m) {
  MULTI_GET(m);
  return m->full_barrier();
}
int pdhg_multi_info(pdhg_multi* m, const char* key, int* value) {
  MULTI_GET(m);
  if (!key || !value) return fail(PDHG_ERR_ARG, "null argument");
  const std::string k(key);
  if (k == "ndev") *value = m->P;
  else if (k == "long_modes") *value = m->K;
  else if (k == "parts") *value = m->parts;
  else if (k == "peer_fold") *value = m->peer_fold ? 1 : 0;
  else if (k.rfind("rows:", 0) == 0) {
    const int r = atoi(k.c_str() + 5);
    if (r < 0 || r >= m->P) return fail(PDHG_ERR_ARG, "slab %d of %d", r, m->P);
    *value = m->j1[r] - m->j0[r];
  } else if (k.rfind("device:", 0) == 0) {   // the HIP device slab r computes on (its context's device)
    const int r = atoi(k.c_str() + 7);
    if (r < 0 || r >= m->P) return fail(PDHG_ERR_ARG, "slab %d of %d", r, m->P);
    return slab_device(m->s[r], value);
  } else return fail(PDHG_ERR_ARG, "unknown key '%s'", key);
  return PDHG_OK;
}
int pdhg_multi_profile(pdhg_multi* m, int enable) {
  MULTI_GET(m);
  int rc = m->full_barrier();
  if (rc) return rc;
  m->prof = enable != 0;
  m->marks_used = 0;
  return PDHG_OK;
}
int pdhg_multi_phase_ms(pdhg_multi* m, const char* phase, double* total_ms, int* steps) {
  MULTI_GET(m);
  if (!phase || !total_ms || !steps) return fail(PDHG_ERR_ARG, "null argument");
  // marks: 0 start, 1 residual done, 2 forward sweeps + carry planes issued, 3 fix-up + backward + update,
  // 4 primal sums folded, 5 dual sub-iterations (with their sums), 6 outer sums
  static const struct { const char* name; int m0, m1; } kPh[] = {
      {"residual", 0, 1}, {"forward", 1, 2}, {"backward", 2, 3}, {"allreduce", 3, 4}, {"dual", 4, 5},
      {"outer", 5, 6}, {"step", 0, 6}};
  for (const auto& ph : kPh)
    if (!strcmp(ph.name, phase)) return m->phase_ms(ph.m0, ph.m1, total_ms, steps);
  *total_ms = 0.0;
  *steps = 0;
  return PDHG_OK;
}

}  // extern "C"
