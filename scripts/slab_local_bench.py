"""Per-slab cost of the t-slab / x-slab decompositions, measured on ONE GPU (run via gpurun).

P slab contexts of one window run in this process (LocalComm: collectives are device copies), so a step
costs the sum of the P slabs' kernels plus the copies; step_ms / P estimates the per-GPU compute time
of a P-GPU run (RCCL transfer time excluded).  Per-kernel-class times come from the contexts' HIP-event
profiles (pdhg_profile_query), summed over slabs and divided by P.

mode "multi": the same t-slabs driven by the native multi-device context (pdhg_create_multi with the device
list [0] * P: one host thread, per-slab main + side streams, per-neighbour events), with the per-phase times
of slab 0's stream (pdhg_multi_phase_ms: cross-slab waits included).

usage: python scripts/slab_local_bench.py [tslab|xslab|multi] [config] [P] [steps]
"""
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(ROOT, "pdhg-optimal-control_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "tslab"
    cfg = sys.argv[2] if len(sys.argv) > 2 else "c3"
    P = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    egno, ndim, epsl, nx, ny, nt = bench.CONFIGS[cfg]
    T = nt - 1
    xs, ys = bench.grid(ndim, nx, ny)
    dt = 1.0 / (nt - 1)
    g = np.sin(np.pi * xs)[:, None] + np.sin(np.pi * ys)[None, :]
    if mode == "multi":
        from pdhg_amd.multi import MultiContext
        m = MultiContext(egno, nx, ny, T, 2.0 / nx, 2.0 / ny, dt, xs, ys, devices=[0] * P, epsl=epsl)
        m.init_state(g)
        m.set_stop_rules(converge=True, nan=False)
        tau, sigma = 0.1 / 1.5, 0.1 * 1.5
        m.iterate(2, tau, sigma, 1e-6, 1)
        m.synchronize()
        m.profile(True)
        t0 = time.perf_counter()
        st = m.iterate(steps, tau, sigma, 1e-6, 1)
        m.synchronize()
        el = time.perf_counter() - t0
        ph = {k: v / steps for k, v in m.phase_ms(reset=False).items()}
        print(json.dumps({"mode": mode, "config": cfg, "P": P, "steps": steps, "iters": st["iters_run"],
                          "step_ms": el / steps * 1e3, "per_slab_ms": el / steps * 1e3 / P,
                          "long_modes": m.info("long_modes"), "parts": m.info("parts"),
                          "phase_ms_slab0_stream": ph}), flush=True)
        m.close()
        return
    if mode == "tslab":
        from pdhg_amd.slab import LocalComm, SlabContext, SlabRunner
        slabs = [SlabContext(r, P, T, egno, nx, ny, 2.0 / nx, 2.0 / ny, dt, xs, ys, epsl=epsl) for r in range(P)]
        for s in slabs:
            s.init_state(g)
        runner = SlabRunner(slabs, LocalComm(P))
    else:
        from pdhg_amd.xslab import LocalComm, XSlabContext, XSlabRunner
        slabs = [XSlabContext(r, P, egno, nx, ny, T, 2.0 / nx, 2.0 / ny, dt, xs, ys, epsl=epsl) for r in range(P)]
        for s in slabs:
            s.init_global_state(g)
        runner = XSlabRunner(slabs, LocalComm(P))
    for s in slabs:
        s.set_stop_rules(converge=True, nan=False)
    tau, sigma = 0.1 / 1.5, 0.1 * 1.5
    runner.iterate(2, tau, sigma, 1e-6, 1)
    torch.cuda.synchronize()
    for s in slabs:
        s.profile_enable(True)
    t0 = time.perf_counter()
    st = runner.iterate(steps, tau, sigma, 1e-6, 1)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    kern = {}
    for cls in ("residual", "precond", "update", "dual"):
        tot = sum(s.profile_query(cls)[0] for s in slabs)
        kern[cls] = tot / steps / P
    print(json.dumps({"mode": mode, "config": cfg, "P": P, "steps": steps, "iters": st["iters"],
                      "step_ms": el / steps * 1e3, "per_slab_ms": el / steps * 1e3 / P,
                      "kernel_ms_per_slab": kern, "kernel_sum_ms_per_slab": sum(kern.values())}), flush=True)


if __name__ == "__main__":
    main()
