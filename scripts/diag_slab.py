"""Diagnostic (GPU): single context vs t-slabs, iteration by iteration, from the reference initial state.

usage: python scripts/diag_slab.py egno nx ny T P epsl iters [env=val ...]
Prints per iteration the relative L2 distance of phi, rho and the four alp arrays between the single context
and the slabs (LocalComm, the bench's schedule), and the err1 / err2 of both.
"""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(ROOT, "pdhg-optimal-control_amd")]

import numpy as np  # noqa: E402


def rel(a, b):
    nb = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / (nb if nb > 0 else 1.0))


def main():
    egno, nx, ny, T, P = (int(v) for v in sys.argv[1:6])
    epsl, iters = float(sys.argv[6]), int(sys.argv[7])
    for kv in sys.argv[8:]:
        k, v = kv.split("=")
        os.environ[k] = v
    import torch
    from pdhg_amd.context import PDHGContext
    from pdhg_amd.slab import LocalComm, SlabContext, SlabRunner, join_state
    xs = np.linspace(0.0, 2.0, nx, endpoint=False)
    ys = np.linspace(0.0, 2.0, ny, endpoint=False)
    G = {"dx": 2.0 / nx, "dy": 2.0 / ny, "dt": 1.0 / max(T, 40), "xs": xs, "ys": ys}
    g = np.sin(np.pi * xs)[:, None] + np.sin(np.pi * ys)[None, :]     # set_fns.py:20 (egno 1/2)
    tau, sigma = 0.1 / 1.5, 0.1 * 1.5
    ref = PDHGContext(egno, 2, nx, ny, T, G["dx"], G["dy"], G["dt"], xs, ys, epsl=epsl, precision="fp32")
    ref.init_state(g)
    slabs = [SlabContext(r, P, T, egno, nx, ny, G["dx"], G["dy"], G["dt"], G["xs"], G["ys"], epsl=epsl)
             for r in range(P)]
    for s in slabs:
        s.init_state(g)
    print("single: fused", ref.path_info("fused_residual"), "fast_xt", ref.path_info("fast_xt"), "half_real",
          ref.path_info("half_real"), "| slab0: fused", slabs[0].path_info("fused_residual"), "fast_xt",
          slabs[0].path_info("fast_xt"), flush=True)
    runner = SlabRunner(slabs, LocalComm(P))
    for it in range(1, iters + 1):
        a = ref.iterate(1, tau, sigma, -1.0, 1)
        b = runner.iterate(1, tau, sigma, -1.0, 1)
        torch.cuda.synchronize()
        sr = ref.get_state()
        ss = join_state([s.get_state() for s in slabs])
        d = [rel(ss[0], sr[0]), rel(ss[1], sr[1])] + [rel(x, y) for x, y in zip(ss[2], sr[2])]
        print("it {} phi {:.2e} rho {:.2e} alp {} | err1 {:.6e} {:.6e} err2 {:.6e} {:.6e}".format(
            it, d[0], d[1], " ".join("{:.1e}".format(v) for v in d[2:]), a["err1"], b["err1"], a["err2"], b["err2"]),
            flush=True)
        if it in (1, 2):   # where in (t, x, y) the phi difference sits
            diff = np.abs(ss[0] - sr[0])
            per_t = diff.reshape(T + 1, -1).max(axis=1)
            print("   phi |diff| max per t row:", " ".join("{:.1e}".format(v) for v in per_t[:: max(1, T // 16)]))
            rdiff = np.abs(ss[1] - sr[1])
            print("   rho |diff| max per t row:", " ".join("{:.1e}".format(v) for v in rdiff.reshape(T, -1).max(axis=1)))
            print("   phi |diff| max per t row (all):", " ".join("{:.1e}".format(v) for v in per_t))
            per_x = diff.max(axis=(0, 2))
            print("   phi |diff| max per x (every nx/16):", " ".join("{:.1e}".format(v) for v in per_x[:: nx // 16]))
            print("   argmax", np.unravel_index(np.argmax(diff), diff.shape), "max", float(diff.max()))
    for s in slabs:
        s.close()
    ref.close()


if __name__ == "__main__":
    main()
