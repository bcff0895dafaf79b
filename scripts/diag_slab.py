"""Slab runner vs single context, one outer iteration at a time (GPU diagnostics for a failing slab case).
usage: python scripts/diag_slab.py egno nx ny T P k [n] [exchange] [overlap]"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))   # tests/_problems.py builds the inputs with it
sys.path.insert(0, os.path.join(HERE, "..", "pdhg-optimal-control_amd"))
from _problems import make_problem, rel  # noqa: E402


def main():
    import torch
    from pdhg_amd.context import PDHGContext
    from pdhg_amd.slab import LocalComm, SlabContext, SlabRunner, join_state, slab_bounds, split_state
    a = sys.argv[1:]
    egno, nx, ny, T, nr, k = (int(v) for v in a[:6])
    n = int(a[6]) if len(a) > 6 else 6
    exchange = a[7] if len(a) > 7 else "neighbour"
    overlap = (a[8] != "0") if len(a) > 8 else True
    P = make_problem(egno, 2, nx, ny, T, 0.0)
    tau, sigma = 0.1 / 1.5, 0.1 * 1.5
    ref = PDHGContext(egno, 2, nx, ny, T, P["dx"], P["dy"], P["dt"], P["xs"], P["ys"], epsl=0.0,
                      precision="fp32", rho_alp_iters=k)
    ref.set_state(P["phi"], P["rho"], P["alp"])
    slabs = [SlabContext(r, nr, T, egno, nx, ny, P["dx"], P["dy"], P["dt"], P["xs"], P["ys"], epsl=0.0,
                         rho_alp_iters=k) for r in range(nr)]
    print("slab T", [s.T for s in slabs], "fast_xt", [s.path_info("fast_xt") for s in slabs], flush=True)
    for s, part in zip(slabs, split_state(P["phi"], P["rho"], P["alp"], slab_bounds(T, nr))):
        s.set_state(*part)
    runner = SlabRunner(slabs, LocalComm(nr), overlap=overlap, exchange=exchange)
    print("n_long", runner.n_long, flush=True)
    for it in range(1, n + 1):
        st_r = ref.iterate(1, tau, sigma, -1.0, k)
        st = runner.iterate(1, tau, sigma, -1.0, k)
        torch.cuda.synchronize()
        phi_r, rho_r, alp_r = ref.get_state()
        parts = [s.get_state() for s in slabs]
        phi_s, rho_s, alp_s = join_state(parts)
        fin = [bool(np.isfinite(x[0]).all() and np.isfinite(x[1]).all()) for x in parts]
        print("it", it, "ref", {q: st_r[q] for q in ("iters_run", "status", "err1", "err2") if q in st_r},
              "slab", {q: st[q] for q in ("iters", "status", "err1", "err2") if q in st}, "finite", fin,
              "phi", "%.3e" % rel(phi_s, phi_r), "rho", "%.3e" % rel(rho_s, rho_r), flush=True)
        if not all(fin):
            for r, x in enumerate(parts):
                bad = np.argwhere(~np.isfinite(x[0]))
                print("  slab", r, "phi nonfinite", len(bad), bad[:5].tolist(), flush=True)
            break
        # rows of phi with the largest deviation
        d = np.abs(phi_s - phi_r).reshape(phi_s.shape[0], -1).max(axis=1)
        print("  phi max |d| per row", np.array2string(d, precision=2), flush=True)


if __name__ == "__main__":
    main()
