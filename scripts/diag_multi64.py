"""Diagnostic (round 5): determinism of the fp64 single context, the Python slab driver and the multi-device context
at C4's 8-slab decomposition (nx = 8192, y cut to 256, T = 128, epsl = 0.1, 2 iterations from the reference state)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pdhg-optimal-control_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
from _problems import make_problem, rel  # noqa: E402

TAU, SIGMA = 0.1 / 1.5, 0.1 * 1.5
egno, nx, ny, T, nr, epsl, n = 2, 8192, 256, 128, 8, 0.1, int(sys.argv[1]) if len(sys.argv) > 1 else 2
P = make_problem(egno, 2, nx, ny, 1, epsl, seeded=False)
g = P["g"][0]
dt = 1.0 / T


def single():
    from pdhg_amd.context import PDHGContext
    c = PDHGContext(egno, 2, nx, ny, T, P["dx"], P["dy"], dt, P["xs"], P["ys"], epsl=epsl, precision="fp64")
    c.init_state(g)
    st = c.iterate(n, TAU, SIGMA, -1.0, 1)
    out = c.get_state()
    c.close()
    return st, out


def multi():
    from pdhg_amd.multi import MultiContext
    m = MultiContext(egno, nx, ny, T, P["dx"], P["dy"], dt, P["xs"], P["ys"], devices=[0] * nr, epsl=epsl,
                     precision="fp64")
    m.init_state(g)
    st = m.iterate(n, TAU, SIGMA, -1.0, 1)
    out = m.get_state()
    m.close()
    return st, out


def runner():
    import torch
    from pdhg_amd.slab import LocalComm, SlabContext, SlabRunner, join_state
    slabs = [SlabContext(r, nr, T, egno, nx, ny, P["dx"], P["dy"], dt, P["xs"], P["ys"], epsl=epsl, precision="fp64")
             for r in range(nr)]
    for s in slabs:
        s.init_state(g)
    st = SlabRunner(slabs, LocalComm(nr)).iterate(n, TAU, SIGMA, -1.0, 1)
    torch.cuda.synchronize()
    out = join_state([s.get_state() for s in slabs])
    for s in slabs:
        s.close()
    return st, out


def main():
  runs = {}
  for name, fn in (("single0", single), ("single1", single), ("runner0", runner), ("multi0", multi), ("multi1", multi),
                 ("multi2", multi), ("runner1", runner)):
    runs[name] = fn()
    report(name, runs[name], runs["single0"][1])


def report(name, run, ref):
    st, out = run
    d = {"phi": rel(out[0], ref[0]), "rho": rel(out[1], ref[1])}
    rows = [float(rel(out[1][j], ref[1][j])) for j in range(T)]
    bad = [j for j, v in enumerate(rows) if not v <= 1e-10]
    print(name, {a: "%.2e" % b for a, b in d.items()}, "err1 %.6e" % st.get("err1"), "bad rho rows", bad[:20],
          flush=True)


if __name__ == "__main__":
    main()
