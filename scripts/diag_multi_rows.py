"""Diagnostic (round 5): where the multi-device context's intermittent C4 fp64 mismatch starts -- per slab and row,
after iteration 1 and after iteration 2 (kernel plane copies, which raised the failure rate)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "scripts")]
import diag_multi64 as D  # noqa: E402
from _problems import rel  # noqa: E402

os.environ["PDHG_MULTI_KCOPY"] = "1"
D.n = 1
ref1 = D.single()[1]
D.n = 2
ref2 = D.single()[1]
bounds = [(j * D.T // D.nr, (j + 1) * D.T // D.nr) for j in range(D.nr)]


def rows_bad(out, ref, what):
    a, b = out[what], ref[what]
    return [j for j in range(a.shape[0]) if not rel(a[j], b[j]) <= 1e-12]


from pdhg_amd.multi import MultiContext  # noqa: E402
P = D.P
for rep in range(10):
    D.runner()
    m = MultiContext(D.egno, D.nx, D.ny, D.T, P["dx"], P["dy"], D.dt, P["xs"], P["ys"], devices=[0] * D.nr,
                     epsl=D.epsl, precision="fp64")
    m.init_state(D.g)
    m.iterate(1, D.TAU, D.SIGMA, -1.0, 1)
    o1 = m.get_state()
    m.iterate(1, D.TAU, D.SIGMA, -1.0, 1)
    o2 = m.get_state()
    m.close()
    b1 = {w: rows_bad(o1, ref1, i) for i, w in ((0, "phi"), (1, "rho"))}
    b2 = {w: rows_bad(o2, ref2, i) for i, w in ((0, "phi"), (1, "rho"))}
    a2 = [k for k in range(4) if not rel(o2[2][k], ref2[2][k]) <= 1e-12]
    print("rep", rep, "it1 bad", {k: v[:12] for k, v in b1.items()}, "it2 bad", {k: v[:40] for k, v in b2.items()},
          "alp arrays bad", a2, flush=True)
