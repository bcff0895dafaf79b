"""Diagnostic (round 5): 10 multi-device runs per copy mode (runtime D2D copies vs kernel copies), interleaved with
the Python slab driver, at C4's decomposition (fp64, epsl 0.1, 2 iterations): count the runs that leave the single
context's result."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "scripts")]
import diag_poison as DP  # noqa: E402,F401
import diag_multi64 as D  # noqa: E402
from _problems import rel  # noqa: E402

ref = D.single()
bad = {"0": 0, "1": 0}
for rep in range(10):
    for kc in ("0", "1"):
        os.environ["PDHG_MULTI_KCOPY"] = kc
        D.runner()
        st, out = D.multi()
        ok = rel(out[0], ref[1][0]) < 1e-12
        bad[kc] += 0 if ok else 1
        print("rep", rep, "kcopy", kc, "ok" if ok else "BAD %.2e" % rel(out[0], ref[1][0]), flush=True)
print("failures:", bad, flush=True)
