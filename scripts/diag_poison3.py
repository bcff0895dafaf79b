"""Diagnostic (round 5): repeated multi-device runs at C4's decomposition (fp64, epsl 0.1, 2 iterations) after the
Python slab driver and poisoned memory, with the runtime's D2D copies and with kernel copies (PDHG_MULTI_KCOPY)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "scripts")]
import diag_poison as DP  # noqa: E402
import diag_multi64 as D  # noqa: E402

ref = D.single()
for kc in ("0", "1", "0", "1"):
    os.environ["PDHG_MULTI_KCOPY"] = kc
    for rep in range(3):
        D.report("runner kcopy{} {}".format(kc, rep), D.runner(), ref[1])
        DP.poison(150)
        D.report("multi kcopy{} {}".format(kc, rep), D.multi(), ref[1])
