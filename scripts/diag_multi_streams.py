"""Diagnostic (round 5): failure rate of the multi-device context at C4's decomposition (fp64, epsl 0.1, 2
iterations) with planes received on per-slab side streams vs on the main streams (PDHG_MULTI_ONESTREAM), kernel
plane copies (PDHG_MULTI_KCOPY=1, the configuration that failed 4 / 10)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "scripts")]
import diag_multi64 as D  # noqa: E402
from _problems import rel  # noqa: E402

ref = D.single()
os.environ["PDHG_MULTI_KCOPY"] = sys.argv[1] if len(sys.argv) > 1 else "1"
bad = {"0": 0, "1": 0}
for rep in range(10):
    for one in ("0", "1"):
        os.environ["PDHG_MULTI_ONESTREAM"] = one
        D.runner()
        st, out = D.multi()
        ok = rel(out[0], ref[1][0]) < 1e-12
        bad[one] += 0 if ok else 1
        print("rep", rep, "onestream", one, "ok" if ok else "BAD %.2e" % rel(out[0], ref[1][0]), flush=True)
print("failures (onestream 0 / 1):", bad, flush=True)
