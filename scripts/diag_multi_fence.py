"""Diagnostic (round 5): failure rate of the multi-device context at C4's decomposition (fp64, epsl 0.1, 2
iterations) with and without the step fence (PDHG_MULTI_STEP_FENCE), kernel plane copies (PDHG_MULTI_KCOPY=1)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "scripts")]
import diag_multi64 as D  # noqa: E402
from _problems import rel  # noqa: E402

ref = D.single()
os.environ["PDHG_MULTI_KCOPY"] = "1"
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 12
bad = {"0": 0, "1": 0}
for rep in range(reps):
    for fence in ("0", "1"):
        os.environ["PDHG_MULTI_STEP_FENCE"] = fence
        D.runner()
        st, out = D.multi()
        ok = rel(out[0], ref[1][0]) < 1e-12
        bad[fence] += 0 if ok else 1
        print("rep", rep, "fence", fence, "ok" if ok else "BAD %.2e" % rel(out[0], ref[1][0]), flush=True)
print("failures (fence 0 / 1):", bad, flush=True)
