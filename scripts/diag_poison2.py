"""Diagnostic (round 5): which part of the multi-device context reads unwritten memory -- poisoned runs of the multi
context at C4's decomposition across parts / iterations / precision (scripts/diag_poison.py)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "scripts")]
import diag_poison as DP  # noqa: E402,F401  (imports diag_multi64 as D and defines poison)
import diag_multi64 as D  # noqa: E402

for n in (1, 2):
    D.n = n
    ref = D.single()
    for env in ({}, {"PDHG_MULTI_PARTS": "1"}):
        os.environ.pop("PDHG_MULTI_PARTS", None)
        os.environ.update(env)
        DP.poison(200)
        D.report("n{} {}".format(n, env), D.multi(), ref[1])
os.environ.pop("PDHG_MULTI_PARTS", None)
