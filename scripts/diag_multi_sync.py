"""Diagnostic (round 5): bisect the multi-device context's intermittent C4 fp64 mismatch with full barriers at
step() phase boundaries (PDHG_MULTI_SYNC bit i = mark i: 1 residual, 2 forward + carries, 3 backward + update,
4 primal sums, 5 dual, 6 outer), kernel plane copies (PDHG_MULTI_KCOPY=1, which raised the failure rate)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "scripts")]
import diag_multi64 as D  # noqa: E402
from _problems import rel  # noqa: E402

ref = D.single()
os.environ["PDHG_MULTI_KCOPY"] = "1"
masks = sys.argv[1:] or ["0", "0x7e", "0x02", "0x04", "0x08", "0x10", "0x20", "0x40"]
for mask in masks:
    os.environ["PDHG_MULTI_SYNC"] = mask
    bad = 0
    for rep in range(6):
        D.runner()
        st, out = D.multi()
        bad += 0 if rel(out[0], ref[1][0]) < 1e-12 else 1
    print("mask", mask, "failures", bad, "/ 6", flush=True)
