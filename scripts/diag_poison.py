"""Diagnostic (round 5): run the single fp64 context, the Python slab driver and the multi-device context at C4's
8-slab decomposition after filling (and releasing) most of the device memory with NaN, so that any read of a device
buffer no kernel wrote shows up as NaN / a wrong value instead of the zeros of fresh pages."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pdhg-optimal-control_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "scripts")]
import torch  # noqa: E402


def poison(gb):
    xs = []
    for _ in range(int(gb)):
        t = torch.empty(1 << 27, dtype=torch.float64, device="cuda")   # 1 GiB
        t.fill_(float("nan"))
        xs.append(t)
    torch.cuda.synchronize()
    del xs
    torch.cuda.empty_cache()


which = sys.argv[1] if len(sys.argv) > 1 else "all"
prec = sys.argv[2] if len(sys.argv) > 2 else "fp64"
import diag_multi64 as D  # noqa: E402   (module-level runs disabled below)

if __name__ == "__main__":
  ref = D.single()                      # fresh memory
  for name, fn in (("single", D.single), ("runner", D.runner), ("multi", D.multi)):
    for rep in range(2):
      poison(200)
      D.report("{}_poisoned{}".format(name, rep), fn(), ref[1])
