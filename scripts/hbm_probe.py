"""Practical HBM rates on this box (PyTorch's own copy / fill / sum kernels over 4 GiB tensors), the yardstick
the kernels' achieved TB/s are read against next to the 8 TB/s spec.
usage: python scripts/hbm_probe.py [GiB]"""
import json
import sys

import torch


def rate(fn, nbytes, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    return {"ms": ms, "TB/s": nbytes / ms / 1e9}


def main():
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
    n = int(gib * 2**30) // 4
    x = torch.empty(n, dtype=torch.float32, device="cuda").uniform_()
    y = torch.empty_like(x)
    out = {
        "bytes_per_array": 4 * n,
        "copy (read + write)": rate(lambda: y.copy_(x), 8 * n),
        "fill (write)": rate(lambda: y.fill_(1.0), 4 * n),
        "sum (read)": rate(lambda: x.sum(), 4 * n),
        "axpy y += 2x (2 reads + write)": rate(lambda: y.add_(x, alpha=2.0), 12 * n),
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
