"""Multi-pass dual loop vs the per-sub-iteration kernels on one dual call and on outer iterations (GPU diagnostics).
usage: python scripts/diag_dual_multi.py [prec] [k]"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
sys.path.insert(0, os.path.join(HERE, "..", "pdhg-optimal-control_amd"))
from _problems import device_ctx, make_problem  # noqa: E402

TAU, SIGMA = 0.1 / 1.5, 0.1 * 1.5


def diff(a, b):
    a, b = np.asarray(a), np.asarray(b)
    d = np.abs(a - b)
    return "n_diff {} max {:.3e} rel {:.3e}".format(int(np.count_nonzero(a != b)), float(d.max()),
                                                     float(d.max() / max(np.abs(b).max(), 1e-300)))


def main():
    prec = sys.argv[1] if len(sys.argv) > 1 else "fp32"
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    P = make_problem(1, 2, 32, 256, 3, 0.0)
    rng = np.random.default_rng(5)
    phi_bar = P["phi"] + 0.02 * rng.standard_normal(P["phi"].shape)
    res = {}
    for multi in ("0", "1"):
        os.environ["PDHG_DUAL_MULTI"] = multi
        ctx = device_ctx(P, prec, rho_alp_iters=k)
        print("multi", multi, "path", ctx.path_info("dual_multi"), flush=True)
        ctx.set_state(P["phi"], P["rho"], P["alp"])
        ctx.set_phi_bar(phi_bar)
        used = ctx.update_dual(SIGMA, 1e-6, k)
        _, rho, alp = ctx.get_state()
        res[multi] = [(used, rho, alp)]
        ctx.set_state(P["phi"], P["rho"], P["alp"])
        for it in range(3):
            st = ctx.iterate(1, TAU, SIGMA, 1e-6, k)
            phi, rho, alp = ctx.get_state()
            res[multi].append((st["inner_total"], phi, rho, alp))
        ctx.close()
    (u0, r0, a0), (u1, r1, a1) = res["0"][0], res["1"][0]
    print("update_dual: used", u0, u1, "rho", diff(r1, r0), "alp", [diff(x, y) for x, y in zip(a1, a0)], flush=True)
    for it in range(1, 4):
        (n0, p0, r0, a0), (n1, p1, r1, a1) = res["0"][it], res["1"][it]
        print("iterate", it, "inner", n0, n1, "phi", diff(p1, p0), "rho", diff(r1, r0),
              "alp", [diff(x, y) for x, y in zip(a1, a0)], flush=True)


if __name__ == "__main__":
    main()
