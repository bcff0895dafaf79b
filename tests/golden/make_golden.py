"""Generate the golden fixtures in this directory from the float64 oracle (oracle/pdhg_oracle.py).

The JAX reference cannot run in this container (jax/jaxlib/einshape/tensorflow absent), so these
vectors are the oracle's own outputs: they pin the oracle against regressions (CPU tests) and give
the GPU tests fixed inputs/outputs.  Cases follow SURVEY.md §4:
(egno, ndim, epsl, bc) in {(1,1,0,0), (2,1,0.1,0), (1,2,0,(0,0)), (2,2,0.1,(0,0)), (3,2,0,(1,0))},
T in {1, 4}, seeded state.  Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
sys.path.insert(0, os.path.join(HERE, ".."))
import pdhg_oracle as O  # noqa: E402
from _problems import make_problem, oracle_fns  # noqa: E402

CASES = [(1, 1, 32, 1, 0.0), (2, 1, 32, 1, 0.1), (1, 2, 16, 12, 0.0), (2, 2, 16, 12, 0.1), (3, 2, 16, 12, 0.0)]
TAU, SIGMA = 0.1 / 1.5, 0.1 * 1.5


def case_name(egno, ndim, nx, ny, epsl, T):
    return "golden_e{}_d{}_{}x{}_eps{}_T{}.npz".format(egno, ndim, nx, ny, epsl, T)


def generate(egno, ndim, nx, ny, epsl, T):
    P = make_problem(egno, ndim, nx, ny, T, epsl)
    primal, dual = oracle_fns(P)
    out = {"phi": P["phi"], "rho": P["rho"], "alp": np.stack(P["alp"]), "dt": P["dt"], "dx": P["dx"], "dy": P["dy"],
           "xs": P["xs"], "ys": P["ys"] if P["ys"] is not None else np.zeros(0), "tau": TAU, "sigma": SIGMA,
           "meta": np.array([egno, ndim, nx, ny, T]), "epsl": epsl}
    out["primal_phi"] = primal(P["phi"], P["rho"], 70.0, P["alp"], TAU, P["dt"], P["dsp"], P["fns"], P["fv"], epsl,
                               P["x_arr"], None)
    pb = 2 * out["primal_phi"] - P["phi"]
    r1, a1, e1 = O.update_dual_oneiter(pb, P["rho"], 70.0, P["alp"], SIGMA, P["dt"], P["dsp"], epsl, P["x_arr"], None,
                                       P["bc"], P["fns"], ndim)
    out["dual_rho"], out["dual_alp"], out["dual_err"] = r1, np.stack(a1), e1
    phi, rho, alp = P["phi"], P["rho"], P["alp"]
    errs = []
    for it in range(10):
        phi_n = primal(phi, rho, 70.0, alp, TAU, P["dt"], P["dsp"], P["fns"], P["fv"], epsl, P["x_arr"], None)
        rho_n, alp_n = dual(2 * phi_n - phi, rho, 70.0, alp, SIGMA, P["dt"], P["dsp"], epsl, P["fns"], P["x_arr"],
                            None, ndim, -1.0)
        errs.append(O.outer_errors(phi, phi_n, rho, rho_n, alp, alp_n))
        phi, rho, alp = phi_n, rho_n, alp_n
        if it + 1 in (1, 2, 10):
            out["it{}_phi".format(it + 1)] = phi
            out["it{}_rho".format(it + 1)] = rho
            out["it{}_alp".format(it + 1)] = np.stack(alp)
    out["errs"] = np.array(errs)
    return out


def all_cases():
    for egno, ndim, nx, ny, epsl in CASES:
        for T in (1, 4):
            yield egno, ndim, nx, ny, epsl, T


if __name__ == "__main__":
    for c in all_cases():
        np.savez_compressed(os.path.join(HERE, case_name(*c)), **generate(*c))
        print("wrote", case_name(*c))
