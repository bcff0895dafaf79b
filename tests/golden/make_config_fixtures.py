"""Sampled float64-oracle fixtures for the kernel instantiations the BASELINE configs run.

The bench configs (BASELINE.json configs[1..4]) select size-specialised kernels: the warp-specialised
x transform at nx = 4096 with closed-form pivots over T = 200 rows (C3), the 512-thread ny = 4096 row
kernels and the fused-residual dual (C3), the nx / ny = 2048 kernels at T = 100 (C2), the half-real
nx = 8192 x transform and the ny = 8192 four-row kernels (C4), the four-step 65536-point DHT with
T = 400 (C1).  The oracle needs 20 s to 6 min per iteration at these sizes, too slow for a GPU test's
time limit, so this script runs it here once and keeps, per run, the oracle's state at a fixed set of
sampled points plus full-array norms and the err1/err2 of the last iteration; the GPU tests compare
the device state at the same points (tests/test_gpu_configs.py).

Runs ("kind_e<epsl>_n<iterations>"):
  ref     from the reference initial state (phi = g, rho = c_on_rho, alp = 0; utils_pdhg_solver.py:123-137);
  seeded  from the seeded rough parity state of SURVEY.md §8(d) (drives every mask / clip branch; from the
          reference state the first primal update is exactly zero: the terminal c/dt cancels -rho/dt).
The initial state is rounded to float32 first, so the oracle starts from exactly what the fp32 device
holds.  Every run also stores "e32": how far the same oracle, executed in float32 from the same state
(pdhg_oracle follows a float32 input through the preconditioner: complex64 FFTs and Thomas), lands from
its float64 result at the sampled points -- the accuracy the reference algorithm itself reaches in
float32.  Three effects make it large at these sizes: with epsl > 0 the reference's explicit
sigma*epsl*Lap(phi_bar) dual term amplifies rounding by ~sigma*epsl*8/dx^2 per iteration (5e5 at
dx = 2/4096); from a rough state the H1 preconditioner recovers low modes of U from a residual dominated
by high ones (float32 FFT round-off relative to |R|); and the controls follow one-sided differences of
phi_bar, whose float32 precision is ulp(phi)/(dx*|grad phi|) (~1e-3 at C1's dx = 2/65536).  The tests bound
each quantity by the larger of a fixed bound and a multiple of e32.  (The "sens" entries are the older
calibration of the first fixtures: the float64 oracle's change under one float32 rounding of the initial
values only; no longer generated.)
rho_alp_iters = 1, dt = 1/max(T, 40) (tests/_problems.make_problem).
Run:  python tests/golden/make_config_fixtures.py [name ...]
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
sys.path.insert(0, os.path.join(HERE, ".."))
import pdhg_oracle as O  # noqa: E402
from _problems import make_problem, oracle_fns  # noqa: E402

TAU, SIGMA = 0.1 / 1.5, 0.1 * 1.5
NSAMPLE = 8192

# name: (egno, ndim, nx, ny, T, [(kind, epsl, iterations), ...], what it pins)
CASES = {
    "c3_ws_T200": (2, 2, 4096, 16, 200, [("ref", 0.1, 1), ("ref", 0.0, 10), ("seeded", 0.1, 1)],
                   "C3 x transform: k_precond_xt_ws_2d<4096> and closed-form pivots at T = 200"),
    "c3_fr_4096x256": (2, 2, 4096, 256, 32, [("ref", 0.1, 1), ("ref", 0.0, 10), ("seeded", 0.1, 1)],
                       "C3 x transform with the fused-residual dual and 8-row fast kernels (nx = 4096)"),
    "c3_rows_ny4096": (2, 2, 64, 4096, 32, [("ref", 0.1, 1), ("ref", 0.0, 10), ("seeded", 0.1, 1)],
                       "C3 row kernels: ny = 4096 fused residual / update with 512 threads"),
    "c2_x2048": (1, 2, 2048, 256, 100, [("ref", 0.0, 10), ("seeded", 0.0, 2)], "C2 x transform nx = 2048 at T = 100"),
    "c2_rows_ny2048": (1, 2, 256, 2048, 100, [("ref", 0.0, 10), ("seeded", 0.0, 2)],
                       "C2 row kernels ny = 2048 at T = 100"),
    "c4_halfreal_x8192": (2, 2, 8192, 256, 16, [("ref", 0.1, 1), ("ref", 0.0, 6), ("seeded", 0.1, 1)],
                          "C4 half-real x transform nx = 8192 (warp-specialised) at T = 16"),
    "c4_rows_ny8192": (2, 2, 64, 8192, 16, [("ref", 0.1, 1), ("ref", 0.0, 10), ("seeded", 0.1, 1)],
                       "C4 row kernels ny = 8192 (4 rows per group)"),
    "c1_exact": (1, 1, 65536, 1, 400, [("ref", 0.0, 10), ("seeded", 0.0, 2)],
                 "C1 exactly: egno 1, nx = 65536, T = 400 (four-step DHT)"),
}


def fixture_path(name):
    return os.path.join(HERE, "cfg_{}.npz".format(name))


def run_tag(kind, epsl, n):
    return "{}_e{}_n{}".format(kind, epsl, n)


def sample_idx(size, seed):
    rng = np.random.default_rng(seed)
    return np.unique(rng.integers(0, size, NSAMPLE * 11 // 10))[:NSAMPLE]


def live_alp(P, alp):
    """The live control component of each alp array (the 2-D arrays carry one zero component)."""
    if P["ndim"] == 1 or P["egno"] == 3:
        return [a[..., 0] for a in alp]
    return [a[..., 0 if i < 2 else 1] for i, a in enumerate(alp)]


def f32(a):
    return np.asarray(a, dtype=np.float32).astype(np.float64)


def initial_state(egno, ndim, nx, ny, T, kind, epsl):
    """The run's initial state as the device holds it (float32-rounded), in the reference layouts."""
    P = make_problem(egno, ndim, nx, ny, T, epsl, seeded=(kind == "seeded"))
    P["phi"], P["rho"], P["alp"] = f32(P["phi"]), f32(P["rho"]), tuple(f32(a) for a in P["alp"])
    return P


def iterate(P, phi, rho, alp, n, log=None):
    primal, dual = oracle_fns(P)
    phi1 = None
    t0 = time.time()
    for it in range(n):
        phi_n = primal(phi, rho, 70.0, alp, TAU, P["dt"], P["dsp"], P["fns"], P["fv"], P["epsl"], P["x_arr"], None)
        if it == 0:
            phi1 = phi_n
        rho_n, alp_n = dual(2 * phi_n - phi, rho, 70.0, alp, SIGMA, P["dt"], P["dsp"], P["epsl"], P["fns"],
                            P["x_arr"], None, P["ndim"], -1.0)
        e1, e2 = O.outer_errors(phi, phi_n, rho, rho_n, alp, alp_n)
        phi, rho, alp = phi_n, rho_n, alp_n
        if log:
            print("  {} it {} err1 {:.3e} err2 {:.3e} ({:.0f} s)".format(log, it + 1, e1, e2, time.time() - t0),
                  flush=True)
    return phi1, phi, rho, alp, (e1, e2)


def rel(a, b):
    nb = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / (nb if nb > 0 else 1.0))


def generate(name):
    """Oracle runs of one case; runs already present in an existing fixture file are kept."""
    egno, ndim, nx, ny, T, runs, _ = CASES[name]
    out = {"meta": np.array([egno, ndim, nx, ny, T]), "tau": TAU, "sigma": SIGMA}
    tags = [run_tag(*r) for r in runs]
    if os.path.exists(fixture_path(name)):
        with np.load(fixture_path(name)) as old:
            out.update({k: old[k] for k in old.files if k.split("__")[0] in tags})
    for (kind, epsl, n), tag in zip(runs, tags):
        if tag + "__err" in out:
            continue
        P = initial_state(egno, ndim, nx, ny, T, kind, epsl)
        ip = sample_idx(P["phi"].size, 1000 + len(tag))
        ir = sample_idx(P["rho"].size, 2000 + len(tag))
        phi1, phi, rho, alp, err = iterate(P, P["phi"], P["rho"], P["alp"], n, log="{} {}".format(name, tag))
        o = {"idx_phi": ip, "idx_rho": ir, "epsl": epsl, "iters": n, "seeded": int(kind == "seeded"),
             "phi1": phi1.reshape(-1)[ip], "U1": ((phi1 - P["phi"]) / TAU).reshape(-1)[ip],
             "phi1_norm": np.linalg.norm(phi1), "phi": phi.reshape(-1)[ip], "rho": rho.reshape(-1)[ir],
             "phi_norm": np.linalg.norm(phi), "rho_norm": np.linalg.norm(rho), "err": np.array(err)}
        for a, arr in enumerate(live_alp(P, alp)):
            o["alp{}".format(a)] = arr.reshape(-1)[ir]
            o["alp{}_norm".format(a)] = np.linalg.norm(arr)
        out.update({tag + "__" + k: v for k, v in o.items()})
        del P, phi1, phi, rho, alp
    for (kind, epsl, n), tag in zip(runs, tags):
        if tag + "__e32" not in out:
            out[tag + "__e32"] = float32_run(egno, ndim, nx, ny, T, kind, epsl, n, {k.split("__", 1)[1]: v for k, v in
                                                                                 out.items() if k.startswith(tag + "__")},
                                             log="{} {}".format(name, tag))
    out["runs"] = np.array(tags)
    return out


def float32_run(egno, ndim, nx, ny, T, kind, epsl, n, o, log=None):
    """The oracle executed in float32 from the run's initial state, compared with the stored float64 samples:
    [phi1, U1, phi, rho, alp0.., err1] relative L2 at the sampled points (err1: relative difference)."""
    P = initial_state(egno, ndim, nx, ny, T, kind, epsl)
    f = np.float32
    phi0 = P["phi"].astype(f)
    P["x_arr"] = P["x_arr"].astype(f)
    phi1, phi, rho, alp, err = iterate(P, phi0, P["rho"].astype(f), tuple(a.astype(f) for a in P["alp"]), n)
    assert phi.dtype == np.float32 and rho.dtype == np.float32
    ip, ir = o["idx_phi"], o["idx_rho"]
    U1 = (phi1.astype(np.float64) - phi0) / TAU
    e = [rel(phi1.reshape(-1)[ip], o["phi1"]), rel(U1.reshape(-1)[ip], o["U1"]), rel(phi.reshape(-1)[ip], o["phi"]),
         rel(rho.reshape(-1)[ir], o["rho"])]
    for a, arr in enumerate(live_alp(P, alp)):
        e.append(rel(arr.reshape(-1)[ir], o["alp{}".format(a)]))
    e1 = float(o["err"][0])
    e.append(abs(float(err[0]) - e1) / e1 if e1 > 0 else abs(float(err[0])))
    if log:
        print("  {} float32 oracle vs float64: {}".format(log, " ".join("{:.2e}".format(v) for v in e)), flush=True)
    return np.array(e)


if __name__ == "__main__":
    for name in (sys.argv[1:] or list(CASES)):
        t0 = time.time()
        np.savez_compressed(fixture_path(name), **generate(name))
        print("wrote", fixture_path(name), "in {:.0f} s".format(time.time() - t0), flush=True)
