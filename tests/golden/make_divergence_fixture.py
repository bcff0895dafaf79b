"""Fixture pinning the reference algorithm's divergence on C3's FULL spatial plane (BASELINE.json configs[3]:
egno 2, ndim 2, epsl 0.1, nx = ny = 4096, dt = 1/200 as nt = 201).

The bench times C3 as one window of T = 200 rows and reports the first iteration at which phi' or rho'
turns non-finite (11 on the device).  That is the reference's own instability: its dual step holds the
explicit sigma*epsl*Lap(phi_bar) term (update_fns_in_pdhg.py:58-70), whose amplification sigma*epsl*8/dx^2
~ 5e5 per iteration at dx = 2/4096 no step size in the reference's back-off range cures.  This script runs
the float64 oracle on the 4096^2 plane with a short window (T = 4 rows, the same dt) from the reference
initial state (phi = g, rho = 70, alp = 0; utils_pdhg_solver.py:123-137), one rho_alp_iter, until phi' or
rho' holds a NaN -- the reference's own test, jnp.isnan (utils_pdhg_solver.py:78-80), which an inf does not
trip -- and stores per iteration: |phi'|, |rho'|, |alp'| (Frobenius over the finite entries), err1, err2,
whether every entry of phi' and rho' is finite, and the first NaN iteration ("first_nonfinite", the name the
bench uses for the same event).  tests/test_gpu_divergence.py runs the device (fp32 and fp64) on
the same window and compares.

The growth is geometric (|rho| x ~3000 per iteration after a few iterations): float32 overflows near iteration
13 while float64 takes ~90 iterations to reach a NaN -- too long for the CPU oracle (2.5 min per iteration here).
So the fixture keeps the first max_iters iterations (|.|_F and max |.| per iteration; first_nonfinite = 0 when no
NaN occurred within them), which pin (a) the device's norm sequence in fp64 and in fp32 while finite, and (b) the
iteration at which the values outgrow float32 (max |rho'| or |phi'| > 3.4e38), where the fp32 device's first
non-finite iteration must fall.

The float32 run (argument f32: inputs rounded to float32, the oracle's arithmetic in float32 as in
make_config_fixtures.py's e32 pass) pins the fp32 device: there fp32 rounding (1e-7 relative) seeds the unstable
modes, which then grow ~3000-fold per iteration, so the float32 trajectory leaves the float64 one after ~2
iterations and reaches a NaN long before float64 does.

Run:  python tests/golden/make_divergence_fixture.py [T] [max_iters] [f32]   (~2.5 min per iteration at T = 4, 6 cores)

Perturbed pointwise variant (argument "points_ulp"): the same run from phi_0 multiplied by (1 + u), u = +-2^-52 with
random signs (np.random.default_rng(7)), at the same sample points -> divergence_c3_plane_T4_points_ulp.npz.  Its
distance to the "points" fixture is how far two float64 runs of the reference algorithm that differ by one rounding
drift apart through the instability: the spread any float64 implementation has against the oracle pointwise.

Other-FFT-library variant (argument "points_npfft", round 5): the same float64 run with every FFT of the oracle
through numpy.fft instead of scipy.fft (a different pocketfft build: the two differ by ~4e-16 relative on one
transform) -> divergence_c3_plane_T4_points_npfft.npz.  It is the like-for-like spread of the reference algorithm
on another FFT library -- what the reference itself (XLA's FFT) could differ from the oracle by -- without the
one-ulp perturbation of every input entry that "points_ulp" applies.

Device-t-solve variant (argument "points_devthomas", round 5): the same float64 run with the oracle's Thomas solve
(utils_precond.py:10-40, complex Thomas scan) replaced by the device's algebra for the same tridiagonal systems
(kernels_xt_f64.hpp: cancellation-free pivot recurrence s = dd + h, g = 1/(1+s), h = s g forward, closed-form pivots
g_k = e^-th E_{k+1}/E_{k+2} backward) -> divergence_c3_plane_T4_points_devthomas.npz: the spread of the reference
algorithm under another, equally exact float64 formulation of one of its steps.

Pointwise variant (argument "points"): the float64 oracle's phi' and rho' at NPTS fixed sample points of the plane
(rows 1..T of phi', every row of rho'; indices from np.random.default_rng(20250117)) after each of the first
max_iters iterations -> divergence_c3_plane_T{T}_points.npz.  tests/test_gpu_divergence.py compares the fp64
device's values at the same points pointwise (relative L2 over the sample, per iteration), so the check covers
the state itself, not only its norms.
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import pdhg_oracle as O  # noqa: E402

TAU, SIGMA = 0.1 / 1.5, 0.1 * 1.5


def setup(nx, ny, T, dt, epsl, dtype=np.float64):
    egno, ndim = 2, 2
    x_arr = O.make_grid(ndim, nx, ny, egno)
    g = O.set_up_J(egno, ndim, (2.0, 2.0))(x_arr)
    fns = O.set_up_example_fns(egno, ndim, 0)
    dsp = (2.0 / nx, 2.0 / ny)
    bc = O.default_bc(egno, ndim)
    fv = O.compute_Dxx_fft_fv(ndim, (nx, ny), dsp, bc)
    primal, dual = O.make_update_fns(ndim, bc, rho_alp_iters=1)
    if dtype == np.float32:   # the oracle in float32 (as make_config_fixtures.py's e32 pass): inputs rounded
        x_arr = x_arr.astype(dtype)
    phi = np.repeat(g, T + 1, axis=0).astype(dtype)
    rho = np.full((T, nx, ny), 70.0, dtype=dtype)
    alp = tuple(np.zeros((T, nx, ny, 2), dtype=dtype) for _ in range(4))
    return dict(x_arr=x_arr, g=g, fns=fns, dsp=dsp, fv=fv, primal=primal, dual=dual, phi=phi, rho=rho, alp=alp,
                dt=dt, epsl=epsl)


NPTS = 4096


def sample_points(T, nx, ny, n=NPTS):
    """Fixed sample of the plane: (t, x, y) for phi rows 1..T and for rho rows 0..T-1."""
    rng = np.random.default_rng(20250117)
    pt = rng.integers(1, T + 1, n), rng.integers(0, nx, n), rng.integers(0, ny, n)
    rt = rng.integers(0, T, n), rng.integers(0, nx, n), rng.integers(0, ny, n)
    return np.stack(pt), np.stack(rt)


def run(S, max_iters, log=True):
    phi, rho, alp = S["phi"], S["rho"], S["alp"]
    pts = S.get("points")
    rows = []
    first = 0
    t0 = time.time()
    for it in range(1, max_iters + 1):
        phi_n = S["primal"](phi, rho, 70.0, alp, TAU, S["dt"], S["dsp"], S["fns"], S["fv"], S["epsl"], S["x_arr"],
                            None)
        with np.errstate(all="ignore"):
            rho_n, alp_n = S["dual"](2 * phi_n - phi, rho, 70.0, alp, SIGMA, S["dt"], S["dsp"], S["epsl"], S["fns"],
                                     S["x_arr"], None, 2, -1.0)
            e1, e2 = O.outer_errors(phi, phi_n, rho, rho_n, alp, alp_n)
            fin = bool(np.isfinite(phi_n).all() and np.isfinite(rho_n).all())
            nan = bool(np.isnan(phi_n).any() or np.isnan(rho_n).any())
            d = np.float64   # norms of float32 states in float64 (they outgrow float32 before the entries do)
            nphi = float(np.linalg.norm(phi_n[np.isfinite(phi_n)].astype(d)))
            nrho = float(np.linalg.norm(rho_n[np.isfinite(rho_n)].astype(d)))
            nalp = float(np.sqrt(sum(np.sum(np.where(np.isfinite(a), a, 0.0).astype(d) ** 2) for a in alp_n)))
            mphi = float(np.nanmax(np.abs(phi_n)))
            mrho = float(np.nanmax(np.abs(rho_n)))
        rows.append([it, nphi, nrho, nalp, e1, e2, 1.0 if fin else 0.0, mphi, mrho])
        if pts is not None:
            S["phi_pts"].append(phi_n[tuple(pts[0])].astype(np.float64))
            S["rho_pts"].append(rho_n[tuple(pts[1])].astype(np.float64))
        if S.get("out"):
            save(S["out"], np.array(rows), 0, S)
        if log:
            print("it {:3d} |phi| {:.6e} |rho| {:.6e} |alp| {:.6e} err1 {:.3e} err2 {:.3e} finite {} nan {} ({:.0f} s)"
                  .format(it, nphi, nrho, nalp, e1, e2, fin, nan, time.time() - t0), flush=True)
        phi, rho, alp = phi_n, rho_n, alp_n
        if nan:
            first = it
            break
    return np.array(rows), first


def save(out, rows, first, S):
    T = S["phi"].shape[0] - 1
    nx, ny = S["phi"].shape[1:]
    if S.get("points") is not None:
        np.savez_compressed(out, rows=rows, meta=np.array([2, 2, nx, ny, T]), dt=S["dt"], epsl=S["epsl"], tau=TAU,
                            sigma=SIGMA, phi_idx=S["points"][0], rho_idx=S["points"][1],
                            phi_pts=np.array(S["phi_pts"]), rho_pts=np.array(S["rho_pts"]))
        return
    np.savez_compressed(out, rows=rows, first_nonfinite=first, meta=np.array([2, 2, nx, ny, T]), dt=S["dt"],
                        epsl=S["epsl"], tau=TAU, sigma=SIGMA,
                        columns=np.array(["iter", "phi_norm", "rho_norm", "alp_norm", "err1", "err2", "finite",
                                          "phi_absmax", "rho_absmax"]))


if __name__ == "__main__":
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    max_iters = int(sys.argv[2]) if len(sys.argv) > 2 else 24
    f32 = len(sys.argv) > 3 and sys.argv[3] == "f32"   # the float32 oracle (until its first NaN)
    points = len(sys.argv) > 3 and sys.argv[3] in ("points", "points_ulp", "points_npfft", "points_devthomas")
    devth = len(sys.argv) > 3 and sys.argv[3] == "points_devthomas"
    if devth:
        def dev_thomas(dl, d, du, b):
            """M x = b with M = ae tridiag(-1, dd + 2, -1), last diagonal dd + 1 (H1_precond_2d's systems), in the
            device's algebra (kernels_xt_f64.hpp)."""
            ae = -float(np.real(dl[1]))
            dd = (np.real(d[0]) - 2.0 * ae) / ae
            T = b.shape[0]
            h = np.ones_like(dd)
            bp = np.zeros_like(b[0])
            bps = []
            for k in range(T - 1):
                s_ = dd + h
                g_ = 1.0 / (1.0 + s_)
                h = s_ * g_
                bp = (b[k] / ae + bp) * g_
                bps.append(bp)
            x = (b[T - 1] / ae + bp) / (dd + h)
            out = [None] * T
            out[T - 1] = x
            dl_ = 0.5 * dd
            th = np.maximum(np.log1p(dl_ + np.sqrt(dl_ * (dl_ + 2.0))), 1e-300)
            for k in range(T - 2, -1, -1):
                g_ = np.exp(-th) * np.expm1(-2.0 * th * (k + 1)) / np.expm1(-2.0 * th * (k + 2))
                x = bps[k] + g_ * x
                out[k] = x
            return np.stack(out)
        O.tridiagonal_solve = dev_thomas
    ulp = len(sys.argv) > 3 and sys.argv[3] == "points_ulp"
    npfft = len(sys.argv) > 3 and sys.argv[3] == "points_npfft"
    if npfft:   # the oracle's FFTs through numpy.fft (periodic bc: fft2 / ifft2 only)
        import types
        sf = O.sfft
        O.sfft = types.SimpleNamespace(
            fft2=lambda a, axes=(-2, -1), workers=None: np.fft.fft2(a, axes=axes),
            ifft2=lambda a, axes=(-2, -1), workers=None: np.fft.ifft2(a, axes=axes),
            fft=lambda a, axis=-1, workers=None: np.fft.fft(a, axis=axis),
            ifft=lambda a, axis=-1, workers=None: np.fft.ifft(a, axis=axis),
            dct=sf.dct, idct=sf.idct)
    nx = ny = 4096
    S = setup(nx, ny, T, 1.0 / 200, 0.1, np.float32 if f32 else np.float64)
    out = os.path.join(HERE, "divergence_c3_plane_T{}{}.npz".format(
        T, "_f32" if f32 else "_points_ulp" if ulp else "_points_npfft" if npfft else "_points_devthomas" if devth
        else "_points" if points else ""))
    if points:
        S.update(points=sample_points(T, nx, ny), phi_pts=[], rho_pts=[])
    if ulp:
        sgn = np.where(np.random.default_rng(7).random(S["phi"].shape) < 0.5, -1.0, 1.0)
        S["phi"] = S["phi"] * (1.0 + sgn * 2.0 ** -52)
    S["out"] = out            # rewritten after every iteration (a partial run is usable)
    rows, first = run(S, max_iters)
    save(out, rows, first, S)
    print("wrote", out, "first NaN iteration", first or "(none within {})".format(max_iters), flush=True)
