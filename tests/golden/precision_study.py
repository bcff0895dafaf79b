"""Where does the float32 reference algorithm lose phi accuracy at the bench configs?  (study, CPU)

Runs the float64 oracle and variants of it in which chosen quantities are held in float32, from the
same float32-rounded initial state as tests/golden/make_config_fixtures.py, and prints the relative L2
distance of phi / rho / alp from the float64 run after n iterations.  Variants:
  f32        everything float32 (the fixtures' e32)
  phi64      phi, phi_bar and their finite differences in float64; rho, alp, residual, preconditioner float32
  phi64rho64 as phi64 with rho also float64
  off32      phi held as g + delta with delta float32; differences of g in float64 rounded to float32 once
  pre64      everything float32 except the H1 preconditioner (FFT + Thomas) in float64
  fft64      float32 except the preconditioner's FFTs (Thomas float32, spectrum rounded to complex64 between)
  th64       float32 except the preconditioner's Thomas solve (FFTs float32)
  dth32      float32 with the device's Thomas algebra (cancellation-free pivot recurrence forward, closed-form
             pivots backward; kernels_xt_dma.hpp) instead of the reference's
  dth64      as dth32 with the recurrences in float64 and b' stored as float32 between the sweeps
usage: python tests/golden/precision_study.py <case> <variant> [...]   (cases as make_config_fixtures.CASES)
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, HERE)
import pdhg_oracle as O  # noqa: E402
from make_config_fixtures import CASES, initial_state, live_alp, TAU, SIGMA  # noqa: E402
from _problems import oracle_fns  # noqa: E402

F32, F64 = np.float32, np.float64
_DEC = ["Dx_right_decreasedim", "Dx_left_decreasedim", "Dy_right_decreasedim", "Dy_left_decreasedim",
        "Dxx_decreasedim", "Dyy_decreasedim"]
_ORIG = {n: getattr(O, n) for n in _DEC + ["Dt_decreasedim", "H1_precond_1d", "H1_precond_2d"]}
STATE = {}


def _patch(variant):
    for n, f in _ORIG.items():
        setattr(O, n, f)
    if variant in ("phi64", "phi64rho64"):
        for n in _DEC + ["Dt_decreasedim"]:
            f = _ORIG[n]
            setattr(O, n, (lambda f: lambda phi, *a: f(phi, *a).astype(F32) if variant == "phi64" else f(phi, *a))(f))
    if variant == "off32":
        G = STATE["G"]

        def mk(f):
            def g(phi, *a):
                return f(G, *a).astype(F32) + f(phi, *a)   # phi passed = delta_bar (float32)
            return g
        for n in _DEC:
            setattr(O, n, mk(_ORIG[n]))
    if variant in ("fft64", "th64"):
        fdt = np.complex128 if variant == "fft64" else np.complex64
        tdt = np.complex128 if variant == "th64" else np.complex64

        def pre2(src, fv, dt, bc, C=1.0):
            nt, nx, ny = src.shape
            v = O.sfft.fft2(src[1:].astype(fdt), axes=(1, 2), workers=O._WORKERS).astype(tdt)
            dl, du, diag = O._lap_t(nt - 1, dt, tdt)
            tb = np.broadcast_to(-np.asarray(fv).astype(tdt), (nt - 1, nx, ny)) + diag[:, None, None] + C
            part = O.tridiagonal_solve(dl, tb, du, v).astype(fdt)
            upd = O.sfft.ifft2(part, axes=(1, 2), workers=O._WORKERS).real.astype(F32)
            return np.concatenate([np.zeros((1, nx, ny), dtype=F32), upd], axis=0)

        def pre1(src, fv, dt, bc, C=1.0, pow=1, Ct=1):
            nt, nx = src.shape
            v = O.sfft.fft(src[1:].astype(fdt), axis=1, workers=O._WORKERS).astype(tdt)
            tb = (np.broadcast_to(-np.asarray(fv).astype(tdt), (nt - 1, nx)) + C) ** pow
            dl, du, diag = O._lap_t(nt - 1, dt, tdt)
            part = O.tridiagonal_solve(dl * Ct, tb + diag[:, None] * Ct, du * Ct, v).astype(fdt)
            upd = O.sfft.ifft(part, axis=1, workers=O._WORKERS).real.astype(F32)
            return np.concatenate([np.zeros((1, nx), dtype=F32), upd], axis=0)
        O.H1_precond_2d, O.H1_precond_1d = pre2, pre1
    if variant in ("dth32", "dth64"):
        adt = np.float64 if variant == "dth64" else F32

        def dev_thomas(v, lam, dt, C):
            """v: [T, modes] complex64 spectrum rows 1..T; lam: [modes] symbol; returns x (complex64)."""
            T = v.shape[0]
            ae = 1.0 / (dt * dt)
            dd = ((C - lam.astype(F32)).astype(F32) * F32(1.0 / ae)).astype(adt)
            inv_ae = adt(1.0 / ae)
            h = np.ones_like(dd)
            b = np.zeros(v.shape[1:], dtype=np.complex128 if adt == np.float64 else np.complex64)
            bp = np.empty(v.shape, dtype=np.complex64)
            for k in range(T):
                rhs = v[k].astype(b.dtype) * inv_ae
                if k < T - 1:
                    s_ = dd + h
                    g_ = adt(1) / (adt(1) + s_)
                    b = (rhs + b) * g_
                    h = s_ * g_
                else:
                    b = (rhs + b) / (dd + h)
                bp[k] = b.astype(np.complex64)    # stored between the sweeps
            dl = adt(0.5) * dd
            th = np.maximum(np.log1p(dl + np.sqrt(dl * (dl + adt(2)))), adt(1e-20))
            E2 = np.expm1(adt(-2) * th * adt(T))
            x = bp[T - 1].astype(b.dtype)
            out = np.empty(v.shape, dtype=np.complex64)
            out[T - 1] = x.astype(np.complex64)
            for k in range(T - 2, -1, -1):
                E1 = np.expm1(adt(-2) * th * adt(k + 1))
                g_ = np.exp(-th) * E1 / E2
                x = bp[k].astype(b.dtype) + g_ * x
                E2 = E1
                out[k] = x.astype(np.complex64)
            return out

        def pre2(src, fv, dt, bc, C=1.0):
            nt, nx, ny = src.shape
            v = O.sfft.fft2(src[1:].astype(np.complex64), axes=(1, 2), workers=O._WORKERS)
            x = dev_thomas(v.reshape(nt - 1, -1), np.real(fv).reshape(-1), dt, C).reshape(v.shape)
            upd = O.sfft.ifft2(x, axes=(1, 2), workers=O._WORKERS).real.astype(F32)
            return np.concatenate([np.zeros((1, nx, ny), dtype=F32), upd], axis=0)
        O.H1_precond_2d = pre2
    if variant == "pre64":
        for n in ("H1_precond_1d", "H1_precond_2d"):
            f = _ORIG[n]
            setattr(O, n, (lambda f: lambda src, *a, **k: f(src.astype(F64), *a, **k).astype(F32))(f))


def run(name, variant, n_override=None, kind="ref", epsl=None):
    egno, ndim, nx, ny, T, runs, _ = CASES[name]
    kind_, epsl_, n = [r for r in runs if r[0] == kind and (epsl is None or r[1] == epsl)][0]
    n = n_override or n
    P = initial_state(egno, ndim, nx, ny, T, kind_, epsl_)
    primal, dual = oracle_fns(P)
    g = np.broadcast_to(P["g"], P["phi"].shape).astype(F64)
    STATE["G"] = g
    _patch(variant)
    if variant == "f64":
        phi, rho, alp = P["phi"], P["rho"], P["alp"]
        x_arr = P["x_arr"]
    else:
        lo = F64 if variant == "phi64rho64" else F32
        rho = P["rho"].astype(lo)
        alp = tuple(a.astype(F32) for a in P["alp"])
        x_arr = P["x_arr"].astype(F32)
        if variant in ("phi64", "phi64rho64"):
            phi = P["phi"].astype(F64)
        elif variant == "off32":
            phi = (P["phi"] - g).astype(F32)
        else:
            phi = P["phi"].astype(F32)
    t0 = time.time()
    for it in range(n):
        phi_n = primal(phi, rho, 70.0, alp, TAU, P["dt"], P["dsp"], P["fns"], P["fv"], epsl_, x_arr, None)
        if variant in ("phi64", "phi64rho64"):
            phi_n = phi_n.astype(F64)
        elif phi_n.dtype != phi.dtype:
            phi_n = phi_n.astype(phi.dtype)
        rho, alp = dual(2 * phi_n - phi, rho, 70.0, alp, SIGMA, P["dt"], P["dsp"], epsl_, P["fns"], x_arr, None,
                        ndim, -1.0)
        if variant == "phi64":
            rho, alp = rho.astype(F32), tuple(a.astype(F32) for a in alp)
        phi = phi_n
    _patch("f64")
    if variant == "off32":
        phi = g + phi.astype(F64)
    return phi.astype(F64), rho.astype(F64), [a.astype(F64) for a in live_alp(P, alp)], time.time() - t0


def rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


if __name__ == "__main__":
    name = sys.argv[1]
    kind = os.environ.get("KIND", "ref")
    epsl = float(os.environ["EPSL"]) if "EPSL" in os.environ else None
    n = int(os.environ["N"]) if "N" in os.environ else None
    ref = run(name, "f64", n, kind, epsl)
    print("{} {} f64 done in {:.0f} s".format(name, kind, ref[3]), flush=True)
    for v in sys.argv[2:]:
        r = run(name, v, n, kind, epsl)
        print("{:>11s}: phi {:.2e} rho {:.2e} alp {} ({:.0f} s)".format(
            v, rel(r[0], ref[0]), rel(r[1], ref[1]),
            " ".join("{:.1e}".format(rel(a, b)) for a, b in zip(r[2], ref[2]) if np.linalg.norm(b) > 0), r[3]),
            flush=True)
