"""t-slab decomposition of the H1 preconditioner's t-solve -- CPU restatement (TEST INFRASTRUCTURE).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; it is the
checker for the multi-GPU path, never part of it.

The reference solves (C - Dxx - Dyy - Dtt) u = r with a Thomas sweep over all T unknown rows of a mode
(utils_precond.py:10-35, :142-178).  Split the rows into P contiguous slabs [j0, j1).  Both recurrences
are affine in the carry that enters a slab and their coefficients do not depend on the data:

  forward   b_k = (r_k/ae + b_{k-1}) g_k       ->  b_k = b0_k + P_k c,     P_k = prod_{i=j0..k} g_i
  backward  x_k = b_k + g_k x_{k+1}            ->  x_{j0} = X0 + G y,      G = prod_{i=j0..j1-1} g_i

with b0 the slab's sweep from a zero carry, c = b_{j0-1} (the upstream slab's last b), y = x_{j1} (the
downstream slab's first x) and X0 = sum_k P'_k b_k (P'_k = prod_{i=j0..k-1} g_i).  So one iteration is:
local forward (b0, D = b0_{j1-1}) -> allgather D -> prefix scan c_q = D_q + G_q c_{q-1} -> fix-up
b = b0 + P c and X0 -> allgather X0 -> suffix scan y_q = X0_{q+1} + G_{q+1} y_{q+1} -> local backward
from y.  This module restates that sequence on numpy arrays and must reproduce the monolithic
tridiagonal_solve of pdhg_oracle.py for every P.
"""
import numpy as np

import pdhg_oracle as O


def slab_bounds(T, P):
    """Contiguous near-equal row ranges [(j0, j1)] of T rows over P slabs (the first T % P get one more)."""
    base, extra = divmod(T, P)
    out, j = [], 0
    for q in range(P):
        n = base + (1 if q < extra else 0)
        out.append((j, j + n))
        j += n
    return out


def pivots(diag, ae):
    """g_k = ae / u_k, u_k = d_k - ae g_{k-1} (the monolithic Thomas pivots, utils_precond.py:19-22)."""
    g = np.empty_like(diag)
    prev = np.zeros_like(diag[0])
    for k in range(diag.shape[0]):
        prev = ae / (diag[k] - ae * prev)
        g[k] = prev
    return g


def local_forward(r, g, ae, j0, j1):
    """Zero-carry forward sweep of one slab: b0 rows, the outgoing plane D and G = prod g."""
    b0 = np.empty_like(r[j0:j1])
    bp = np.zeros_like(r[0])
    G = np.ones_like(g[0])
    for k in range(j0, j1):
        bp = (r[k] / ae + bp) * g[k]
        b0[k - j0] = bp
        G = G * g[k]
    return b0, bp, G


def carry_in(D, G, q):
    """c_{q-1} of slab q: prefix scan c = D_p + G_p c over the upstream slabs p < q."""
    c = np.zeros_like(D[0])
    for p in range(q):
        c = D[p] + G[p] * c
    return c


def fixup(b0, g, j0, c):
    """b = b0 + P c and X0 = sum_k P'_k b_k (the slab's zero-right-carry backward result at j0)."""
    b = np.empty_like(b0)
    Pk = np.ones_like(g[0])
    x0 = np.zeros_like(b0[0])
    for i in range(b0.shape[0]):
        x0 = x0 + Pk * (b0[i] + Pk * g[j0 + i] * c)   # P'_k = Pk before the update
        Pk = Pk * g[j0 + i]
        b[i] = b0[i] + Pk * c
    return b, x0


def right_carry(X0, G, q):
    """y_q = x_{j1} of slab q: suffix scan y = X0_p + G_p y over the downstream slabs p > q."""
    y = np.zeros_like(X0[0])
    for p in range(len(X0) - 1, q, -1):
        y = X0[p] + G[p] * y
    return y


def local_backward(b, g, j0, y):
    x = np.empty_like(b)
    xc = y
    for i in range(b.shape[0] - 1, -1, -1):
        xc = b[i] + g[j0 + i] * xc
        x[i] = xc
    return x


def thomas_slabs(diag, r, ae, P):
    """Solve -ae x_{k-1} + d_k x_k - ae x_{k+1} = r_k (x_{-1} = x_T = 0) over P slabs."""
    T = diag.shape[0]
    bounds = slab_bounds(T, P)
    g = pivots(diag, ae)
    fw = [local_forward(r, g, ae, j0, j1) for (j0, j1) in bounds]
    D = [f[1] for f in fw]
    G = [f[2] for f in fw]
    fx = [fixup(fw[q][0], g, bounds[q][0], carry_in(D, G, q)) for q in range(P)]
    X0 = [f[1] for f in fx]
    x = [local_backward(fx[q][0], g, bounds[q][0], right_carry(X0, G, q)) for q in range(P)]
    return np.concatenate(x, axis=0)


def h1_precond_2d_slabs(source_term, fv, dt, C, P):
    """H1_precond_2d (bc (0, 0)) with the t-solve split over P slabs (utils_precond.py:142-178)."""
    nt, nx, ny = source_term.shape
    v = np.fft.fft2(source_term[1:], axes=(1, 2))
    T = nt - 1
    ae = 1.0 / (dt * dt)
    diag = np.broadcast_to(-fv, (T, nx, ny)) + C + 2 * ae
    diag = np.array(diag)
    diag[-1] -= ae                                   # Neumann last row (utils_precond.py:130)
    part = thomas_slabs(diag, v, ae, P)
    upd = np.fft.ifft2(part, axes=(1, 2)).real
    return np.concatenate([np.zeros((1, nx, ny)), upd], axis=0)


def monolithic_tridiag(diag, r, ae):
    """The reference-form solve of the same system (pdhg_oracle.tridiagonal_solve)."""
    T = diag.shape[0]
    dl = np.full(T, -ae)
    dl[0] = 0.0
    du = np.full(T, -ae)
    du[-1] = 0.0
    return O.tridiagonal_solve(dl, diag, du, r)


# ---- single-exchange variant: X0_q is affine in the slab's incoming carry -------------------------
#   X0_q = S1_q + c_{q-1} S2_q,   S1 = sum_k P'_k b0_k (data),  S2 = sum_k P'_k P_k (iteration-invariant)
# so ONE allgather of (D, S1) per iteration lets every slab fold both scans locally.

def s_sums(b0, g, j0):
    """S1 = sum P'_k b0_k and S2 = sum P'_k P_k over the slab's rows (P'_k = prod g_{j0..k-1})."""
    Pk = np.ones_like(g[0])
    s1 = np.zeros_like(b0[0])
    s2 = np.zeros_like(g[0])
    for i in range(b0.shape[0]):
        s1 = s1 + Pk * b0[i]
        s2 = s2 + Pk * Pk * g[j0 + i]
        Pk = Pk * g[j0 + i]
    return s1, s2


def carries_single(D, S1, G, S2, q):
    """(c_{q-1}, y_q) of slab q from everybody's (D, S1, G, S2)."""
    P = len(D)
    cin = [np.zeros_like(D[0])]
    for p in range(P - 1):
        cin.append(D[p] + G[p] * cin[p])          # cin[p] = carry INTO slab p
    y = np.zeros_like(D[0])
    for p in range(P - 1, q, -1):
        y = (S1[p] + cin[p] * S2[p]) + G[p] * y   # X0_p + G_p y
    return cin[q], y


def thomas_slabs_single(diag, r, ae, P):
    T = diag.shape[0]
    bounds = slab_bounds(T, P)
    g = pivots(diag, ae)
    fw = [local_forward(r, g, ae, j0, j1) for (j0, j1) in bounds]
    ss = [s_sums(fw[q][0], g, bounds[q][0]) for q in range(P)]
    D, G = [f[1] for f in fw], [f[2] for f in fw]
    S1, S2 = [s[0] for s in ss], [s[1] for s in ss]
    out = []
    for q, (j0, j1) in enumerate(bounds):
        c, y = carries_single(D, S1, G, S2, q)
        b, _ = fixup(fw[q][0], g, j0, c)
        out.append(local_backward(b, g, j0, y))
    return np.concatenate(out, axis=0)


# ---- neighbour-exchange variant: only the long-range modes need every slab's planes ---------------
#   G_q = prod g over slab q depends only on the mode; where G_q < delta for every slab the far terms
#   G_{q-1} c_in(q-1) and G_{q+1} y_{q+1} are below delta relative, so
#     c_in(q) = D_{q-1},   y_q = S1_{q+1} + (D_q + G_q c_in(q)) S2_{q+1}
#   (kernels_common.hpp k_slab_fix_nb); the other ("long-range") modes fold exactly.

def long_range_mask(G, delta):
    """Modes where some slab's gain reaches delta (they take the exact all-slab folds)."""
    return ~(np.max(np.abs(np.stack(G)), axis=0) < delta)


def carries_neighbour(D, S1, G, S2, q, long_mask):
    P = len(D)
    c = D[q - 1] if q > 0 else np.zeros_like(D[0])
    if q + 1 < P:
        y = S1[q + 1] + (D[q] + G[q] * c) * S2[q + 1]
    else:
        y = np.zeros_like(D[0])
    ce, ye = carries_single(D, S1, G, S2, q)
    return np.where(long_mask, ce, c), np.where(long_mask, ye, y)


def thomas_slabs_neighbour(diag, r, ae, P, delta=2.0 ** -40):
    T = diag.shape[0]
    bounds = slab_bounds(T, P)
    g = pivots(diag, ae)
    fw = [local_forward(r, g, ae, j0, j1) for (j0, j1) in bounds]
    ss = [s_sums(fw[q][0], g, bounds[q][0]) for q in range(P)]
    D, G = [f[1] for f in fw], [f[2] for f in fw]
    S1, S2 = [s[0] for s in ss], [s[1] for s in ss]
    mask = long_range_mask(G, delta)
    out = []
    for q, (j0, j1) in enumerate(bounds):
        c, y = carries_neighbour(D, S1, G, S2, q, mask)
        b, _ = fixup(fw[q][0], g, j0, c)
        out.append(local_backward(b, g, j0, y))
    return np.concatenate(out, axis=0), mask
