"""t-slab decomposition (multi-GPU design) -- CPU checks.

The partitioned Thomas sweep (oracle/slab_oracle.py) must reproduce the monolithic reference-form
solve for every slab count, including uneven slabs and one-row slabs."""
import numpy as np
import pytest

import pdhg_oracle as O
import slab_oracle as S

rng = np.random.default_rng(7)


@pytest.mark.parametrize("T,P", [(1, 1), (5, 1), (5, 2), (7, 3), (8, 8), (13, 4), (40, 8)])
def test_thomas_slabs_equals_monolithic(T, P):
    M = 17
    ae = 1.0 / (0.05 ** 2)
    lam = -rng.uniform(0, 5e3, M)
    diag = np.tile(1.0 - lam + 2 * ae, (T, 1))
    diag[-1] -= ae
    r = rng.standard_normal((T, M)) + 1j * rng.standard_normal((T, M))
    ref = S.monolithic_tridiag(diag.astype(complex), r, ae)
    out = S.thomas_slabs(diag, r, ae, P)
    assert np.allclose(out, ref, rtol=1e-11, atol=1e-12 * np.abs(ref).max())


@pytest.mark.parametrize("T,P", [(5, 2), (7, 3), (8, 8), (40, 8)])
def test_single_exchange_variant_equals_monolithic(T, P):
    M = 11
    ae = 1.0 / (0.05 ** 2)
    diag = np.tile(1.0 + rng.uniform(0, 5e3, M) + 2 * ae, (T, 1))
    diag[-1] -= ae
    r = rng.standard_normal((T, M))
    ref = S.monolithic_tridiag(diag, r, ae)
    assert np.allclose(S.thomas_slabs_single(diag, r, ae, P), ref, rtol=1e-11, atol=1e-12 * np.abs(ref).max())


@pytest.mark.parametrize("T,P", [(12, 3), (40, 8), (200, 8)])
def test_neighbour_exchange_variant_equals_monolithic(T, P):
    """Short-range modes (every slab gain < 2^-40) use only the adjacent slabs' planes; the error stays
    at the level of the exact variants.  The symbol spans low (long-range) and high frequencies."""
    M = 64
    dt = 1.0 / T
    ae = 1.0 / dt ** 2
    lam = -4.0 * np.sin(np.pi * np.arange(M) / (2 * M)) ** 2 * (M / 0.05) ** 2
    diag = np.tile(1.0 - lam + 2 * ae, (T, 1))
    diag[-1] -= ae
    r = rng.standard_normal((T, M))
    ref = S.monolithic_tridiag(diag, r, ae)
    out, mask = S.thomas_slabs_neighbour(diag, r, ae, P)
    assert 0 < mask.sum() < M          # both classes present
    assert np.allclose(out, ref, rtol=1e-10, atol=1e-11 * np.abs(ref).max())


def test_slab_bounds_cover_rows():
    for T in (1, 7, 200):
        for P in (1, 2, 3, 8):
            if P > T:
                continue
            b = S.slab_bounds(T, P)
            assert b[0][0] == 0 and b[-1][1] == T
            assert all(b[q][1] == b[q + 1][0] and b[q][1] > b[q][0] for q in range(P - 1))


@pytest.mark.parametrize("P", [2, 3, 5])
def test_h1_precond_2d_slabs_equals_oracle(P):
    nt, nx, ny = 11, 8, 6
    dx, dy, dt = 2 / nx, 2 / ny, 0.02
    fv = O.compute_Dxx_fft_fv(2, (nx, ny), (dx, dy), (0, 0))
    src = rng.standard_normal((nt, nx, ny))
    ref = O.H1_precond_2d(src, fv, dt, (0, 0), C=1.0)
    out = S.h1_precond_2d_slabs(src, fv, dt, 1.0, P)
    assert np.allclose(out, ref, rtol=1e-10, atol=1e-12)


def test_split_join_state_roundtrip():
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "pdhg-optimal-control_amd"))
    from pdhg_amd.slab import join_state, slab_bounds, split_state
    T = 7
    phi = rng.standard_normal((T + 1, 4, 3))
    rho = rng.standard_normal((T, 4, 3))
    alp = tuple(rng.standard_normal((T, 4, 3, 2)) for _ in range(4))
    for P in (1, 2, 3, 7):
        parts = split_state(phi, rho, alp, slab_bounds(T, P))
        assert [p[1].shape[0] for p in parts] == [j1 - j0 for j0, j1 in slab_bounds(T, P)]
        phi2, rho2, alp2 = join_state(parts)
        assert np.array_equal(phi2, phi) and np.array_equal(rho2, rho)
        assert all(np.array_equal(a, b) for a, b in zip(alp2, alp))
