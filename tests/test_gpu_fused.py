"""Fused residual path (k_dual_lds_2d FR + k_res_fwdy_fused_2d) vs the float64 oracle and vs the unfused
kernels (pytest -m gpu).

With rho_alp_iters = 1 the fp32 dual sweep also forms the next primal's continuity residual
(update_fns_in_pdhg.py:72-96) from the rho', alp' it has just written; the residual kernel only completes
the terms at its 8-row x 256-column tile edges.  PDHG_FUSE_RES=1 forces the path on grids smaller than the
default threshold, =0 turns it off.  Bounds: the fp32 bounds of test_gpu_parity (phi 1e-5, rho 2e-4 after
10 iterations from the seeded state); fused vs unfused device runs agree to fp32 reassociation (1e-5).

fp64 (ny = 2048 / 4096: the sweep k_dual_lds_2d<.., double, 2> on 128-column strips, the residual in 4-row
half-tile tasks of k_res_fwdy_fused_2d<.., 4, 512, double>; ny = 8192, C4's: 2-row quarter-tile tasks,
k_res_fwdy_fused_2d<.., 8192, 2, 512, double>): against the float64 oracle at 1e-9 (phi, rho; the fp64 bar of
test_gpu_configs) and against the unfused fp64 kernels at 1e-12; at C4's full 8192^2 plane (the half-real
spectrum, one column per block: 16-B chunk stores) against the unfused kernels.
"""
import numpy as np
import pytest

from _problems import device_ctx, make_problem, rel
from test_gpu_parity import SIGMA, TAU, _oracle_iterate

pytestmark = pytest.mark.gpu

FUSED = [
    # egno, ndim, nx, ny, T, epsl
    (1, 2, 256, 256, 3, 0.0),
    (2, 2, 256, 512, 5, 1e-5),   # 2 strips along y: strip-edge columns through p.ey
    (1, 2, 512, 1024, 4, 1e-5),  # 4 strips, 64 row groups
    (2, 2, 64, 256, 1, 0.0),     # T = 1: the residual row is formed after the loop only
    (2, 2, 128, 1024, 2, 1e-4),
]
IDS = ["e{}d{}_{}x{}_T{}_eps{}".format(*c) for c in FUSED]
# epsl = 0.1 at these dx is the reference's unstable regime (explicit sigma*epsl*Lap in the dual, see
# test_fp32_from_reference_init): fp32 rounding is amplified every iteration, so there the fused path is
# held to the unfused path's own distance from the oracle
UNSTABLE = [(2, 2, 256, 512, 3, 0.1), (1, 2, 256, 256, 2, 0.1)]
UNSTABLE_IDS = ["e{}d{}_{}x{}_T{}_eps{}".format(*c) for c in UNSTABLE]


FUSED64 = [
    (2, 2, 32, 2048, 4, 1e-5),
    (1, 2, 16, 2048, 3, 0.0),
    (2, 2, 24, 4096, 2, 1e-4),   # 3 tiles of 8 rows = 6 half-tile tasks per time row; 32 strips
    (2, 2, 32, 8192, 3, 1e-5),   # ny = 8192: 4 quarter-tile tasks per tile, 64 strips
    (1, 2, 24, 8192, 2, 0.0),
]
IDS64 = ["e{}d{}_{}x{}_T{}_eps{}".format(*c) for c in FUSED64]


def _c4_plane(T, epsl):
    """C4's 8192^2 plane with a window of T rows, without window-sized host state: the grid and g (a one-row
    make_problem), the reference initial state formed on the device (init_state), and a seeded rough rho (set_state)."""
    P = make_problem(2, 2, 8192, 8192, 1, epsl, seeded=False)
    P.update(T=T, dt=1.0 / max(T, 40), g=P["g"][0])
    rho = 70.0 * np.random.default_rng(11).uniform(0.5, 1.5, (T, 8192, 8192))
    return P, rho


def _ctx(P, fuse, monkeypatch, precision="fp32"):
    monkeypatch.setenv("PDHG_FUSE_RES", "1" if fuse else "0")
    monkeypatch.setenv("PDHG_SHORT_T", "0")   # these windows are short: keep the 8-row (fusable) dual
    ctx = device_ctx(P, precision)
    assert ctx.path_info("fused_residual") == (1 if fuse else 0)
    if precision == "fp64" and fuse:
        assert ctx.path_info("dual_ypl") == 2
        assert ctx.path_info("res64" if P["ny"] < 8192 else "ip_rows") == 1
    return ctx


def _run(P, fuse, n, monkeypatch, precision="fp32"):
    ctx = _ctx(P, fuse, monkeypatch, precision)
    ctx.set_state(P["phi"], P["rho"], P["alp"])
    st = ctx.iterate(n, TAU, SIGMA, -1.0, 1)
    assert st["iters_run"] == n and st["status"] == 0
    out = ctx.get_state()
    ctx.close()
    return out, st


@pytest.mark.parametrize("case", FUSED, ids=IDS)
def test_fused_iterate_vs_oracle(native, case, monkeypatch):
    P = make_problem(*case)
    n = 10
    phi_o, rho_o, alp_o, e1_o, e2_o = _oracle_iterate(P, n)
    (phi_d, rho_d, alp_d), st = _run(P, True, n, monkeypatch)
    assert rel(phi_d, phi_o) < 1e-5
    assert rel(rho_d, rho_o) < 2e-4
    for a_d, a_o in zip(alp_d, alp_o):
        assert rel(a_d, a_o) < 2e-4
    assert abs(st["err1"] - e1_o) <= 1e-2 * e1_o


@pytest.mark.parametrize("case", UNSTABLE, ids=UNSTABLE_IDS)
def test_fused_unstable_regime_no_worse_than_unfused(native, case, monkeypatch):
    P = make_problem(*case)
    n = 3
    phi_o, rho_o, alp_o, _, _ = _oracle_iterate(P, n)
    errs = []
    for fuse in (False, True):
        (phi_d, rho_d, alp_d), _ = _run(P, fuse, n, monkeypatch)
        errs.append([rel(phi_d, phi_o), rel(rho_d, rho_o)] + [rel(a, b) for a, b in zip(alp_d, alp_o)])
    unf, fus = errs
    for f, u in zip(fus, unf):
        assert f <= 2.0 * u + 1e-6, (fus, unf)


@pytest.mark.parametrize("case", FUSED, ids=IDS)
def test_fused_matches_unfused(native, case, monkeypatch):
    """Same kernels up to where the residual is formed: the states after a few iterations agree to
    fp32 reassociation, and so do the err1/err2 stop quantities."""
    P = make_problem(*case)
    (s0, st0), (s1, st1) = [_run(P, fuse, 4, monkeypatch) for fuse in (False, True)]
    assert rel(s1[0], s0[0]) < 1e-5
    assert rel(s1[1], s0[1]) < 1e-5
    for a1, a0 in zip(s1[2], s0[2]):
        assert rel(a1, a0) < 1e-5
    assert abs(st1["err1"] - st0["err1"]) <= 1e-4 * st0["err1"]
    assert abs(st1["err2"] - st0["err2"]) <= 1e-4 * st0["err2"]


def test_fused_dropin_calls_and_state_reset(native, monkeypatch):
    """The per-call drop-ins (update_primal / update_dual) use the fused residual after a fused dual;
    set_state invalidates it (the next primal forms the residual from the new rho, alp)."""
    P = make_problem(2, 2, 256, 512, 3, 1e-5)
    ref = _ctx(P, False, monkeypatch)
    ctx = _ctx(P, True, monkeypatch)
    for c in (ref, ctx):
        c.set_state(P["phi"], P["rho"], P["alp"])
        for _ in range(3):
            c.update_primal(TAU)
            c.update_dual(SIGMA, -1.0, 1)
    for a, b in zip(ctx.get_state(), ref.get_state()):
        if isinstance(a, tuple):
            for x, y in zip(a, b):
                assert rel(x, y) < 1e-5
        else:
            assert rel(a, b) < 1e-5
    # new state: a stale fused residual would give the old state's primal
    rng = np.random.default_rng(7)
    rho2 = P["rho"] * rng.uniform(0.8, 1.2, P["rho"].shape)
    for c in (ref, ctx):
        c.set_state(P["phi"], rho2, P["alp"])
        c.update_primal(TAU)
    assert rel(ctx.get_state()[0], ref.get_state()[0]) < 1e-6
    ref.close()
    ctx.close()


@pytest.mark.parametrize("case", FUSED64, ids=IDS64)
def test_fused_fp64_vs_oracle_and_unfused(native, case, monkeypatch):
    """fp64 fused residual: 6 iterations from the seeded state against the float64 oracle and the unfused fp64
    kernels (update_fns_in_pdhg.py:72-96 formed by the sweep, tile / strip edges completed by the residual)."""
    P = make_problem(*case)
    n = 6
    phi_o, rho_o, alp_o, e1_o, _ = _oracle_iterate(P, n)
    (s0, st0), (s1, st1) = [_run(P, fuse, n, monkeypatch, "fp64") for fuse in (False, True)]
    assert rel(s1[0], phi_o) < 1e-9 and rel(s1[1], rho_o) < 1e-9
    for a_d, a_o in zip(s1[2], alp_o):
        assert rel(a_d, a_o) < 1e-7
    assert abs(st1["err1"] - e1_o) <= 1e-7 * e1_o
    for a, b in zip((s1[0], s1[1]) + tuple(s1[2]), (s0[0], s0[1]) + tuple(s0[2])):
        assert rel(a, b) < 1e-12
    assert abs(st1["err2"] - st0["err2"]) <= 1e-10 * st0["err2"]


@pytest.mark.parametrize("prec,case", [("fp32", (2, 2, 256, 512, 5, 1e-5)), ("fp32", (1, 2, 512, 1024, 4, 1e-5)),
                                       ("fp64", (2, 2, 32, 2048, 4, 1e-5))], ids=["fp32_e2", "fp32_e1", "fp64_e2"])
@pytest.mark.parametrize("fuse", [True, False], ids=["fr", "nofr"])
def test_dual_neighbour_sync_bitwise(native, monkeypatch, prec, case, fuse):
    """k_dual_lds_2d with the per-step block barrier replaced by neighbour counts in LDS (PDHG_DUAL_NBSYNC=1):
    the same arithmetic in the same order, so the states after 4 iterations are bitwise those of the barrier
    form, with and without the fused residual."""
    P = make_problem(*case)
    out = []
    for nb in ("0", "1"):
        monkeypatch.setenv("PDHG_DUAL_NBSYNC", nb)
        out.append(_run(P, fuse, 4, monkeypatch, prec))
    (s0, st0), (s1, st1) = out
    for a, b in zip((s1[0], s1[1]) + tuple(s1[2]), (s0[0], s0[1]) + tuple(s0[2])):
        assert np.array_equal(a, b)
    assert st1["err1"] == st0["err1"] and st1["err2"] == st0["err2"]


@pytest.mark.parametrize("epsl,n", [pytest.param(0.0, 4, marks=pytest.mark.extended), (0.1, 2)])
def test_fused_fp64_c4_plane(native, monkeypatch, epsl, n):
    """C4's 8192^2 plane in fp64 (T = 3): the half-real x blocks (B = 1), so every fused-residual chunk is the two
    rows of a task at one ky (a 16-B store) -- against the unfused fp64 kernels (ip_rows): phi, rho within 1e-12.
    The controls too at epsl = 0; at epsl = 0.1 (sigma*epsl/dx^2 = 2.5e5 at C4's dx) the residual's other
    association (formed in the sweep) moves a few controls that sit at their clamp by more: 1e-8 (measured 2.8e-9)."""
    if epsl == 0.0:   # extended tier: the seeded rough state in every array
        P = make_problem(2, 2, 8192, 8192, 3, epsl)
        (s0, st0), (s1, st1) = [_run(P, fuse, n, monkeypatch, "fp64") for fuse in (False, True)]
        for a, b in zip(s1[2], s0[2]):
            assert rel(a, b) < 1e-12
    else:             # the reference initial state + a seeded rough rho (no window-sized host copies of alp)
        P, rho = _c4_plane(3, epsl)
        out = []
        for fuse in (False, True):
            ctx = _ctx(P, fuse, monkeypatch, "fp64")
            try:
                ctx.init_state(P["g"])
                ctx.set_state(rho=rho)
                st = ctx.iterate(n, TAU, SIGMA, -1.0, 1)
                assert st["iters_run"] == n and st["status"] == 0
                out.append((ctx.get_state(alp=False), st))
            finally:
                ctx.close()
        (s0, st0), (s1, st1) = out
        assert abs(st1["err2"] - st0["err2"]) <= 1e-8 * st0["err2"]   # err2 sums the controls' changes
    assert rel(s1[0], s0[0]) < 1e-12 and rel(s1[1], s0[1]) < 1e-12
    assert abs(st1["err1"] - st0["err1"]) <= 1e-10 * st0["err1"]


def test_fp64_update_c4_plane_fast_vs_generic(native, monkeypatch):
    """fp64 at C4's 8192^2 plane: the inverse DHT_y + update through the fast row kernel on 2-row tasks
    (k_invy_update_fast_2d<8192, 2, ..., double>, 16-B chunks of the half-real spectrum) against the generic row-pair
    kernel (PDHG_UPD8192=0): the same float64 arithmetic up to the transform's association, 1e-12 after 3 iterations."""
    P, rho = _c4_plane(3, 0.0)
    out = []
    for flag in ("1", "0"):
        monkeypatch.setenv("PDHG_UPD8192", flag)
        ctx = device_ctx(P, "fp64")
        try:
            assert ctx.path_info("upd8192") == int(flag) and ctx.path_info("half_real") == 1
            ctx.init_state(P["g"])
            ctx.set_state(rho=rho)
            st = ctx.iterate(3, TAU, SIGMA, -1.0, 1)
            out.append((ctx.get_state(alp=False), st))
        finally:
            ctx.close()
    (s1, st1), (s0, st0) = out
    assert rel(s1[0], s0[0]) < 1e-12 and rel(s1[1], s0[1]) < 1e-12
    assert abs(st1["err1"] - st0["err1"]) <= 1e-10 * st0["err1"]
    assert abs(st1["err2"] - st0["err2"]) <= 1e-10 * st0["err2"]   # err2 sums the controls' changes too


@pytest.mark.parametrize("prec", ["fp64", "fp32"])
def test_c4_task_order_spectrum_bitwise(native, monkeypatch, prec):
    """C4's 8192^2 plane (half-real x blocks, B = 1): the fused residual's spectrum in task order + the LDS-tiled
    transpose into the blocked layout (to_c4, k_res_fwdy_fused_transpose_2d) against the fused residual's direct
    16-B chunk stores (PDHG_C4_TO=0): the same values moved another way, so the states agree bit for bit."""
    P, rho = _c4_plane(3, 0.1)
    out = []
    for flag in ("1", "0"):
        monkeypatch.setenv("PDHG_C4_TO", flag)
        ctx = _ctx(P, True, monkeypatch, prec)
        try:
            assert ctx.path_info("to_c4") == int(flag) and ctx.path_info("half_real") == 1
            ctx.init_state(P["g"])
            ctx.set_state(rho=rho)
            st = ctx.iterate(3, TAU, SIGMA, -1.0, 1)
            out.append((ctx.get_state(alp=False), st))
        finally:
            ctx.close()
    (s1, st1), (s0, st0) = out
    assert np.array_equal(s1[0], s0[0]) and np.array_equal(s1[1], s0[1])
    # err1 / err2 sum every state array (the controls included): equal sums, bit for bit
    assert st1["err1"] == st0["err1"] and st1["err2"] == st0["err2"]
