"""The kernel instantiations every BASELINE config runs, against the float64 oracle (pytest -m gpu).

Each case below selects, and asserts through ``pdhg_path_info``, the size-specialised kernels of one
bench config (BASELINE.json configs[1..4]) at the window length the config uses where that matters
(closed-form Thomas pivots at T = 200 / 400, utils_precond.py:10-35, :142-178):

  c3_ws_T200         C3's x transform k_precond_xt_ws_2d<4096,1,false>, pivots over T = 200
  c3_fr_4096x256     the same x transform under the fused-residual dual (update_fns_in_pdhg.py:72-96,
                     150-165) and the 8-row fast kernels at nx = 4096
  c3_rows_ny4096     C3's row kernels: k_res_fwdy_fused_2d<2,4096,8,512>, k_invy_update_fast_2d<4096,8,512>
  c2_x2048           C2's x transform at nx = 2048, T = 100 (fused residual on, as at 2048^2)
  c2_rows_ny2048     C2's ny = 2048 row kernels, T = 100
  c4_halfreal_x8192  C4's half-real nx = 8192 warp-specialised x transform (no fused residual, as at 8192^2)
  c4_rows_ny8192     C4's ny = 8192 four-row kernels
  c1_exact           C1 itself: egno 1, 1-D, nx = 65536, T = 400 (four-step DHT, 1-D Thomas)

The fp64 oracle needs 20 s - 6 min per iteration at these sizes, so tests/golden/make_config_fixtures.py
ran it once (from the float32-rounded initial state the device holds) and kept the oracle state at 8192
sampled points per array, the full-array norms, the last iteration's err1/err2, and "e32": how far the
same oracle executed in float32 (complex64 FFTs and Thomas) lands from its float64 result -- the accuracy
the reference algorithm itself reaches in float32.  The device runs the same iterations in fp32 and is
compared on those points.

Bounds (relative L2 over the sampled points; every achieved value is also written to
gpurun_out/parity.jsonl -> profiles/parity_r03.json):
  phi, epsl = 0 runs (the ref state and the seeded rough state): FIXED 1e-6 after the first primal
  update and 1e-5 (the north-star bound) after the run, on every default kernel path -- no e32 escape.
  Measured on the device (round 3): ref runs 5e-8 - 4.4e-7 (C1 2.5e-7, C3-T200 1.3e-7), seeded C1
  6.4e-6, C2 3.3e-8.  The float32 ORACLE is worse than that at T = 200 / 400 (e32 = 1.6e-5 at C3-T200,
  4.7e-5 at C1): tests/golden/precision_study.py locates all of it in the reference's Thomas recurrence
  (utils_precond.py:10-35) run in float32 -- with the Thomas solve alone in float64 the float32 oracle
  lands at 4.1e-7 -- while the device's cancellation-free pivot recurrence with closed-form backward
  pivots, emulated in float32 by the same study ("dth32"), lands at 5.7e-7.
  Other quantities keep max(fixed, K32 x e32), K32 = 4, because fp32 storage itself limits them:
  rho, epsl = 0.1: the explicit sigma*epsl*Lap(phi_bar) dual term amplifies the float32 representation
    of phi_bar by ~sigma*epsl*8/dx^2 = 5e5 at dx = 2/4096 (rho after one iteration: 4.9e-5 in the
    float32 oracle and on the device; 3e-8 with phi / phi_bar alone held in float64, precision_study
    "phi64");
  alp: the controls follow one-sided differences of phi_bar, whose float32 precision is
    ulp(phi)/(dx |grad phi|) (9.4e-4 at C1's dx = 2/65536; 4.9e-5 with phi in float64);
  phi, epsl = 0.1 seeded runs: from a rough state the residual is dominated by the epsl*Lap(rho) term
    at high frequency (|R| ~ 1e7) while U = H1^-1 R lives in the low modes, so the float32 rounding of R
    itself bounds U (U1 1.1e-4 in the float32 oracle, 1.2e-4 on the device; phi1 1.4e-5 / 1.5e-5 at
    C3-T200): precision_study moves it neither with the transforms in float64 (1.4e-5) nor with the
    t-solve in float64 (1.7e-5), only with rho and the residual in float64 (2e-10).
Runs with epsl = 0.1 therefore stop after one iteration; test_one_step_eps below checks a further
iteration (the fused residual formed by the first dual sweep) from the device's own state, against the
oracle in float64 and in float32 from that state.
"""
import os

import numpy as np
import pytest

from _problems import device_ctx, make_problem, oracle_fns, rel

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
TAU, SIGMA = 0.1 / 1.5, 0.1 * 1.5
K32 = 4.0        # device error <= K32 x (oracle in float32 vs oracle in float64), or the fixed bound

# name: (environment for the context, expected pdhg_path_info values)
CASES = {
    "c3_ws_T200": ({"PDHG_XT_BATCH": "0"}, {"fast_xt": 2, "half_real": 0}),
    "c3_fr_4096x256": ({"PDHG_FUSE_RES": "1", "PDHG_XT_BATCH": "0"}, {"fast_xt": 2, "fused_residual": 1, "rows_rw": 8,
                                                                   "fast_dual": 8}),
    "c3_rows_ny4096": ({"PDHG_FUSE_RES": "1"}, {"fused_residual": 1, "rows_rw": 8, "res_threads": 512,
                                                "upd_threads": 512, "fast_dual": 8}),
    "c2_x2048": ({"PDHG_FUSE_RES": "1", "PDHG_XT_BATCH": "0"}, {"fast_xt": 1, "fused_residual": 1, "rows_rw": 8}),
    "c2_rows_ny2048": ({"PDHG_FUSE_RES": "1"}, {"fused_residual": 1, "rows_rw": 8, "res_threads": 512,
                                                "upd_threads": 512}),
    "c4_halfreal_x8192": ({"PDHG_FUSE_RES": "0"}, {"fast_xt": 5, "half_real": 1, "fused_residual": 0}),
    # the warp-specialised half-real x transform (the default before round 5; PDHG_XT_DMA_HR=0)
    "c4_halfreal_x8192@ws": ({"PDHG_FUSE_RES": "0", "PDHG_XT_DMA_HR": "0"}, {"fast_xt": 2, "half_real": 1}),
    "c4_rows_ny8192": ({"PDHG_FUSE_RES": "0"}, {"rows_rw": 4, "fused_residual": 0, "res_threads": 1024,
                                                "upd_threads": 1024}),
    # the fused residual at ny = 8192: 4-row half-tile tasks of the 8-row sweep (k_res_fwdy_fused_2d<.., 8192, 4, 512>)
    "c4_rows_ny8192@fr": ({"PDHG_FUSE_RES": "1", "PDHG_SHORT_T": "0"}, {"rows_rw": 4, "fused_residual": 1,
                                                                        "res_threads": 512, "fast_dual": 8}),
    "c1_exact": ({}, {"fourstep": 1, "glb_line": 1, "thomas_chunk": 1, "fs16": 1, "fs_wide": 0, "fused_residual": 1}),
    "c1_exact@wide": ({"PDHG_FS16": "0"}, {"fourstep": 1, "fs16": 0, "fs_wide": 1}),
    "c1_exact@tile16": ({"PDHG_FS16": "0", "PDHG_FS_WIDE": "0"}, {"fourstep": 1, "fs16": 0, "fs_wide": 0}),
    "c1_exact@thomas1": ({"PDHG_THOMAS_CHUNK": "0"}, {"fourstep": 1, "fs16": 1, "thomas_chunk": 0}),
    # the row-batched x transform (k_precond_xt_batch_2d) on the same fixtures
    "c3_ws_T200@batch": ({"PDHG_XT_BATCH": "1", "PDHG_XT_DMA": "0"}, {"fast_xt": 3}),
    "c3_fr_4096x256@batch": ({"PDHG_FUSE_RES": "1", "PDHG_XT_BATCH": "1", "PDHG_XT_DMA": "0"},
                             {"fast_xt": 3, "fused_residual": 1}),
    # the LDS-DMA staged x transform (k_precond_xt_dma_2d)
    "c3_ws_T200@dma": ({"PDHG_XT_BATCH": "1", "PDHG_XT_DMA": "1"}, {"fast_xt": 4}),
    "c3_fr_4096x256@dma": ({"PDHG_FUSE_RES": "1", "PDHG_XT_BATCH": "1", "PDHG_XT_DMA": "1"},
                           {"fast_xt": 4, "fused_residual": 1}),
    "c2_x2048@batch": ({"PDHG_FUSE_RES": "1", "PDHG_XT_BATCH": "1"}, {"fast_xt": 3, "fused_residual": 1}),
    # the fused residual with 1024 threads (k_res_fwdy_fused_2d<2,4096,8,1024>)
    "c3_rows_ny4096@nt1024": ({"PDHG_FUSE_RES": "1", "PDHG_HALF_NT": "2"}, {"fused_residual": 1, "res_threads": 1024}),
}


# The default tier runs each config's DEFAULT fp32 kernels (C3: the LDS-DMA x transform, the 8-row fused rows; C2: the
# row-batched x transform; C4: the half-real DMA x transform, the 4-row rows with and without the fused residual; C1:
# the 16 x 4096 split with the chunked t-solve); the other schedules (tuning alternatives kept selectable by
# environment) are the extended tier (PDHG_TESTS=full)
EXTENDED_CASES = {"c3_ws_T200", "c3_fr_4096x256", "c2_x2048", "c4_halfreal_x8192@ws", "c1_exact@wide", "c1_exact@tile16",
                  "c1_exact@thomas1", "c3_ws_T200@batch", "c3_fr_4096x256@batch", "c3_rows_ny4096@nt1024"}


def _tier(names, extended):
    return [pytest.param(n, marks=pytest.mark.extended) if n in extended else n for n in names]


# non-default schedules whose phi keeps the e32 escape on epsl = 0 runs: the one-thread-per-mode 1-D t-solve
# (PDHG_THOMAS_CHUNK=0; measured 1.6e-5 on C1's seeded state against 6.4e-6 for the default chunked solve)
PHI_E32_ESCAPE = {"c1_exact@thomas1"}


def _fixture(name):
    path = os.path.join(HERE, "golden", "cfg_{}.npz".format(name))
    if not os.path.exists(path):
        pytest.fail("missing fixture {} (python tests/golden/make_config_fixtures.py {})".format(path, name))
    return np.load(path)


def _live(ndim, egno, alp):
    if ndim == 1 or egno == 3:
        return [a[..., 0] for a in alp]
    return [a[..., 0 if i < 2 else 1] for i, a in enumerate(alp)]


def _f32_state(P):
    f = lambda a: np.asarray(a, dtype=np.float32).astype(np.float64)  # noqa: E731
    return f(P["phi"]), f(P["rho"]), tuple(f(a) for a in P["alp"])


def _norm_dev(x, ref_norm):
    return abs(np.linalg.norm(x) / float(ref_norm) - 1)


@pytest.mark.parametrize("name", _tier(CASES, EXTENDED_CASES))
def test_config_instantiation(native, name, monkeypatch, parity_log):
    env, expect = CASES[name]
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    F = _fixture(name.split("@")[0])
    egno, ndim, nx, ny, T = (int(v) for v in F["meta"])
    failures = []
    for tag in [str(t) for t in F["runs"]]:
        g = lambda k: F[tag + "__" + k]  # noqa: E731
        epsl, n, seeded = float(g("epsl")), int(g("iters")), bool(int(g("seeded")))
        ip, ir = g("idx_phi"), g("idx_rho")
        e32 = g("e32")    # [phi1, U1, phi, rho, alp0.., err1]
        # phi: the north-star bound 1e-5 (1e-6 after the first update) as a FIXED bound on every epsl = 0 run
        # (ref and seeded), no e32 escape; runs with epsl > 0 keep the escape (see the module docstring)
        fixed_phi = epsl == 0.0 and name not in PHI_E32_ESCAPE
        tol = {"phi1": 1e-6 if fixed_phi else max(1e-6, K32 * e32[0]), "U1": max(5e-4, K32 * e32[1]),
               "phi": 1e-5 if fixed_phi else max(1e-5, K32 * e32[2]),
               "rho": max(2e-4 if seeded else 1e-5, K32 * e32[3]), "err1": max(1e-3, K32 * e32[-1])}
        for a in range(len(e32) - 5):
            tol["alp{}".format(a)] = max(1e-3 if seeded else 1e-4, K32 * e32[4 + a])
        P = make_problem(egno, ndim, nx, ny, T, epsl, seeded=seeded)
        phi0, rho0, alp0 = _f32_state(P)
        ctx = device_ctx(P, "fp32")
        try:
            for key, val in expect.items():
                assert ctx.path_info(key) == val, (name, key, ctx.path_info(key), val)
            ctx.set_state(phi0, rho0, alp0)
            ctx.update_primal(TAU)
            phi1 = ctx.get_state()[0]
            m = {"phi1": rel(phi1.reshape(-1)[ip], g("phi1")), "phi1_norm": _norm_dev(phi1, g("phi1_norm"))}
            if seeded:   # the primal update itself (zero from the reference state)
                m["U1"] = rel((phi1.reshape(-1)[ip] - phi0.reshape(-1)[ip]) / TAU, g("U1"))
            del phi1
            ctx.set_state(phi0, rho0, alp0)
            st = ctx.iterate(n, TAU, SIGMA, -1.0, 1)
            phi, rho, alp = ctx.get_state()
            m["phi"], m["phi_norm"] = rel(phi.reshape(-1)[ip], g("phi")), _norm_dev(phi, g("phi_norm"))
            m["rho"], m["rho_norm"] = rel(rho.reshape(-1)[ir], g("rho")), _norm_dev(rho, g("rho_norm"))
            for a, arr in enumerate(_live(ndim, egno, alp)):
                ref = g("alp{}".format(a))
                if np.linalg.norm(ref) > 0:
                    m["alp{}".format(a)] = rel(arr.reshape(-1)[ir], ref)
                    m["alp{}_norm".format(a)] = _norm_dev(arr, g("alp{}_norm".format(a)))
            e1_o = float(g("err")[0])
            m["err1"] = abs(st["err1"] - e1_o) / e1_o if e1_o > 0 else abs(st["err1"])
        finally:
            ctx.close()
        print("CFG {} {}: {} | e32 {}".format(name, tag, " ".join("{}={:.2e}".format(k, v) for k, v in m.items()),
                                              " ".join("{:.1e}".format(v) for v in e32)), flush=True)
        parity_log("test_config_instantiation", "{}/{}".format(name, tag), m,
                   {k: tol[k[:-5] if k.endswith("_norm") else k] for k in m}, e32=[float(v) for v in e32],
                   iters=n, epsl=epsl, seeded=seeded)
        if not (st["iters_run"] == n and st["status"] == 0 and not st["nan_seen"]):
            failures.append((tag, "run", st))
        for k, v in m.items():
            bound = tol[k[:-5] if k.endswith("_norm") else k]
            if not v <= bound:
                failures.append((tag, k, v, bound))
    assert not failures, failures


# one further iteration from the device's own state (epsl = 0.1, seeded rough state): the fused residual
# formed by the first dual sweep feeds the second primal update.  Short windows with the C3/C4 kernels
# forced (PDHG_XT_WS=1 selects the warp-specialised x transform below T = 16), so the oracle runs here.
ONE_STEP = {
    # name: (egno, nx, ny, T, env, expected path)
    "ws_fr_4096x256": (2, 4096, 256, 4, {"PDHG_XT_BATCH": "0", "PDHG_XT_WS": "1", "PDHG_FUSE_RES": "1"},
                       {"fast_xt": 2, "fused_residual": 1}),
    "rows_ny4096_fr": (2, 64, 4096, 4, {"PDHG_FUSE_RES": "1"}, {"fused_residual": 1, "res_threads": 512}),
    "halfreal_x8192": (2, 8192, 16, 4, {}, {"fast_xt": 5, "half_real": 1}),
    "halfreal_x8192_ws": (2, 8192, 16, 4, {"PDHG_XT_DMA_HR": "0"}, {"fast_xt": 2, "half_real": 1}),
    "rows_ny8192": (2, 64, 8192, 4, {}, {"rows_rw": 4}),
    "batch_fr_4096x256": (2, 4096, 256, 8, {"PDHG_XT_BATCH": "1", "PDHG_XT_DMA": "0", "PDHG_FUSE_RES": "1"},
                          {"fast_xt": 3, "fused_residual": 1}),
    "batch_x2048_T6": (1, 2048, 256, 6, {"PDHG_XT_BATCH": "1"}, {"fast_xt": 3}),   # partial last batch
    "dma_fr_4096x256": (2, 4096, 256, 8, {"PDHG_XT_BATCH": "1", "PDHG_XT_DMA": "1", "PDHG_FUSE_RES": "1"},
                        {"fast_xt": 4, "fused_residual": 1}),
    "dma_4096_T7": (1, 4096, 256, 7, {"PDHG_XT_BATCH": "1", "PDHG_XT_DMA": "1"}, {"fast_xt": 4}),   # odd T
}


@pytest.mark.extended
@pytest.mark.parametrize("nx,T", [(4096, 37), (2048, 9), (1024, 4), (512, 3)])
def test_batched_x_transform_matches_ws(native, monkeypatch, nx, T):
    """The row-batched x transform against the warp-specialised / single-role kernel on the same state: the
    same arithmetic per mode in another schedule (3 iterations from the seeded state, fp32: <= 1e-6)."""
    P = make_problem(2, 2, nx, 256, T, 0.0, seeded=True)
    out = []
    for batch in ("0", "1"):
        monkeypatch.setenv("PDHG_XT_BATCH", batch)   # 0: warp-specialised (nx = 4096, T >= 16) / single-role
        monkeypatch.setenv("PDHG_XT_DMA", "0")
        ctx = device_ctx(P, "fp32")
        try:
            assert ctx.path_info("fast_xt") == (3 if batch == "1" else (2 if (nx == 4096 and T >= 16) else 1))
            ctx.set_state(*_f32_state(P))
            ctx.iterate(3, TAU, SIGMA, -1.0, 1)
            out.append(ctx.get_state())
        finally:
            ctx.close()
    assert rel(out[1][0], out[0][0]) < 1e-6 and rel(out[1][1], out[0][1]) < 1e-6


@pytest.mark.extended
@pytest.mark.parametrize("T", [50, 9, 5, 4])
def test_dma_halfreal_matches_ws(native, monkeypatch, T):
    """The LDS-DMA half-real x transform (k_precond_xt_dma_2d<4096, true>, C4's nx = 8192) against the
    warp-specialised half-real kernel on the same state: the same modes per item (k, k + N) and Thomas algebra,
    both reading lam(k + N) as the host's lam(N - k) from LDS (even symmetry; the subtraction form -4/dx^2 - lam(k)
    cancels in float32); 3 iterations, fp32 <= 1e-6 (the two kernels differ only in how rows are staged)."""
    P = make_problem(2, 2, 8192, 64, T, 0.0, seeded=True)
    out = []
    for dma in ("0", "1"):
        monkeypatch.setenv("PDHG_XT_DMA_HR", dma)
        ctx = device_ctx(P, "fp32")
        try:
            assert ctx.path_info("fast_xt") == (5 if dma == "1" else 2) and ctx.path_info("half_real") == 1
            ctx.set_state(*_f32_state(P))
            ctx.iterate(3, TAU, SIGMA, -1.0, 1)
            out.append(ctx.get_state())
        finally:
            ctx.close()
    assert rel(out[1][0], out[0][0]) < 1e-6 and rel(out[1][1], out[0][1]) < 1e-6
    assert rel(np.stack(out[1][2]), np.stack(out[0][2])) < 1e-5


@pytest.mark.extended
@pytest.mark.parametrize("T", [37, 8, 5, 4])
def test_dma_x_transform_matches_batched(native, monkeypatch, T):
    """The LDS-DMA staged x transform against the row-batched one on the same state (same arithmetic per mode,
    2 rows per batch instead of 4: partial batches at both sweep ends for odd T; 3 iterations, fp32 <= 1e-6)."""
    P = make_problem(2, 2, 4096, 256, T, 0.0, seeded=True)
    out = []
    monkeypatch.setenv("PDHG_XT_BATCH", "1")
    for dma in ("0", "1"):
        monkeypatch.setenv("PDHG_XT_DMA", dma)
        ctx = device_ctx(P, "fp32")
        try:
            assert ctx.path_info("fast_xt") == (4 if dma == "1" else 3)
            ctx.set_state(*_f32_state(P))
            ctx.iterate(3, TAU, SIGMA, -1.0, 1)
            out.append(ctx.get_state())
        finally:
            ctx.close()
    assert rel(out[1][0], out[0][0]) < 1e-6 and rel(out[1][1], out[0][1]) < 1e-6


@pytest.mark.parametrize("name", _tier(ONE_STEP, {"ws_fr_4096x256", "halfreal_x8192_ws", "batch_fr_4096x256"}))
def test_one_step_eps(native, name, monkeypatch, parity_log):
    """Device iteration 2 vs one oracle iteration from the device's iteration-1 state (float32 values, so the
    oracle starts from exactly the device's state).  Bounds: the larger of the seeded-state bounds (phi 1e-5,
    rho 2e-4, alp 1e-3) and K32 x the distance between that oracle step in float32 and in float64."""
    egno, nx, ny, T, env, expect = ONE_STEP[name]
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    P = make_problem(egno, 2, nx, ny, T, 0.1, seeded=True)
    ctx = device_ctx(P, "fp32")
    try:
        for key, val in expect.items():
            assert ctx.path_info(key) == val, (name, key, ctx.path_info(key), val)
        ctx.set_state(*_f32_state(P))
        st1 = ctx.iterate(1, TAU, SIGMA, -1.0, 1)
        s1 = ctx.get_state()
        st2 = ctx.iterate(1, TAU, SIGMA, -1.0, 1)
        s2 = ctx.get_state()
    finally:
        ctx.close()
    assert st1["status"] == 0 and st2["status"] == 0
    primal, dual = oracle_fns(P)

    def step(phi, rho, alp):
        phi_n = primal(phi, rho, 70.0, alp, TAU, P["dt"], P["dsp"], P["fns"], P["fv"], 0.1, P["x_arr"], None)
        rho_n, alp_n = dual(2 * phi_n - phi, rho, 70.0, alp, SIGMA, P["dt"], P["dsp"], 0.1, P["fns"], P["x_arr"],
                            None, 2, -1.0)
        return phi_n, rho_n, alp_n
    o = step(*s1)
    f = np.float32
    P["x_arr"] = P["x_arr"].astype(f)
    p = step(s1[0].astype(f), s1[1].astype(f), tuple(a.astype(f) for a in s1[2]))   # the oracle in float32
    assert p[0].dtype == f
    live_o, live_p, live_d = (_live(2, egno, x[2]) for x in (o, p, s2))
    m = {"phi": (rel(s2[0], o[0]), max(1e-5, K32 * rel(p[0], o[0]))),
         "rho": (rel(s2[1], o[1]), max(2e-4, K32 * rel(p[1], o[1])))}
    for a in range(4):
        if np.linalg.norm(live_o[a]) > 0:
            m["alp{}".format(a)] = (rel(live_d[a], live_o[a]), max(1e-3, K32 * rel(live_p[a], live_o[a])))
    parity_log("test_one_step_eps", name, {k: v for k, (v, b) in m.items()}, {k: b for k, (v, b) in m.items()})
    print("ONESTEP {}: {}".format(name, " ".join("{}={:.2e}(<{:.1e})".format(k, v, b) for k, (v, b) in m.items())),
          flush=True)
    assert all(v <= b for v, b in m.values()), m


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
@pytest.mark.parametrize("nx,T,egno", [(65536, 100, 1), (4096, 33, 2), (1024, 400, 1), (256, 1, 2), (512, 17, 1)])
def test_chunked_thomas_matches_one_thread_per_mode(native, monkeypatch, nx, T, egno, prec):
    """1-D t-solve in 32-row chunks (k_thomas_chunk_1d: chunk carries folded through LDS) against the
    one-thread-per-mode recurrence (k_thomas_1d) on the same state: 3 iterations from the reference state,
    fp32, <= 1e-6 (same algebra, another association of the products).  From the seeded rough state the two
    fp32 results differ by up to 2e-5 at nx = 65536 (both within the float32 oracle's own 6.5e-5 of the
    float64 one there: test_config_instantiation c1_exact / c1_exact@thomas1).  fp64: 16-row chunks, one per
    half-wave (T = 17: an odd chunk count, the last half-wave's chunk empty), <= 1e-12."""
    P = make_problem(egno, 1, nx, 1, T, 0.0, seeded=False)
    out = []
    for chunk in ("0", "1"):
        monkeypatch.setenv("PDHG_THOMAS_CHUNK", chunk)
        ctx = device_ctx(P, prec)
        try:
            assert ctx.path_info("thomas_chunk") == int(chunk)
            ctx.set_state(*(_f32_state(P) if prec == "fp32" else (P["phi"], P["rho"], P["alp"])))
            ctx.iterate(3, TAU, SIGMA, -1.0, 1)
            out.append(ctx.get_state())
        finally:
            ctx.close()
    bar = 1e-6 if prec == "fp32" else 1e-12
    assert rel(out[1][0], out[0][0]) < bar and rel(out[1][1], out[0][1]) < bar


# The parity path: the same fixtures in the reference's arithmetic (fp64; jaxsrc/update_fns_in_pdhg.py:10).  Every
# run of every fixture -- the epsl = 0.1 runs of C3 / C4 included -- at FIXED bounds with no float32 escape: the
# north-star 1e-5 on phi, rho and every control, and the fp64 bar 1e-9 on phi / rho (the device and the oracle run
# the same float64 algorithm from the same state; measured ~1e-13).  The fp64 kernels at each fixture's shape are
# asserted through pdhg_path_info (k_precond_xt_f64_2d at nx = 4096 and its half-real form at C4's nx = 8192, the
# 4-row fast row kernels at ny = 2048 / 4096, the generic row kernels on one padded in-place line at C4's ny = 8192,
# the time-marching dual).
FP64_CASES = {
    "c3_ws_T200": {"f64_xt": 1},
    "c3_fr_4096x256": {"f64_xt": 1, "dual64": 1},
    "c3_rows_ny4096": {"res64": 1, "dual64": 1},
    "c2_x2048": {"dual64": 1, "f64_xt": 1},   # k_precond_xt_f64_2d<2048, 512, false, BPR> (round 5)
    "c2_x2048+generic": {"dual64": 1, "f64_xt": 0},   # the generic runtime-radix kernel it replaced
    "c2_x2048+v1": {"f64_xt": 1},   # the A/B shapes of the nx = 2048 kernel (PDHG_XT64_VAR)
    "c2_x2048+v2": {"f64_xt": 1},
    "c2_x2048+v3": {"f64_xt": 1},
    "c2_rows_ny2048": {"res64": 1, "dual64": 1},
    "c1_exact": {"glb_line": 1, "fs16": 1},   # the 16 x 4096 split on complex doubles (kernels_fs16.hpp)
    "c4_halfreal_x8192": {"f64_xt": 1, "half_real": 1, "dual64": 1},   # k_precond_xt_f64_2d<4096, 512, HR>
    "c4_rows_ny8192": {"ip_rows": 1, "dual64": 1},   # row pairs transformed in one padded in-place line (FFTIp)
    # the fp64 fused residual (k_dual_lds_2d<.., double, 2> FR + k_res_fwdy_fused_2d<.., 4, 512, double>), the
    # default at C3's size, forced on the fixture's smaller grid
    "c3_rows_ny4096+fr": {"res64": 1, "dual64": 1, "fused_residual": 1, "dual_ypl": 2},
    "c2_rows_ny2048+fr": {"res64": 1, "dual64": 1, "fused_residual": 1, "dual_ypl": 2},
}
FP64_ENV = {"fr": {"PDHG_FUSE_RES": "1", "PDHG_SHORT_T": "0"}, "generic": {"PDHG_XT64": "0"},
           "v1": {"PDHG_XT64_VAR": "1"}, "v2": {"PDHG_XT64_VAR": "2"}, "v3": {"PDHG_XT64_VAR": "3"}}
FP64_BAR = 1e-9


def test_fp64_fs16_matches_generic(native, monkeypatch):
    """fp64 C1 (nx = 65536, T = 400): the 16 x 4096 split against the generic Stockham passes over global scratch
    (PDHG_FS16=0), both the same float64 arithmetic up to the transform's association: 2 iterations from the
    seeded state, every state array within 1e-12."""
    F = _fixture("c1_exact")
    egno, ndim, nx, ny, T = (int(v) for v in F["meta"])
    P = make_problem(egno, ndim, nx, ny, T, 0.0, seeded=True)
    out = []
    for flag in ("1", "0"):
        monkeypatch.setenv("PDHG_FS16", flag)
        ctx = device_ctx(P, "fp64")
        try:
            assert ctx.path_info("fs16") == int(flag)
            ctx.set_state(P["phi"], P["rho"], P["alp"])
            st = ctx.iterate(2, TAU, SIGMA, -1.0, 1)
            assert st["iters_run"] == 2 and st["status"] == 0
            out.append(ctx.get_state() + (st,))
        finally:
            ctx.close()
    (p1, r1, a1, s1), (p0, r0, a0, s0) = out
    assert rel(p1, p0) < 1e-12 and rel(r1, r0) < 1e-12
    for x, y in zip(a1, a0):
        assert rel(x, y) < 1e-12
    assert abs(s1["err1"] - s0["err1"]) <= 1e-10 * s0["err1"]


@pytest.mark.parametrize("name", _tier(FP64_CASES, {"c2_x2048+generic", "c2_x2048+v1", "c2_x2048+v2", "c2_x2048+v3"}))
def test_config_fp64_fixed_bounds(native, name, parity_log, monkeypatch):
    fixture, _, variant = name.partition("+")
    for k, v in FP64_ENV.get(variant, {}).items():
        monkeypatch.setenv(k, v)
    F = _fixture(fixture)
    egno, ndim, nx, ny, T = (int(v) for v in F["meta"])
    failures = []
    for tag in [str(t) for t in F["runs"]]:
        g = lambda k: F[tag + "__" + k]  # noqa: E731
        epsl, n, seeded = float(g("epsl")), int(g("iters")), bool(int(g("seeded")))
        ip, ir = g("idx_phi"), g("idx_rho")
        P = make_problem(egno, ndim, nx, ny, T, epsl, seeded=seeded)
        phi0, rho0, alp0 = _f32_state(P)
        ctx = device_ctx(P, "fp64")
        try:
            for key, val in FP64_CASES[name].items():
                assert ctx.path_info(key) == val, (name, key, ctx.path_info(key), val)
            ctx.set_state(phi0, rho0, alp0)
            st = ctx.iterate(n, TAU, SIGMA, -1.0, 1)
            phi, rho, alp = ctx.get_state()
        finally:
            ctx.close()
        m = {"phi": rel(phi.reshape(-1)[ip], g("phi")), "rho": rel(rho.reshape(-1)[ir], g("rho"))}
        for a, arr in enumerate(_live(ndim, egno, alp)):
            ref = g("alp{}".format(a))
            if np.linalg.norm(ref) > 0:
                m["alp{}".format(a)] = rel(arr.reshape(-1)[ir], ref)
        e1_o = float(g("err")[0])
        m["err1"] = abs(st["err1"] - e1_o) / e1_o if e1_o > 0 else abs(st["err1"])
        tol = {k: 1e-5 for k in m}
        tol["phi"] = tol["rho"] = FP64_BAR
        parity_log("test_config_fp64_fixed_bounds", "{}/{}".format(name, tag), m, tol, iters=n, epsl=epsl,
                   seeded=seeded)
        if not (st["iters_run"] == n and st["status"] == 0 and not st["nan_seen"]):
            failures.append((tag, "run", st))
        failures += [(tag, k, v, tol[k]) for k, v in m.items() if not v <= tol[k]]
    assert not failures, failures
