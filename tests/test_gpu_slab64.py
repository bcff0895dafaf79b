"""t-slab decomposition in fp64 -- the reference's arithmetic (jaxsrc/update_fns_in_pdhg.py:10, set_fns.py:7) --
on the GPU: P slab contexts on one device through LocalComm against the single fp64 context of
the same window, for every x transform a fp64 slab runs (the generic runtime-radix kernel incl. egno 3's DCT, the
fp64 nx = 4096 kernel and its half-real nx = 8192 form with their slab phases, kernels_xt_f64.hpp) and both
residual forms (the 4-row kernels with the halo row split off at ny = 2048 / 4096, the generic row kernels over
the whole slab after the halo otherwise; the fused residual), plus one epsl = 0.1 step against the fp64 oracle.

Bounds: the slab path rounds the distributed t-solve's carry sums in another association than the single
context's sweep, in double: relative L2 <= 1e-11 after 6 iterations from the seeded state (measured values go to
parity_log); one step against the oracle <= 1e-9, the fp64 single context's own bar (test_gpu_configs.py)."""
import numpy as np
import pytest

from _problems import make_problem, oracle_fns, rel

pytestmark = pytest.mark.gpu

TAU, SIGMA = 0.1 / 1.5, 0.1 * 1.5
TOL = 1e-11

CASES = [
    # (egno, nx, ny, T, P, k, expected path_info)
    (1, 512, 256, 6, 2, 1, {"f64_xt": 1, "res64": 0}),        # fp64 x kernel at nx = 512 (B = 2), generic rows
    (2, 4096, 256, 50, 2, 1, {"f64_xt": 1}),                  # 25-row slabs (C3's on 8 GPUs): fp64 nx = 4096 kernel
    (2, 4096, 256, 11, 3, 1, {"f64_xt": 1}),                  # 4 + 4 + 3 rows
    (2, 8192, 256, 5, 2, 1, {"f64_xt": 1, "half_real": 1}),   # C4's nx: half-real split
    (1, 512, 256, 3, 3, 1, {"f64_xt": 1}),                    # one-row slabs: the halo row is the whole slab
    # slabs of 2 and 1 rows: every slab takes the window's column-block width (B = 2; ADVICE r5: a 1-row slab kept
    # B = 8 next to its neighbour's B = 2 and the exchanged carry planes were misindexed)
    (1, 512, 256, 3, 2, 1, {"f64_xt": 1}),
    (3, 512, 256, 9, 3, 1, {"f64_xt": 0}),                    # egno 3: the generic kernel's DCT slab phases
    (1, 512, 2048, 8, 2, 1, {"res64": 1}),                    # 4-row residual kernels, halo row split off
    (2, 512, 2048, 12, 3, 2, {"res64": 1}),                   # two buffer sets, dual sub-iterations
    (2, 4096, 2048, 8, 2, 1, {"res64": 1, "f64_xt": 1}),      # C3's x extent with the 4-row row kernels
    # the reference's default dual loop (rho_alp_iters = 10 with early exit, update_fns_in_pdhg.py:167-180) at C3's x
    # extent: two buffer sets per slab, the global exit decision through the per-sub-iteration sums
    (2, 4096, 256, 20, 2, 10, {"f64_xt": 1}),
    # C3's whole plane (what bench.py --gpus N runs per slab): the fused fp64 sweep inside the slabs by default
    # (T = 8: the reference layouts' host copies of a 4096^2 window -- alp with its dead components -- cost 4 GB a row)
    (2, 4096, 4096, 8, 2, 1, {"res64": 1, "f64_xt": 1, "fused_residual": 1, "dual_ypl": 2}),
]


def _ids(cases):
    return ["e{}_{}x{}_T{}_P{}_k{}".format(*c[:6]) for c in cases]


def _run_pair(P, nr, k, n, path=None, egno=None, alp=None):
    """alp (default: below C3's 4096^2 plane): compare the controls too; at 4096^2 their reference-layout host copies
    (dead components included) cost more than the whole run, and err2 (compared) sums their changes anyway."""
    if alp is None:
        alp = P["nx"] * P["ny"] < 4096 * 4096
    import torch
    from pdhg_amd.context import PDHGContext
    from pdhg_amd.slab import LocalComm, SlabContext, SlabRunner, join_state, slab_bounds, split_state
    egno = P["egno"]
    T = P["T"]
    ref = PDHGContext(egno, 2, P["nx"], P["ny"], T, P["dx"], P["dy"], P["dt"], P["xs"], P["ys"], epsl=P["epsl"],
                      precision="fp64", rho_alp_iters=k)
    try:
        ref.set_state(P["phi"], P["rho"], P["alp"])
        st_ref = ref.iterate(n, TAU, SIGMA, -1.0, k)
        want = ref.get_state(alp=alp)
    finally:
        ref.close()
    slabs = [SlabContext(r, nr, T, egno, P["nx"], P["ny"], P["dx"], P["dy"], P["dt"], P["xs"], P["ys"],
                         epsl=P["epsl"], rho_alp_iters=k, precision="fp64") for r in range(nr)]
    try:
        for s in slabs:
            for key, v in (path or {}).items():
                assert s.path_info(key) == v, (key, s.path_info(key), v)
        for s, part in zip(slabs, split_state(P["phi"], P["rho"], P["alp"], slab_bounds(T, nr))):
            s.set_state(*part)
        runner = SlabRunner(slabs, LocalComm(nr))
        assert runner.b[0]["DS"].dtype == torch.float64   # exchange planes in the slabs' precision
        st = runner.iterate(n, TAU, SIGMA, -1.0, k)
        torch.cuda.synchronize()
        parts = [s.get_state(alp=alp) for s in slabs]
        got = join_state(parts) if alp else join_state([(a, b, ()) for a, b, _ in parts])[:2] + (None,)
    finally:
        for s in slabs:
            s.close()
    return st, st_ref, got, want


def _metrics(st, st_ref, got, want):
    m = {"phi": rel(got[0], want[0]), "rho": rel(got[1], want[1]),
         "err1": abs(st["err1"] - st_ref["err1"]) / abs(st_ref["err1"]),
         "err2": abs(st["err2"] - st_ref["err2"]) / abs(st_ref["err2"])}
    if got[2] is not None:
        m["alp"] = rel(np.stack(got[2]), np.stack(want[2]))
    return m


@pytest.mark.parametrize("egno,nx,ny,T,nr,k,path", CASES, ids=_ids(CASES))
def test_fp64_slabs_match_single_context(native, parity_log, egno, nx, ny, T, nr, k, path):
    P = make_problem(egno, 2, nx, ny, T, 0.0)
    n = 6
    st, st_ref, got, want = _run_pair(P, nr, k, n, path)
    assert st["iters"] == st_ref["iters_run"] == n
    assert st["inner_total"] == st_ref["inner_total"]
    m = _metrics(st, st_ref, got, want)
    bounds = {key: TOL for key in m}
    parity_log("test_fp64_slabs_match_single_context", "e{}_{}x{}_T{}_P{}_k{}".format(egno, nx, ny, T, nr, k), m,
               bounds)
    assert all(m[key] <= bounds[key] for key in m), m


def test_fp64_slabs_generic_x_kernel(native, parity_log, monkeypatch):
    """The generic runtime-radix x kernel's slab phases in fp64 (PDHG_XT64=0: 8 columns per block at nx = 512)."""
    monkeypatch.setenv("PDHG_XT64", "0")
    P = make_problem(2, 2, 512, 256, 7, 0.0)
    st, st_ref, got, want = _run_pair(P, 3, 1, 6, {"f64_xt": 0})
    m = _metrics(st, st_ref, got, want)
    parity_log("test_fp64_slabs_generic_x_kernel", "e2_512x256_T7_P3", m, {key: TOL for key in m})
    assert all(v <= TOL for v in m.values()), m


@pytest.mark.parametrize("nx,ny,T,nr", [(512, 2048, 16, 2), (512, 2048, 9, 3), (64, 8192, 8, 2)],
                         ids=["T16_P2", "T9_P3", "ny8192_T8_P2"])
def test_fp64_slabs_fused_residual(native, parity_log, monkeypatch, nx, ny, T, nr):
    """The fp64 fused sweep (k_dual_lds_2d<.., double, 2> forming the next residual, k_res_fwdy_fused_2d on
    half-tile tasks) inside t-slabs: the halo launch of row 0, the last row completed from the next slab's
    rho row 0 -- against the fused single fp64 context."""
    monkeypatch.setenv("PDHG_FUSE_RES", "1")
    P = make_problem(2, 2, nx, ny, T, 0.0)
    st, st_ref, got, want = _run_pair(P, nr, 1, 6, {"fused_residual": 1, "res64": 1 if ny < 8192 else 0})
    m = _metrics(st, st_ref, got, want)
    bounds = {key: TOL for key in m}
    parity_log("test_fp64_slabs_fused_residual", "e2_{}x{}_T{}_P{}".format(nx, ny, T, nr), m, bounds)
    assert all(m[key] <= bounds[key] for key in m), m


@pytest.mark.parametrize("egno", [2, 3])
def test_fp64_slab_eps_one_step_vs_oracle(native, parity_log, egno):
    """epsl = 0.1 from the seeded rough state through the fp64 t-slab phases (4 slabs of 4 rows) for one
    iteration against the fp64 oracle: the fixed 1e-9 of the fp64 single context (no float32 escape)."""
    import torch
    from pdhg_amd.slab import LocalComm, SlabContext, SlabRunner, join_state, slab_bounds, split_state
    nx, ny, T, nr = 512, 512, 16, 4
    P = make_problem(egno, 2, nx, ny, T, 0.1, seeded=True)
    slabs = [SlabContext(r, nr, T, egno, nx, ny, P["dx"], P["dy"], P["dt"], P["xs"], P["ys"], epsl=0.1,
                         precision="fp64") for r in range(nr)]
    try:
        for s, part in zip(slabs, split_state(P["phi"], P["rho"], P["alp"], slab_bounds(T, nr))):
            s.set_state(*part)
        SlabRunner(slabs, LocalComm(nr)).iterate(1, TAU, SIGMA, -1.0, 1)
        torch.cuda.synchronize()
        got = join_state([s.get_state() for s in slabs])
    finally:
        for s in slabs:
            s.close()
    primal, dual = oracle_fns(P)
    phi_n = primal(P["phi"], P["rho"], 70.0, P["alp"], TAU, P["dt"], P["dsp"], P["fns"], P["fv"], 0.1, P["x_arr"],
                   None)
    rho_n, alp_n = dual(2 * phi_n - P["phi"], P["rho"], 70.0, P["alp"], SIGMA, P["dt"], P["dsp"], 0.1, P["fns"],
                        P["x_arr"], None, 2, -1.0)
    m = {"phi": rel(got[0], phi_n), "rho": rel(got[1], rho_n)}
    for a in range(4):
        if np.linalg.norm(alp_n[a]) > 0:
            m["alp%d" % a] = rel(got[2][a], alp_n[a])
    b = {key: 1e-9 for key in m}
    parity_log("test_fp64_slab_eps_one_step_vs_oracle", "e{}_512x512_T16_P4".format(egno), m, b)
    assert all(m[key] <= b[key] for key in m), (m, b)


def test_fp64_multi_context_small(native, parity_log):
    """The native multi-device context in fp64 (planes moved as doubles between the slabs' buffers) against the
    single fp64 context: 3 slabs on device 0."""
    from pdhg_amd.multi import MultiContext
    from pdhg_amd.context import PDHGContext
    nx, ny, T, nr, n = 4096, 256, 24, 3, 4
    P = make_problem(2, 2, nx, ny, T, 0.0, seeded=False)
    g = P["g"][0]
    ref = PDHGContext(2, 2, nx, ny, T, P["dx"], P["dy"], P["dt"], P["xs"], P["ys"], precision="fp64")
    try:
        ref.init_state(g)
        st_ref = ref.iterate(n, TAU, SIGMA, -1.0, 1)
        want = ref.get_state()
    finally:
        ref.close()
    m_ = MultiContext(2, nx, ny, T, P["dx"], P["dy"], P["dt"], P["xs"], P["ys"], devices=[0] * nr,
                      precision="fp64")
    try:
        assert m_.info("peer_fold") == 0   # gather fold unless PDHG_MULTI_PEER_FOLD=1
        m_.init_state(g)
        st = m_.iterate(n, TAU, SIGMA, -1.0, 1)
        got = m_.get_state()
    finally:
        m_.close()
    assert st["iters_run"] == st_ref["iters_run"] == n
    m = {"phi": rel(got[0], want[0]), "rho": rel(got[1], want[1]),
         "err1": abs(st["err1"] - st_ref["err1"]) / st_ref["err1"]}
    parity_log("test_fp64_multi_context_small", "e2_4096x256_T24_P3", m, {k: TOL for k in m})
    assert all(v <= TOL for v in m.values()), m


def test_fp64_slabs_task_order_spectrum(native, parity_log, monkeypatch):
    """The task-order residual spectrum (PDHG_TC_SPEC=1, the default of windows of >= 100 rows at C3's extents,
    i.e. of 2-slab C3 runs) inside fp64 t-slabs: row-range residual launches and the x kernel's forward-sweep parts
    read it; against the single fp64 context with the same layout, 1e-11."""
    monkeypatch.setenv("PDHG_TC_SPEC", "1")
    P = make_problem(2, 2, 4096, 4096, 8, 0.0)
    st, st_ref, got, want = _run_pair(P, 2, 1, 6, {"tc_spec": 1, "fused_residual": 1})
    m = _metrics(st, st_ref, got, want)
    parity_log("test_fp64_slabs_task_order_spectrum", "e2_4096x4096_T8_P2", m, {key: TOL for key in m})
    assert all(v <= TOL for v in m.values()), m


def test_fp64_slabs_c4_task_order(native, parity_log, monkeypatch):
    """C4's task-order residual spectrum + transpose (to_c4) inside fp64 t-slabs: the fused residual's row-range
    launches (interior rows, then the halo row) transpose their own rows.  C4's 8192^2 plane, 4 rows in 2 slabs,
    epsl = 0.1, from the reference initial state with a seeded rough rho (no window-sized control arrays on the
    host); against the single fp64 context with the same layout, 1e-11 (phi, rho, err1, err2)."""
    import torch
    from pdhg_amd.context import PDHGContext
    from pdhg_amd.slab import LocalComm, SlabContext, SlabRunner, slab_bounds
    monkeypatch.setenv("PDHG_FUSE_RES", "1")
    monkeypatch.setenv("PDHG_SHORT_T", "0")
    G = make_problem(2, 2, 8192, 8192, 1, 0.1, seeded=False)
    T, nr, n = 4, 2, 4
    dt = 1.0 / 40
    g = G["g"][0]
    rho = 70.0 * np.random.default_rng(13).uniform(0.5, 1.5, (T, 8192, 8192))
    ref = PDHGContext(2, 2, 8192, 8192, T, G["dx"], G["dy"], dt, G["xs"], G["ys"], epsl=0.1, precision="fp64")
    try:
        assert ref.path_info("to_c4") == 1
        ref.init_state(g)
        ref.set_state(rho=rho)
        st_ref = ref.iterate(n, TAU, SIGMA, -1.0, 1)
        want = ref.get_state(alp=False)
    finally:
        ref.close()
    slabs = [SlabContext(r, nr, T, 2, 8192, 8192, G["dx"], G["dy"], dt, G["xs"], G["ys"], epsl=0.1, precision="fp64")
             for r in range(nr)]
    try:
        assert all(s.path_info("to_c4") == 1 for s in slabs)
        for s, (j0, j1) in zip(slabs, slab_bounds(T, nr)):
            s.init_state(g)
            s.set_state(rho=rho[j0:j1])
        st = SlabRunner(slabs, LocalComm(nr)).iterate(n, TAU, SIGMA, -1.0, 1)
        torch.cuda.synchronize()
        parts = [s.get_state(alp=False) for s in slabs]
    finally:
        for s in slabs:
            s.close()
    phi = np.concatenate([parts[0][0]] + [p[0][1:] for p in parts[1:]], axis=0)
    rho_s = np.concatenate([p[1] for p in parts], axis=0)
    m = {"phi": rel(phi, want[0]), "rho": rel(rho_s, want[1]),
         "err1": abs(st["err1"] - st_ref["err1"]) / st_ref["err1"],
         "err2": abs(st["err2"] - st_ref["err2"]) / st_ref["err2"]}
    parity_log("test_fp64_slabs_c4_task_order", "e2_8192x8192_T4_P2_eps0.1", m, {k: TOL for k in m})
    assert all(v <= TOL for v in m.values()), m
