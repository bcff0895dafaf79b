"""The t-slab decomposition at the decompositions the BASELINE configs run on 8 GPUs (SURVEY.md 8(e),
BASELINE.json configs[3..4]), on the one-GPU box:

  * C3 on 8 GPUs: T = 200 rows in 8 slabs of 25 (the LDS-DMA x transform inside every slab), nx = 4096;
  * C4 on 8 GPUs: nx = 8192 (the half-real LDS-DMA x transform inside every slab) with slabs of
    16 rows (T = 128, P = 8);
  * epsl = 0.1 (configs 3/4 run with it), two iterations from the reference state;

each driven three ways -- the Python slab driver over LocalComm (pdhg_amd/slab.py, the bench's schedule:
halos and carry planes on a side stream, two column-block parts), the native multi-device context
(pdhg_create_multi, csrc/pdhg_multi.hpp: one host thread, per-slab side streams, per-neighbour events) and,
for C3's rows, eight processes over gloo (DistComm, the one-process-per-GPU form bench.py --gpus 8 runs) --
against the single context of the same window (which test_gpu_configs.py pins to the oracle), plus an
epsl = 0.1 one-step slab run against the fp64 oracle itself.  Achieved errors go to parity_log.
The spatial y extent is cut to 256 (512 for the oracle case) so every case fits the test time limit; the
kernels selected along x and t are the ones of the full configs (asserted through pdhg_path_info)."""
import os

import numpy as np
import pytest

from _problems import device_ctx, make_problem, oracle_fns, rel

pytestmark = pytest.mark.gpu

TAU, SIGMA = 0.1 / 1.5, 0.1 * 1.5
K32 = 4.0

DECOMP = {
    # name: (egno, nx, ny, T, P, epsl, iterations, expected slab path); from the reference initial state
    # (init_state: phi = g, rho = 70, alp = 0), whose first primal update is zero, so iteration 2 is the
    # first to exercise every phase
    "c3_p8": (2, 4096, 256, 200, 8, 0.0, 4, {"fast_xt": 4}),
    "c3_p8_eps": (2, 4096, 256, 200, 8, 0.1, 2, {"fast_xt": 4}),
    "c4_p8": (2, 8192, 256, 128, 8, 0.0, 4, {"fast_xt": 5, "half_real": 1}),
    "c4_p8_eps": (2, 8192, 256, 128, 8, 0.1, 2, {"fast_xt": 5, "half_real": 1}),
}
# bounds against the single context: fp32 rounding of another association of the same sums (the
# distributed t-solve) for epsl = 0; with epsl = 0.1 from the rough state the explicit sigma*epsl*Lap(phi_bar)
# term amplifies that phi_bar rounding ~5e5-fold into rho (test_gpu_configs.py docstring)
BOUNDS = {0.0: {"phi": 2e-5, "rho": 2e-4, "alp": 2e-4}, 0.1: {"phi": 2e-5, "rho": 2e-3, "alp": 2e-2}}
# fp64 (the reference's arithmetic, jaxsrc/update_fns_in_pdhg.py:10): the same decomposition in double, against
# the single fp64 context -- the distributed t-solve's other association of the carry sums rounds in the last
# bits only
BOUNDS64 = {0.0: {"phi": 1e-12, "rho": 1e-12, "alp": 1e-12}, 0.1: {"phi": 1e-12, "rho": 1e-12, "alp": 1e-12}}
# fp64 slab kernels: the fp64 x transform with its slab phases (kernels_xt_f64.hpp; half-real at nx = 8192)
PATH64 = {4096: {"f64_xt": 1}, 8192: {"f64_xt": 1, "half_real": 1}}
CASES = [(n, "fp32") for n in DECOMP] + [(n, "fp64") for n in DECOMP]
IDS = ["{}@{}".format(n, p) for n, p in CASES]
# The default tier runs the bench's driver in the arithmetic it is run in (SlabRunner, fp64, at both configs' own
# epsl = 0.1 decompositions) plus the other driver once (the multi-device context at C4's, fp64; its fp32 form is
# held to the single context by test_gpu_multi.py); the full cross product is the extended tier (PDHG_TESTS=full)
KEEP = {"slabrunner": {("c3_p8_eps", "fp64"), ("c4_p8_eps", "fp64")},
        "multi": {("c4_p8_eps", "fp64")}}


def _cases(driver):
    return [c if c in KEEP[driver] else pytest.param(*c, marks=pytest.mark.extended) for c in CASES]


def _grid(egno, nx, ny, T, epsl):
    """make_problem's grid, spacings and g without the window-sized state arrays (the reference initial
    state is formed on the device by init_state)."""
    G = make_problem(egno, 2, nx, ny, 1, epsl, seeded=False)
    G.update(T=T, dt=1.0 / max(T, 40), g=G["g"][0])
    return G


def _single(P, n, prec="fp32"):
    ref = device_ctx(P, prec)
    try:
        ref.init_state(P["g"])
        st = ref.iterate(n, TAU, SIGMA, -1.0, 1)
        return st, ref.get_state()
    finally:
        ref.close()


def _check(name, got, want, st, st_ref, epsl, parity_log, driver, prec="fp32"):
    b = (BOUNDS64 if prec == "fp64" else BOUNDS)[epsl]
    m = {"phi": rel(got[0], want[0]), "rho": rel(got[1], want[1]),
         "alp": rel(np.stack(got[2]), np.stack(want[2])),
         "err1": abs(st["err1"] - st_ref["err1"]) / st_ref["err1"]}
    bounds = dict(b, err1=(1e-3 if epsl == 0.0 else 1e-2) if prec == "fp32" else 1e-12)
    parity_log("test_gpu_decomp", "{}/{}@{}".format(name, driver, prec), m, bounds)
    assert all(m[k] <= bounds[k] for k in m), (name, driver, m, bounds)


@pytest.mark.parametrize("name,prec", _cases("slabrunner"), ids=IDS)
def test_slab_runner_at_config_decomposition(native, name, prec, parity_log):
    import torch
    from pdhg_amd.slab import LocalComm, SlabContext, SlabRunner, join_state
    egno, nx, ny, T, nr, epsl, n, path = DECOMP[name]
    if prec == "fp64":
        path = PATH64[nx]
    P = _grid(egno, nx, ny, T, epsl)
    st_ref, want = _single(P, n, prec)
    slabs = [SlabContext(r, nr, T, egno, nx, ny, P["dx"], P["dy"], P["dt"], P["xs"], P["ys"], epsl=epsl,
                         precision=prec) for r in range(nr)]
    try:
        for s in slabs:
            for k, v in path.items():
                assert s.path_info(k) == v, (name, k, s.path_info(k), v)
        for s in slabs:
            s.init_state(P["g"])
        runner = SlabRunner(slabs, LocalComm(nr))   # the bench's schedule: overlap, neighbour carries, 2 parts
        assert runner.parts == 2 and runner.side is not None
        st = runner.iterate(n, TAU, SIGMA, -1.0, 1)
        torch.cuda.synchronize()
        got = join_state([s.get_state() for s in slabs])
    finally:
        for s in slabs:
            s.close()
    assert st["iters"] == st_ref["iters_run"] == n
    _check(name, got, want, st, st_ref, epsl, parity_log, "slabrunner", prec)


@pytest.mark.parametrize("name,prec", _cases("multi"), ids=IDS)
def test_multi_context_at_config_decomposition(native, name, prec, parity_log):
    from pdhg_amd.multi import MultiContext
    egno, nx, ny, T, nr, epsl, n, _ = DECOMP[name]
    P = _grid(egno, nx, ny, T, epsl)
    st_ref, want = _single(P, n, prec)
    m = MultiContext(egno, nx, ny, T, P["dx"], P["dy"], P["dt"], P["xs"], P["ys"], devices=[0] * nr, epsl=epsl,
                     precision=prec)
    try:
        assert m.info("ndev") == nr and m.info("parts") == 2
        assert all(m.info("device:%d" % r) == 0 for r in range(nr))   # each slab computes on its listed device
        m.init_state(P["g"])
        m.profile(True)
        st = m.iterate(n, TAU, SIGMA, -1.0, 1)
        ph = m.phase_ms(reset=False)
        got = m.get_state()
    finally:
        m.close()
    assert st["iters_run"] == st_ref["iters_run"] == n
    assert ph.get("step", 0.0) > 0.0 and all(v >= 0.0 for v in ph.values()), ph
    _check(name, got, want, st, st_ref, epsl, parity_log, "multi", prec)


def test_multi_handle_is_not_a_context(native):
    """A pdhg_multi* passed to a pdhg_ctx entry point (and the reverse) is rejected, not dereferenced."""
    import ctypes
    from pdhg_amd import _native as N
    from pdhg_amd.multi import MultiContext
    P = make_problem(1, 2, 512, 256, 4, 0.0)
    m = MultiContext(1, 512, 256, 4, P["dx"], P["dy"], P["dt"], P["xs"], P["ys"], devices=[0, 0])
    ctx = device_ctx(P, "fp32")
    lib = N.load()
    try:
        st = N.pdhg_stats()
        assert lib.pdhg_iterate(m._h, 1, TAU, SIGMA, -1.0, 1, ctypes.byref(st)) == N.PDHG_ERR_ARG
        assert lib.pdhg_update_primal(m._h, TAU) == N.PDHG_ERR_ARG
        assert lib.pdhg_destroy(m._h) == N.PDHG_ERR_ARG
        assert lib.pdhg_multi_iterate(ctx._h, 1, TAU, SIGMA, -1.0, 1, ctypes.byref(st)) == N.PDHG_ERR_ARG
        assert lib.pdhg_multi_destroy(ctx._h) == N.PDHG_ERR_ARG
        assert not hasattr(m, "update_primal")   # MultiContext exposes only the whole-window calls
    finally:
        ctx.close()
        m.close()


@pytest.mark.parametrize("egno", [2, 3])
def test_slab_eps_one_step_vs_oracle(native, parity_log, egno):
    """epsl = 0.1 through the t-slab phases (4 slabs of 4 rows, fused residual off / on as selected, seeded
    rough state) for one iteration against the fp64 oracle: bounds as test_gpu_configs.test_one_step_eps --
    the larger of the seeded-state bounds and K32 x the float32 oracle's own distance.  egno 3: bc (1, 0), the
    DCT x transform's slab phases (jaxsrc/set_fns.py:96-111, utils/utils_precond.py:159-174)."""
    import torch
    from pdhg_amd.slab import LocalComm, SlabContext, SlabRunner, join_state, slab_bounds, split_state
    nx, ny, T, nr = 512, 512, 16, 4
    P = make_problem(egno, 2, nx, ny, T, 0.1, seeded=True)
    f = np.float32
    phi0, rho0 = P["phi"].astype(f).astype(np.float64), P["rho"].astype(f).astype(np.float64)
    alp0 = tuple(a.astype(f).astype(np.float64) for a in P["alp"])
    slabs = [SlabContext(r, nr, T, egno, nx, ny, P["dx"], P["dy"], P["dt"], P["xs"], P["ys"], epsl=0.1)
             for r in range(nr)]
    try:
        for s, part in zip(slabs, split_state(phi0, rho0, alp0, slab_bounds(T, nr))):
            s.set_state(*part)
        SlabRunner(slabs, LocalComm(nr)).iterate(1, TAU, SIGMA, -1.0, 1)
        torch.cuda.synchronize()
        got = join_state([s.get_state() for s in slabs])
    finally:
        for s in slabs:
            s.close()
    primal, dual = oracle_fns(P)

    def step(phi, rho, alp, x_arr):
        phi_n = primal(phi, rho, 70.0, alp, TAU, P["dt"], P["dsp"], P["fns"], P["fv"], 0.1, x_arr, None)
        rho_n, alp_n = dual(2 * phi_n - phi, rho, 70.0, alp, SIGMA, P["dt"], P["dsp"], 0.1, P["fns"], x_arr, None,
                            2, -1.0)
        return phi_n, rho_n, alp_n
    o = step(phi0, rho0, alp0, P["x_arr"])
    p32 = step(phi0.astype(f), rho0.astype(f), tuple(a.astype(f) for a in alp0), P["x_arr"].astype(f))
    m = {"phi": rel(got[0], o[0]), "rho": rel(got[1], o[1])}
    b = {"phi": max(1e-5, K32 * rel(p32[0], o[0])), "rho": max(2e-4, K32 * rel(p32[1], o[1]))}
    for a in range(4):
        m["alp%d" % a] = rel(got[2][a], o[2][a])
        b["alp%d" % a] = max(1e-3, K32 * rel(p32[2][a], o[2][a]))
    parity_log("test_slab_eps_one_step_vs_oracle", "e{}_512x512_T16_P4".format(egno), m, b)
    assert all(m[k] <= b[k] for k in m), (m, b)


def _gloo_worker(rank, world, port, paths, d, out):
    import sys
    sys.path[:0] = paths
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:{}".format(port), rank=rank, world_size=world)
    try:
        from pdhg_amd.slab import DistComm, SlabContext, SlabRunner, slab_bounds
        meta = np.load(os.path.join(d, "meta.npy"))
        egno, nx, ny, T, n = (int(v) for v in meta)
        P = _grid(egno, nx, ny, T, 0.0)
        j0, j1 = slab_bounds(T, world)[rank]
        s = SlabContext(rank, world, T, egno, nx, ny, P["dx"], P["dy"], P["dt"], P["xs"], P["ys"])
        s.init_state(P["g"])
        st = SlabRunner([s], DistComm()).iterate(n, TAU, SIGMA, -1.0, 1)
        torch.cuda.synchronize()
        phi, rho, _ = s.get_state()
        # phi row 0 of a slab r > 0 is its halo (the previous slab's phi_bar row, join_state drops it):
        # compare the rows the slab owns
        h = 0 if rank == 0 else 1
        phi_r = np.load(os.path.join(d, "phi.npy"), mmap_mode="r")[j0 + h:j1 + 1]
        rho_r = np.load(os.path.join(d, "rho.npy"), mmap_mode="r")[j0:j1]
        out.put((rank, int(st["iters"]), float(st["err1"]), rel(phi[h:], phi_r), rel(rho, rho_r)))
        s.close()
    finally:
        dist.destroy_process_group()


def test_tslab_distcomm_gloo_p8(native, tmp_path, parity_log):
    """Eight processes on the one GPU over gloo (DistComm: halos point to point, neighbour carry planes,
    allreduces, as bench.py --gpus 8 runs them over RCCL), C3's decomposition along t (8 slabs of 25 rows,
    the LDS-DMA x transform at nx = 4096, y cut to 256): every rank's rows against the single context."""
    import socket
    import torch.multiprocessing as mp
    egno, nx, ny, T, n, world = 2, 4096, 256, 200, 3, 8
    P = _grid(egno, nx, ny, T, 0.0)
    st_ref, (phi_r, rho_r, _) = _single(P, n)
    np.save(tmp_path / "meta.npy", np.array([egno, nx, ny, T, n]))
    np.save(tmp_path / "phi.npy", phi_r)
    np.save(tmp_path / "rho.npy", rho_r)
    del phi_r, rho_r, P
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    here = os.path.dirname(os.path.abspath(__file__))
    paths = [os.path.abspath(os.path.join(here, p)) for p in ("../pdhg-optimal-control_amd", "../oracle", ".")]
    q = mp.get_context("spawn").Queue()
    mp.spawn(_gloo_worker, args=(world, port, paths, str(tmp_path), q), nprocs=world, join=True)
    res = sorted(q.get() for _ in range(world))
    worst = {"phi": max(r[3] for r in res), "rho": max(r[4] for r in res),
             "err1": max(abs(r[2] - st_ref["err1"]) / st_ref["err1"] for r in res)}
    parity_log("test_tslab_distcomm_gloo_p8", "c3_4096x256_T200_P8", worst, {"phi": 2e-5, "rho": 2e-4, "err1": 1e-3})
    assert all(r[1] == n for r in res), res
    assert worst["phi"] < 2e-5 and worst["rho"] < 2e-4 and worst["err1"] < 1e-3, (worst, res)
