"""x-slab decomposition on the GPU: P x-slab contexts on one device, exchanging halo
rows and the transposed spectrum through LocalComm, must reproduce the single-context iteration
(pdhg_iterate) of the same window -- same state after n outer iterations within fp32 rounding, same
error history and stop decisions -- for T = 1 (the reference's marching default) and longer windows,
the x-transform kernels x-slab windows select (one-row, single-role, half-real, generic) and k = 1 / k > 1.
The single-context path is itself pinned to the oracle by test_gpu_parity.py; one case here also
checks the x-slab state against the fp64 oracle directly.  fp64 x-slabs (the reference's arithmetic,
jaxsrc/update_fns_in_pdhg.py:10; ny = 2048 / 4096) against the single fp64 context at 1e-11 and the fp64 oracle at
1e-9, incl. the multi-process path over gloo."""
import numpy as np
import pytest

from _problems import make_problem, oracle_fns, rel

pytestmark = pytest.mark.gpu

CASES = [
    # (egno, nx, ny, T, P, k, epsl)
    (1, 512, 256, 1, 2, 1, 0.0),     # T = 1 (marching default): k_precond_x_t1_2d
    (2, 512, 256, 1, 4, 1, 0.1),
    (1, 512, 256, 3, 2, 3, 0.0),     # two buffer sets (rho_alp_iters > 1), T = 3
    (2, 512, 512, 2, 1, 1, 0.0),     # one slab: the halo ring is the slab itself
    (1, 512, 256, 1, 8, 1, 0.0),     # 64-row slabs
    (2, 4096, 256, 1, 2, 1, 0.0),    # nx = 4096, T = 1: k_precond_x_t1_2d<4096>
    (2, 8192, 256, 1, 2, 1, 0.0),    # half-real x blocks (C4's nx)
    (1, 256, 256, 2, 2, 1, 0.0),     # generic x kernel (runtime plan)
    (2, 384, 256, 1, 2, 1, 0.0),     # non-power-of-two nx (radix-3 plan), 192-row slabs
    (1, 512, 256, 1, 2, 3, 0.0),     # T = 1 with two buffer sets: the row-per-thread dual's live-row mask
    (2, 512, 256, 2, 4, 1, 0.0),     # T = 2: short-window kernels (single-role x transform, row-per-thread dual)
    (2, 512, 256, 8, 2, 1, 0.0),     # T = 8: 8-row LDS dual, single-role x transform
    # egno 3 (bc (1, 0): Neumann x edges, DCT along x in the generic x kernel on the transposed lines)
    (3, 512, 256, 1, 2, 1, 0.0),
    (3, 256, 256, 2, 4, 1, 0.0),     # the inner slabs exchange with both neighbours, the outer ones replicate
    (3, 384, 256, 1, 2, 3, 0.0),     # non-power-of-two DCT plan, two buffer sets
    (3, 512, 256, 4, 2, 1, 1e-3),    # (epsl = 0.1 diverges in the single context here: NaN within 6 iterations)
]


def _xslabs(P, nranks, k, precision="fp32"):
    from pdhg_amd.xslab import XSlabContext
    return [XSlabContext(r, nranks, P["egno"], P["nx"], P["ny"], P["T"], P["dx"], P["dy"], P["dt"], P["xs"], P["ys"],
                         epsl=P["epsl"], rho_alp_iters=k, precision=precision) for r in range(nranks)]


def _state(slabs):
    from pdhg_amd.xslab import join_rows
    parts = [s.get_state() for s in slabs]
    phi = join_rows(slabs, [p[0] for p in parts])
    rho = join_rows(slabs, [p[1] for p in parts])
    alp = [join_rows(slabs, [p[2][a] for p in parts]) for a in range(4)]
    return phi, rho, alp


@pytest.mark.parametrize("egno,nx,ny,T,nr,k,epsl", CASES,
                         ids=[f"e{c[0]}_{c[1]}x{c[2]}_T{c[3]}_P{c[4]}_k{c[5]}_eps{c[6]}" for c in CASES])
def test_xslabs_match_single_context(native, egno, nx, ny, T, nr, k, epsl):
    import torch
    from pdhg_amd.context import PDHGContext
    from pdhg_amd.xslab import LocalComm, XSlabRunner
    P = make_problem(egno, 2, nx, ny, T, epsl)
    tau, sigma, n = 0.1 / 1.5, 0.1 * 1.5, 6
    ref = PDHGContext(egno, 2, nx, ny, T, P["dx"], P["dy"], P["dt"], P["xs"], P["ys"], epsl=epsl,
                      precision="fp32", rho_alp_iters=k)
    ref.set_state(P["phi"], P["rho"], P["alp"])
    st_ref = ref.iterate(n, tau, sigma, -1.0, k)
    phi_r, rho_r, alp_r = ref.get_state()

    slabs = _xslabs(P, nr, k)
    for s in slabs:
        assert s.nloc == nx // nr and s.nx == s.nloc + 16
        s.set_global_state(P["phi"], P["rho"], P["alp"])
    runner = XSlabRunner(slabs, LocalComm(nr))
    st = runner.iterate(n, tau, sigma, -1.0, k)
    torch.cuda.synchronize()
    phi_s, rho_s, alp_s = _state(slabs)
    assert not st_ref["nan_seen"] and not st["nan_seen"]
    assert st["iters"] == st_ref["iters_run"] == n
    assert st["inner_total"] == st_ref["inner_total"]
    assert rel(phi_s, phi_r) < 2e-5
    assert rel(rho_s, rho_r) < 2e-4
    assert rel(np.stack(alp_s), np.stack(alp_r)) < 2e-4
    assert abs(st["err1"] - st_ref["err1"]) <= 1e-4 * st_ref["err1"]
    assert abs(st["err2"] - st_ref["err2"]) <= 1e-4 * st_ref["err2"]
    for s in slabs:
        s.close()
    ref.close()


def test_xslab_vs_oracle(native):
    """Two x-slabs, 10 iterations from the seeded state, against the fp64 oracle (the north-star bound)."""
    import torch
    from pdhg_amd.xslab import LocalComm, XSlabRunner
    P = make_problem(2, 2, 512, 256, 1, 0.0)
    tau, sigma, n = 0.1 / 1.5, 0.1 * 1.5, 10
    primal, dual = oracle_fns(P)
    phi, rho, alp = P["phi"], P["rho"], P["alp"]
    for _ in range(n):
        phi_n = primal(phi, rho, 70.0, alp, tau, P["dt"], P["dsp"], P["fns"], P["fv"], P["epsl"], P["x_arr"], None)
        rho, alp = dual(2 * phi_n - phi, rho, 70.0, alp, sigma, P["dt"], P["dsp"], P["epsl"], P["fns"], P["x_arr"],
                        None, 2, -1.0)
        phi = phi_n
    slabs = _xslabs(P, 2, 1)
    for s in slabs:
        s.set_global_state(P["phi"], P["rho"], P["alp"])
    XSlabRunner(slabs, LocalComm(2)).iterate(n, tau, sigma, -1.0, 1)
    torch.cuda.synchronize()
    phi_s, rho_s, _ = _state(slabs)
    assert rel(phi_s, phi) < 1e-5
    assert rel(rho_s, rho) < 1e-5


def test_xslab_convergence_stop(native):
    """The global stop decision (all-reduced err1/err2) ends every slab at the single context's iteration."""
    import torch
    from pdhg_amd.context import PDHGContext
    from pdhg_amd.xslab import LocalComm, XSlabRunner
    P = make_problem(1, 2, 512, 256, 1, 0.0, seeded=False)
    tau, sigma, eps = 0.1 / 1.5, 0.1 * 1.5, 1e-3
    ref = PDHGContext(1, 2, 512, 256, 1, P["dx"], P["dy"], P["dt"], P["xs"], P["ys"], precision="fp32")
    ref.set_state(P["phi"], P["rho"], P["alp"])
    st_ref = ref.iterate(3000, tau, sigma, eps, 1)
    assert st_ref["status"] == 1
    slabs = _xslabs(P, 4, 1)
    for s in slabs:
        s.init_global_state(P["g"])
    st = XSlabRunner(slabs, LocalComm(4)).iterate(3000, tau, sigma, eps, 1)
    torch.cuda.synchronize()
    assert st["status"] == 1
    assert abs(st["iters"] - st_ref["iters_run"]) <= 1
    assert rel(_state(slabs)[0], ref.get_state()[0]) < 1e-4


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
def test_multi_step_xslab(native, prec):
    """Window marching over x-slabs (T = 1 windows, warm starts) against the single-context marching (fp64: the
    reference's arithmetic at C2's ny, the same stop iterations and states to 1e-10)."""
    import torch
    from pdhg_amd.context import PDHGContext
    from pdhg_amd.xslab import LocalComm, XSlabRunner, multi_step_xslab
    ny = 2048 if prec == "fp64" else 256
    P = make_problem(2, 2, 512, ny, 1, 0.0, seeded=False)
    nt, eps, s_par = 4, 1e-3, 0.1
    slabs = _xslabs(P, 2, 1, prec)
    res, errs = multi_step_xslab(XSlabRunner(slabs, LocalComm(2)), P["g"], nt, 70.0, stepsz_param=s_par,
                                 N_maxiter=3000, eps=eps)
    torch.cuda.synchronize()
    phi_x = np.concatenate([r[1] for r in res], axis=1)
    rho_x = np.concatenate([r[2] for r in res], axis=1)
    assert phi_x.shape == (nt, 512, ny) and rho_x.shape == (nt - 1, 512, ny)
    # single context, same marching (utils_pdhg_solver.py:193-206)
    ref = PDHGContext(2, 2, 512, ny, 1, P["dx"], P["dy"], P["dt"], P["xs"], P["ys"], precision=prec)
    phi0 = np.repeat(P["g"], 2, axis=0)
    rho0, alp0 = np.full((1, 512, ny), 70.0), tuple(np.zeros((1, 512, ny, 2)) for _ in range(4))
    phis, rhos, iters = [], [], []
    for i in range(nt - 1):
        ref.set_state(phi0, rho0, alp0)
        st = ref.iterate(3000, s_par / 1.5, s_par * 1.5, eps, 1)
        assert st["status"] == 1
        iters.append(st["iters_run"])
        phi_c, rho_c, alp_c = ref.get_state()
        phis.append(phi_c[:-1] if i < nt - 2 else phi_c)
        rhos.append(rho_c)
        phi0, rho0, alp0 = phi0 + (phi_c[-1:] - phi0[0:1]), rho_c, alp_c
    tol_phi, tol_rho = (1e-10, 1e-10) if prec == "fp64" else (1e-4, 1e-3)
    assert rel(phi_x, np.concatenate(phis)) < tol_phi
    assert rel(rho_x, np.concatenate(rhos)) < tol_rho
    if prec == "fp64":
        assert res[0][0] == max(iters), (res[0][0], iters)
    for s in slabs:
        s.close()
    ref.close()


def test_xslab_rejects_unsupported(native):
    from pdhg_amd import _native as N
    from pdhg_amd.xslab import XSlabContext
    P = make_problem(1, 2, 512, 256, 1, 0.0)
    with pytest.raises(N.PDHGError):      # 512 rows do not split into 3 slabs
        XSlabContext(0, 3, 1, 512, 256, 1, P["dx"], P["dy"], P["dt"], P["xs"], P["ys"])
    with pytest.raises(N.PDHGError):      # 4-row slabs (not a multiple of 8)
        XSlabContext(0, 128, 1, 512, 256, 1, P["dx"], P["dy"], P["dt"], P["xs"], P["ys"])
    with pytest.raises(N.PDHGError):      # fp64 needs the fp64 row kernels (ny = 2048 / 4096)
        XSlabContext(0, 2, 1, 512, 256, 1, P["dx"], P["dy"], P["dt"], P["xs"], P["ys"], precision="fp64")


FP64_CASES = [
    # (egno, nx, ny, T, P, k, epsl, expected path_info of the slabs)
    (2, 512, 2048, 1, 2, 1, 0.0, {"t1_xt64": 1, "res64": 1, "dual64": 1}),   # C2's ny, the marching default T = 1
    (2, 512, 2048, 1, 4, 1, 0.1, {"t1_xt64": 1}),
    (1, 256, 2048, 1, 2, 1, 0.0, {"t1_xt64": 0, "f64_xt": 0}),              # generic x kernel (nx = 256)
    (1, 512, 2048, 1, 2, 3, 0.0, {"t1_xt64": 1}),                           # two buffer sets, k = 3
    (2, 512, 2048, 3, 2, 3, 0.0, {"f64_xt": 1}),                            # fp64 x kernel (nx = 512, B = 2)
    (2, 2048, 2048, 2, 4, 1, 0.0, {"f64_xt": 1}),                           # C2's nx: b' in registers
    (2, 4096, 2048, 1, 2, 1, 0.0, {"t1_xt64": 1}),                          # C3's nx, one-row x kernel
    (2, 512, 4096, 4, 2, 1, 0.0, {"f64_xt": 1, "fast_dual": 8}),            # ny = 4096, 8-row LDS dual
    (3, 512, 2048, 1, 2, 1, 0.0, {"f64_xt": 0}),                            # egno 3: Neumann x edges, DCT
    (3, 256, 2048, 2, 4, 1, 0.0, {"f64_xt": 0}),
]


@pytest.mark.parametrize("egno,nx,ny,T,nr,k,epsl,path", FP64_CASES,
                         ids=[f"e{c[0]}_{c[1]}x{c[2]}_T{c[3]}_P{c[4]}_k{c[5]}_eps{c[6]}" for c in FP64_CASES])
def test_fp64_xslabs_match_single_context(native, parity_log, egno, nx, ny, T, nr, k, epsl, path):
    """fp64 x-slabs against the single fp64 context: the same kernels on the same rows (the x transform on the
    transposed whole lines), so the states agree to the summation order of the stop sums: 1e-11."""
    import torch
    from pdhg_amd.context import PDHGContext
    from pdhg_amd.xslab import LocalComm, XSlabRunner
    P = make_problem(egno, 2, nx, ny, T, epsl)
    tau, sigma, n = 0.1 / 1.5, 0.1 * 1.5, 6
    ref = PDHGContext(egno, 2, nx, ny, T, P["dx"], P["dy"], P["dt"], P["xs"], P["ys"], epsl=epsl,
                      precision="fp64", rho_alp_iters=k)
    try:
        ref.set_state(P["phi"], P["rho"], P["alp"])
        st_ref = ref.iterate(n, tau, sigma, -1.0, k)
        phi_r, rho_r, alp_r = ref.get_state()
    finally:
        ref.close()
    slabs = _xslabs(P, nr, k, "fp64")
    try:
        for s in slabs:
            for key, v in path.items():
                assert s.path_info(key) == v, (key, s.path_info(key), v)
            s.set_global_state(P["phi"], P["rho"], P["alp"])
        runner = XSlabRunner(slabs, LocalComm(nr))
        assert runner.b[0]["send"].dtype == torch.float64
        st = runner.iterate(n, tau, sigma, -1.0, k)
        torch.cuda.synchronize()
        phi_s, rho_s, alp_s = _state(slabs)
    finally:
        for s in slabs:
            s.close()
    assert not st_ref["nan_seen"] and not st["nan_seen"]
    assert st["iters"] == st_ref["iters_run"] == n
    assert st["inner_total"] == st_ref["inner_total"]
    m = {"phi": rel(phi_s, phi_r), "rho": rel(rho_s, rho_r), "alp": rel(np.stack(alp_s), np.stack(alp_r)),
         "err1": abs(st["err1"] - st_ref["err1"]) / st_ref["err1"],
         "err2": abs(st["err2"] - st_ref["err2"]) / st_ref["err2"]}
    b = {key: 1e-11 for key in m}
    parity_log("test_fp64_xslabs_match_single_context", f"e{egno}_{nx}x{ny}_T{T}_P{nr}_k{k}_eps{epsl}", m, b)
    assert all(m[key] <= b[key] for key in m), m


@pytest.mark.parametrize("egno,epsl,n", [(2, 0.0, 10), (2, 0.1, 1), (3, 0.0, 10)])
def test_fp64_xslab_vs_oracle(native, parity_log, egno, epsl, n):
    """fp64 x-slabs (P = 4, T = 1) from the seeded state against the fp64 oracle: the fp64 single context's 1e-9."""
    import torch
    from pdhg_amd.xslab import LocalComm, XSlabRunner
    P = make_problem(egno, 2, 512, 2048, 1, epsl)
    tau, sigma = 0.1 / 1.5, 0.1 * 1.5
    primal, dual = oracle_fns(P)
    phi, rho, alp = P["phi"], P["rho"], P["alp"]
    for _ in range(n):
        phi_n = primal(phi, rho, 70.0, alp, tau, P["dt"], P["dsp"], P["fns"], P["fv"], P["epsl"], P["x_arr"], None)
        rho, alp = dual(2 * phi_n - phi, rho, 70.0, alp, sigma, P["dt"], P["dsp"], P["epsl"], P["fns"], P["x_arr"],
                        None, 2, -1.0)
        phi = phi_n
    slabs = _xslabs(P, 4, 1, "fp64")
    try:
        for s in slabs:
            s.set_global_state(P["phi"], P["rho"], P["alp"])
        XSlabRunner(slabs, LocalComm(4)).iterate(n, tau, sigma, -1.0, 1)
        torch.cuda.synchronize()
        phi_s, rho_s, alp_s = _state(slabs)
    finally:
        for s in slabs:
            s.close()
    m = {"phi": rel(phi_s, phi), "rho": rel(rho_s, rho)}
    for a in range(4):
        if np.linalg.norm(alp[a]) > 0:
            m["alp%d" % a] = rel(alp_s[a], alp[a])
    b = {key: 1e-9 for key in m}
    parity_log("test_fp64_xslab_vs_oracle", f"e{egno}_512x2048_T1_P4_eps{epsl}_n{n}", m, b)
    assert all(m[key] <= b[key] for key in m), m


def _dist_worker(rank, world, port, paths, out, prec="fp32"):
    import sys
    sys.path[:0] = paths
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:{}".format(port), rank=rank, world_size=world)
    try:
        from pdhg_amd.context import PDHGContext
        from pdhg_amd.xslab import DistComm, XSlabContext, XSlabRunner
        ny = 2048 if prec == "fp64" else 256
        P = make_problem(2, 2, 512, ny, 1, 0.0)
        tau, sigma, n = 0.1 / 1.5, 0.1 * 1.5, 6
        ref = PDHGContext(2, 2, 512, ny, 1, P["dx"], P["dy"], P["dt"], P["xs"], P["ys"], precision=prec)
        ref.set_state(P["phi"], P["rho"], P["alp"])
        st_ref = ref.iterate(n, tau, sigma, -1.0, 1)
        phi_r = ref.get_state()[0]
        ref.close()
        s = XSlabContext(rank, world, 2, 512, ny, 1, P["dx"], P["dy"], P["dt"], P["xs"], P["ys"], precision=prec)
        s.set_global_state(P["phi"], P["rho"], P["alp"])
        st = XSlabRunner([s], DistComm()).iterate(n, tau, sigma, -1.0, 1)
        torch.cuda.synchronize()
        phi_s = s.live_rows(s.get_state()[0])
        e = rel(phi_s, phi_r[:, s.x0:s.x0 + s.nloc])
        out.put((rank, st["iters"], st_ref["iters_run"], e, abs(st["err1"] - st_ref["err1"]) / st_ref["err1"]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
def test_xslab_distcomm_gloo_rehearsal(native, prec):
    """The multi-process path (DistComm: allgather / all-to-all / allreduce over torch.distributed) with two
    ranks on the one GPU over gloo (host-staged): each rank's rows match the single context (fp64: 1e-11)."""
    import os
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    here = os.path.dirname(os.path.abspath(__file__))
    paths = [os.path.join(here, "..", "pdhg-optimal-control_amd"), os.path.join(here, "..", "oracle"), here]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.spawn(_dist_worker, args=(2, port, [os.path.abspath(p) for p in paths], q, prec), nprocs=2, join=True)
    res = sorted(q.get() for _ in range(2))
    tol_phi, tol_err = (1e-11, 1e-11) if prec == "fp64" else (2e-5, 1e-4)
    for rank, it, it_ref, e_phi, e_err1 in res:
        assert it == it_ref == 6, res
        assert e_phi < tol_phi and e_err1 < tol_err, res
