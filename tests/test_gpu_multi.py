"""Multi-device context (include/pdhg.h pdhg_create_multi, csrc/pdhg_multi.hpp): one host
thread driving P t-slabs with device-to-device plane copies and fixed-order sum folds.  On the one-GPU box the
device list repeats device 0 (the same code path as distinct devices, with same-device copies instead of
peer copies).  It must reproduce the single-context iteration (pdhg_iterate) of the same window within fp32
rounding, and the Python slab driver (pdhg_amd.slab, LocalComm) closely: same kernels, same exchanges."""
import numpy as np
import pytest

from _problems import make_problem, rel

pytestmark = pytest.mark.gpu

CASES = [
    # (egno, nx, ny, T, P, k)
    (1, 512, 256, 6, 2, 1),
    (2, 512, 256, 7, 3, 1),
    (2, 512, 256, 40, 4, 1),     # 10-row slabs: neighbour-only carries for the short-range modes
    (1, 512, 256, 5, 5, 3),      # one-row slabs, dual sub-iterations with early exit
    (2, 4096, 256, 50, 2, 1),    # 25-row slabs: the LDS-DMA x transform
    (3, 512, 256, 9, 3, 1),      # egno 3: bc (1, 0), the generic DCT x kernel's slab phases
]


# the peer-pointer fold (opt-in, PDHG_MULTI_PEER_FOLD=1) on the first case by default, on all in the extended tier
PARAMS = [pytest.param(*c, f, marks=() if (f == "0" or i == 0) else (pytest.mark.extended,))
          for i, c in enumerate(CASES) for f in ("1", "0")]
IDS = [f"e{c[0]}_{c[1]}x{c[2]}_T{c[3]}_P{c[4]}_k{c[5]}-{'peer' if f == '1' else 'gather'}_fold"
       for c in CASES for f in ("1", "0")]


@pytest.mark.parametrize("egno,nx,ny,T,nr,k,fold", PARAMS, ids=IDS)
def test_multi_matches_single_context(native, egno, nx, ny, T, nr, k, fold, monkeypatch):
    """fold 1: every slab folds the P sum vectors itself from their owners' buffers (peer pointers; on one GPU
    local ones), alternating contribution buffers; fold 0: gather on slab 0, fold, copy back."""
    import torch
    monkeypatch.setenv("PDHG_MULTI_PEER_FOLD", fold)
    from pdhg_amd.context import PDHGContext
    from pdhg_amd.multi import MultiContext
    from pdhg_amd.slab import LocalComm, SlabContext, SlabRunner, join_state, slab_bounds, split_state
    P = make_problem(egno, 2, nx, ny, T, 0.0)
    tau, sigma, n = 0.1 / 1.5, 0.1 * 1.5, 6
    ref = PDHGContext(egno, 2, nx, ny, T, P["dx"], P["dy"], P["dt"], P["xs"], P["ys"], epsl=0.0,
                      precision="fp32", rho_alp_iters=k)
    ref.set_state(P["phi"], P["rho"], P["alp"])
    st_ref = ref.iterate(n, tau, sigma, -1.0, k)
    phi_r, rho_r, alp_r = ref.get_state()
    ref.close()

    m = MultiContext(egno, nx, ny, T, P["dx"], P["dy"], P["dt"], P["xs"], P["ys"], devices=[0] * nr,
                     epsl=0.0, rho_alp_iters=k)
    assert m.info("ndev") == nr
    assert m.info("peer_fold") == int(fold)
    assert [m.info("rows:%d" % i) for i in range(nr)] == [j1 - j0 for j0, j1 in slab_bounds(T, nr)]
    m.set_state(P["phi"], P["rho"], P["alp"])
    st = m.iterate(n, tau, sigma, -1.0, k)
    phi_m, rho_m, alp_m = m.get_state()
    m.close()
    assert st["iters_run"] == st_ref["iters_run"] == n
    assert rel(phi_m, phi_r) < 2e-5
    assert rel(rho_m, rho_r) < 2e-4
    assert rel(np.stack(alp_m), np.stack(alp_r)) < 2e-4
    assert abs(st["err1"] - st_ref["err1"]) <= 1e-3 * st_ref["err1"]
    assert abs(st["err2"] - st_ref["err2"]) <= 1e-3 * st_ref["err2"]

    # the Python driver of the same slabs (serial halos, neighbour exchange): same kernels and exchanges
    slabs = [SlabContext(r, nr, T, egno, nx, ny, P["dx"], P["dy"], P["dt"], P["xs"], P["ys"], epsl=0.0,
                         rho_alp_iters=k) for r in range(nr)]
    for s, part in zip(slabs, split_state(P["phi"], P["rho"], P["alp"], slab_bounds(T, nr))):
        s.set_state(*part)
    SlabRunner(slabs, LocalComm(nr), overlap=False, exchange="neighbour").iterate(n, tau, sigma, -1.0, k)
    torch.cuda.synchronize()
    phi_s, rho_s, _ = join_state([s.get_state() for s in slabs])
    for s in slabs:
        s.close()
    assert rel(phi_m, phi_s) < 1e-6 and rel(rho_m, rho_s) < 1e-6


def test_multi_state_round_trip_and_errors(native):
    from pdhg_amd import _native as N
    from pdhg_amd.multi import MultiContext
    P = make_problem(2, 2, 512, 256, 7, 0.0, seeded=True)
    m = MultiContext(2, 512, 256, 7, P["dx"], P["dy"], P["dt"], P["xs"], P["ys"], devices=[0, 0, 0])
    m.set_state(P["phi"], P["rho"], P["alp"])
    phi, rho, alp = m.get_state()
    f = np.float32
    assert np.array_equal(phi, P["phi"].astype(f).astype(np.float64))
    assert np.array_equal(rho, P["rho"].astype(f).astype(np.float64))
    assert all(np.array_equal(a, b.astype(f).astype(np.float64)) for a, b in zip(alp, P["alp"]))
    m.close()
    with pytest.raises(N.PDHGError):   # more devices than rows
        MultiContext(2, 512, 256, 2, P["dx"], P["dy"], P["dt"], P["xs"], P["ys"], devices=[0, 0, 0])
    Q = make_problem(1, 2, 48, 40, 4, 0.0)
    with pytest.raises(N.PDHGError):   # nx = 48: no fast x-transform kernel for the slabs
        MultiContext(1, 48, 40, 4, Q["dx"], Q["dy"], Q["dt"], Q["xs"], Q["ys"], devices=[0, 0])
