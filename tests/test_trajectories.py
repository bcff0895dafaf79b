"""Trajectory consumers of alp (run_example.py:18-155) vs the per-sample oracle restatement (CPU)."""
import numpy as np
import pytest

import traj_oracle as TO
from pdhg_amd import run_example as RE, set_fns, trajectories as TR


def _field(shape, seed):
    return 0.5 * np.random.default_rng(seed).standard_normal(shape)


@pytest.mark.parametrize("egno,method", [(1, "linear"), (2, "nearest")])
@pytest.mark.parametrize("epsl", [0.0, 0.1])
def test_traj_1d_matches_oracle(egno, method, epsl):
    nx, nt, P, T = 24, 9, 2.0, 1.0
    x_arr = np.linspace(0.0, P, nx, endpoint=False)
    t_arr = np.linspace(0.0, T, nt)
    alp = _field((2, nt - 1, nx), egno)
    fns = set_fns.set_up_example_fns(egno, 1, 0)
    x0 = np.linspace(0.0, P, 7)
    a_p, x_p = TR.compute_traj_1d(x0, alp, fns.f_fn, nt, x_arr, t_arr, P, T, epsl, method,
                                  rng=np.random.default_rng(5))
    a_o, x_o = TO.compute_traj_1d(x0, alp, fns.f_fn, nt, x_arr, t_arr, P, T, epsl, method,
                                  rng=np.random.default_rng(5))
    assert a_p.shape == (nt - 1, 7, 1) and x_p.shape == (nt, 7)
    assert np.allclose(a_p, a_o, rtol=1e-12, atol=1e-13) and np.allclose(x_p, x_o, rtol=1e-12, atol=1e-13)


@pytest.mark.parametrize("bc,center", [(0, False), (1, True), (2, False)])
def test_extend_bdry_matches_virtual_grid(bc, center):
    n, P = 6, 2.0
    x = np.linspace(0.0, P, n, endpoint=False) - (P / 2 if center else 0.0)
    val = _field((3, n, 4, 2), 3)
    for lo, hi in ((-2.5, 0.3), (0.1, 1.9), (-0.2, 5.1), (-4.9, 3.3)):
        xe, ve = TR.extend_bdry_2d(x, lo, hi, val, P, axis=1, bc=bc, center=center)
        e = TO.VirtualExtension(x, lo, hi, P, bc, center)
        assert len(xe) == e.size == ve.shape[1]
        for i in range(e.size):
            assert abs(xe[i] - e.coord(i)) < 1e-12
            src = e.source(i)
            ref = np.zeros_like(val[:, 0]) if src[0] == "zero" else val[:, src[1]]
            assert np.array_equal(ve[:, i], ref)
        val2 = val.transpose(0, 2, 1, 3)                   # the same lines along axis 2
        ye, we = TR.extend_bdry_2d(x, lo, hi, val2, P, axis=2, bc=bc, center=center)
        assert np.array_equal(ye, xe) and np.array_equal(we, ve.transpose(0, 2, 1, 3))


@pytest.mark.parametrize("egno,method", [(1, "linear"), (2, "nearest"), (3, "linear")])
def test_traj_2d_matches_oracle(egno, method):
    nx, ny, nt, P, T = 10, 8, 6, 2.0, 1.0
    center = egno == 3
    x1 = np.linspace(0.0, P, nx, endpoint=False) - (P / 2 if center else 0.0)
    x2 = np.linspace(0.0, P, ny, endpoint=False) - (P / 2 if center else 0.0)
    n_ctrl = 1 if egno == 3 else 2
    alp = _field((4, nt - 1, nx, ny, n_ctrl), 10 + egno)
    if egno == 3:
        alp[2:] = 0.0
    bc = (1, 0) if egno == 3 else (0, 0)
    fns = set_fns.set_up_example_fns(egno, 2, 0)
    x0 = TR.trajectory_samples(egno, 2, 4, P, P, 0.0)
    if egno != 3:
        x0 = x0 + np.array([0.013, -0.021])       # off-grid starts
    args = (x0, alp, fns.f_fn, nt, x1, x2, np.linspace(0.0, T, nt), P, P, T, bc, (center, center), 0.05, method)
    a_p, x_p = TR.compute_traj_2d(*args, rng=np.random.default_rng(9))
    a_o, x_o = TO.compute_traj_2d(*args, rng=np.random.default_rng(9))
    assert a_p.shape == (nt - 1, len(x0), n_ctrl) and x_p.shape == (nt, len(x0), 2)
    assert np.allclose(a_p, a_o, rtol=1e-11, atol=1e-12) and np.allclose(x_p, x_o, rtol=1e-11, atol=1e-12)


def test_run_example_writes_trajectories(tmp_path, monkeypatch):
    """--plot with --plot_traj_num_1d computes the trajectories from the solved alp (run_example.py:342-393) and
    writes them next to the results; the solve itself is replaced by a stub here (CPU test)."""
    nx, nt = 16, 5

    def fake_solve(ndim, n_ctrl, egno, epsl, fns, nx_, ny, nt_, *a, **k):
        rng = np.random.default_rng(0)
        phi = rng.standard_normal((nt_, nx_))
        alp = 0.3 * rng.standard_normal((2, nt_ - 1, nx_, 1))
        return [(3, phi, np.ones((nt_ - 1, nx_)), alp)], [np.zeros((1, 2))]
    monkeypatch.setattr(RE, "solve_HJ", fake_solve)
    RE.main(["--egno", "1", "--ndim", "1", "--nx", str(nx), "--nt", str(nt), "--plot", "1", "--plot_traj_num_1d", "5",
             "--out", str(tmp_path), "--save", "0"])
    files = list(tmp_path.rglob("traj_*.npz"))
    assert len(files) == 1
    z = np.load(files[0])
    assert z["traj_x"].shape == (nt, 5) and z["traj_alp"].shape == (nt - 1, 5, 1)
