"""The run_example.py-style driver (pdhg_amd/run_example.py; reference run_example.py:157-440).

CPU: flags and grid.  GPU: an end-to-end C0-shaped run (egno 1, 1-D, nx = 160, nt = 41, windows of
time_step_per_PDHG = 2, capped iterations) through the device, against the oracle's solve_HJ."""
import numpy as np
import pytest

import pdhg_oracle as O
from pdhg_amd import run_example as R


@pytest.mark.parametrize("egno,ndim", [(1, 1), (2, 2), (3, 2)])
def test_grid_matches_reference_construction(egno, ndim):
    x, t = R.make_grid(ndim, egno, 12, 10, 5, 2.0, 2.0, 1.0)
    assert np.array_equal(x, O.make_grid(ndim, 12, 10, egno))
    assert t.shape[0] == 5 and t[-1].item() == 1.0


def test_flags_defaults_are_the_reference_defaults():
    F = R.build_parser().parse_args([])
    assert (F.egno, F.ndim, F.nt, F.nx, F.ny, F.stepsz_param, F.time_step_per_PDHG, F.eps, F.c_on_rho) == \
        (1, 1, 11, 20, 20, 0.1, 2, 1e-6, 70.0)


@pytest.mark.gpu
def test_c0_end_to_end_matches_oracle(native, tmp_path):
    args = ["--egno", "1", "--ndim", "1", "--nx", "160", "--nt", "41", "--N_maxiter", "300", "--print_freq", "100",
            "--precision", "fp64", "--out", str(tmp_path)]
    res_d, errs_d = R.main(args)
    res_o, errs_o = O.solve_HJ(1, 1, 0.0, 160, 1, 41, N_maxiter=300, print_freq=100)
    assert len(res_d) == len(res_o)
    for (n_d, phi_d, rho_d, alp_d), (n_o, phi_o, rho_o, alp_o) in zip(res_d, res_o):
        assert n_d == n_o
        assert np.linalg.norm(phi_d - phi_o) <= 1e-9 * np.linalg.norm(phi_o)
        assert np.linalg.norm(rho_d - rho_o) <= 1e-9 * np.linalg.norm(rho_o)
