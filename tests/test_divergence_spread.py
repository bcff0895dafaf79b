"""CPU check of the pointwise bounds of tests/test_gpu_divergence.py against the committed yardstick fixtures
(tests/golden/make_divergence_fixture.py): the float64 oracle's phi' / rho' at 4096 fixed points of C3's full
plane (T = 4, eps 0.1), per iteration, as run by the reference algorithm (scipy.fft), on numpy.fft, and with its
Thomas solve (utils_precond.py:10-40) in the device's exact-arithmetic-equivalent pivot algebra (kernels_xt_f64.hpp).

* through iteration PTS_TIGHT every reformulation stays within the tight bound PTS_TOL (the north-star 1e-5), so
  holding the device to it there is fair;
* after it one exact reformulation of one step moves the points by more than PTS_TOL_LATE, so the late bound is no
  looser than the spread of an equally valid float64 implementation;
* numpy.fft vs scipy.fft (the same FFT family) is far tighter than both: it is not the yardstick."""
import os

import numpy as np

from test_gpu_divergence import PTS_TIGHT, PTS_TOL, PTS_TOL_LATE

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _spread(variant):
    a = np.load(os.path.join(G, "divergence_c3_plane_T4_points.npz"))
    b = np.load(os.path.join(G, "divergence_c3_plane_T4_points_{}.npz".format(variant)))
    assert np.array_equal(a["phi_idx"], b["phi_idx"]) and np.array_equal(a["rho_idx"], b["rho_idx"])
    rel = lambda x, y: float(np.linalg.norm(x - y) / np.linalg.norm(y))  # noqa: E731
    n = a["phi_pts"].shape[0]
    return ([rel(b["phi_pts"][i], a["phi_pts"][i]) for i in range(n)],
            [rel(b["rho_pts"][i], a["rho_pts"][i]) for i in range(n)])


def test_pointwise_bounds_vs_reformulation_spread():
    phi, rho = _spread("devthomas")
    assert max(phi[:PTS_TIGHT] + rho[:PTS_TIGHT]) < PTS_TOL, (phi, rho)
    assert max(phi[PTS_TIGHT:] + rho[PTS_TIGHT:]) > PTS_TOL_LATE, (phi, rho)
    nphi, nrho = _spread("npfft")
    assert max(nphi + nrho) < 0.1 * max(phi[PTS_TIGHT:] + rho[PTS_TIGHT:])
