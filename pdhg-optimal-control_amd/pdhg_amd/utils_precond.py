"""Setup-time symbol of the preconditioner (jaxsrc/utils/utils_precond.py:42-71).

Only ``compute_Dxx_fft_fv`` is host-side in the reference too (it is computed
once by solve_HJ, run_example.py:191).  The device path does not consume it:
the kernels use the analytic periodic symbol  -2(1 - cos(2 pi k / n)) / dx^2,
which is exactly the FFT of the reference's stencil up to roundoff.  It is
kept so callers that pass ``fv`` through the reference signatures still work.
"""
import numpy as np


def compute_Dxx_fft_fv(ndim, nspatial, dspatial, bc):
    if ndim == 1:
        (nx,), (dx,) = nspatial, dspatial
        if bc != 0:
            raise NotImplementedError
        k = np.arange(nx)
        return (-2.0 * (1.0 - np.cos(2 * np.pi * k / nx)) / dx ** 2).astype(np.complex128)
    if ndim == 2:
        (nx, ny), (dx, dy) = nspatial, dspatial
        if tuple(bc) != (0, 0):
            raise NotImplementedError("bc {} (egno 3's DCT symbol) is not implemented yet".format(bc))
        lx = -2.0 * (1.0 - np.cos(2 * np.pi * np.arange(nx) / nx)) / dx ** 2
        ly = -2.0 * (1.0 - np.cos(2 * np.pi * np.arange(ny) / ny)) / dy ** 2
        return (lx[:, None] + ly[None, :]).astype(np.complex128)
    raise NotImplementedError
