"""Setup-time symbol of the preconditioner (jaxsrc/utils/utils_precond.py:42-71).

Only ``compute_Dxx_fft_fv`` is host-side in the reference too (it is computed
once by solve_HJ, run_example.py:191).  The device path does not consume it:
the kernels use the analytic periodic symbol  -2(1 - cos(2 pi k / n)) / dx^2,
which is exactly the FFT of the reference's stencil up to roundoff, and for bc (1, 0)
(egno 3) the reference's fft_y(dct_x(lap)) in closed form:
DCT-II(x stencil)[kx] + 2 cos(pi kx / 2nx) * lam_y[ky].  It is kept so callers that pass
``fv`` through the reference signatures still work.
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
        ly = -2.0 * (1.0 - np.cos(2 * np.pi * np.arange(ny) / ny)) / dy ** 2
        k = np.arange(nx)
        if tuple(bc) == (0, 0):
            lx = -2.0 * (1.0 - np.cos(2 * np.pi * k / nx)) / dx ** 2
            return (lx[:, None] + ly[None, :]).astype(np.complex128)
        if tuple(bc) == (1, 0):
            c2 = lambda n: 2.0 * np.cos(np.pi * k * (2 * n + 1) / (2 * nx))   # DCT-II of e_n
            lx = (-2.0 * c2(0) + c2(1) + c2(nx - 1)) / dx ** 2
            return (lx[:, None] + c2(0)[:, None] * ly[None, :]).astype(np.complex128)
        raise NotImplementedError("bc {}".format(bc))
    raise NotImplementedError
