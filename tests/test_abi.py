"""C ABI checks that need no GPU: the library builds/loads, exports every symbol declared in
include/pdhg.h, and validates arguments / reports a missing device with a status + message."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pdhg.h")


@pytest.fixture(scope="module")
def lib():
    import __graft_entry__
    __graft_entry__.build()
    from pdhg_amd import _native
    return _native


def header_functions():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(pdhg_\w+)\s*\(", txt, flags=re.M)))


def test_header_and_binding_agree(lib):
    assert header_functions() == sorted(lib.EXPORTS)


def test_library_exports_every_header_symbol(lib):
    out = subprocess.check_output(["nm", "-D", "--defined-only", lib.LIB_PATH]).decode()
    exported = set(re.findall(r" T (pdhg_\w+)", out))
    missing = [f for f in header_functions() if f not in exported]
    assert not missing, missing
    L = lib.load()
    for f in header_functions():
        assert hasattr(L, f)


def test_abi_version_and_struct_layout(lib):
    L = lib.load()
    assert L.pdhg_abi_version() == 1
    # pdhg_problem: 10 ints + 8 doubles + 2 pointers
    assert ctypes.sizeof(lib.pdhg_problem) == 10 * 4 + 8 * 8 + 2 * 8


def _prob(lib, **kw):
    p = lib.pdhg_problem()
    xs = np.linspace(0, 2, 16, endpoint=False)
    p.egno, p.ndim, p.nx, p.ny, p.T, p.precision, p.rho_alp_iters = 1, 1, 16, 1, 4, 4, 1
    p.dx, p.dt, p.C, p.pow_, p.Ct, p.c_on_rho = 2 / 16, 0.025, 1.0, 1.0, 1.0, 70.0
    p.xs = lib.dptr(xs)
    for k, v in kw.items():
        setattr(p, k, v)
    return p, xs


@pytest.mark.parametrize("field,value", [("egno", 4), ("ndim", 3), ("T", 0), ("precision", 2), ("nx", 2),
                                         ("rho_alp_iters", 0), ("dt", 0.0)])
def test_create_rejects_bad_arguments(lib, field, value):
    L = lib.load()
    p, xs = _prob(lib, **{field: value})
    h = ctypes.c_void_p()
    rc = L.pdhg_create(ctypes.byref(p), 0, ctypes.byref(h))
    assert rc == lib.PDHG_ERR_ARG
    assert L.pdhg_last_error().decode()


def test_create_unsupported_bc(lib):
    L = lib.load()
    p, xs = _prob(lib, bc_x=1)
    h = ctypes.c_void_p()
    assert L.pdhg_create(ctypes.byref(p), 0, ctypes.byref(h)) == lib.PDHG_ERR_UNSUPPORTED


def test_no_device_is_an_error_not_a_fallback(lib):
    """Without a GPU the product path fails loudly (there is no CPU fallback)."""
    if lib.device_count() > 0:
        pytest.skip("a GPU is visible")
    L = lib.load()
    p, xs = _prob(lib)
    h = ctypes.c_void_p()
    assert L.pdhg_create(ctypes.byref(p), 0, ctypes.byref(h)) == lib.PDHG_ERR_HIP
    from pdhg_amd.context import PDHGContext
    with pytest.raises(lib.PDHGError):
        PDHGContext(1, 1, 16, 1, 4, 2 / 16, 0.0, 0.025, xs)


def test_null_context_calls(lib):
    L = lib.load()
    assert L.pdhg_update_primal(None, 0.1) == lib.PDHG_ERR_ARG
    assert L.pdhg_destroy(None) == lib.PDHG_OK


def test_xslab_create_validates_before_device(lib):
    """pdhg_create_xslab checks the decomposition (rank range, ndim, bc, row split) and pdhg_create's problem
    checks (here an unknown precision; fp32 and fp64 are both x-slab precisions) before it touches a device."""
    L = lib.load()
    xs = np.linspace(0, 2, 64, endpoint=False)
    ys = np.linspace(0, 2, 256, endpoint=False)

    def prob(**kw):
        p = lib.pdhg_problem()
        p.egno, p.ndim, p.nx, p.ny, p.T, p.precision, p.rho_alp_iters = 1, 2, 64, 256, 1, 4, 1
        p.dx, p.dy, p.dt, p.C, p.pow_, p.Ct, p.c_on_rho = 2 / 64, 2 / 256, 0.025, 1.0, 1.0, 1.0, 70.0
        p.xs, p.ys = lib.dptr(xs), lib.dptr(ys)
        for k, v in kw.items():
            setattr(p, k, v)
        return p

    h = ctypes.c_void_p()
    for (rank, nranks, kw, code) in [(2, 2, {}, lib.PDHG_ERR_ARG), (0, 0, {}, lib.PDHG_ERR_ARG),
                                     (0, 2, {"precision": 2}, lib.PDHG_ERR_ARG),
                                     (0, 2, {"ndim": 1, "ny": 1}, lib.PDHG_ERR_UNSUPPORTED),
                                     (0, 2, {"bc_x": 2}, lib.PDHG_ERR_UNSUPPORTED),   # Dirichlet x edges
                                     (0, 3, {}, lib.PDHG_ERR_UNSUPPORTED),      # 64 rows / 3
                                     (0, 16, {}, lib.PDHG_ERR_UNSUPPORTED)]:    # 4-row slabs
        p = prob(**kw)
        assert L.pdhg_create_xslab(ctypes.byref(p), rank, nranks, 0, ctypes.byref(h)) == code, (rank, nranks, kw)
        assert L.pdhg_last_error().decode()
    # phase calls on a non-slab / null context fail with a status, not a crash
    assert L.pdhg_xslab_residual(None) == lib.PDHG_ERR_ARG
