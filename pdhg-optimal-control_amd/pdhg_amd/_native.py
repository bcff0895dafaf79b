"""ctypes binding of libpdhg.so (C ABI in include/pdhg.h).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc, gfx950).
There is no CPU fallback: importing this module raises if the shared object
is missing, and every call raises ``PDHGError`` on a non-zero status.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libpdhg.so")

PDHG_OK = 0
PDHG_ERR_ARG = -1
PDHG_ERR_UNSUPPORTED = -2
PDHG_ERR_HIP = -3
PDHG_ERR_STATE = -4
PDHG_ERR_NOMEM = -5

# every symbol declared in include/pdhg.h
EXPORTS = (
    "pdhg_last_error", "pdhg_abi_version", "pdhg_device_count", "pdhg_create", "pdhg_destroy",
    "pdhg_set_state", "pdhg_get_state", "pdhg_get_phi_bar", "pdhg_set_phi_bar", "pdhg_get_rows", "pdhg_init_state",
    "pdhg_update_primal", "pdhg_update_dual", "pdhg_errors", "pdhg_inner_error", "pdhg_iterate", "pdhg_set_stop_rules", "pdhg_synchronize",
    "pdhg_device_bytes", "pdhg_path_info", "pdhg_profile_enable", "pdhg_profile_query", "pdhg_algorithmic_bytes",
    # t-slab decomposition (multi-GPU)
    "pdhg_create_slab", "pdhg_set_stream", "pdhg_slab_plane_size", "pdhg_slab_begin", "pdhg_slab_carry_gain",
    "pdhg_slab_residual", "pdhg_slab_forward", "pdhg_slab_fixup", "pdhg_slab_long_modes", "pdhg_slab_fixup_nb", "pdhg_slab_backward", "pdhg_slab_primal_finalize", "pdhg_slab_dual",
    "pdhg_slab_dual_finalize", "pdhg_slab_outer", "pdhg_slab_outer_finalize", "pdhg_slab_plane_out",
    "pdhg_slab_plane_in", "pdhg_slab_status", "pdhg_slab_part_modes", "pdhg_slab_forward_part",
    "pdhg_slab_carry_out_part", "pdhg_slab_fixup_nb_part", "pdhg_slab_backward_part", "pdhg_slab_update",
    # x-slab decomposition (multi-GPU for T = 1 windows)
    "pdhg_create_xslab", "pdhg_xslab_layout", "pdhg_xslab_sizes", "pdhg_xslab_halo_out", "pdhg_xslab_halo_in",
    "pdhg_xslab_residual", "pdhg_xslab_wire", "pdhg_xslab_precond", "pdhg_xslab_update",
    # multi-device context (one host thread, t-slabs over a device list)
    "pdhg_create_multi", "pdhg_multi_destroy", "pdhg_multi_set_state", "pdhg_multi_get_state",
    "pdhg_multi_iterate", "pdhg_multi_set_stop_rules", "pdhg_multi_synchronize", "pdhg_multi_info",
    "pdhg_multi_profile", "pdhg_multi_phase_ms", "pdhg_multi_init_state", "pdhg_build_id",
)


class PDHGError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("pdhg status {}: {}".format(code, msg))
        self.code = code


class PDHGUnsupported(PDHGError, NotImplementedError):
    pass


class pdhg_problem(ctypes.Structure):
    _fields_ = [
        ("egno", ctypes.c_int), ("ndim", ctypes.c_int), ("bc_x", ctypes.c_int), ("bc_y", ctypes.c_int),
        ("nx", ctypes.c_int), ("ny", ctypes.c_int), ("T", ctypes.c_int), ("precision", ctypes.c_int),
        ("rho_alp_iters", ctypes.c_int), ("reserved0", ctypes.c_int),
        ("dx", ctypes.c_double), ("dy", ctypes.c_double), ("dt", ctypes.c_double),
        ("epsl", ctypes.c_double), ("c_on_rho", ctypes.c_double),
        ("C", ctypes.c_double), ("pow_", ctypes.c_double), ("Ct", ctypes.c_double),
        ("xs", ctypes.POINTER(ctypes.c_double)), ("ys", ctypes.POINTER(ctypes.c_double)),
    ]


class pdhg_stats(ctypes.Structure):
    _fields_ = [
        ("iters_run", ctypes.c_int), ("status", ctypes.c_int), ("inner_last", ctypes.c_int),
        ("inner_total", ctypes.c_int), ("err1", ctypes.c_double), ("err2", ctypes.c_double),
        ("err_inner", ctypes.c_double), ("rho_min", ctypes.c_double), ("rho_max", ctypes.c_double),
        ("nan_seen", ctypes.c_int), ("first_nan_iter", ctypes.c_int),
    ]


_lib = None


def load():
    """Load libpdhg.so once; raises ImportError if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError("libpdhg.so not built at {} — run __graft_entry__.build()".format(LIB_PATH))
    # PyTorch-ROCm ships its own HIP runtime; if libpdhg.so (built against /opt/rocm) initialises HIP
    # first, torch later reports "No HIP GPUs are available".  Load torch's runtime first whenever
    # torch is installed (the multi-GPU driver and the bench use it for RCCL and streams).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(LIB_PATH)
    P = ctypes.c_void_p
    dp = ctypes.POINTER(ctypes.c_double)
    sig = {
        "pdhg_last_error": ([], ctypes.c_char_p),
        "pdhg_abi_version": ([], ctypes.c_int),
        "pdhg_device_count": ([ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
        "pdhg_create": ([ctypes.POINTER(pdhg_problem), ctypes.c_int, ctypes.POINTER(P)], ctypes.c_int),
        "pdhg_destroy": ([P], ctypes.c_int),
        "pdhg_set_state": ([P, dp, dp, dp], ctypes.c_int),
        "pdhg_get_state": ([P, dp, dp, dp], ctypes.c_int),
        "pdhg_get_phi_bar": ([P, dp], ctypes.c_int),
        "pdhg_set_phi_bar": ([P, dp], ctypes.c_int),
        "pdhg_get_rows": ([P, ctypes.c_int, ctypes.c_int, dp, dp, dp, dp], ctypes.c_int),
        "pdhg_init_state": ([P, dp], ctypes.c_int),
        "pdhg_update_primal": ([P, ctypes.c_double], ctypes.c_int),
        "pdhg_update_dual": ([P, ctypes.c_double, ctypes.c_double, ctypes.c_int, ctypes.POINTER(ctypes.c_int)],
                             ctypes.c_int),
        "pdhg_errors": ([P, dp, dp], ctypes.c_int),
        "pdhg_inner_error": ([P, dp], ctypes.c_int),
        "pdhg_iterate": ([P, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_int,
                          ctypes.POINTER(pdhg_stats)], ctypes.c_int),
        "pdhg_set_stop_rules": ([P, ctypes.c_int, ctypes.c_int], ctypes.c_int),
        "pdhg_synchronize": ([P], ctypes.c_int),
        "pdhg_device_bytes": ([P, ctypes.POINTER(ctypes.c_ulonglong)], ctypes.c_int),
        "pdhg_path_info": ([P, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
        "pdhg_profile_enable": ([P, ctypes.c_int], ctypes.c_int),
        "pdhg_profile_query": ([P, ctypes.c_char_p, dp, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
        "pdhg_algorithmic_bytes": ([P, ctypes.c_int, ctypes.c_char_p, dp], ctypes.c_int),
        "pdhg_create_slab": ([ctypes.POINTER(pdhg_problem), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                              ctypes.POINTER(P)], ctypes.c_int),
        "pdhg_set_stream": ([P, P], ctypes.c_int),
        "pdhg_slab_plane_size": ([P, ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_ulonglong)],
                                 ctypes.c_int),
        "pdhg_slab_begin": ([P], ctypes.c_int),
        "pdhg_slab_carry_gain": ([P, P], ctypes.c_int),
        "pdhg_slab_residual": ([P, ctypes.c_int], ctypes.c_int),
        "pdhg_slab_forward": ([P, ctypes.c_double], ctypes.c_int),
        "pdhg_slab_fixup": ([P, P, P, ctypes.c_int, ctypes.c_int], ctypes.c_int),
        "pdhg_slab_long_modes": ([P, P, ctypes.c_int, ctypes.c_double, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
        "pdhg_slab_fixup_nb": ([P, P, P, P, P, ctypes.c_int, ctypes.c_int], ctypes.c_int),
        "pdhg_slab_backward": ([P, ctypes.c_double, P], ctypes.c_int),
        "pdhg_slab_primal_finalize": ([P, P], ctypes.c_int),
        "pdhg_slab_dual": ([P, ctypes.c_double, ctypes.c_int, ctypes.c_int, P, ctypes.c_int], ctypes.c_int),
        "pdhg_slab_dual_finalize": ([P, ctypes.c_double, ctypes.c_int, P], ctypes.c_int),
        "pdhg_slab_outer": ([P, ctypes.c_int, P], ctypes.c_int),
        "pdhg_slab_outer_finalize": ([P, ctypes.c_double, ctypes.c_int, P], ctypes.c_int),
        "pdhg_slab_plane_out": ([P, ctypes.c_int, P], ctypes.c_int),
        "pdhg_slab_plane_in": ([P, ctypes.c_int, P], ctypes.c_int),
        "pdhg_slab_status": ([P, ctypes.POINTER(pdhg_stats)], ctypes.c_int),
        "pdhg_slab_part_modes": ([P, ctypes.c_int, ctypes.c_int] + [ctypes.POINTER(ctypes.c_ulonglong)] * 2,
                                 ctypes.c_int),
        "pdhg_slab_forward_part": ([P, ctypes.c_double, ctypes.c_int, ctypes.c_int], ctypes.c_int),
        "pdhg_slab_carry_out_part": ([P, P, ctypes.c_int, ctypes.c_int], ctypes.c_int),
        "pdhg_slab_fixup_nb_part": ([P, P, P, P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int],
                                    ctypes.c_int),
        "pdhg_slab_backward_part": ([P, ctypes.c_double, ctypes.c_int, ctypes.c_int], ctypes.c_int),
        "pdhg_slab_update": ([P, ctypes.c_double, P], ctypes.c_int),
        "pdhg_create_xslab": ([ctypes.POINTER(pdhg_problem), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                               ctypes.POINTER(P)], ctypes.c_int),
        "pdhg_xslab_layout": ([P] + [ctypes.POINTER(ctypes.c_int)] * 4, ctypes.c_int),
        "pdhg_xslab_sizes": ([P] + [ctypes.POINTER(ctypes.c_ulonglong)] * 3, ctypes.c_int),
        "pdhg_xslab_halo_out": ([P, ctypes.c_int, P], ctypes.c_int),
        "pdhg_xslab_halo_in": ([P, ctypes.c_int, P, P], ctypes.c_int),
        "pdhg_xslab_residual": ([P], ctypes.c_int),
        "pdhg_xslab_wire": ([P, ctypes.c_int, P], ctypes.c_int),
        "pdhg_xslab_precond": ([P], ctypes.c_int),
        "pdhg_xslab_update": ([P, ctypes.c_double, P], ctypes.c_int),
        "pdhg_create_multi": ([ctypes.POINTER(pdhg_problem), ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                               ctypes.POINTER(P)], ctypes.c_int),
        "pdhg_multi_destroy": ([P], ctypes.c_int),
        "pdhg_multi_set_state": ([P, dp, dp, dp], ctypes.c_int),
        "pdhg_multi_get_state": ([P, dp, dp, dp], ctypes.c_int),
        "pdhg_multi_iterate": ([P, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                ctypes.POINTER(pdhg_stats)], ctypes.c_int),
        "pdhg_multi_set_stop_rules": ([P, ctypes.c_int, ctypes.c_int], ctypes.c_int),
        "pdhg_multi_synchronize": ([P], ctypes.c_int),
        "pdhg_multi_info": ([P, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
        "pdhg_multi_profile": ([P, ctypes.c_int], ctypes.c_int),
        "pdhg_multi_init_state": ([P, dp], ctypes.c_int),
        "pdhg_multi_phase_ms": ([P, ctypes.c_char_p, dp, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
        "pdhg_build_id": ([], ctypes.c_char_p),
    }
    missing = set(EXPORTS) - set(sig)
    if missing:
        raise ImportError("no ctypes signature for {}".format(sorted(missing)))
    for name, (args, res) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    _lib = lib
    return lib


def check(rc):
    if rc != PDHG_OK:
        msg = load().pdhg_last_error().decode("utf-8", "replace")
        if rc == PDHG_ERR_UNSUPPORTED:
            raise PDHGUnsupported(rc, msg)
        raise PDHGError(rc, msg)
    return rc


def dptr(a):
    """float64 C-contiguous array -> double*; None -> NULL."""
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def device_count():
    n = ctypes.c_int(0)
    check(load().pdhg_device_count(ctypes.byref(n)))
    return n.value
