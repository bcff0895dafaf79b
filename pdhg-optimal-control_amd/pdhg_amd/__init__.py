"""MI355X-native PDHG for Hamilton–Jacobi optimal control (drop-in for TingweiMeng/PDHG-optimal-control's hot path).

Modules mirror the reference's ``jaxsrc`` entry points:

* ``set_fns``             set_up_J, set_up_numerical_L, set_up_example_fns
* ``update_fns_in_pdhg``  update_primal_1d/2d, update_dual_oneiter, update_dual_alternative
* ``utils_pdhg_solver``   PDHG_solver_oneiter, PDHG_multi_step (+ make_update_fns)
* ``utils_precond``       compute_Dxx_fft_fv
* ``solver``              save, load_solution, load_middle_solution

Compute runs in ``libpdhg.so`` (HIP, gfx950) through ``context.PDHGContext``.
"""
from . import _native  # noqa: F401

__all__ = ["set_fns", "update_fns_in_pdhg", "utils_pdhg_solver", "utils_precond", "solver", "context"]
