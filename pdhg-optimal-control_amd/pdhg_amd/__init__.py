"""MI355X-native PDHG for Hamilton–Jacobi optimal control (drop-in for TingweiMeng/PDHG-optimal-control's hot path).

Modules mirror the reference's ``jaxsrc`` entry points:

* ``set_fns``             set_up_J, set_up_numerical_L, set_up_example_fns
* ``update_fns_in_pdhg``  update_primal_1d/2d, update_dual_oneiter, update_dual_alternative
* ``utils_pdhg_solver``   PDHG_solver_oneiter, PDHG_multi_step (+ make_update_fns)
* ``utils_precond``       compute_Dxx_fft_fv
* ``solver``              save, load_solution, load_middle_solution
* ``run_example``         the reference's CLI driver (flags, solve_HJ, npz results)

Multi-GPU (no reference counterpart): ``slab`` (t-slabs of one window: halos + distributed Thomas over
RCCL) and ``xslab`` (x-slabs for the T = 1 marching default: halo rows + all-to-all spectrum transposes).

Compute runs in ``libpdhg.so`` (HIP, gfx950) through ``context.PDHGContext``.
"""
from . import _native  # noqa: F401

__all__ = ["set_fns", "update_fns_in_pdhg", "utils_pdhg_solver", "utils_precond", "solver", "context",
           "run_example", "slab", "xslab"]
