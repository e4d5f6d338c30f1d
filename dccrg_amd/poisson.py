"""Python mirror of the reference's ``Poisson_Solve`` (tests/poisson/poisson_solve.hpp:156-1056)
over the device solver of the C ABI (``dccrgx_poisson_cache`` / ``dccrgx_poisson_solve``).

The reference keeps rhs and solution in ``Poisson_Cell`` (51-86); here they are
fp64 fields of the grid, by default the ones named ``"rhs"`` and ``"solution"``.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, lib
from .grid import Field


def _ids(cells):
    a = np.ascontiguousarray(np.asarray(cells if cells is not None else [], dtype=np.uint64))
    return a, (a.ctypes.data_as(C.c_void_p) if a.size else None)


class Poisson_Solve:
    """Same parameters and defaults as the reference constructors (166-201)."""

    def __init__(self, max_iterations=1000, min_iterations=0, stop_residual=1e-15, p_of_norm=2.0,
                 stop_after_residual_increase=10.0, verbose=False):
        self.max_iterations = int(max_iterations)
        self.min_iterations = int(min_iterations)
        self.stop_residual = float(stop_residual)
        self.p_of_norm = float(p_of_norm)
        self.stop_after_residual_increase = float(stop_after_residual_increase)
        self.verbose = bool(verbose)
        self.iterations = 0
        self.residual = None

    def set_verbosity(self, given):
        self.verbose = bool(given)

    def set_max_iterations(self, given):
        self.max_iterations = int(given)

    def set_min_iterations(self, given):
        self.min_iterations = int(given)

    @staticmethod
    def _fields(grid, rhs, solution):
        rhs = rhs if rhs is not None else grid.fields["rhs"]
        solution = solution if solution is not None else grid.fields["solution"]
        assert isinstance(rhs, Field) and isinstance(solution, Field)
        return rhs, solution

    def cache_system_info(self, cells, grid, cells_to_skip=None, rhs=None, solution=None):
        """827-971: classify (local cells boundary, then skip, then solve) and
        compute the geometry factors on the device."""
        rhs, solution = self._fields(grid, rhs, solution)
        a, pa = _ids(cells)
        b, pb = _ids(cells_to_skip)
        check(lib().dccrgx_poisson_cache(grid.h, rhs.id, solution.id, pa, a.size, pb, b.size))

    def _run(self, cells, grid, cells_to_skip, cache_is_up_to_date, rhs, solution, failsafe):
        if not cache_is_up_to_date:
            self.cache_system_info(cells, grid, cells_to_skip, rhs, solution)
        it, res = C.c_uint(), C.c_double()
        check(lib().dccrgx_poisson_solve(grid.h, self.max_iterations, self.min_iterations, self.stop_residual,
                                         self.p_of_norm, self.stop_after_residual_increase, int(failsafe),
                                         C.byref(it), C.byref(res)))
        self.iterations, self.residual = it.value, res.value
        if self.verbose and grid.rank == 0:
            what = "norm" if failsafe else "residual"
            print(f"iterations: {self.iterations}, {what}: {self.residual}")
        return self.iterations, self.residual

    def solve(self, cells, grid, cells_to_skip=None, cache_is_up_to_date=False, rhs=None, solution=None):
        """251-522: BiCG; the solution field ends as the best solution found."""
        return self._run(cells, grid, cells_to_skip, cache_is_up_to_date, rhs, solution, False)

    def solve_failsafe(self, cells, grid, cells_to_skip=None, cache_is_up_to_date=False, rhs=None, solution=None):
        """531-634: Jacobi-like iteration."""
        return self._run(cells, grid, cells_to_skip, cache_is_up_to_date, rhs, solution, True)

    @staticmethod
    def field(grid, name):
        """The solver's per-cell state as a read-only Field ("p0", "r0",
        "scaling_factor", "f_x_pos", "type", ...)."""
        fid = C.c_int()
        check(lib().dccrgx_poisson_field(grid.h, name.encode(), C.byref(fid)))
        dt = np.int32 if name == "type" else np.float64
        return Field(grid, fid.value, "poisson." + name, dt, False)
