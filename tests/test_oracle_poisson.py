"""The oracle's Poisson restatement (tests/poisson/poisson_solve.hpp) pinned
against the reference's own Poisson known-answer tests:

* poisson3d.cpp:122-238 — 8^3 periodic grid refined twice around
  (pi, pi/2, 4 pi), default solver, PASSED iff the level-0-averaged 2-norm
  error < 0.35 (poisson3d.cpp:227);
* poisson1d_boundary.cpp:108-221 — 1-D grids of 8..4096 cells with skip and
  boundary cells, solver (10000, 0, 1e-15, 2, 100): the error norm must not
  grow with resolution.

The reference itself cannot be built here (dccrg.hpp needs Zoltan and
Boost), so these thresholds are the parity anchor of the Poisson rows."""
import math

import numpy as np
import pytest

from oracle import oracle as O
from poisson_cases import (boundary1d_classes, boundary1d_rhs, boundary1d_solution, center_refine_select,
                                 level0_avg_norm, poisson3d_lengths, poisson3d_solution)


def oracle_poisson3d(n=8, R=2, rounds=2):
    o = O.Grid((n, n, n), R, (True, True, True), 0, 1)
    L0 = poisson3d_lengths(n)
    o.set_geometry((0, 0, 0), L0)
    for _ in range(rounds):
        ids, _ = o.cells()
        c, L = o.geometry(ids)
        for i in ids[center_refine_select(c, L)]:
            o.refine_completely(int(i))
        o.stop_refining()
    ids, _ = o.cells()
    c, L = o.geometry(ids)
    o.po_set(ids, -(81.0 / 16.0) * poisson3d_solution(c), np.zeros(ids.size), np.zeros(ids.size, np.int32))
    return o, ids, c, L, L0


def test_poisson3d_kat():
    o, ids, c, L, L0 = oracle_poisson3d()
    assert np.unique(L[:, 0]).size == 3  # levels 0, 1, 2 present
    it, res = o.po_solve()
    norm = level0_avg_norm(ids, o.po_get(ids)[:, 0], c, L, 8, L0)
    assert norm < 0.35, norm  # poisson3d.cpp:227


def test_uniform_scaling_factors():
    """set_scaling_factor 696-819 on a uniform periodic grid: f = 1/dx^2 per
    direction, scaling factor = -sum f."""
    o = O.Grid((4, 5, 6), 0, (True, True, True), 0, 1)
    dx = (0.5, 0.25, 2.0)
    o.set_geometry((0, 0, 0), dx)
    ids, _ = o.cells()
    o.po_set(ids, np.ones(ids.size), np.zeros(ids.size), np.zeros(ids.size, np.int32))
    o.po_solve(max_iterations=1)
    out = o.po_get(ids)
    for d in range(3):
        np.testing.assert_allclose(out[:, 8 + 2 * d], 1 / dx[d] ** 2, rtol=1e-15)
        np.testing.assert_allclose(out[:, 9 + 2 * d], 1 / dx[d] ** 2, rtol=1e-15)
    np.testing.assert_allclose(out[:, 7], -2 * sum(1 / x ** 2 for x in dx), rtol=1e-15)


def oracle_boundary1d(cells):
    nx = cells + 4
    h = 2 * math.pi / cells
    o = O.Grid((nx, 1, 1), 0, (False, False, False), 0, 1)
    o.set_geometry((-2 * h, 0, 0), (h, 1, 1))
    ids, _ = o.cells()
    c, _ = o.geometry(ids)
    ix = (ids - 1).astype(np.int64)
    solve, bdy, skip = boundary1d_classes(ix, nx)
    x = c[:, 0]
    rhs = np.where(solve | bdy, boundary1d_rhs(x), 0.0)
    sol = np.where(bdy, boundary1d_solution(x), 0.0)
    types = np.where(solve, 0, np.where(skip, 2, 1)).astype(np.int32)
    o.po_set(ids, rhs, sol, types)
    return o, ids, x, solve


@pytest.mark.parametrize("max_cells", [512])
def test_poisson1d_boundary_kat(max_cells):
    old = float("inf")
    cells = 8
    while cells <= max_cells:
        o, ids, x, solve = oracle_boundary1d(cells)
        o.po_solve(10000, 0, 1e-15, 2, 100)
        sol = o.po_get(ids)[:, 0]
        norm = math.sqrt(float(np.sum((sol[solve] - boundary1d_solution(x[solve])) ** 2)))
        assert norm <= old, (cells, norm, old)  # poisson1d_boundary.cpp:208-219
        old = norm
        cells *= 2


def test_failsafe_converges():
    """solve_failsafe 531-634 on the 3-D case reaches its stop residual."""
    o, ids, c, L, L0 = oracle_poisson3d(n=4, rounds=1)
    it, norm = o.po_solve(max_iterations=20000, stop_residual=1e-9, failsafe=True)
    assert norm <= 1e-9 and it < 20000


def test_poisson1d_reference_fixture_and_oracle():
    """tests/poisson/poisson1d.cpp:147-350 on the oracle: 1-D periodic grids
    of n cells (x, y and z orientation) solved by BiCG (10, 0, 1e-7, 2, 10),
    offset to zero in the last cell, must lie within the 2-norm 3e-7 of the
    reference's own serial solution (tests/golden/poisson1d_ref.npz, from
    reference_poisson_solve.hpp compiled unmodified) and of each other."""
    from poisson_cases import (POISSON1D_SOLVER, POISSON1D_THRESHOLD, offset_last, p_norm,
                               poisson1d_reference)

    for n in (8, 16, 64, 256, 1024):
        ref, rhs = poisson1d_reference(n)
        assert abs(float(np.sum(rhs))) < 1e-12 and abs(ref[-1]) < 1e-9  # the recurrence ends near 0
        h = 2 * math.pi / n
        sols = []
        for d in range(3):
            length = [1, 1, 1]
            length[d] = n
            L0 = [1.0, 1.0, 1.0]
            L0[d] = h
            o = O.Grid(tuple(length), 0, (True, True, True), 0, 1)
            o.set_geometry((0, 0, 0), tuple(L0))
            ids, _ = o.cells()
            o.po_set(ids, rhs[ids.astype(np.int64) - 1], np.zeros(ids.size), np.zeros(ids.size, np.int32))
            o.po_solve(*POISSON1D_SOLVER)
            sol = offset_last(o.po_get(ids)[:, 0])
            assert p_norm(sol, ref) <= POISSON1D_THRESHOLD, (n, d, p_norm(sol, ref))
            sols.append(sol)
        for a in range(3):
            for b in range(a + 1, 3):
                assert p_norm(sols[a], sols[b]) <= POISSON1D_THRESHOLD
