"""Poisson test cases shared by the oracle and GPU tests: the reference's
tests/poisson drivers restated (mesh, right-hand side, norms)."""
import math

import numpy as np


def poisson3d_solution(c):
    """poisson3d.cpp:44-52"""
    return np.sin(c[:, 0]) * np.cos(2 * c[:, 1]) * np.sin(c[:, 2] / 4)


def center_refine_select(centers, lengths):
    """poisson3d.cpp:177-189: cells touching the point (pi, pi/2, 4 pi)."""
    mn, mx = centers - lengths / 2, centers + lengths / 2
    return ((mn[:, 0] < 1.01 * math.pi) & (mx[:, 0] > 0.99 * math.pi) & (mn[:, 1] < 0.51 * math.pi)
            & (mx[:, 1] > 0.49 * math.pi) & (mn[:, 2] < 4.01 * math.pi) & (mx[:, 2] > 3.99 * math.pi))


def poisson3d_lengths(n):
    """poisson3d.cpp:146-149 level-0 cell lengths for an n^3 grid."""
    return (2 * math.pi / n, 1 * math.pi / n, 8 * math.pi / n)


def level0_avg_norm(ids, sol, centers, lengths, n, L0):
    """get_p_norm of poisson3d.cpp:61-119 (p = 2): solution averaged over each
    level-0 parent (weight 8^-lvl) against the analytic value at its center."""
    lvl = np.round(np.log2(L0[0] / lengths[:, 0])).astype(int)
    k = (np.floor(centers[:, 0] / L0[0]).astype(np.int64) + n * np.floor(centers[:, 1] / L0[1]).astype(np.int64)
         + n * n * np.floor(centers[:, 2] / L0[2]).astype(np.int64))
    avg = np.zeros(n ** 3)
    np.add.at(avg, k, sol / 8.0 ** lvl)
    j = np.arange(n ** 3)
    c0 = np.stack([(j % n + 0.5) * L0[0], ((j // n) % n + 0.5) * L0[1], (j // (n * n) + 0.5) * L0[2]], axis=1)
    return math.sqrt(float(np.sum((avg - poisson3d_solution(c0)) ** 2)))


def boundary1d_solution(x):
    """poisson1d_boundary.cpp:42-50"""
    return np.sin(x) ** 2


def boundary1d_rhs(x):
    return 2 * (np.cos(x) ** 2 - np.sin(x) ** 2)


def boundary1d_classes(ix, nx):
    """poisson1d_boundary.cpp:141-164: outermost cells skipped, next ones
    boundary cells, the rest solved -> (solve mask, boundary mask, skip mask)."""
    skip = (ix == 0) | (ix == nx - 1)
    bdy = (ix == 1) | (ix == nx - 2)
    return ~(skip | bdy), bdy, skip


# ---- poisson1d.cpp / poisson2d.cpp / poisson1d_amr.cpp ----------------------
GOLDEN = __import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "poisson1d_ref.npz")
POISSON1D_SIZES = [8 << k for k in range(13)]  # 8 ... 32768 (poisson1d.cpp:149-154)
POISSON1D_SOLVER = (10, 0, 1e-7, 2, 10)        # Poisson_Solve solver(10, 0, 1e-7, 2, 10, false), :164
POISSON1D_THRESHOLD = 3e-7                     # norm_threshold, :283


def poisson1d_reference(n):
    """(solution, rhs) of the reference's serial solver for n cells
    (tests/golden/poisson1d_ref.npz, made by tests/golden/make_poisson_ref.py
    from tests/poisson/reference_poisson_solve.hpp compiled unmodified)."""
    with np.load(GOLDEN) as z:
        return z[f"n{n}"].copy(), z[f"rhs{n}"].copy()


def offset_last(sol_by_index):
    """offset_solution (poisson1d.cpp:90-121): zero in the last cell."""
    return sol_by_index - sol_by_index[-1]


def p_norm(a, b, p=2.0):
    return float(np.sum(np.abs(a - b) ** p) ** (1.0 / p))


def poisson2d_solution(x, y):
    """poisson2d.cpp:37-45"""
    return np.sin(x) * np.cos(2 * y)


def poisson2d_rhs(x, y):
    return -5 * poisson2d_solution(x, y)


def poisson2d_cases(max_cells=128):
    """The (cells_x, cells_y) sequence of poisson2d.cpp:150-165, whose loop
    bounds move inside the loops: 4x4, 8x4, 4x8, 8x8, 16x8, 8x16, ...,
    128x128 (the C loops executed as written)."""
    out = []
    lo, hi = 4, 8
    cy = lo
    while cy <= hi:
        cx = lo
        while cx <= hi:
            if cy == 2 * cx:
                lo = hi
                if hi < max_cells:
                    hi *= 2
            out.append((cx, cy))
            cx *= 2
        cy *= 2
    return out


def amr1d_solution(x):
    """poisson1d_amr.cpp:37-45"""
    return np.sin(x / 2) ** 2


def amr1d_rhs(x):
    return 0.5 * (np.cos(x / 2) ** 2 - np.sin(x / 2) ** 2)


def amr1d_normalize(sol, lvl, exact):
    """normalize_solution (poisson1d_amr.cpp:47-105): offset so that the
    8^-level weighted averages of solution and analytic agree."""
    w = 1.0 / 8.0 ** lvl
    return sol - (np.sum(w * sol) / np.sum(w) - np.sum(w * exact) / np.sum(w))
