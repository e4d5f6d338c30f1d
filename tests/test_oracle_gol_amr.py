"""The oracle's restatement of the refined game of life
(tests/game_of_life/solve.hpp:37-170, get_live_neighbors), pinned by the
reference's own differential test tests/game_of_life/unrefined2d.cpp:
played on a refined grid, every leaf's state equals the state of its
level-0 parent in the same game played on the unrefined grid
(unrefined2d.cpp:215-240), at every step.  The live cells are the
reference's patterns (tests/game_of_life/initialize.hpp:28-89) on its
15 x 15 x 1 grid; the reference refines/unrefines randomly each step
(refine.hpp), this restatement refines a random set once (no unrefinement in
scope) with children inheriting the parent's state (refined2d.cpp:212-220)."""
import numpy as np
import pytest

from oracle import oracle as O

GRID = 15  # unrefined2d.cpp:108 base_length, direction 'z' -> (15, 15, 1)


def unrefined2d_live_cells(n=GRID):
    """initialize.hpp:28-89 get_live_cells(grid_size = n): blinker, toad,
    beacon, glider, block, beehive (ids of the level-0 grid)."""
    live = {198, 199, 200}  # blinker
    live |= {188, 189, 190, 188 + 1 + n, 188 + 2 + n, 188 + 3 + n}  # toad
    b = 137
    live |= {b, b + 1, b - n, b + 1 - n, b + 2 - 2 * n, b + 3 - 2 * n, b + 2 - 3 * n, b + 3 - 3 * n}  # beacon
    g = 143
    live |= {g + 1, g + 2 - n, g - 2 * n, g + 1 - 2 * n, g + 2 - 2 * n}  # glider
    k = 47
    live |= {k, k + 1, k - n, k + 1 - n}  # block
    h = 51
    live |= {h - n, h + 1, h + 2, h + 1 - 2 * n, h + 2 - 2 * n, h + 3 - n}  # beehive
    return live


def refined_pair(length, periodic, frac, seed, live0):
    """(refined oracle grid, unrefined oracle grid), both initialised from the
    level-0 live set `live0`; children inherit their parent's state."""
    o = O.Grid(length, 1, periodic, 1, 1)
    ids, _ = o.cells()
    rng = np.random.default_rng(seed)
    for c in rng.choice(ids, size=int(frac * ids.size), replace=False):
        o.refine_completely(int(c))
    o.stop_refining()
    leaves, _ = o.cells()
    par = o.mapping.batch(leaves)["level0_parent"]
    o.gola_set(leaves, np.array([1 if int(p) in live0 else 0 for p in par], np.uint32))
    u = O.Grid(length, 0, periodic, 1, 1)
    uids, _ = u.cells()
    u.gol_set(uids, np.array([1 if int(c) in live0 else 0 for c in uids], np.uint32))
    return o, u, leaves, par


@pytest.mark.parametrize("frac,seed", [(0.5, 0), (0.3, 1), (1.0, 2)])
def test_unrefined2d_patterns_refined_equals_unrefined(frac, seed):
    length = (GRID, GRID, 1)
    o, u, leaves, par = refined_pair(length, (False, False, False), frac, seed, unrefined2d_live_cells())
    assert leaves.size > GRID * GRID  # something was refined
    for step in range(25):  # unrefined2d.cpp:183
        o.gola_steps(1)
        u.gol_steps(1)
        assert np.array_equal(o.gola_get(leaves), u.gol_get(par)), f"step {step}"


@pytest.mark.parametrize("periodic", [(False, False, False), (True, True, True)])
def test_3d_random_refined_equals_unrefined(periodic):
    """3-D: the game explodes within a step or two (26 neighbors), so each
    round starts from fresh sparse level-0 states and plays one turn."""
    length = (8, 7, 6)
    n0 = length[0] * length[1] * length[2]
    for seed in range(5):
        rng = np.random.default_rng(100 + seed)
        live0 = {int(c) for c in np.nonzero(rng.random(n0) < 0.06)[0] + 1}
        o, u, leaves, par = refined_pair(length, periodic, 0.4, seed, live0)
        o.gola_steps(1)
        u.gol_steps(1)
        assert np.array_equal(o.gola_get(leaves), u.gol_get(par)), f"seed {seed}"


def test_2d_random_long_game():
    """A 2-D grid (z length 1) never exceeds 8 live level-0 neighbors."""
    length = (24, 20, 1)
    rng = np.random.default_rng(5)
    live0 = {int(c) for c in np.nonzero(rng.random(480) < 0.35)[0] + 1}
    o, u, leaves, par = refined_pair(length, (True, True, False), 0.5, 9, live0)
    for step in range(30):
        o.gola_steps(1)
        u.gol_steps(1)
        assert np.array_equal(o.gola_get(leaves), u.gol_get(par)), f"step {step}"


def test_list_overflow_aborts_like_reference():
    """solve.hpp:98-101: more than 8 distinct live level-0 neighbors abort."""
    o = O.Grid((3, 3, 3), 1, (False, False, False), 1, 1)
    ids, _ = o.cells()
    o.gola_set(ids, np.ones(ids.size, np.uint32))
    with pytest.raises(RuntimeError, match="No more room"):
        o.gola_steps(1)
