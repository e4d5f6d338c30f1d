"""Refined game of life (tests/game_of_life/solve.hpp:37-170)
on the GPU: bit-exact against the oracle's literal restatement at every
step, the reference's own differential property (unrefined2d.cpp:215-240:
refined game == unrefined game per level-0 parent) through the product on
both sides, the reference's abort on list overflow as an error status, and a
3-rank emulated run (both fields halo-exchanged between the phases) equal to
one rank."""
import numpy as np
import pytest

import dccrg_amd
from helpers import make_pair
from oracle import oracle as O
from test_gpu_multirank import emulated_exchange, views
from test_oracle_gol_amr import GRID, unrefined2d_live_cells

pytestmark = pytest.mark.gpu

LIST = np.dtype((np.uint64, 8))


def refined_oracle(length, periodic, frac, seed):
    o = O.Grid(length, 1, periodic, 1, 1)
    ids, _ = o.cells()
    rng = np.random.default_rng(seed)
    for c in rng.choice(ids, size=int(frac * ids.size), replace=False):
        o.refine_completely(int(c))
    o.stop_refining()
    return o


def product_on(o, length, periodic):
    leaves, owners = o.cells()
    g = dccrg_amd.Dccrg(0, 1, 0).set_initial_length(length).set_maximum_refinement_level(1)
    g.set_periodic(*periodic).set_neighborhood_length(1).initialize()
    g.set_cells(leaves, owners)
    st = g.add_field("is_alive", np.uint32)
    ls = g.add_field("gol_list", LIST)
    return g, st, ls


def states_by_parent(o, ids, live0):
    par = o.mapping.batch(ids)["level0_parent"]
    return np.array([1 if int(p) in live0 else 0 for p in par], np.uint32), par


@pytest.mark.parametrize("length,periodic,frac,seed,density,steps", [
    ((15, 15, 1), (False, False, False), 0.5, 0, None, 25),
    ((24, 20, 1), (True, True, False), 0.5, 9, 0.35, 30),
    ((20, 1, 16), (True, False, False), 0.3, 4, 0.3, 20),
    ((9, 8, 7), (False, False, False), 0.4, 1, 0.05, 1),
    ((9, 8, 7), (True, True, True), 0.4, 2, 0.05, 1),
])
def test_refined_game_matches_oracle(gpu, length, periodic, frac, seed, density, steps):
    o = refined_oracle(length, periodic, frac, seed)
    g, st, ls = product_on(o, length, periodic)
    n0 = length[0] * length[1] * length[2]
    if density is None:
        live0 = unrefined2d_live_cells()
    else:
        rng = np.random.default_rng(seed + 50)
        live0 = {int(c) for c in np.nonzero(rng.random(n0) < density)[0] + 1}
    slots = g.slot_ids()[: g.n_local]
    a0, _ = states_by_parent(o, slots, live0)
    st.set(a0)
    o.gola_set(slots, a0)
    for step in range(steps):
        g.update_copies_of_remote_neighbors()
        g.get_live_neighbors(st, ls)
        o.gola_steps(1)
        assert np.array_equal(st.get(0, g.n_local), o.gola_get(slots)), f"step {step}"
    g.close()


@pytest.mark.parametrize("length,periodic,frac,seed,density", [
    ((15, 15, 1), (False, False, False), 0.5, 0, 0.3),
    ((24, 20, 1), (True, True, False), 0.5, 9, 0.3),
    ((9, 8, 7), (True, True, True), 0.4, 2, 0.05),
    ((2, 2, 3), (True, True, True), 0.5, 3, 0.3),
])
def test_collected_lists_match_oracle(gpu, length, periodic, frac, seed, density):
    """The lists data[1..8] after the collect loop, entry for entry (level-0
    parents of live neighbors in first-seen order, error_cell padded)."""
    o = refined_oracle(length, periodic, frac, seed)
    g, st, ls = product_on(o, length, periodic)
    n0 = length[0] * length[1] * length[2]
    rng = np.random.default_rng(seed + 7)
    live0 = {int(c) for c in np.nonzero(rng.random(n0) < density)[0] + 1}
    slots = g.slot_ids()[: g.n_local]
    a0, _ = states_by_parent(o, slots, live0)
    st.set(a0)
    o.gola_set(slots, a0)
    g.gol_amr_collect(st, ls)
    got = ls.get(0, g.n_local).reshape(-1, 8)
    assert np.array_equal(got, o.gola_collect(slots))
    g.close()


def test_unrefined2d_differential_through_product(gpu):
    """unrefined2d.cpp:104-240 with the product on both sides: the refined
    grid (random half of the cells refined, children inherit the state)
    plays get_live_neighbors, the unrefined grid plays the plain game."""
    length = (GRID, GRID, 1)
    o = refined_oracle(length, (False, False, False), 0.5, 3)
    g, st, _ = product_on(o, length, (False, False, False))
    ls = g.fields["gol_list"]
    live0 = unrefined2d_live_cells()
    slots = g.slot_ids()[: g.n_local]
    a0, par = states_by_parent(o, slots, live0)
    st.set(a0)
    u = dccrg_amd.Dccrg(0, 1, 0).set_initial_length(length).set_maximum_refinement_level(0)
    u.set_neighborhood_length(1).initialize()
    us = u.add_field("is_alive", np.uint32)
    uslots = u.slot_ids()[: u.n_local]
    us.set(np.array([1 if int(c) in live0 else 0 for c in uslots], np.uint32))
    pos = {int(c): i for i, c in enumerate(uslots)}
    idx = np.array([pos[int(p)] for p in par])
    for step in range(25):
        g.get_live_neighbors(st, ls)
        u.gol_step(us)
        u.gol_commit(us)
        assert np.array_equal(st.get(0, g.n_local), us.get(0, u.n_local)[idx]), f"step {step}"
    g.close()
    u.close()


def test_list_overflow_is_an_error(gpu):
    """solve.hpp:98-101 aborts on a 9th live level-0 neighbor; the product
    returns DCCRGX_EINVAL with the reference's message."""
    o = O.Grid((3, 3, 3), 1, (False, False, False), 1, 1)
    g, st, ls = product_on(o, (3, 3, 3), (False, False, False))
    st.set(np.ones(g.n_local, np.uint32))
    with pytest.raises(dccrg_amd.DccrgError, match="No more room"):
        g.gol_amr_collect(st, ls)
    g.close()


def test_siblings_disagreeing_is_an_error(gpu):
    """solve.hpp:81-90: a dead neighbor whose level-0 parent was already
    recorded alive through a sibling aborts the reference."""
    length = (4, 4, 1)
    o = O.Grid(length, 1, (False, False, False), 1, 1)
    o.refine_completely(6)  # level-0 cell (1, 1, 0)
    o.stop_refining()
    g, st, ls = product_on(o, length, (False, False, False))
    slots = g.slot_ids()[: g.n_local]
    par = o.mapping.batch(slots)["level0_parent"]
    a = np.zeros(slots.size, np.uint32)
    kids = np.sort(slots[par == 6])
    a[np.isin(slots, kids[:1])] = 1  # first child (lowest id) alive, its siblings dead
    st.set(a)
    o.gola_set(slots, a)
    with pytest.raises(RuntimeError, match="should not be alive"):
        o.gola_steps(1)
    with pytest.raises(dccrg_amd.DccrgError, match="recorded alive"):
        g.gol_amr_collect(st, ls)
    g.close()


def test_three_rank_emulation_equals_one_rank(gpu):
    length, P = (12, 10, 1), 3
    gs, o = views(length, 1, (True, False, False), 1, P, rounds=1, frac=0.3, seed=5)
    ref, _ = make_pair(length, 1, (True, False, False), 1, rounds=1, frac=0.3, seed=5)
    rng = np.random.default_rng(2)
    live0 = {int(c) for c in np.nonzero(rng.random(120) < 0.35)[0] + 1}
    rs = ref.add_field("is_alive", np.uint32)
    rl = ref.add_field("gol_list", LIST)
    rslots = ref.slot_ids()[: ref.n_local]
    rs.set(states_by_parent(o, rslots, live0)[0])
    for g in gs:
        st = g.add_field("is_alive", np.uint32)
        g.add_field("gol_list", LIST)
        sl = g.slot_ids()[: g.n_local]
        st.set(states_by_parent(o, sl, live0)[0])
    for _ in range(8):
        emulated_exchange(gs, ["is_alive", "gol_list"])
        for g in gs:
            g.gol_amr_collect(g.fields["is_alive"], g.fields["gol_list"])
        emulated_exchange(gs, ["is_alive", "gol_list"])
        for g in gs:
            g.gol_amr_spread(g.fields["is_alive"], g.fields["gol_list"])
        ref.get_live_neighbors(rs, rl)
    final = dict(zip(rslots.tolist(), rs.get(0, ref.n_local).tolist()))
    for g in gs:
        sl = g.slot_ids()[: g.n_local]
        assert np.array_equal(g.fields["is_alive"].get(0, g.n_local), np.array([final[int(c)] for c in sl]))
    for g in gs + [ref]:
        g.close()


def test_turn_equals_split_phases_and_clears_lists(gpu):
    """dccrgx_get_live_neighbors (the whole turn, lists kept in masks and
    every local list error_cell at the end, solve.hpp:163) gives the states
    of the split form (collect, halo, spread) at every step, on a list field
    holding garbage before the first turn and after the mesh changes."""
    length = (24, 20, 1)
    o = refined_oracle(length, (True, True, False), 0.5, 9)
    g, st, ls = product_on(o, length, (True, True, False))
    h, hst, hls = product_on(o, length, (True, True, False))
    rng = np.random.default_rng(59)
    live0 = {int(c) for c in np.nonzero(rng.random(480) < 0.35)[0] + 1}
    slots = g.slot_ids()[: g.n_local]
    a0, _ = states_by_parent(o, slots, live0)
    st.set(a0)
    hst.set(a0)
    ls.set(np.full((g.n_slots, 8), 5, np.uint64))
    for step in range(18):
        if step == 9:
            # the mesh changes between turns: three level-0
            # leaves refined, one level-1 family merged, on both grids; the
            # rebuild drops the record that the inner lists are zero, and the
            # list field is filled with garbage again
            sl = g.slot_ids()[: g.n_local]
            lv0 = sl[sl <= np.uint64(480)][:3]
            lv1 = sl[sl > np.uint64(480)][:1]
            for x in (g, h):
                for c in lv0:
                    x.refine_completely(int(c))
                for c in lv1:
                    x.unrefine_completely(int(c))
                x.stop_refining()
            assert np.array_equal(g.slot_ids(), h.slot_ids())
            assert not np.array_equal(g.slot_ids()[: g.n_local], sl), "the mesh did not change"
            ls.set(np.full((g.n_slots, 8), 7, np.uint64))
        g.get_live_neighbors(st, ls)
        h.gol_amr_collect(hst, hls)
        h.update_copies_of_remote_neighbors()
        h.gol_amr_spread(hst, hls)
        assert np.array_equal(st.get(0, g.n_local), hst.get(0, h.n_local)), f"step {step}"
        assert not np.any(ls.get(0, g.n_local)), f"step {step}: lists not cleared"
    g.close()
    h.close()


def test_turn_with_disagreeing_families_follows_the_reference(gpu):
    """One refined level-0 cell with a single live child: the family
    disagrees, so the geometric collect gives way to the exact per-entry
    walk, and the turn does what the reference's loop does - abort when some
    row meets a dead child after the live one (solve.hpp:81-90; children 0-6
    here), else (child 7, always met last) the oracle's states."""
    length = (6, 6, 1)
    for k in (0, 3, 7):
        o = O.Grid(length, 1, (False, False, False), 1, 1)
        o.refine_completely(15)
        o.stop_refining()
        g, st, ls = product_on(o, length, (False, False, False))
        slots = g.slot_ids()[: g.n_local]
        kids = np.sort(slots[slots > np.uint64(36)])
        a = (slots == kids[k]).astype(np.uint32)
        st.set(a)
        o.gola_set(slots, a)
        if k == 7:
            o.gola_steps(1)
            g.get_live_neighbors(st, ls)
            assert np.array_equal(st.get(0, g.n_local), o.gola_get(slots))
        else:
            with pytest.raises(RuntimeError, match="should not be alive"):
                o.gola_steps(1)
            with pytest.raises(dccrg_amd.DccrgError, match="recorded alive"):
                g.get_live_neighbors(st, ls)
        g.close()
