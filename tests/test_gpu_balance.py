"""Repartition (balance_load, make_new_partition
dccrg.hpp:8349-8581, continue/finish_balance_load 3899-4147) on one GPU
through detached per-rank views: every view moves to the same new partition
(the reference's pin path: a pinned cell goes to its process, the rest stay,
8426-8518), its structures must equal the oracle's per-rank views of that
partition, the payload of every cell that stays must survive the rebuild,
and - with the migrated payloads moved in wire order by the test, as RCCL
does between real ranks - a game of life continued on the new partition
must equal one rank's."""
import numpy as np
import pytest

import dccrg_amd
from helpers import make_pair
from test_gpu_multirank import emulated_exchange, views

pytestmark = pytest.mark.gpu


def pinned_partition(ids, owners, P, frac, seed):
    """make_new_partition's pin path: pinned cells move to their process."""
    rng = np.random.default_rng(seed)
    new = owners.copy()
    pick = rng.choice(ids.size, size=int(frac * ids.size), replace=False)
    new[pick] = rng.integers(0, P, size=pick.size)
    return new


def check_views(gs, o, P):
    for r, g in enumerate(gs):
        assert np.array_equal(g.local_cells(), o.rank_cells(r, "local"))
        assert np.array_equal(g.inner_cells(), o.rank_cells(r, "inner"))
        assert np.array_equal(g.outer_cells(), o.rank_cells(r, "outer"))
        assert np.array_equal(g.remote_cells(), o.rank_cells(r, "remote_bdy"))
        for p in range(P):
            if p != r:
                assert np.array_equal(g.get_cells_to_send(p), o.cells_to_send(r, p)), (r, p)
                assert np.array_equal(g.get_cells_to_receive(p), o.cells_to_receive(r, p)), (r, p)


@pytest.mark.parametrize("length,R,periodic,hood,P,rounds", [
    ((10, 8, 6), 0, (False, False, False), 1, 3, 0),
    ((8, 8, 4), 2, (True, True, False), 1, 4, 2),
    ((6, 6, 6), 1, (True, False, True), 0, 2, 1),
])
def test_repartition_views_and_payload(gpu, length, R, periodic, hood, P, rounds):
    gs, o = views(length, R, periodic, hood, P, rounds, 0.15, 3)
    ids, owners = gs[0].get_cell_process()
    o_ids, o_own = o.cells()
    assert np.array_equal(ids, o_ids) and np.array_equal(owners, o_own)
    val = lambda c: (c * np.uint64(2654435761) + np.uint64(7)) & np.uint64(0xFFFFFFFF)  # noqa: E731
    for g in gs:
        f = g.add_field("val", np.uint32)
        f.set(val(g.slot_ids()[: g.n_local]).astype(np.uint32))
    new = pinned_partition(ids, owners, P, 0.3, 11)
    before = [set(g.local_cells().tolist()) for g in gs]
    for g in gs:
        g.balance_load_to(ids, new)
        got_ids, got_own = g.get_cell_process()
        assert np.array_equal(got_ids, ids) and np.array_equal(got_own, new)
    o.set_cells(ids, new)
    check_views(gs, o, P)
    for r, g in enumerate(gs):
        sl = g.slot_ids()[: g.n_local]
        stay = np.array([int(c) in before[r] for c in sl])
        got = g.fields["val"].get(0, g.n_local)
        assert np.array_equal(got[stay], val(sl[stay]).astype(np.uint32)), f"rank {r}: stayed payload changed"
    for g in gs:
        g.close()


def test_game_continues_on_new_partition(gpu):
    length, P, steps = (12, 10, 8), 3, 4
    gs, o = views(length, 1, (True, False, True), 1, P, rounds=1, frac=0.2, seed=4)
    ref, _ = make_pair(length, 1, (True, False, True), 1, rounds=1, frac=0.2, seed=4)
    rng = np.random.default_rng(8)
    rids = ref.slot_ids()[: ref.n_local]
    a0 = (rng.random(rids.size) < 0.3).astype(np.uint32)
    state = dict(zip(rids.tolist(), a0.tolist()))
    rs = ref.add_field("is_alive", np.uint32)
    rs.set(a0)
    for g in gs:
        st = g.add_field("is_alive", np.uint32)
        st.set(np.array([state[int(c)] for c in g.slot_ids()[: g.n_local]], np.uint32))

    def play(k):
        for _ in range(k):
            emulated_exchange(gs, ["is_alive"])
            for g in gs:
                g.gol_step(g.fields["is_alive"], "inner")
                g.gol_step(g.fields["is_alive"], "outer")
                g.gol_commit(g.fields["is_alive"])
            ref.gol_step(rs)
            ref.gol_commit(rs)

    play(steps)
    ids, owners = gs[0].get_cell_process()
    new = pinned_partition(ids, owners, P, 0.4, 5)
    # the migration's wire content: each moved cell's payload from its old owner
    moved = {}
    for r, g in enumerate(gs):
        sl = g.slot_ids()[: g.n_local]
        vals = g.fields["is_alive"].get(0, g.n_local)
        for c, v in zip(sl.tolist(), vals.tolist()):
            moved[c] = v
    for g in gs:
        g.balance_load_to(ids, new)
    for r, g in enumerate(gs):
        sl = g.slot_ids()[: g.n_local]
        cur = g.fields["is_alive"].get(0, g.n_local)
        idx = np.searchsorted(ids, sl)
        incoming = owners[idx] != r
        cur[incoming] = np.array([moved[int(c)] for c in sl[incoming]], np.uint32)
        g.fields["is_alive"].set(cur)
    play(steps)
    final = dict(zip(rids.tolist(), rs.get(0, ref.n_local).tolist()))
    for g in gs:
        sl = g.slot_ids()[: g.n_local]
        assert np.array_equal(g.fields["is_alive"].get(0, g.n_local), np.array([final[int(c)] for c in sl]))
    for g in gs + [ref]:
        g.close()


def test_single_rank_balance(gpu):
    g, _ = make_pair((6, 5, 4), 0, (False, False, False), 1)
    ids, owners = g.get_cell_process()
    assert np.all(owners == 0)
    f = g.add_field("v", np.float64)
    f.set(np.arange(g.n_local, dtype=np.float64))
    g.pin(int(ids[3]), 0)
    g.balance_load()
    g.balance_load_to(ids, owners)
    assert np.array_equal(f.get(0, g.n_local), np.arange(g.n_local, dtype=np.float64))
    with pytest.raises(dccrg_amd.DccrgError, match="out of range"):
        g.balance_load_to(ids, owners + 1)
    g.close()


def test_iterators_test1_invariants_over_random_partitions(gpu):
    """tests/iterators/test1.cpp: a 1000 x 1 x 1 grid, neighborhood length 3,
    five rounds of random load balancing; after each, every rank's inner
    cells are exactly its local cells whose neighbors_of and neighbors_to are
    all local, outer cells the rest, and every remote cell on the process
    boundary is a non-local neighbor of a local cell.  The random partition
    is the test's (RANDOM partitioner, here a seeded owner per cell through
    balance_load_to), the invariants are the reference's."""
    P = 3
    gs = []
    for r in range(P):
        g = dccrg_amd.Dccrg(r, P, 0).set_initial_length((1000, 1, 1)).set_neighborhood_length(3)
        g.set_maximum_refinement_level(0).initialize()
        gs.append(g)
    rng = np.random.default_rng(21)
    for _ in range(5):
        ids, _ = gs[0].get_cell_process()
        new = rng.integers(0, P, size=ids.size).astype(np.int32)
        for g in gs:
            g.balance_load_to(ids, new)
        for r, g in enumerate(gs):
            inner_ref, outer_ref, remote_ref = set(), set(), set()
            for c in g.local_cells().tolist():
                assert g.is_local(c)
                nb = [i for i, _ in g.get_neighbors_of(c)] + [i for i, _ in g.get_neighbors_to(c)]
                nonlocal_nb = [i for i in nb if not g.is_local(i)]
                (outer_ref if nonlocal_nb else inner_ref).add(c)
                remote_ref.update(nonlocal_nb)
            assert set(g.inner_cells().tolist()) == inner_ref
            assert set(g.outer_cells().tolist()) == outer_ref
            assert set(g.remote_cells().tolist()) == remote_ref
            assert np.all(new[np.searchsorted(ids, g.local_cells())] == r)
    for g in gs:
        g.close()
