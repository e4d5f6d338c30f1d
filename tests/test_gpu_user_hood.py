"""User neighborhoods (add_neighborhood dccrg.hpp:6383-6520,
update_user_neighbors 8974-8980, the id's send / receive lists 8590-8752):
neighbor lists per id against the oracle's literal find_neighbors_of walk
with the user offsets, the reference's neighbor_list_length KAT
(tests/user_neighborhood/neighbor_list_length.cpp), neighbors_to as the
inverse of neighbors_of, per-rank send / receive lists of an id on detached
views, and add_neighborhood's refusals."""
import json
import os

import numpy as np
import pytest

import dccrg_amd
from helpers import make_pair
from test_gpu_multirank import views

pytestmark = pytest.mark.gpu


def random_hood(rng, L, k):
    if L == 0:
        faces = [(-1, 0, 0), (1, 0, 0), (0, -1, 0), (0, 1, 0), (0, 0, -1), (0, 0, 1)]
        pick = rng.choice(6, size=k, replace=False)
        return [faces[i] for i in pick]
    items = [(x, y, z) for z in range(-L, L + 1) for y in range(-L, L + 1) for x in range(-L, L + 1)
             if (x, y, z) != (0, 0, 0)]
    pick = rng.choice(len(items), size=k, replace=False)
    return [items[i] for i in pick]


@pytest.mark.parametrize("length,R,periodic,L,rounds,k", [
    ((6, 5, 4), 0, (False, False, False), 1, 0, 5),
    ((6, 6, 6), 2, (True, True, False), 1, 2, 7),
    ((5, 5, 5), 1, (True, True, True), 2, 1, 11),
    ((6, 6, 4), 2, (False, True, True), 0, 2, 3),
])
def test_user_hood_lists_match_oracle(gpu, length, R, periodic, L, rounds, k):
    g, o = make_pair(length, R, periodic, L, rounds, 0.15, 9)
    rng = np.random.default_rng(3)
    hood = random_hood(rng, L, k)
    assert g.add_neighborhood(7, hood)
    cells = g.local_cells()
    nof = {}
    for c in cells.tolist():
        got = g.get_neighbors_of(c, 7)
        nid, off = o.neighbors_of_hood(c, hood)
        assert [i for i, _ in got] == nid.tolist(), c
        assert [list(x) for _, x in got] == off.tolist(), c
        nof[c] = set(i for i, _ in got)
    # neighbors_to of an id: the cells whose id-stencil lists this cell
    inv = {c: set() for c in cells.tolist()}
    for c, ns in nof.items():
        for n in ns:
            inv[n].add(c)
    for c in cells.tolist():
        assert set(i for i, _ in g.get_neighbors_to(c, 7)) == inv[c], c
    # the default lists are untouched
    nid, off = o.neighbors_of(int(cells[0]))
    assert [i for i, _ in g.get_neighbors_of(int(cells[0]))] == nid.tolist()
    g.remove_neighborhood(7)
    assert g.get_neighbors_of(int(cells[0]), 7) is None
    g.close()


def test_neighbor_list_length_kat(gpu, golden_dir):
    k = json.load(open(os.path.join(golden_dir, "kat_hood_counts.json")))
    g = dccrg_amd.Dccrg(0, 1, 0).set_initial_length(k["length"]).set_periodic(*[bool(p) for p in k["periodic"]])
    g.set_maximum_refinement_level(k["R"]).set_neighborhood_length(k["hood_len"]).initialize()
    cells = g.local_cells()
    for i, h in enumerate(k["hoods"]):
        hid = None
        if h["hood"] is not None:
            hid = 100 + i
            assert g.add_neighborhood(hid, h["hood"])
        for c in cells[::7].tolist():
            of = g.get_neighbors_of(c, hid)
            assert len(set(of)) == h["n_of"], (h["name"], c)
            assert len(set(i for i, _ in g.get_neighbors_to(c, hid))) == h["n_to"], (h["name"], c)
        if hid is not None:
            g.remove_neighborhood(hid)
    g.close()


@pytest.mark.parametrize("length,R,periodic,L,P,rounds", [
    ((10, 6, 5), 0, (False, False, False), 1, 3, 0),
    ((6, 6, 6), 2, (True, True, False), 1, 4, 2),
    ((8, 6, 4), 1, (True, False, True), 2, 2, 1),
])
def test_user_hood_update_lists(gpu, length, R, periodic, L, P, rounds):
    gs, o = views(length, R, periodic, L, P, rounds, 0.15, 5)
    rng = np.random.default_rng(4)
    hood = random_hood(rng, L, 4 if L else 2)
    for g in gs:
        assert g.add_neighborhood(3, hood)
    ids, owners = o.cells()
    owner = dict(zip(ids.tolist(), owners.tolist()))
    recv = {}
    for r in range(P):
        for c in ids[owners == r].tolist():
            nid, _ = o.neighbors_of_hood(c, hood)
            for n in nid.tolist():
                if owner[n] != r:
                    recv.setdefault((r, owner[n]), set()).add(n)
    for r, g in enumerate(gs):
        for p in range(P):
            if p == r:
                continue
            exp_r = sorted(recv.get((r, p), ()))
            exp_s = sorted(recv.get((p, r), ()))
            assert g.get_cells_to_receive(p, 3).tolist() == exp_r, (r, p)
            assert g.get_cells_to_send(p, 3).tolist() == exp_s, (r, p)
            # a user id's lists are a subset of the default ones
            assert set(exp_r) <= set(g.get_cells_to_receive(p).tolist())
    for g in gs:
        g.close()


def test_add_neighborhood_refusals(gpu):
    g, _ = make_pair((5, 5, 5), 0, (True, True, True), 1)
    assert not g.add_neighborhood(dccrg_amd.grid.DEFAULT_HOOD, [(1, 0, 0)])
    assert g.add_neighborhood(1, [(1, 0, 0)])
    assert not g.add_neighborhood(1, [(0, 1, 0)])  # existing id
    assert not g.add_neighborhood(2, [(2, 0, 0)])  # outside the default length 1
    assert not g.add_neighborhood(3, [(0, 0, 0)])
    g.close()
    f, _ = make_pair((5, 5, 5), 0, (True, True, True), 0)
    assert f.add_neighborhood(1, [(0, 0, -1), (1, 0, 0)])
    assert not f.add_neighborhood(2, [(1, 1, 0)])  # face neighborhood: unit face offsets only
    f.close()
