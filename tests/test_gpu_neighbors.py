"""Device neighbor construction vs the oracle (literal restatement of the
reference's walk, dccrg.hpp:4339-4861, face lists 2806-2933), bit-exact:
ids, stencil order, offsets, neighbors_to sets, face lists, iterator sets."""
import numpy as np
import pytest

from helpers import compare_neighbors, make_pair, make_pair_refined_by_product

pytestmark = pytest.mark.gpu

UNIFORM = [
    ((1, 1, 1), (False, False, False), 0), ((1, 1, 1), (True, True, True), 1), ((1, 1, 1), (True, True, True), 2),
    ((3, 1, 1), (False, False, False), 1), ((1, 3, 1), (True, False, True), 1), ((2, 2, 2), (True, True, True), 1),
    ((5, 4, 3), (False, False, False), 1), ((5, 4, 3), (True, True, True), 1), ((6, 5, 4), (True, False, True), 2),
    ((7, 3, 2), (False, True, False), 0), ((10, 10, 10), (True, True, True), 2), ((15, 15, 1), (False, False, False), 1),
]


@pytest.mark.parametrize("length,periodic,hood", UNIFORM)
def test_uniform(gpu, length, periodic, hood):
    g, o = make_pair(length, 0, periodic, hood)
    assert compare_neighbors(g, o) == int(np.prod(length))
    g.close()


REFINED = [
    ((1, 1, 1), 1, (False, False, False), 1, 1, 1.0, 0),
    ((1, 1, 1), 1, (True, True, True), 1, 1, 1.0, 1),
    ((2, 1, 1), 1, (False, False, False), 0, 1, 0.5, 2),
    ((4, 4, 4), 2, (False, False, False), 1, 2, 0.15, 3),
    ((4, 4, 4), 2, (True, True, True), 1, 2, 0.15, 4),
    ((5, 3, 4), 2, (True, False, True), 0, 2, 0.2, 5),
    ((6, 6, 2), 2, (True, True, False), 0, 2, 0.2, 6),
    ((3, 3, 3), 3, (False, True, False), 1, 3, 0.1, 7),
    ((4, 4, 4), 2, (True, True, True), 2, 2, 0.1, 8),
    ((8, 8, 8), 2, (False, False, False), 1, 2, 0.05, 9),
]


@pytest.mark.parametrize("length,R,periodic,hood,rounds,frac,seed", REFINED)
def test_refined(gpu, length, R, periodic, hood, rounds, frac, seed):
    g, o = make_pair(length, R, periodic, hood, rounds, frac, seed)
    gi = np.sort(g.local_cells())
    oi, _ = o.cells()
    assert np.array_equal(gi, oi)
    compare_neighbors(g, o)
    g.close()


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_refinement_closure_matches(gpu, seed):
    """refine_completely + stop_refining (induce_refines 9591-9720 closure,
    children inherit owners) give the same leaf set as the oracle."""
    g, o = make_pair_refined_by_product((4, 3, 3), 2, (seed % 2 == 0, False, True), seed % 3, 2, 0.2, seed)
    oi, _ = o.cells()
    assert np.array_equal(np.sort(g.local_cells()), oi)
    compare_neighbors(g, o)
    g.close()


def test_face_cache_kat_through_product(gpu, golden_dir):
    """The reference's own face-neighbor KATs (tests/get_neighbors_/test1.cpp),
    checked through the device face lists: the first face neighbor per
    direction is the cached neighbors_ entry."""
    import json
    import os

    import dccrg_amd

    cases = json.load(open(os.path.join(golden_dir, "kat_face_cache.json")))
    for c in cases:
        g = dccrg_amd.Dccrg(0, 1, 0)
        g.set_initial_length(c["length"]).set_maximum_refinement_level(c["R"]).set_periodic(*c["periodic"])
        g.set_neighborhood_length(c["hood"]).initialize()
        for r in c["refine"]:
            g.refine_completely(r)
        if c["refine"]:
            g.stop_refining()
        for cell, exp in c["expected"].items():
            fl = g.get_face_neighbors_of(int(cell))
            first = {}
            for nid, d in fl:
                first.setdefault(d, nid)
            got = [first.get(d, 0) for d in (-1, 1, -2, 2, -3, 3)]
            assert got == exp, (c, cell, fl)
        g.close()


def test_large_uniform_counts(gpu):
    """Full-size property: on a 256x256x64 non-periodic grid with hood 1 the
    neighbor count of a cell is prod over dims of (#valid of {-1,0,1}) - 1."""
    g, _ = make_pair((256, 256, 64), 0, (False, False, False), 1)
    ptr, ids, offs = g.csr("of")
    slots = g.slot_ids()
    idx = slots - 1
    x, y, z = idx % 256, (idx // 256) % 256, idx // (256 * 256)

    def nv(v, n):
        return 1 + (v > 0) + (v < n - 1)

    exp = nv(x, 256) * nv(y, 256) * nv(z, 64) - 1
    assert np.array_equal(np.diff(ptr.astype(np.int64)), exp)
    g.close()
