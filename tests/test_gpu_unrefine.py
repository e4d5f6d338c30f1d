"""Unrefinement and the refine overrides through the product (SURVEY §8 f1:
unrefine_completely 2560, dont_unrefine 2679, dont_refine 2744,
stop_refining 3461 = override_refines 9991 + induce_refines 9591 +
override_unrefines 9796 + execute_refines 10104) against the oracle's
literal restatement, one rank: after every stop_refining the leaf set, the
neighbor lists and the removed cells equal the oracle's; the removed cells'
payloads are exposed on the parent's process and the merged parents start
zeroed.  Several ranks: tests/test_gpu_transport.py::sc_unrefine."""
import numpy as np
import pytest

from helpers import compare_neighbors, make_pair_refined_by_product

pytestmark = pytest.mark.gpu


def val(ids):
    return ((np.asarray(ids, np.uint64) * np.uint64(2654435761) + np.uint64(7)) & np.uint64(0xFFFFFFFF)).astype(
        np.uint32)


def _round(g, o, rng, p_unref, p_dont_unref, p_ref, p_dont_ref):
    ids = g.local_cells()
    lv = np.array([g.get_refinement_level(int(c)) for c in ids])
    R = g.get_maximum_refinement_level()
    for c, l in zip(ids.tolist(), lv.tolist()):
        u = rng.random()
        if l > 0 and u < p_unref:
            assert g.unrefine_completely(c) == o.unrefine_completely(c)
        elif l > 0 and u < p_unref + p_dont_unref:
            assert g.dont_unrefine(c) and o.dont_unrefine(c)
        elif l < R and u < p_unref + p_dont_unref + p_ref:
            # both refuse a cell in, or next to a coarser one in, the dont_refine
            # set kept from the last stop_refining (2477-2491)
            assert g.refine_completely(c) == o.refine_completely(c)
        elif u < p_unref + p_dont_unref + p_ref + p_dont_ref:
            assert g.dont_refine(c) and o.dont_refine(c)


@pytest.mark.parametrize("case", [
    dict(length=(8, 8, 4), R=2, per=(False, False, False), hood=1, seed=1),
    dict(length=(6, 5, 4), R=2, per=(True, True, False), hood=0, seed=2),
    dict(length=(5, 5, 5), R=1, per=(True, False, True), hood=2, seed=3),
])
def test_unrefine_matches_oracle(gpu, case):
    g, o = make_pair_refined_by_product(case["length"], case["R"], case["per"], case["hood"], 2, 0.15, case["seed"])
    f = g.add_field("val", np.uint32)
    rng = np.random.default_rng(case["seed"] + 100)
    merged_any = False
    for it in range(4):
        f.set(val(g.slot_ids()[: g.n_local]))
        before = set(g.local_cells().tolist())
        _round(g, o, rng, 0.5, 0.05, 0.04 if it % 2 else 0.0, 0.02)
        g.stop_refining()
        o.stop_refining()
        oids, _ = o.cells()
        assert np.array_equal(g.local_cells(), oids), it
        compare_neighbors(g, o)
        rid, _ = o.removed()
        got = g.get_removed_cells()
        assert np.array_equal(np.sort(got), rid), it
        merged_any = merged_any or rid.size > 0
        # removed payloads: the children's values; parents zeroed; the rest kept
        assert np.array_equal(f.get_removed(), val(got))
        now = g.slot_ids()[: g.n_local]
        v = f.get(0, g.n_local)
        for c, x in zip(now.tolist(), v.tolist()):
            if c in before:
                assert x == int(val([c])[0])
        if got.size:
            par = set(g.mapping_batch(got)["parent"].tolist())
            pos = {c: i for i, c in enumerate(now.tolist())}
            for c in par:
                assert v[pos[c]] == 0
    assert merged_any
    g.close()


def test_unrefine_refusals(gpu):
    g, o = make_pair_refined_by_product((4, 4, 4), 2, (False, False, False), 1, 0, 0.0, 5)
    assert g.unrefine_completely(1) and o.unrefine_completely(1)  # level 0: no-op, true
    assert not g.unrefine_completely(10 ** 9)  # not a local leaf
    for gg in (g, o):
        gg.refine_completely(22)
        gg.stop_refining()
    kids = g.mapping_batch(np.array([22], np.uint64))["siblings"]  # level 0: [22, 0, ...]
    ch = [int(c) for c in np.sort(g.local_cells()) if g.get_refinement_level(int(c)) == 1
          and int(g.mapping_batch(np.array([c], np.uint64))["parent"][0]) == 22]
    assert len(ch) == 8 and int(kids[0][0]) == 22
    for gg in (g, o):
        gg.refine_completely(ch[0])
        gg.stop_refining()
    # the first child now has children: its siblings cannot be unrefined
    assert not g.unrefine_completely(ch[1])
    assert not o.unrefine_completely(ch[1])
    # dont_unrefine / dont_refine of cells that are not local leaves
    assert not g.dont_unrefine(ch[0]) and not g.dont_refine(10 ** 9)
    g.close()
