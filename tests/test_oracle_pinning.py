"""Pin the oracle (CPU restatement, oracle/dccrg_oracle.cpp) to the reference:
its own Mapping/Cartesian_Geometry compiled as-is (mapping_ref.json) and the
known answers of its own tests (kat_*.json).  CPU only."""
import json
import math
import os

import numpy as np
import pytest

from oracle import oracle as O


def _load(golden_dir, name):
    with open(os.path.join(golden_dir, name)) as f:
        return json.load(f)


def test_mapping_matches_reference_headers(golden_dir):
    for g in _load(golden_dir, "mapping_ref.json"):
        m = O.Mapping(g["length"], g["max_ref_lvl"])
        assert m.last_cell == g["last_cell"]
        assert m.max_possible_level() == g["max_possible_level"]
        ids = np.array([r["id"] for r in g["ids"]], np.uint64)
        b = m.batch(ids)
        for i, r in enumerate(g["ids"]):
            assert b["level"][i] == r["level"], r
            if r["level"] < 0:
                continue
            assert list(b["indices"][i]) == r["indices"], r
            assert b["length"][i] == r["length"]
            assert b["parent"][i] == r["parent"]
            assert b["child"][i] == r["child"]
            assert b["level0_parent"][i] == r["level0_parent"]
            assert list(b["siblings"][i]) == r["siblings"]
        q = g["queries"]
        got = m.from_indices([x["indices"] for x in q], [x["level"] for x in q])
        assert [int(v) for v in got] == [x["cell"] for x in q]


def test_geometry_matches_reference_headers(golden_dir):
    for g in _load(golden_dir, "mapping_ref.json"):
        recs = [r for r in g["ids"] if r["level"] >= 0]
        if np.prod(g["length"]) > 4096:
            continue
        grid = O.Grid(g["length"], g["max_ref_lvl"])
        grid.set_geometry(g["start"], g["level_0_cell_length"])
        c, L = grid.geometry(np.array([r["id"] for r in recs], np.uint64))
        for i, r in enumerate(recs):
            assert list(c[i]) == r["center"], r  # bit-exact fp64
            assert list(L[i]) == r["cell_length"], r


@pytest.mark.parametrize("case_i", range(52))
def test_face_cache_kat(golden_dir, case_i):
    cases = _load(golden_dir, "kat_face_cache.json")
    if case_i >= len(cases):
        pytest.skip("no such case")
    c = cases[case_i]
    g = O.Grid(c["length"], c["R"], c["periodic"], c["hood"])
    for r in c["refine"]:
        g.refine_completely(r)
    if c["refine"]:
        g.stop_refining()
    ids, _ = g.cells()
    for cell, exp in c["expected"].items():
        assert int(cell) in set(int(i) for i in ids)
        assert [int(v) for v in g.neighbors_(int(cell))] == exp, (c, cell)


def test_face_neighbor_count_kat(golden_dir):
    for c in _load(golden_dir, "kat_face_counts.json"):
        g = O.Grid(c["length"], c["R"], c["periodic"], c["hood"])
        for r in c["refine"]:
            g.refine_completely(r)
        if c["refine"]:
            g.stop_refining()
        ids, _ = g.cells()
        assert sorted(int(i) for i in ids) == sorted(int(k) for k in c["counts"]), c
        for cell, n in c["counts"].items():
            nid, _ = g.face_neighbors_of(int(cell))
            assert len(nid) == n, (c, cell)
            if cell in c["first"]:
                assert int(nid[0]) == c["first"][cell]


def test_neighbor_list_length_kat(golden_dir):
    k = _load(golden_dir, "kat_hood_counts.json")
    g = O.Grid(k["length"], k["R"], k["periodic"], k["hood_len"])
    ids, _ = g.cells()
    for h in k["hoods"]:
        for cell in ids[::37]:
            if h["hood"] is None:
                nid, off = g.iterator_neighbors_of(int(cell))
                assert len(nid) == h["n_of"]
                tid, _ = g.neighbors_to(int(cell))
                assert len(tid) == h["n_to"]
            else:
                nid, off = g.neighbors_of_hood(int(cell), h["hood"])
                assert len(set(zip(nid.tolist(), map(tuple, off.tolist())))) == h["n_of"]
                inv = [[-a, -b, -c] for a, b, c in h["hood"]]
                tid, _ = g.neighbors_of_hood(int(cell), inv)
                assert len(set(tid.tolist())) == h["n_to"]


def test_game_of_life_kat(golden_dir):
    k = _load(golden_dir, "kat_gol.json")["game_of_life_test"]
    g = O.Grid(k["length"], k["R"], k["periodic"], k["hood_len"])
    ids, _ = g.cells()
    alive0 = np.isin(ids, np.array(k["initial_live"], np.uint64)).astype(np.uint32)
    g.gol_set(ids, alive0)
    pos = {int(c): i for i, c in enumerate(ids)}
    for step in range(k["steps"]):
        st = g.gol_get(ids)
        for c in k["always_alive"]:
            assert st[pos[c]], (step, c)
        for c in (k["alive_even"] if step % 2 == 0 else k["alive_odd"]):
            assert st[pos[c]], (step, c)
        for c in k["glider"].get(str(step), []):
            assert st[pos[c]], (step, c)
        g.gol_steps(1)


def test_blinker_kat(golden_dir):
    k = _load(golden_dir, "kat_gol.json")["simple_game_of_life"]
    g = O.Grid(k["length"], k["R"], k["periodic"], k["hood_len"])
    ids, _ = g.cells()
    g.gol_set(ids, np.isin(ids, np.array(k["initial_live"], np.uint64)).astype(np.uint32))
    pos = {int(c): i for i, c in enumerate(ids)}
    for turn in range(k["steps"]):
        g.gol_steps(1)
        st = g.gol_get(ids)
        for c in k["always_alive"]:
            assert st[pos[c]]
        even = turn % 2 == 0
        for c in k["alive_after_even_turn"]:
            assert bool(st[pos[c]]) == even
        for c in k["dead_after_even_turn"]:
            assert bool(st[pos[c]]) != even


def test_grid_file_block_matches_reference_writers(golden_dir):
    """save_grid_data's internal grid block as the reference's own Mapping /
    Grid_Topology / Cartesian_Geometry writers produce it
    (oracle/ref_write_probe.cpp -> tests/golden/grid_file_ref.json)."""
    for c in _load(golden_dir, "grid_file_ref.json"):
        b = O.grid_block_bytes(c["length"], c["R"], c["hood"], c["periodic"], c["start"], c["l0"])
        assert b.hex() == c["block_hex"]
        assert len(b) == c["sizes"][3]
