"""Game of life on the device (structured kernel for uniform single-rank
grids, CSR kernel otherwise) vs the oracle and the reference's KATs:
bit-exact uint32 state."""
import json
import os

import numpy as np
import pytest

import dccrg_amd
from helpers import make_pair

pytestmark = pytest.mark.gpu


def _alive(ids, p=0.25, seed=0):
    # seeded alive(id) rule: splitmix64(id ^ 0x5DEECE66D) < p*2^64
    z = (ids.astype(np.uint64) ^ np.uint64(0x5DEECE66D)) + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    z = z ^ (z >> np.uint64(31))
    return (z < np.uint64(int(p * 2 ** 64))).astype(np.uint32)


def _run(g, o, steps):
    st = g.add_field("is_alive", np.uint32)
    ids = g.slot_ids()
    a0 = _alive(ids)
    st.set(a0)
    o.gol_set(ids, a0)
    for _ in range(steps):
        g.gol_step(st)
        g.gol_commit(st)
    o.gol_steps(steps)
    return st.get(0, g.n_local), o.gol_get(ids[: g.n_local])


@pytest.mark.parametrize("length,periodic", [((16, 12, 10), (False, False, False)), ((16, 12, 10), (True, True, True)),
                                             ((70, 9, 33), (True, False, True)), ((1, 1, 1), (True, True, True)),
                                             ((2, 3, 1), (True, True, False)), ((64, 8, 40), (False, True, False)),
                                             # 256-multiples of x: the 16-B-per-lane kernel
                                             ((256, 8, 12), (False, False, False)), ((256, 6, 9), (True, True, True)),
                                             ((512, 5, 40), (True, False, False)), ((256, 1, 1), (True, True, True))])
def test_structured_matches_oracle(gpu, length, periodic):
    g, o = make_pair(length, 0, periodic, 1)
    got, exp = _run(g, o, 6)
    assert np.array_equal(got, exp)
    g.close()


@pytest.mark.parametrize("hood", [0, 2])
def test_csr_uniform_matches_oracle(gpu, hood):
    g, o = make_pair((9, 8, 7), 0, (True, False, True), hood)
    got, exp = _run(g, o, 4)
    assert np.array_equal(got, exp)
    g.close()


def test_csr_refined_matches_oracle(gpu):
    g, o = make_pair((6, 6, 6), 2, (False, True, False), 1, rounds=2, frac=0.15, seed=3)
    got, exp = _run(g, o, 4)
    assert np.array_equal(got, exp)
    g.close()


def _kat_grid(k):
    g = dccrg_amd.Dccrg(0, 1, 0)
    g.set_initial_length(k["length"]).set_maximum_refinement_level(k["R"]).set_periodic(*k["periodic"])
    g.set_neighborhood_length(k["hood_len"]).initialize()
    return g


def test_reference_kat_game_of_life_test(gpu, golden_dir):
    k = json.load(open(os.path.join(golden_dir, "kat_gol.json")))["game_of_life_test"]
    g = _kat_grid(k)
    st = g.add_field("is_alive", np.uint32)
    ids = g.slot_ids()
    st.set(np.isin(ids, np.array(k["initial_live"], np.uint64)).astype(np.uint32))
    pos = {int(c): i for i, c in enumerate(ids)}
    for step in range(k["steps"]):
        s = st.get()
        for c in k["always_alive"] + (k["alive_even"] if step % 2 == 0 else k["alive_odd"]) + k["glider"].get(
                str(step), []):
            assert s[pos[c]], (step, c)
        g.gol_step(st)
        g.gol_commit(st)
    g.close()


def test_reference_kat_blinker(gpu, golden_dir):
    k = json.load(open(os.path.join(golden_dir, "kat_gol.json")))["simple_game_of_life"]
    g = _kat_grid(k)
    st = g.add_field("is_alive", np.uint32)
    ids = g.slot_ids()
    st.set(np.isin(ids, np.array(k["initial_live"], np.uint64)).astype(np.uint32))
    pos = {int(c): i for i, c in enumerate(ids)}
    for turn in range(k["steps"]):
        g.gol_step(st)
        g.gol_commit(st)
        s = st.get()
        even = turn % 2 == 0
        assert all(s[pos[c]] for c in k["always_alive"])
        assert all(bool(s[pos[c]]) == even for c in k["alive_after_even_turn"])
        assert all(bool(s[pos[c]]) != even for c in k["dead_after_even_turn"])
    g.close()


def _numpy_gol(a, steps):
    """Independent vectorized checker (non-periodic, 26-point) for full sizes."""
    a = a.astype(np.uint8)
    for _ in range(steps):
        p = np.pad(a, 1)
        c = np.zeros(a.shape, np.uint8)
        for dz in (0, 1, 2):
            for dy in (0, 1, 2):
                for dx in (0, 1, 2):
                    if dx == dy == dz == 1:
                        continue
                    c += p[dz:dz + a.shape[0], dy:dy + a.shape[1], dx:dx + a.shape[2]]
        a = np.where(c == 3, 1, np.where(c == 2, a, 0)).astype(np.uint8)
    return a


def test_config2_full_size(gpu):
    """BASELINE config 2 (1024x1024x64, hood 1, non-periodic) for 3 steps
    against an independent vectorized checker at full size."""
    nx, ny, nz = 1024, 1024, 64
    g = dccrg_amd.Dccrg(0, 1, 0).set_initial_length((nx, ny, nz)).set_neighborhood_length(1)
    g.set_maximum_refinement_level(0).initialize()
    st = g.add_field("is_alive", np.uint32)
    ids = np.arange(1, nx * ny * nz + 1, dtype=np.uint64)
    a0 = _alive(ids)
    st.set(a0)
    for _ in range(3):
        g.gol_step(st)
        g.gol_commit(st)
    got = st.get().reshape(nz, ny, nx)
    exp = _numpy_gol(a0.reshape(nz, ny, nx), 3)
    assert np.array_equal(got, exp)
    g.close()
