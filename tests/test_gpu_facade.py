"""The C++ drop-in facade (include/dccrg.hpp) end to end on the GPU: the
example programs (built in-tree by __graft_entry__.build()) run as separate
processes and their results equal the oracle's game of life.
game_of_life_items is the reference's examples/game_of_life.cpp loop
(cell.neighbors_of / neighbor.data over the iteration items) next to the
device sweep; game_of_life is BASELINE config 1's driver on the device sweep."""
import os
import re
import subprocess

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "examples", "bin")


def alive0(ids):
    z = (ids ^ np.uint64(0x5DEECE66D)) + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    z = z ^ (z >> np.uint64(31))
    return (z < np.uint64(int(0.2 * 2 ** 64))).astype(np.uint32)


def oracle_game(nx, ny, turns):
    o = O.Grid((nx, ny, 1), 0, (False, False, False), 1, 1)
    ids, _ = o.cells()
    o.gol_set(ids, alive0(ids))
    o.gol_steps(turns)
    a = o.gol_get(ids)
    return int(a.sum()), int(ids[a > 0].astype(np.uint64).sum())


def run(args):
    exe = os.path.join(BIN, args[0])
    if not os.path.exists(exe):
        pytest.fail(f"{exe} missing: run __graft_entry__.build() first")
    r = subprocess.run([exe] + [str(a) for a in args[1:]], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_reference_style_item_loop_matches_oracle(gpu):
    out = run(["game_of_life_items", 48, 40, 12])
    m = re.search(r"live (\d+) idsum (\d+) agree (\d)", out)
    assert m and m.group(3) == "1", out
    assert (int(m.group(1)), int(m.group(2))) == oracle_game(48, 40, 12)


def test_config1_driver_matches_oracle(gpu):
    out = run(["game_of_life", 20])
    m = re.search(r"cells (\d+) turns (\d+) live (\d+)", out)
    assert m, out
    assert int(m.group(1)) == 250000
    assert int(m.group(3)) == oracle_game(500, 500, 20)[0]
