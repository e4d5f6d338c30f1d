"""The C++ drop-in facade (include/dccrg.hpp) end to end on the GPU.

1. The reference's own examples/game_of_life.cpp (BASELINE config 1: 500 x
   500 x 1, neighborhood 1, 100 turns, host loops over cell.neighbors_of /
   neighbor.data, the start / wait halo split), compiled against the facade
   with only its include line changed (examples/bin/ref_game_of_life, built
   by __graft_entry__.build()), runs under mpiexec at 1 and 2 ranks sharing
   the GPU (the library's host exchange over MPI).  The facade dumps the
   state the example's rand() produced as it enters turn 1 and the state
   after the last turn (DCCRGX_DUMP_CELLS); the latter must equal the
   oracle's 100-turn game from the former.
2. The repo's config-1 driver on the device sweep (examples/bin/game_of_life)
   at 1 and 2 ranks against the oracle."""
import os
import re
import subprocess

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "examples", "bin")
MPIEXEC = "/opt/conda/bin/mpiexec"
LEN = (500, 500, 1)


def alive0(ids):
    z = (ids ^ np.uint64(0x5DEECE66D)) + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    z = z ^ (z >> np.uint64(31))
    return (z < np.uint64(int(0.2 * 2 ** 64))).astype(np.uint32)


def mpirun(exe, P, args=(), env=None):
    path = os.path.join(BIN, exe)
    if not os.path.exists(path):
        pytest.fail(f"{path} missing: run __graft_entry__.build() first")
    cmd = [MPIEXEC, "-n", str(P), path] + [str(a) for a in args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


@pytest.mark.parametrize("P", [1, 2])
def test_reference_example_matches_oracle(gpu, tmp_path, P):
    dump = tmp_path / "cells"
    env = dict(os.environ, DCCRGX_DUMP_CELLS=str(dump))
    out = mpirun("ref_game_of_life", P, env=env)
    assert "Game played at" in out
    rec = np.dtype([("id", "<u8"), ("alive", "<u4"), ("count", "<u4")])

    def load(when):
        d = {}
        for r in range(P):
            raw = np.fromfile(f"{dump}.{when}.{r}", dtype=rec)
            d.update(zip(raw["id"].tolist(), raw["alive"].tolist()))
        return d

    init = load("initial")  # the example's rand() state, as it entered turn 1
    ids = np.array(sorted(init), np.uint64)
    a0 = np.array([init[int(c)] for c in ids], np.uint32)
    assert 0.15 < a0.mean() < 0.25  # rand() / RAND_MAX < 0.2
    o = O.Grid(LEN, 0, (False, False, False), 1, 1)
    o.gol_set(ids, a0)
    o.gol_steps(100)
    exp = dict(zip(ids.tolist(), o.gol_get(ids).tolist()))
    got = load("final")
    assert len(got) == 500 * 500
    assert got == exp


@pytest.mark.parametrize("P", [1, 2])
def test_config1_driver_matches_oracle(gpu, P):
    out = mpirun("game_of_life", P, [30])
    m = re.search(r"cells (\d+) turns (\d+) live (\d+)", out)
    assert m, out
    assert int(m.group(1)) == 250000
    o = O.Grid(LEN, 0, (False, False, False), 1, 1)
    ids, _ = o.cells()
    o.gol_set(ids, alive0(ids))
    o.gol_steps(30)
    assert int(m.group(3)) == int(o.gol_get(ids).sum())


def test_advection_device_members(gpu):
    """examples/advection_device.cpp: the reference's adaptive advection loop
    (tests/advection/2d.cpp, adapt every step, cfl 0.5) through the facade's
    device members only (add_field<double>, advection_initialize / _step /
    _commit / _check_adaptation / _adapt, advection_max_time_step), at 1 and
    2 processes: mass conserved over the steps (1e-13
    relative), cells created and removed, and the same counts and mass at
    both process counts."""
    res = {}
    for P in (1, 2):
        out = mpirun("advection_device", P, [16, 12])
        m = re.search(r"cells (\d+) steps (\d+) created (\d+) removed (\d+) mass0 (\S+) mass (\S+)", out)
        assert m, out
        res[P] = m.groups()
    for P in (1, 2):
        _, steps, created, removed, m0, m1 = res[P]
        assert int(steps) == 12 and int(created) > 0 and int(removed) > 0
        assert abs(float(m1) - float(m0)) <= 1e-13 * abs(float(m0)), (P, m0, m1)
    assert res[1][:4] == res[2][:4]
    assert abs(float(res[1][5]) - float(res[2][5])) <= 1e-13 * abs(float(res[1][5]))


@pytest.mark.parametrize("n", [64, 512])
def test_poisson_device_members(gpu, tmp_path, n):
    """examples/poisson_device.cpp: tests/poisson/poisson1d.cpp's solve through
    the facade's poisson_cache / poisson_solve at 1 and 3 processes, within
    the reference's 2-norm threshold (3e-7) of the reference's serial solver
    (tests/golden/poisson1d_ref.npz) after the last-cell offset."""
    from poisson_cases import POISSON1D_THRESHOLD, offset_last, p_norm, poisson1d_reference

    ref, rhs = poisson1d_reference(n)
    rf = tmp_path / "rhs.bin"
    rhs.astype("<f8").tofile(rf)
    sols = []
    for P in (1, 3):
        of = tmp_path / f"sol{P}.bin"
        out = mpirun("poisson_device", P, [n, rf, of])
        assert re.search(rf"cells {n} iterations \d+", out), out
        sols.append(offset_last(np.fromfile(of, dtype="<f8")))
    for s_ in sols:
        assert p_norm(s_, ref) <= POISSON1D_THRESHOLD
    assert p_norm(sols[0], sols[1]) <= POISSON1D_THRESHOLD


CELL_LINE = re.compile(r"Cell (\d+) data \(on process (\d+)\): ([-\d .e+]*)")


def _cell_lines(out):
    rows = []
    for m in CELL_LINE.finditer(out):
        vals = [float(v) for v in m.group(3).split()]
        rows.append((int(m.group(1)), int(m.group(2)), vals))
    return rows


@pytest.mark.parametrize("P", [2, 3])
def test_reference_variable_data_size(gpu, P):
    """tests/variable_data_size/variable_data_size.cpp compiled against the
    facade (include lines only): cell c holds c values c, c+1, ...; the
    program sizes the arriving cells between initialize_ and
    continue_balance_load and prints every cell before and after the
    balance.  Both prints must show every cell once with its own values."""
    rows = _cell_lines(mpirun("ref_variable_data_size", P))
    assert len(rows) == 6, rows
    for phase in (rows[:3], rows[3:]):
        assert sorted(c for c, _, _ in phase) == [1, 2, 3]
        for c, _, vals in phase:
            assert vals == [float(c + i) for i in range(c)]


@pytest.mark.parametrize("P", [2, 3])
def test_reference_variable_neighbour_data(gpu, P):
    """tests/variable_data_size/variable_neighbour_data.cpp against the
    facade: variables1 of every cell and variables2 of its neighbors
    (cell.neighbors_of) through a derived-datatype halo, twice around
    balances; in the last print the halo carries variables1 only, so a
    remote neighbor's variables2 is its freshly sized zeros."""
    out = mpirun("ref_variable_neighbour_data", P)
    rows = _cell_lines(out)
    assert len(rows) == 9, rows
    nbrs = {1: [2], 2: [1, 3], 3: [2]}
    for k, phase in enumerate((rows[:3], rows[3:6], rows[6:])):
        assert sorted(c for c, _, _ in phase) == [1, 2, 3]
        for c, _, vals in phase:
            assert vals[:c] == [float(c + i) for i in range(c)]
            rest = vals[c:]
            for n in nbrs[c]:
                part, rest = rest[:n], rest[n:]
                own = [float(-(n + i)) for i in range(n)]
                if k < 2:
                    assert part == own, (k, c, n, vals)
                else:
                    assert part == own or part == [0.0] * n, (k, c, n, vals)
            assert rest == []


@pytest.mark.parametrize("Ps,Pl", [(1, 1), (3, 2), (2, 3)])
def test_variable_restart(gpu, tmp_path, Ps, Pl):
    """Grid files of variable-size payloads through the facade, the scenario
    of tests/restart/variable_cell_data.cpp (examples/variable_restart.cpp:
    20 x 1 x 1 cells holding `id` ints behind a uint64 count, none when
    id % 4 == 0).  Saved by Ps processes after the cells of every third one
    moved on (an empty rank at Ps = 3), the file is the reference's layout
    (save_grid_data 1089-1740: endianness word, grid block, cell list, then
    each cell's bytes as its datatype describes them, no padding, back to
    back); loaded by Pl processes in two passes (start / continue x2 /
    finish_loading_grid_data), every cell holds its own data, also after a
    balance moves the loaded payloads."""
    import struct

    path = tmp_path / "variable_cell_data.dc"
    out = mpirun("variable_restart", Ps, ["save", path])
    assert out.count("PASS") == Ps, out
    raw = open(path, "rb").read()
    assert struct.unpack_from("<Q", raw, 0)[0] == 0x1234567890ABCDEF
    R = struct.unpack_from("<i", raw, 8 + 24)[0]
    assert raw[8:8 + 87] == O.grid_block_bytes((20, 1, 1), R, 1, (False, False, False), (0, 0, 0), (1, 1, 1))
    total = struct.unpack_from("<Q", raw, 95)[0]
    assert total == 20
    lst = np.frombuffer(raw, "<u8", 2 * total, 103).reshape(-1, 2)
    assert sorted(lst[:, 0].tolist()) == list(range(1, 21))
    pos = 103 + 16 * total
    for cid, off in sorted(lst.tolist(), key=lambda r: r[1]):
        n = cid if cid % 4 else 0
        rec = struct.pack("<Q", n) + np.arange(n, dtype="<i4").tobytes()
        assert off == pos and raw[off:off + len(rec)] == rec, cid
        pos += len(rec)
    assert pos == len(raw)
    out = mpirun("variable_restart", Pl, ["load", path])
    assert out.count("PASS") == Pl, out
    assert sum(int(m) for m in re.findall(r"PASS \d+ (\d+)", out)) == 20


@pytest.mark.parametrize("P", [1, 2])
def test_stretched_geometry_restart(gpu, tmp_path, P):
    """A Stretched_Cartesian_Geometry grid saved and loaded through the facade
    (examples/stretched_restart.cpp): the file's geometry block is the
    reference's Stretched_Cartesian_Geometry::write bytes
    (dccrg_stretched_cartesian_geometry.hpp:652-715: id 2, the coordinate
    counts, the coordinates), and the loaded grid has the same unevenly
    spaced coordinates, payloads and cell centers / lengths."""
    import struct

    path = tmp_path / "stretched.dc"
    out = mpirun("stretched_restart", P, [path])
    assert out.count("PASS") == P, out
    raw = open(path, "rb").read()
    coords = [[0.0, 0.5, 1.5, 3.0, 5.0, 5.25], [-2.0, -1.0, 0.25, 4.0, 4.5], [10.0, 10.5, 12.0, 12.125]]
    block = O.stretched_geometry_block(coords)
    assert struct.unpack_from("<Q", raw, 0)[0] == 0x1234567890ABCDEF
    assert raw[8 + 35:8 + 35 + len(block)] == block
