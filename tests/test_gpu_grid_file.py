"""Grid files (save_grid_data dccrg.hpp:1089-1740,
load_grid_data 1742-2425, layout 1104-1120): the product's file is byte for
byte the oracle's restatement of the layout, whose grid block is pinned to
the reference's own writers (tests/golden/grid_file_ref.json); loading
restores the mesh, geometry and transferred payloads; files from three real
ranks: test_gpu_transport.py::test_save_grid_data_three_ranks."""
import os

import numpy as np
import pytest

import dccrg_amd
from helpers import make_pair
from oracle import oracle as O

pytestmark = pytest.mark.gpu

GEOM = ((0.5, -1.0, 2.0), (0.25, 0.125, 1.5))


def fill(g, seed):
    """Transferred u32 + f64 fields and one local-only f64 field, values by id."""
    ids = g.slot_ids()[: g.n_local]
    a = g.add_field("a", np.uint32)
    b = g.add_field("b", np.float64)
    c = g.add_field("c", np.float64, False)
    a.set((ids * np.uint64(2654435761) + np.uint64(seed)).astype(np.uint32))
    b.set(np.sin(ids.astype(np.float64) * 0.37 + seed))
    c.set(np.full(ids.size, 9.0))
    return ids


def payload(cid, seed):
    v = np.array([(cid * 2654435761 + seed) & 0xFFFFFFFF], np.uint32).tobytes()
    return v + np.array([np.sin(cid * 0.37 + seed)], np.float64).tobytes()


@pytest.mark.parametrize("length,R,periodic,hood,rounds", [
    ((4, 3, 2), 2, (True, False, True), 1, 2),
    ((6, 5, 4), 0, (False, False, False), 2, 0),
])
def test_file_bytes_and_round_trip(gpu, tmp_path, length, R, periodic, hood, rounds):
    g, o = make_pair(length, R, periodic, hood, rounds, 0.2, 3)
    g.set_geometry(*GEOM)
    fill(g, 5)
    path = tmp_path / "grid.dc"
    header = b"user header!"
    g.save_grid_data(path, offset=16, header=header)
    got = open(path, "rb").read()
    block = O.grid_block_bytes(length, R, hood, periodic, *GEOM)
    cells = g.local_cells()
    exp = O.grid_file_bytes(block, header, 16, [cells], lambda c: payload(c, 5))
    assert got == exp
    # load into a fresh grid with the same transferred fields
    h = dccrg_amd.Dccrg(0, 1, 0)
    a = h.add_field("a", np.uint32)
    b = h.add_field("b", np.float64)
    c = h.add_field("c", np.float64, False)
    h.load_grid_data(path, offset=16, header_bytes=len(header))
    assert np.array_equal(h.local_cells(), cells)
    assert h.get_maximum_refinement_level() == R
    ids = h.slot_ids()[: h.n_local]
    assert np.array_equal(a.get(0, h.n_local), (ids * np.uint64(2654435761) + np.uint64(5)).astype(np.uint32))
    assert np.array_equal(b.get(0, h.n_local), np.sin(ids.astype(np.float64) * 0.37 + 5))
    assert np.all(c.get(0, h.n_local) == 0)
    cg, Lg = g.geometry(cells)
    ch, Lh = h.geometry(cells)
    assert np.array_equal(cg, ch) and np.array_equal(Lg, Lh)
    # neighbor structure of the loaded grid matches the original
    for cid in cells[:: max(1, cells.size // 40)].tolist():
        assert h.get_neighbors_of(cid) == g.get_neighbors_of(cid)
    g.close()
    h.close()


def test_load_rejects_bad_files(gpu, tmp_path):
    p = tmp_path / "bad.dc"
    p.write_bytes(b"\0" * 256)
    h = dccrg_amd.Dccrg(0, 1, 0)
    with pytest.raises(dccrg_amd.DccrgError, match="endianness"):
        h.load_grid_data(p)
    h.close()
    h = dccrg_amd.Dccrg(0, 1, 0)
    with pytest.raises(dccrg_amd.DccrgError, match="cannot open"):
        h.load_grid_data(os.path.join(str(tmp_path), "missing.dc"))
    h.close()
    # a grid block the setters would refuse (the neighborhood
    # length, refinement level and lengths of a file are validated)
    import struct

    for hood, R, length in ((99, 0, (4, 4, 4)), (1, 60, (4, 4, 4)), (1, 0, (0, 4, 4))):
        block = O.grid_block_bytes(length, R, hood, (False, False, False), (0, 0, 0), (1, 1, 1))
        p.write_bytes(struct.pack("<Q", 0x1234567890ABCDEF) + block + struct.pack("<Q", 0))
        h = dccrg_amd.Dccrg(0, 1, 0)
        with pytest.raises(dccrg_amd.DccrgError, match="grid file"):
            h.load_grid_data(p)
        h.close()
