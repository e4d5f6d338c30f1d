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


def _counts(ids):
    """tests/restart/variable_cell_data.cpp's cells: id ints (0 .. id - 1) in
    every cell whose id is not a multiple of 4, none in the others (here
    modulo 23, so refined cells stay small)."""
    return np.where(ids % 4 != 0, ids % 23, 0).astype(np.uint64)


def _var_record(cid):
    n = (cid % 23) if cid % 4 else 0
    return (np.array([n], np.uint64).tobytes() + np.arange(n, dtype=np.int32).tobytes()
            + np.array([cid * 0.5], np.float64).tobytes()[2:6])


def _var_fields(g):
    size = g.add_field("size", np.uint64)
    data = g.add_variable_field("data", np.int32)
    tail = g.add_field("tail", np.float64)
    tail.set_window(2, 4)  # four bytes of each element (a datatype narrower than the object)
    return size, data, tail


def test_variable_payload_file_and_round_trip(gpu, tmp_path):
    """save_grid_data of variable-size payloads (1521-1540: what each cell's
    datatype describes, no padding): per cell the u64 count, its ints and a
    4-byte window of an f64, byte for byte as the layout restatement; the
    one-call load (one variable field: the rest of each record) and the split
    load of tests/restart/variable_cell_data.cpp (the counts first, then the
    ints sized from them: start / continue / finish_loading_grid_data 1795,
    2112, 2380) both restore every payload."""
    length, R = (5, 4, 3), 2
    g, o = make_pair(length, R, (True, False, False), 1, 2, 0.25, 7)
    g.set_geometry(*GEOM)
    size, data, tail = _var_fields(g)
    ids = g.slot_ids()[: g.n_local]
    cnt = _counts(ids)
    size.set(cnt)
    data.set([np.arange(int(k), dtype=np.int32) for k in cnt])
    tail.set(ids.astype(np.float64) * 0.5)
    path = tmp_path / "var.dc"
    g.save_grid_data(path, offset=8, header=b"hdr")
    cells = g.local_cells()
    exp = O.grid_file_bytes(O.grid_block_bytes(length, R, 1, (True, False, False), *GEOM), b"hdr", 8, [cells],
                            _var_record)
    assert open(path, "rb").read() == exp
    assert cnt.sum() > 0 and (cnt == 0).any()

    def check(h, sz, dt, tl):
        hid = h.slot_ids()[: h.n_local]
        assert np.array_equal(h.local_cells(), cells)
        k = _counts(hid)
        assert np.array_equal(sz.get(0, h.n_local), k)
        got = dt.get(0, h.n_local)
        assert all(np.array_equal(a, np.arange(int(n), dtype=np.int32)) for a, n in zip(got, k))
        want = np.zeros(h.n_local, np.float64)
        wv, tv = want.view(np.uint8).reshape(-1, 8), (hid.astype(np.float64) * 0.5).view(np.uint8).reshape(-1, 8)
        wv[:, 2:6] = tv[:, 2:6]
        assert np.array_equal(tl.get(0, h.n_local).view(np.uint8), want.view(np.uint8))

    h = dccrg_amd.Dccrg(0, 1, 0)
    f = _var_fields(h)
    h.load_grid_data(path, offset=8, header_bytes=3)
    check(h, *f)
    h.close()

    h = dccrg_amd.Dccrg(0, 1, 0)
    sz, dt, tl = _var_fields(h)
    h.start_loading_grid_data(path, offset=8, header_bytes=3)
    hid = h.slot_ids()[: h.n_local]
    h.continue_loading_grid_data(sz)
    k = sz.get(0, h.n_local)
    assert np.array_equal(k, _counts(hid))
    left = h.grid_file_bytes_left()
    assert np.array_equal(left, 4 * k + 4)
    # a request past a record's end is refused and moves nothing
    with pytest.raises(dccrg_amd.DccrgError, match="fewer bytes left"):
        h.continue_loading_grid_data(dt, k + 2)
    h.continue_loading_grid_data(dt, k)
    h.continue_loading_grid_data(tl)
    assert np.all(h.grid_file_bytes_left() == 0)
    h.finish_loading_grid_data()
    check(h, sz, dt, tl)
    with pytest.raises(dccrg_amd.DccrgError, match="no grid file"):
        h.continue_loading_grid_data(tl)
    g.close()
    h.close()


def test_variable_payload_file_empty_records(gpu, tmp_path):
    """Records of zero bytes (a cell without data, no fixed-size field):
    each cell still gets exactly its own bytes back."""
    g, _ = make_pair((6, 1, 1), 0, (False, False, False), 1, 0, 0.0, 1)
    data = g.add_variable_field("data", np.int32)
    ids = g.slot_ids()[: g.n_local]
    cnt = _counts(ids)
    data.set([np.arange(int(k), dtype=np.int32) + 7 for k in cnt])
    path = tmp_path / "empty.dc"
    g.save_grid_data(path)
    h = dccrg_amd.Dccrg(0, 1, 0)
    d = h.add_variable_field("data", np.int32)
    h.load_grid_data(path)
    hid = h.slot_ids()[: h.n_local]
    got = d.get(0, h.n_local)
    assert all(np.array_equal(a, np.arange(int(n), dtype=np.int32) + 7) for a, n in zip(got, _counts(hid)))
    # two variable-size fields cannot be split without the caller's counts
    h2 = dccrg_amd.Dccrg(0, 1, 0)
    h2.add_variable_field("x", np.int32)
    h2.add_variable_field("y", np.int32)
    with pytest.raises(dccrg_amd.DccrgError, match="several variable-size"):
        h2.load_grid_data(path)
    g.close()
    h.close()
    h2.close()


def test_save_over_longer_file_fixed_size(gpu, tmp_path):
    """save_grid_data of fixed-size fields over an older, longer file at the
    same path: like the reference (MPI_MODE_CREATE | MPI_MODE_WRONLY,
    dccrg.hpp:1131) the file is not truncated, so bytes past the new grid data
    stay (a caller's own bytes there survive), and the one-shot
    load reads every cell exactly (fixed-size records never run to the end of
    the file)."""
    path = tmp_path / "reuse_fixed.dc"
    big, _ = make_pair((9, 2, 1), 0, (False, False, False), 1, 0, 0.0, 1)
    b = big.add_field("value", np.float64)
    b.set(np.full(big.n_local, 3.5))
    big.add_field("pad", np.float64).set(np.full(big.n_local, 9.0))
    big.save_grid_data(path)
    old = open(path, "rb").read()
    g, _ = make_pair((6, 1, 1), 0, (False, False, False), 1, 0, 0.0, 1)
    v = g.add_field("value", np.float64)
    ids = g.slot_ids()[: g.n_local]
    v.set(ids.astype(np.float64) * 0.25)
    g.save_grid_data(path)
    new = open(path, "rb").read()
    assert len(new) == len(old)  # not truncated
    used = 8 + 87 + 8 + 16 * ids.size + 8 * ids.size
    assert new[used:] == old[used:]  # the bytes past the grid data are untouched
    h = dccrg_amd.Dccrg(0, 1, 0)
    hv = h.add_field("value", np.float64)
    h.load_grid_data(path)
    hid = h.slot_ids()[: h.n_local]
    assert np.array_equal(hv.get(0, h.n_local), hid.astype(np.float64) * 0.25)
    for x in (big, g, h):
        x.close()


def test_save_over_longer_file_variable_size(gpu, tmp_path):
    """The same with a variable-size field: the one-shot load infers such a
    field's bytes from the record's end, and the last record ends at the end of
    the file, so save_grid_data cuts the file at the end of its grid data
    (stale bytes of the older file must not become the last cell's
    payload).  Both the one-shot load (sizes inferred) and the split load with
    the sizes the program knows (the reference's way,
    tests/restart/variable_cell_data.cpp) restore every cell exactly."""
    path = tmp_path / "reuse.dc"
    big, _ = make_pair((9, 2, 1), 0, (False, False, False), 1, 0, 0.0, 1)
    d = big.add_variable_field("data", np.int32)
    d.set([np.full(40, 3, np.int32) for _ in range(big.n_local)])
    big.save_grid_data(path)
    old = open(path, "rb").read()
    g, _ = make_pair((6, 1, 1), 0, (False, False, False), 1, 0, 0.0, 1)
    size = g.add_field("size", np.uint64)
    data = g.add_variable_field("data", np.int32)
    ids = g.slot_ids()[: g.n_local]
    cnt = _counts(ids)
    size.set(cnt)
    data.set([np.arange(int(k), dtype=np.int32) + 7 for k in cnt])
    g.save_grid_data(path)
    new = open(path, "rb").read()
    used = 8 + 87 + 8 + 16 * ids.size + int(8 * ids.size + 4 * cnt.sum())
    assert len(old) > used and len(new) == used  # cut at the end of the grid data
    # one-shot: the variable field's sizes from the records
    h1 = dccrg_amd.Dccrg(0, 1, 0)
    h1s = h1.add_field("size", np.uint64)
    h1d = h1.add_variable_field("data", np.int32)
    h1.load_grid_data(path)
    k1 = h1s.get(0, h1.n_local)
    assert np.array_equal(k1, _counts(h1.slot_ids()[: h1.n_local]))
    got1 = h1d.get(0, h1.n_local)
    assert all(np.array_equal(a, np.arange(int(n), dtype=np.int32) + 7) for a, n in zip(got1, k1))
    # split load with the caller's sizes
    h = dccrg_amd.Dccrg(0, 1, 0)
    hs = h.add_field("size", np.uint64)
    hd = h.add_variable_field("data", np.int32)
    h.start_loading_grid_data(path)
    h.continue_loading_grid_data(hs)
    k = hs.get(0, h.n_local)
    hid = h.slot_ids()[: h.n_local]
    assert np.array_equal(k, _counts(hid))
    h.continue_loading_grid_data(hd, k)
    h.finish_loading_grid_data()
    got = hd.get(0, h.n_local)
    assert all(np.array_equal(a, np.arange(int(n), dtype=np.int32) + 7) for a, n in zip(got, k))
    for x in (big, g, h, h1):
        x.close()


def test_stretched_geometry_block_file_and_round_trip(gpu, tmp_path):
    """A grid saved with a Stretched_Cartesian_Geometry carries that
    geometry's block (dccrg_stretched_cartesian_geometry.hpp:652-715: id 2,
    the coordinate counts, the coordinates) where a Cartesian grid has its
    Cartesian block: the file is byte for byte the oracle's layout with that
    block, and loading it returns the block and the payloads; a block of
    another shape is refused."""
    length, R, periodic, hood = (4, 3, 2), 1, (False, True, False), 1
    g, _ = make_pair(length, R, periodic, hood, 1, 0.2, 3)
    coords = [[0.0, 0.5, 1.5, 3.0, 5.0], [-2.0, -1.0, 0.25, 4.0], [10.0, 10.5, 12.0]]
    block = O.stretched_geometry_block(coords)
    g.set_geometry_block(block)
    fill(g, 7)
    path = tmp_path / "stretched.dc"
    g.save_grid_data(path)
    got = open(path, "rb").read()
    exp = O.grid_file_bytes(O.grid_block_stretched_bytes(length, R, hood, periodic, coords), b"", 0,
                            [g.local_cells()], lambda c: payload(c, 7))
    assert got == exp
    h = dccrg_amd.Dccrg(0, 1, 0)
    a = h.add_field("a", np.uint32)
    b = h.add_field("b", np.float64)
    h.add_field("c", np.float64, False)
    h.load_grid_data(path)
    assert h.geometry_block() == block
    assert np.array_equal(h.local_cells(), g.local_cells())
    ids = h.slot_ids()[: h.n_local]
    assert np.array_equal(a.get(0, h.n_local), (ids * np.uint64(2654435761) + np.uint64(7)).astype(np.uint32))
    assert np.array_equal(b.get(0, h.n_local), np.sin(ids.astype(np.float64) * 0.37 + 7))
    # a Cartesian file reads back without a block
    g.set_geometry_block(b"")
    g.save_grid_data(tmp_path / "cart.dc")
    k = dccrg_amd.Dccrg(0, 1, 0)
    for n, t in (("a", np.uint32), ("b", np.float64)):
        k.add_field(n, t)
    k.add_field("c", np.float64, False)
    k.load_grid_data(tmp_path / "cart.dc")
    assert k.geometry_block() == b""
    with pytest.raises(dccrgx_error()):
        g.set_geometry_block(block[:-8])  # the counts promise one more coordinate
    for x in (g, h, k):
        x.close()


def dccrgx_error():
    return dccrg_amd.DccrgError
