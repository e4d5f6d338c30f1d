"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes wrapper over ``oracle/liboracle.so`` (the CPU restatement of the
reference in ``oracle/dccrg_oracle.cpp``).  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module; the product (``dccrg_amd``) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

u64p = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")


def build() -> str:
    path = os.path.join(_HERE, "liboracle.so")
    src = os.path.join(_HERE, "dccrg_oracle.cpp")
    if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", _HERE, "liboracle.so"], check=True)
    return path


def lib():
    global _LIB
    if _LIB is not None:
        return _LIB
    L = C.CDLL(build())
    L.or_last_error.restype = C.c_char_p
    L.or_last_cell.restype = C.c_uint64
    L.or_last_cell.argtypes = [u64p, C.c_int]
    L.or_max_possible_level.argtypes = [u64p]
    L.or_map_batch.argtypes = [u64p, C.c_int, u64p, C.c_size_t, i32p, u64p, u64p, u64p, u64p, u64p, u64p]
    L.or_from_indices_batch.argtypes = [u64p, C.c_int, u64p, i32p, C.c_size_t, u64p]
    L.or_grid_create.restype = C.c_void_p
    L.or_grid_create.argtypes = [u64p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint, C.c_int]
    L.or_grid_destroy.argtypes = [C.c_void_p]
    L.or_grid_set_cells.argtypes = [C.c_void_p, u64p, i32p, C.c_size_t]
    L.or_grid_num_cells.restype = C.c_size_t
    L.or_grid_num_cells.argtypes = [C.c_void_p]
    L.or_grid_cells.argtypes = [C.c_void_p, u64p, i32p]
    L.or_refine_completely.argtypes = [C.c_void_p, C.c_uint64]
    L.or_unrefine_completely.argtypes = [C.c_void_p, C.c_uint64]
    L.or_dont_unrefine.argtypes = [C.c_void_p, C.c_uint64]
    L.or_dont_refine.argtypes = [C.c_void_p, C.c_uint64]
    L.or_removed.restype = C.c_size_t
    L.or_removed.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    L.or_stop_refining.restype = C.c_int64
    L.or_stop_refining.argtypes = [C.c_void_p]
    L.or_neighbors_.argtypes = [C.c_void_p, C.c_uint64, u64p]
    L.or_neighbors.restype = C.c_int64
    L.or_neighbors.argtypes = [C.c_void_p, C.c_uint64, C.c_int, u64p, i32p, C.c_size_t]
    L.or_neighbors_of_hood.restype = C.c_int64
    L.or_neighbors_of_hood.argtypes = [C.c_void_p, C.c_uint64, i32p, C.c_size_t, u64p, i32p, C.c_size_t]
    L.or_face_neighbors.restype = C.c_int64
    L.or_face_neighbors.argtypes = [C.c_void_p, C.c_uint64, u64p, i32p, C.c_size_t]
    L.or_rank_cells.restype = C.c_int64
    L.or_rank_cells.argtypes = [C.c_void_p, C.c_int, C.c_int, u64p, C.c_size_t]
    L.or_rank_list.restype = C.c_int64
    L.or_rank_list.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, u64p, C.c_size_t]
    L.or_gol_set.argtypes = [C.c_void_p, u64p, u32p, C.c_size_t]
    L.or_gol_steps.argtypes = [C.c_void_p, C.c_int]
    L.or_gol_get.argtypes = [C.c_void_p, u64p, u32p, C.c_size_t]
    L.or_gola_set.argtypes = [C.c_void_p, u64p, u32p, C.c_size_t]
    L.or_gola_steps.argtypes = [C.c_void_p, C.c_int]
    L.or_gola_get.argtypes = [C.c_void_p, u64p, u32p, C.c_size_t]
    L.or_gola_collect.argtypes = [C.c_void_p, u64p, u64p, C.c_size_t]
    L.or_set_geometry.argtypes = [C.c_void_p, f64p, f64p]
    L.or_geometry_batch.argtypes = [C.c_void_p, u64p, C.c_size_t, f64p, f64p]
    L.or_adv_initialize.argtypes = [C.c_void_p]
    L.or_adv_prerefine.restype = C.c_int64
    L.or_adv_prerefine.argtypes = [C.c_void_p, C.c_double, C.c_double]
    L.or_adv_max_time_step.restype = C.c_double
    L.or_adv_max_time_step.argtypes = [C.c_void_p]
    L.or_adv_steps.argtypes = [C.c_void_p, C.c_int, C.c_double]
    L.or_adv_check.argtypes = [C.c_void_p, C.c_double, C.c_double, C.c_double]
    L.or_adv_adapt.argtypes = [C.c_void_p, C.c_void_p]
    L.or_adv_get.argtypes = [C.c_void_p, u64p, C.c_size_t, f64p]
    L.or_po_set.argtypes = [C.c_void_p, u64p, f64p, f64p, i32p, C.c_size_t]
    L.or_po_solve.restype = C.c_int64
    L.or_po_solve.argtypes = [C.c_void_p, C.c_uint, C.c_uint, C.c_double, C.c_double, C.c_double, C.c_int,
                              C.c_int, C.POINTER(C.c_double)]
    L.or_po_get.argtypes = [C.c_void_p, u64p, C.c_size_t, f64p]
    _LIB = L
    return L


def _err():
    return lib().or_last_error().decode()


class Mapping:
    """dccrg_mapping.hpp restated (oracle)."""

    def __init__(self, length, max_ref_lvl):
        self.len = np.ascontiguousarray(length, dtype=np.uint64)
        self.R = int(max_ref_lvl)

    @property
    def last_cell(self):
        return int(lib().or_last_cell(self.len, self.R))

    def max_possible_level(self):
        return int(lib().or_max_possible_level(self.len))

    def batch(self, ids):
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        n = ids.size
        lvl = np.empty(n, np.int32)
        ind = np.empty(3 * n, np.uint64)
        clen = np.empty(n, np.uint64)
        par = np.empty(n, np.uint64)
        ch = np.empty(n, np.uint64)
        l0 = np.empty(n, np.uint64)
        sib = np.empty(8 * n, np.uint64)
        lib().or_map_batch(self.len, self.R, ids, n, lvl, ind, clen, par, ch, l0, sib)
        return dict(level=lvl, indices=ind.reshape(n, 3), length=clen, parent=par, child=ch,
                    level0_parent=l0, siblings=sib.reshape(n, 8))

    def from_indices(self, ind, lvl):
        ind = np.ascontiguousarray(np.asarray(ind, dtype=np.uint64).reshape(-1))
        lvl = np.ascontiguousarray(np.asarray(lvl, dtype=np.int32).reshape(-1))
        out = np.empty(lvl.size, np.uint64)
        lib().or_from_indices_batch(self.len, self.R, ind, lvl, lvl.size, out)
        return out


class Grid:
    """Single-address-space restatement of dccrg's global cell structures."""

    def __init__(self, length, max_ref_lvl=0, periodic=(False, False, False), hood_len=1, nprocs=1):
        self.length = tuple(int(x) for x in length)
        self.R = int(max_ref_lvl)
        self.periodic = tuple(bool(p) for p in periodic)
        self.hood_len = int(hood_len)
        self.nprocs = int(nprocs)
        self.h = lib().or_grid_create(np.asarray(self.length, np.uint64), self.R, *[int(p) for p in self.periodic],
                                      self.hood_len, self.nprocs)
        if not self.h:
            raise RuntimeError(_err())
        self.mapping = Mapping(self.length, self.R)

    def __del__(self):
        h = getattr(self, "h", None)
        if h and _LIB is not None:
            _LIB.or_grid_destroy(h)
            self.h = None

    def _chk(self, rc):
        if rc < 0:
            raise RuntimeError(_err())
        return rc

    def cells(self):
        n = lib().or_grid_num_cells(self.h)
        ids = np.empty(n, np.uint64)
        own = np.empty(n, np.int32)
        lib().or_grid_cells(self.h, ids, own)
        return ids, own

    def set_cells(self, ids, owners):
        ids = np.ascontiguousarray(ids, np.uint64)
        owners = np.ascontiguousarray(owners, np.int32)
        self._chk(lib().or_grid_set_cells(self.h, ids, owners, ids.size))

    def refine_completely(self, cell):
        return bool(lib().or_refine_completely(self.h, int(cell)))

    def unrefine_completely(self, cell):
        return bool(self._chk(lib().or_unrefine_completely(self.h, int(cell))))

    def dont_unrefine(self, cell):
        return bool(lib().or_dont_unrefine(self.h, int(cell)))

    def dont_refine(self, cell):
        return bool(lib().or_dont_refine(self.h, int(cell)))

    def removed(self):
        """Cells removed by the last stop_refining (ascending) and their
        parent's process."""
        n = lib().or_removed(self.h, None, None)
        ids = np.empty(n, np.uint64)
        own = np.empty(n, np.int32)
        lib().or_removed(self.h, ids.ctypes.data, own.ctypes.data)
        return ids, own

    def stop_refining(self):
        return self._chk(lib().or_stop_refining(self.h))

    def neighbors_(self, cell):
        out = np.empty(6, np.uint64)
        if lib().or_neighbors_(self.h, int(cell), out) != 0:
            return None
        return out

    def _nl(self, cell, kind):
        cap = 4096
        ids = np.empty(cap, np.uint64)
        offs = np.empty(3 * cap, np.int32)
        n = self._chk(lib().or_neighbors(self.h, int(cell), kind, ids, offs, cap))
        return ids[:n].copy(), offs[: 3 * n].reshape(n, 3).copy()

    def neighbors_of(self, cell):
        """find_neighbors_of in stencil order (dccrg.hpp:4339-4680)."""
        return self._nl(cell, 0)

    def neighbors_to(self, cell):
        """find_neighbors_to, sorted by id (dccrg.hpp:4708-4861)."""
        return self._nl(cell, 1)

    def iterator_neighbors_of(self, cell):
        """cell.neighbors_of of the iterators (dccrg.hpp:11451-11500)."""
        return self._nl(cell, 2)

    def neighbors_of_hood(self, cell, hood):
        hood = np.ascontiguousarray(np.asarray(hood, np.int32).reshape(-1))
        cap = 4096
        ids = np.empty(cap, np.uint64)
        offs = np.empty(3 * cap, np.int32)
        n = self._chk(lib().or_neighbors_of_hood(self.h, int(cell), hood, hood.size // 3, ids, offs, cap))
        return ids[:n].copy(), offs[: 3 * n].reshape(n, 3).copy()

    def face_neighbors_of(self, cell):
        cap = 64
        ids = np.empty(cap, np.uint64)
        dirs = np.empty(cap, np.int32)
        n = self._chk(lib().or_face_neighbors(self.h, int(cell), ids, dirs, cap))
        return ids[:n].copy(), dirs[:n].copy()

    def rank_cells(self, rank, what):
        kinds = {"local": 0, "inner": 1, "outer": 2, "local_bdy": 3, "remote_bdy": 4}
        cap = lib().or_grid_num_cells(self.h) + 1
        out = np.empty(cap, np.uint64)
        n = self._chk(lib().or_rank_cells(self.h, rank, kinds[what], out, cap))
        return out[:n].copy()

    def cells_to_send(self, rank, peer):
        cap = lib().or_grid_num_cells(self.h) + 1
        out = np.empty(cap, np.uint64)
        n = self._chk(lib().or_rank_list(self.h, rank, peer, 0, out, cap))
        return out[:n].copy()

    def cells_to_receive(self, rank, peer):
        cap = lib().or_grid_num_cells(self.h) + 1
        out = np.empty(cap, np.uint64)
        n = self._chk(lib().or_rank_list(self.h, rank, peer, 1, out, cap))
        return out[:n].copy()

    # -- game of life ------------------------------------------------------
    def gol_set(self, ids, alive):
        ids = np.ascontiguousarray(ids, np.uint64)
        alive = np.ascontiguousarray(alive, np.uint32)
        lib().or_gol_set(self.h, ids, alive, ids.size)

    def gol_steps(self, steps):
        self._chk(lib().or_gol_steps(self.h, int(steps)))

    def gol_get(self, ids):
        ids = np.ascontiguousarray(ids, np.uint64)
        out = np.empty(ids.size, np.uint32)
        self._chk(lib().or_gol_get(self.h, ids, out, ids.size))
        return out

    # -- game of life on a refined grid (tests/game_of_life/solve.hpp) ----------
    def gola_set(self, ids, alive):
        ids = np.ascontiguousarray(ids, np.uint64)
        alive = np.ascontiguousarray(alive, np.uint32)
        lib().or_gola_set(self.h, ids, alive, ids.size)

    def gola_steps(self, steps):
        self._chk(lib().or_gola_steps(self.h, int(steps)))

    def gola_get(self, ids):
        ids = np.ascontiguousarray(ids, np.uint64)
        out = np.empty(ids.size, np.uint32)
        self._chk(lib().or_gola_get(self.h, ids, out, ids.size))
        return out

    def gola_collect(self, ids):
        """Only the collect loop (solve.hpp:45-109); the cells' lists data[1..8]."""
        ids = np.ascontiguousarray(ids, np.uint64)
        out = np.empty((ids.size, 8), np.uint64)
        self._chk(lib().or_gola_collect(self.h, ids, out, ids.size))
        return out

    # -- advection ---------------------------------------------------------
    def set_geometry(self, start, level_0_cell_length):
        lib().or_set_geometry(self.h, np.asarray(start, np.float64), np.asarray(level_0_cell_length, np.float64))

    def geometry(self, ids):
        ids = np.ascontiguousarray(ids, np.uint64)
        c = np.empty(3 * ids.size)
        L = np.empty(3 * ids.size)
        lib().or_geometry_batch(self.h, ids, ids.size, c, L)
        return c.reshape(-1, 3), L.reshape(-1, 3)

    def adv_initialize(self):
        self._chk(lib().or_adv_initialize(self.h))

    def adv_prerefine(self, relative_diff=0.025, diff_threshold=0.25):
        return self._chk(lib().or_adv_prerefine(self.h, relative_diff, diff_threshold))

    def adv_max_time_step(self):
        return float(lib().or_adv_max_time_step(self.h))

    def adv_steps(self, steps, dt):
        self._chk(lib().or_adv_steps(self.h, int(steps), float(dt)))

    def adv_check(self, diff_increase, diff_threshold=0.25, unrefine_sensitivity=0.5):
        self._chk(lib().or_adv_check(self.h, float(diff_increase), float(diff_threshold), float(unrefine_sensitivity)))

    def adv_adapt(self):
        out = np.zeros(2, np.int64)
        self._chk(lib().or_adv_adapt(self.h, out.ctypes.data))
        return int(out[0]), int(out[1])

    def adv_get(self, ids):
        ids = np.ascontiguousarray(ids, np.uint64)
        out = np.empty(9 * ids.size)
        self._chk(lib().or_adv_get(self.h, ids, ids.size, out))
        return out.reshape(-1, 9)

    # ---- Poisson (tests/poisson/poisson_solve.hpp) ----
    PO_FIELDS = ("solution", "best_solution", "p0", "p1", "r0", "r1", "A_dot_p0", "scaling_factor",
                 "f_x_neg", "f_x_pos", "f_y_neg", "f_y_pos", "f_z_neg", "f_z_pos", "type")

    def po_set(self, ids, rhs, solution, types):
        """Every leaf once; types 0 solve, 1 boundary, 2 skip."""
        ids = np.ascontiguousarray(ids, np.uint64)
        self._chk(lib().or_po_set(self.h, ids, np.ascontiguousarray(rhs, np.float64),
                                  np.ascontiguousarray(solution, np.float64),
                                  np.ascontiguousarray(types, np.int32), ids.size))

    def po_solve(self, max_iterations=1000, min_iterations=0, stop_residual=1e-15, p_of_norm=2.0,
                 stop_after_residual_increase=10.0, failsafe=False, reverse=False):
        """Returns (iterations, residual).  reverse: visit cells (and sum) in
        descending id order — a second faithful order, to measure the
        reference's own summation-order noise."""
        r = C.c_double(0)
        it = self._chk(lib().or_po_solve(self.h, max_iterations, min_iterations, stop_residual, p_of_norm,
                                         stop_after_residual_increase, int(failsafe), int(reverse), C.byref(r)))
        return int(it), r.value

    def po_get(self, ids):
        ids = np.ascontiguousarray(ids, np.uint64)
        out = np.empty(16 * ids.size)
        self._chk(lib().or_po_get(self.h, ids, ids.size, out))
        return out.reshape(-1, 16)


# -- grid files (save_grid_data, dccrg.hpp:1089-1740; layout 1104-1120) -------
def grid_block_bytes(length, R, hood, periodic, start, l0):
    """The internal grid data block: Mapping::write (dccrg_mapping.hpp:576:
    3 x uint64 length, int max_ref_lvl), the neighborhood length (unsigned,
    dccrg.hpp:1216-1231), Grid_Topology::write (dccrg_topology.hpp:144:
    3 x uint8), Cartesian_Geometry::write (dccrg_cartesian_geometry.hpp:618:
    int geometry id 1, 3 x double start, 3 x double level-0 length)."""
    import struct

    return (struct.pack("<3Qi", *[int(v) for v in length], int(R)) + struct.pack("<I", int(hood))
            + struct.pack("<3B", *[1 if p else 0 for p in periodic])
            + struct.pack("<i3d3d", 1, *[float(v) for v in start], *[float(v) for v in l0]))


def stretched_geometry_block(coordinates):
    """Stretched_Cartesian_Geometry::write (dccrg_stretched_cartesian_geometry.hpp:
    652-715): int geometry id 2, the three coordinate counts as uint64, then
    each dimension's coordinates as doubles (data_size 808-817)."""
    import struct

    out = struct.pack("<i", 2) + struct.pack("<3Q", *[len(c) for c in coordinates])
    for c in coordinates:
        out += struct.pack("<%dd" % len(c), *[float(v) for v in c])
    return out


def grid_block_stretched_bytes(length, R, hood, periodic, coordinates):
    """grid_block_bytes with the stretched geometry's block in place of the
    Cartesian one (the reference's save_grid_data writes geometry.write's bytes
    there, dccrg.hpp:1216-1231)."""
    import struct

    return (struct.pack("<3Qi", *[int(v) for v in length], int(R)) + struct.pack("<I", int(hood))
            + struct.pack("<3B", *[1 if p else 0 for p in periodic]) + stretched_geometry_block(coordinates))


def grid_file_bytes(block, header, offset, cells_by_rank, data_of):
    """A whole grid file as save_grid_data lays it out: `offset` zero bytes
    (untouched by the writer), the user header, uint64 0x1234567890abcdef,
    the block, uint64 total cells, (id, data offset) per cell rank by rank,
    then the cells' data in the same order.  data_of(id) -> bytes."""
    import struct

    head = bytes(offset) + bytes(header) + struct.pack("<Q", 0x1234567890ABCDEF) + bytes(block)
    cells = [int(c) for r in cells_by_rank for c in r]
    head += struct.pack("<Q", len(cells))
    data = [bytes(data_of(c)) for c in cells]
    pos = len(head) + 16 * len(cells)
    lst = b""
    for c, d in zip(cells, data):
        lst += struct.pack("<QQ", c, pos)
        pos += len(d)
    return head + lst + b"".join(data)
