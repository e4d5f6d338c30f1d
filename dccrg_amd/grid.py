"""Python mirror of the reference's ``dccrg::Dccrg<Cell_Data, Geometry>`` host
interface (dccrg.hpp:145-7072) over the C ABI in ``include/dccrgx.h``.

Method names, argument meaning and chaining follow the reference so that
ports of its tests read like the originals; cell payloads are SoA device
fields instead of a ``Cell_Data`` struct.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from ._lib import EINVAL, ENOTFOUND, ERANGE, EXCHANGE_FN, DccrgError, check, lib

REGION = {"all": 0, "inner": 1, "outer": 2}
DEFAULT_HOOD = -0xDCC  # default_neighborhood_id (dccrg.hpp:93)
CELLS = {"local": 0, "inner": 1, "outer": 2, "remote": 3, "all": 4}
CSR_KIND = {"of": 0, "to": 1, "face": 2, "iterator": 3}
# neighbor types of get_cells (dccrg.hpp:95-142)
HAS_NO_NEIGHBOR, HAS_LOCAL_NEIGHBOR_OF, HAS_LOCAL_NEIGHBOR_TO = 0, 1, 2
HAS_REMOTE_NEIGHBOR_OF, HAS_REMOTE_NEIGHBOR_TO = 4, 8
HAS_LOCAL_NEIGHBOR_BOTH, HAS_REMOTE_NEIGHBOR_BOTH = 3, 12


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def _dev_ptr(t):
    """A device address: an int, or a CUDA (HIP) float64 torch tensor's data."""
    if isinstance(t, int):
        return C.c_void_p(t)
    if not (getattr(t, "is_cuda", False) and str(t.dtype) == "torch.float64" and t.is_contiguous()):
        raise TypeError("expected a contiguous float64 tensor on the GPU (or a device address)")
    return C.c_void_p(t.data_ptr())


class Field:
    """One SoA payload array over all slots (local cells, then remote copies)."""

    def __init__(self, grid, fid, name, dtype, transfer):
        self.grid, self.id, self.name, self.dtype, self.transfer = grid, fid, name, np.dtype(dtype), transfer

    def device_ptr(self):
        p = C.c_void_p()
        check(lib().dccrgx_field_device_ptr(self.grid.h, self.id, C.byref(p)))
        return p.value

    def get(self, slot0=0, n=None):
        if n is None:
            n = self.grid.n_slots - slot0
        out = np.empty(n, self.dtype)
        check(lib().dccrgx_field_download(self.grid.h, self.id, slot0, n, _ptr(out)))
        return out

    def set(self, values, slot0=0):
        # subarray dtypes (e.g. (uint64, 8)) take values of shape (n, 8)
        a = np.ascontiguousarray(values, dtype=self.dtype.base)
        check(lib().dccrgx_field_upload(self.grid.h, self.id, slot0, a.nbytes // self.dtype.itemsize, _ptr(a)))

    def get_removed(self):
        """Payloads of the cells removed by the last stop_refining whose
        parent is local, in the order of Dccrg.get_removed_cells(sorted=False)."""
        n = len(self.grid.get_removed_cells(sorted=False))
        out = np.empty(n, self.dtype)
        check(lib().dccrgx_removed_field_download(self.grid.h, self.id, _ptr(out), out.nbytes))
        return out

    def set_transfer(self, transfer: bool):
        self.transfer = bool(transfer)
        check(lib().dccrgx_set_field_transfer(self.grid.h, self.id, int(transfer)))

    def set_window(self, offset, nbytes):
        """The bytes of each element the halo carries (what a Cell_Data's
        get_mpi_datatype describes)."""
        check(lib().dccrgx_set_field_window(self.grid.h, self.id, int(offset), int(nbytes)))


class VariableField:
    """A payload of a different number of bytes per cell (a Cell_Data whose
    get_mpi_datatype describes e.g. a std::vector, tests/variable_data_size):
    one byte pool over all slots.  Values are lists of numpy arrays of
    ``dtype`` (one per cell); the halo, migrations and removed-cell payloads
    carry each cell's bytes and its size."""

    def __init__(self, grid, fid, name, dtype, transfer):
        self.grid, self.id, self.name, self.dtype, self.transfer = grid, fid, name, np.dtype(dtype), transfer

    def sizes(self, slot0=0, n=None):
        """Byte sizes of the cells at slots [slot0, slot0 + n)."""
        if n is None:
            n = self.grid.n_slots - slot0
        out = np.empty(n, np.uint64)
        check(lib().dccrgx_variable_field_sizes(self.grid.h, self.id, slot0, n, _ptr(out)))
        return out

    def resize(self, counts, slot0=0):
        """Element counts of the cells from slot0 on (Cell_Data::...resize):
        each keeps its leading bytes, new bytes are zero."""
        b = np.ascontiguousarray(np.asarray(counts, np.uint64) * np.uint64(self.dtype.itemsize))
        check(lib().dccrgx_variable_field_resize(self.grid.h, self.id, slot0, b.size, _ptr(b)))

    def set(self, values, slot0=0):
        """One array per cell from slot0 on; the cells take their sizes."""
        arrs = [np.ascontiguousarray(v, self.dtype) for v in values]
        self.resize([a.size for a in arrs], slot0)
        raw = np.concatenate([a.view(np.uint8) for a in arrs]) if arrs else np.zeros(0, np.uint8)
        raw = np.ascontiguousarray(raw)
        check(lib().dccrgx_variable_field_upload(self.grid.h, self.id, slot0, len(arrs), _ptr(raw), raw.nbytes))

    def get(self, slot0=0, n=None):
        if n is None:
            n = self.grid.n_slots - slot0
        sz = self.sizes(slot0, n)
        raw = np.empty(int(sz.sum()), np.uint8)
        got = C.c_size_t()
        check(lib().dccrgx_variable_field_download(self.grid.h, self.id, slot0, n, _ptr(raw), raw.nbytes,
                                                     C.byref(got)))
        return _split(raw, sz, self.dtype)

    def get_removed(self):
        """Payloads of the cells removed by the last stop_refining whose
        parent is local (order of Dccrg.get_removed_cells(sorted=False))."""
        n = len(self.grid.get_removed_cells(sorted=False))
        sz = np.zeros(n + 1, np.uint64)
        total = C.c_size_t()
        rc = lib().dccrgx_removed_variable_field_download(self.grid.h, self.id, _ptr(sz), None, 0, C.byref(total))
        if rc != ERANGE:
            check(rc)
        raw = np.empty(total.value, np.uint8)
        check(lib().dccrgx_removed_variable_field_download(self.grid.h, self.id, _ptr(sz), _ptr(raw), raw.nbytes,
                                                           C.byref(total)))
        return _split(raw, sz[:n], self.dtype)


def _split(raw, sizes, dtype):
    out, o = [], 0
    for b in sizes.tolist():
        out.append(raw[o:o + int(b)].view(dtype).copy())
        o += int(b)
    return out


class TorchExchange:
    """Host transport over torch.distributed point-to-point (gloo): the
    exchange primitive of include/dccrgx.h (dccrgx_exchange_fn)."""

    def __init__(self, group=None):
        import torch.distributed as dist

        self.group = group
        self.rank, self.size = dist.get_rank(group), dist.get_world_size(group)
        self.error = None
        self.fn = EXCHANGE_FN(self._exchange)

    def _exchange(self, ctx, send, send_bytes, recv, recv_bytes):
        try:
            import torch
            import torch.distributed as dist

            reqs, outs = [], []
            for p in range(self.size):
                if p == self.rank:
                    continue
                nb = int(send_bytes[p])
                if nb:
                    t = torch.empty(nb, dtype=torch.uint8)
                    C.memmove(t.data_ptr(), send[p], nb)
                    reqs.append(dist.isend(t, p, group=self.group))
                nr = int(recv_bytes[p])
                if nr:
                    t = torch.empty(nr, dtype=torch.uint8)
                    reqs.append(dist.irecv(t, p, group=self.group))
                    outs.append((p, t))
            for r in reqs:
                r.wait()
            for p, t in outs:
                C.memmove(recv[p], t.data_ptr(), t.numel())
            return 0
        except Exception as e:  # reported to the library as a failed exchange
            self.error = e
            return -1


class Dccrg:
    """One grid per process; ``rank``/``size`` and an RCCL bootstrap id replace
    the reference's ``MPI_Comm`` (initialize(comm), dccrg.hpp:472)."""

    def __init__(self, rank=0, size=1, device=0, unique_id: bytes | None = None, exchange: TorchExchange | None = None):
        L = lib()
        h = C.c_void_p()
        self._exchange = exchange  # keeps the callback alive
        if exchange is not None:
            check(L.dccrgx_create_with_exchange(rank, size, device, exchange.fn, None, C.byref(h)))
        else:
            uid = None
            if unique_id is not None:
                # without a unique id the grid is a detached view of rank `rank`
                # (structures only, no halo transport / collectives); with one,
                # an RCCL communicator (also of one rank)
                uid = C.create_string_buffer(bytes(unique_id), 128)
            check(L.dccrgx_create(rank, size, device, uid, C.byref(h)))
        self.h = h
        self.rank, self.size, self.device = rank, size, device
        self.fields = {}

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        check(lib().dccrgx_get_unique_id(buf))
        return buf.raw

    @classmethod
    def from_torch_distributed(cls, device=None, transport="rccl"):
        """Bootstrap from an initialized torch.distributed process group.
        transport "rccl": the library's own RCCL communicator (one GPU per
        rank); "host": torch.distributed point-to-point through the host (any
        number of ranks per GPU, a gloo group)."""
        import torch.distributed as dist

        rank, size = dist.get_rank(), dist.get_world_size()
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", rank))
        if transport == "host":
            return cls(rank, size, device, exchange=TorchExchange())
        obj = [cls.unique_id() if rank == 0 else None]
        if size > 1:
            dist.broadcast_object_list(obj, src=0)
        return cls(rank, size, device, obj[0] if size > 1 else None)

    def close(self):
        if getattr(self, "h", None):
            lib().dccrgx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- setup (dccrg.hpp:8120-8230), chainable ----------------------------
    def set_initial_length(self, length):
        a = (C.c_uint64 * 3)(*[int(x) for x in length])
        check(lib().dccrgx_set_initial_length(self.h, a))
        self.length = tuple(int(x) for x in length)
        return self

    def set_maximum_refinement_level(self, level):
        check(lib().dccrgx_set_maximum_refinement_level(self.h, int(level)))
        return self

    def get_maximum_refinement_level(self):
        v = C.c_int()
        check(lib().dccrgx_get_maximum_refinement_level(self.h, C.byref(v)))
        return v.value

    def set_periodic(self, x, y, z):
        check(lib().dccrgx_set_periodic(self.h, int(x), int(y), int(z)))
        return self

    def set_neighborhood_length(self, n):
        check(lib().dccrgx_set_neighborhood_length(self.h, int(n)))
        return self

    def initialize(self):
        check(lib().dccrgx_initialize(self.h))
        return self

    def set_geometry(self, start, level_0_cell_length):
        s = (C.c_double * 3)(*start)
        l0 = (C.c_double * 3)(*level_0_cell_length)
        check(lib().dccrgx_set_geometry(self.h, s, l0))
        return self

    def set_geometry_block(self, block: bytes):
        """The grid file's geometry block of a Stretched_Cartesian_Geometry
        (dccrg_stretched_cartesian_geometry.hpp:652-715), written by
        save_grid_data instead of the Cartesian block; b"" restores that."""
        b = bytes(block)
        buf = C.create_string_buffer(b, len(b)) if b else None
        check(lib().dccrgx_set_geometry_block(self.h, buf, len(b)))
        return self

    def geometry_block(self) -> bytes:
        """The stretched geometry block a load read (b"" for a Cartesian file)."""
        n = C.c_size_t()
        check(lib().dccrgx_get_geometry_block(self.h, None, 0, C.byref(n)))
        if not n.value:
            return b""
        buf = C.create_string_buffer(n.value)
        check(lib().dccrgx_get_geometry_block(self.h, buf, n.value, C.byref(n)))
        return buf.raw[: n.value]

    def geometry(self, cells):
        """(centers, lengths), each (n, 3): Cartesian_Geometry get_center /
        get_length (dccrg_cartesian_geometry.hpp:282-362) of many cells."""
        ids = np.ascontiguousarray(cells, np.uint64)
        c = np.empty((ids.size, 3))
        L = np.empty((ids.size, 3))
        check(lib().dccrgx_geometry_batch(self.h, _ptr(ids), ids.size, _ptr(c), _ptr(L)))
        return c, L

    def get_center(self, cell):
        return tuple(self.geometry([cell])[0][0])

    def get_length(self, cell):
        return tuple(self.geometry([cell])[1][0])

    # ---- mapping ------------------------------------------------------------
    def get_cell_from_indices(self, indices, level):
        a = (C.c_uint64 * 3)(*[int(x) for x in indices])
        return int(lib().dccrgx_get_cell_from_indices(self.h, a, int(level)))

    def get_indices(self, cell):
        a = (C.c_uint64 * 3)()
        rc = lib().dccrgx_get_indices(self.h, int(cell), a)
        if rc == ENOTFOUND:
            return None
        check(rc)
        return tuple(a)

    def get_refinement_level(self, cell):
        return int(lib().dccrgx_get_refinement_level(self.h, int(cell)))

    def get_last_cell(self):
        return int(lib().dccrgx_get_last_cell(self.h))

    def mapping_batch(self, ids):
        """Device id math for many ids (dccrgx_mapping_batch): dict of level,
        indices (n, 3), length, parent, child, level0_parent, siblings (n, 8)."""
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        lvl = np.empty(ids.size, np.int32)
        out = np.empty((ids.size, 15), np.uint64)
        check(lib().dccrgx_mapping_batch(self.h, ids.ctypes.data, ids.size, lvl.ctypes.data, out.ctypes.data))
        return dict(level=lvl, indices=out[:, 0:3], length=out[:, 3], parent=out[:, 4], child=out[:, 5],
                    level0_parent=out[:, 6], siblings=out[:, 7:15])

    # ---- queries ------------------------------------------------------------
    @property
    def counts(self):
        v = [C.c_size_t() for _ in range(4)]
        check(lib().dccrgx_get_counts(self.h, *[C.byref(x) for x in v]))
        return dict(inner=v[0].value, outer=v[1].value, recv=v[2].value, slots=v[3].value)

    @property
    def n_slots(self):
        return self.counts["slots"]

    @property
    def n_local(self):
        c = self.counts
        return c["inner"] + c["outer"]

    def _u64_query(self, fn, *args, cap=None):
        n = C.c_size_t()
        rc = fn(self.h, *args, None, 0, C.byref(n))
        if rc not in (0, ERANGE):
            check(rc)
        out = np.empty(n.value, np.uint64)
        check(fn(self.h, *args, _ptr(out), out.size, C.byref(n)))
        return out

    def get_cells(self, criteria="local", exact_match=False, neighborhood_id=DEFAULT_HOOD, sorted=True):
        """get_cells (dccrg.hpp:651) - sorted ids.  `criteria`: a list of
        neighbor-type bitmasks (HAS_* below, is_neighbor_type_match 2946-3053;
        [] = every local cell), or a selection name ("local", "inner",
        "outer", "remote", "all")."""
        if isinstance(criteria, str):
            return self._u64_query(lib().dccrgx_get_cells, CELLS[criteria])
        c = np.ascontiguousarray(criteria, np.int32)
        return self._u64_query(lib().dccrgx_get_cells_by_criteria, _ptr(c), c.size, int(exact_match),
                               int(neighborhood_id))

    def local_cells(self):
        return self.get_cells("local")

    def inner_cells(self):
        return self.get_cells("inner")

    def outer_cells(self):
        return self.get_cells("outer")

    def remote_cells(self):
        return self.get_cells("remote")

    def slot_ids(self):
        return self._u64_query(lib().dccrgx_get_slot_ids)

    def get_neighbors_of(self, cell, hood=None):
        """[(id, (x, y, z)), ...] in stencil order (get_neighbors_of, 819), or
        None for a cell that is not local or an unknown neighborhood id (the
        reference returns nullptr).  hood: a user neighborhood id."""
        if hood is not None and hood != DEFAULT_HOOD:
            return self._user_neighbors(cell, hood, 0)
        n = C.c_size_t()
        cap = 4096
        ids = np.empty(cap, np.uint64)
        offs = np.empty(3 * cap, np.int32)
        rc = lib().dccrgx_get_neighbors_of(self.h, int(cell), _ptr(ids), _ptr(offs), cap, C.byref(n))
        if rc == ENOTFOUND:
            return None
        check(rc)
        k = n.value
        return [(int(ids[i]), tuple(int(v) for v in offs[3 * i: 3 * i + 3])) for i in range(k)]

    def get_neighbors_to(self, cell, hood=None):
        if hood is not None and hood != DEFAULT_HOOD:
            return self._user_neighbors(cell, hood, 1)
        n = C.c_size_t()
        cap = 8192
        ids = np.empty(cap, np.uint64)
        rc = lib().dccrgx_get_neighbors_to(self.h, int(cell), _ptr(ids), cap, C.byref(n))
        if rc == ENOTFOUND:
            return None
        check(rc)
        return [(int(i), (0, 0, 0)) for i in ids[: n.value]]

    def _user_neighbors(self, cell, hood, kind):
        n = C.c_size_t()
        rc = lib().dccrgx_get_user_neighbors(self.h, int(hood), int(cell), kind, None, None, 0, C.byref(n))
        if rc == ENOTFOUND:
            return None
        if rc not in (0, ERANGE):
            check(rc)
        k = n.value
        ids = np.empty(max(k, 1), np.uint64)
        offs = np.empty(3 * max(k, 1), np.int32)
        check(lib().dccrgx_get_user_neighbors(self.h, int(hood), int(cell), kind, _ptr(ids), _ptr(offs), k,
                                              C.byref(n)))
        if kind == 1:
            return [(int(i), (0, 0, 0)) for i in ids[:k]]
        return [(int(ids[i]), tuple(int(v) for v in offs[3 * i: 3 * i + 3])) for i in range(k)]

    # ---- user neighborhoods (add_neighborhood, dccrg.hpp:6383) -----------------------
    def add_neighborhood(self, hood, offsets):
        """True if the neighborhood was added; False where the reference
        returns false (default / existing id, offset outside the default
        neighborhood or (0,0,0))."""
        o = np.ascontiguousarray(np.asarray(offsets, np.int32).reshape(-1, 3))
        rc = lib().dccrgx_add_neighborhood(self.h, int(hood), _ptr(o), o.shape[0])
        if rc == EINVAL:
            return False
        check(rc)
        return True

    def remove_neighborhood(self, hood):
        check(lib().dccrgx_remove_neighborhood(self.h, int(hood)))
        return self

    def _user_list(self, hood, peer, receive):
        n = C.c_size_t()
        rc = lib().dccrgx_get_user_update_list(self.h, int(hood), int(peer), int(receive), None, 0, C.byref(n))
        if rc not in (0, ERANGE):
            check(rc)
        out = np.empty(max(n.value, 1), np.uint64)
        check(lib().dccrgx_get_user_update_list(self.h, int(hood), int(peer), int(receive), _ptr(out), n.value,
                                                C.byref(n)))
        return out[: n.value].copy()

    def get_face_neighbors_of(self, cell):
        n = C.c_size_t()
        ids = np.empty(64, np.uint64)
        dirs = np.empty(64, np.int32)
        rc = lib().dccrgx_get_face_neighbors_of(self.h, int(cell), _ptr(ids), _ptr(dirs), 64, C.byref(n))
        if rc == ENOTFOUND:
            return None
        check(rc)
        return [(int(ids[i]), int(dirs[i])) for i in range(n.value)]

    def find_neighbors_of(self, cell, neighborhood):
        """find_neighbors_of(cell, neighborhood) (dccrg.hpp:4339): [(id, (x, y,
        z)), ...] for any list of offsets; raises for a cell this process
        does not know (the reference throws)."""
        o = np.ascontiguousarray(np.asarray(neighborhood, np.int32).reshape(-1, 3))
        n = C.c_size_t()
        rc = lib().dccrgx_find_neighbors_of(self.h, int(cell), _ptr(o), o.shape[0], None, None, 0, C.byref(n))
        if rc not in (0, ERANGE):
            check(rc)
        k = n.value
        ids = np.empty(max(k, 1), np.uint64)
        offs = np.empty(3 * max(k, 1), np.int32)
        check(lib().dccrgx_find_neighbors_of(self.h, int(cell), _ptr(o), o.shape[0], _ptr(ids), _ptr(offs), k,
                                             C.byref(n)))
        return [(int(ids[i]), tuple(int(v) for v in offs[3 * i: 3 * i + 3])) for i in range(k)]

    def get_neighbors_(self):
        """The face-neighbor cache (get_neighbors_, dccrg.hpp:7107): {leaf:
        (-x, +x, -y, +y, -z, +z)} over the leaves whose faces this process
        can resolve (every local leaf)."""
        n = C.c_size_t()
        rc = lib().dccrgx_get_face_cache(self.h, None, None, 0, C.byref(n))
        if rc not in (0, ERANGE):
            check(rc)
        k = n.value
        ids = np.empty(max(k, 1), np.uint64)
        nb = np.empty(6 * max(k, 1), np.uint64)
        check(lib().dccrgx_get_face_cache(self.h, _ptr(ids), _ptr(nb), k, C.byref(n)))
        return {int(ids[i]): tuple(int(v) for v in nb[6 * i: 6 * i + 6]) for i in range(k)}

    def comm_loopback(self, field, slot0, n, dst_slot0):
        """Field slots [slot0, slot0 + n) sent to this process itself through
        the RCCL byte mover, received into [dst_slot0, ...) (transport check)."""
        check(lib().dccrgx_comm_loopback(self.h, field.id, slot0, n, dst_slot0))

    def unpin_all_cells(self):
        check(lib().dccrgx_unpin_all_cells(self.h))
        return self

    def neighbor_entries(self, kind="of"):
        """Number of entries of a local CSR (no download of the entries)."""
        n = C.c_size_t()
        ptr = np.empty(self.n_local + 1, np.uint32)
        rc = lib().dccrgx_download_csr(self.h, CSR_KIND[kind], _ptr(ptr), None, None, 0, C.byref(n))
        if rc not in (0, ERANGE):
            check(rc)
        return int(n.value)

    def csr(self, kind="of"):
        """Bulk download (ptr, ids, aux) of a local CSR in slot order."""
        k = CSR_KIND[kind]
        n = C.c_size_t()
        nl = self.n_local
        ptr = np.empty(nl + 1, np.uint32)
        rc = lib().dccrgx_download_csr(self.h, k, _ptr(ptr), None, None, 0, C.byref(n))
        if rc not in (0, ERANGE):
            check(rc)
        tot = n.value
        ids = np.empty(max(tot, 1), np.uint64)
        aux = np.empty(max(3 * tot, 1), np.int32) if k in (0, 2, 3) else None
        check(lib().dccrgx_download_csr(self.h, k, _ptr(ptr), _ptr(ids), _ptr(aux), tot, C.byref(n)))
        ids = ids[:tot]
        if k in (0, 3):
            aux = aux[: 3 * tot].reshape(tot, 3)
        elif k == 2:
            aux = aux[:tot]
        return ptr, ids, aux

    def is_local(self, cell):
        return bool(lib().dccrgx_is_local(self.h, int(cell)))

    def get_process(self, cell):
        return int(lib().dccrgx_get_process(self.h, int(cell)))

    def get_slot(self, cell):
        return int(lib().dccrgx_get_slot(self.h, int(cell)))

    def get_peers(self):
        n = C.c_size_t()
        buf = np.empty(max(self.size, 1), np.int32)
        check(lib().dccrgx_get_peers(self.h, _ptr(buf), buf.size, C.byref(n)))
        return [int(x) for x in buf[: n.value]]

    def get_cells_to_send(self, peer, hood=None):
        if hood is not None and hood != DEFAULT_HOOD:
            return self._user_list(hood, peer, 0)
        return self._u64_query(lib().dccrgx_get_cells_to_send, int(peer))

    def get_cells_to_receive(self, peer, hood=None):
        if hood is not None and hood != DEFAULT_HOOD:
            return self._user_list(hood, peer, 1)
        return self._u64_query(lib().dccrgx_get_cells_to_receive, int(peer))

    def get_number_of_update_send_cells(self):
        s, r = C.c_uint64(), C.c_uint64()
        check(lib().dccrgx_get_number_of_update_cells(self.h, C.byref(s), C.byref(r)))
        return s.value

    def get_number_of_update_receive_cells(self):
        s, r = C.c_uint64(), C.c_uint64()
        check(lib().dccrgx_get_number_of_update_cells(self.h, C.byref(s), C.byref(r)))
        return r.value

    # ---- refinement -------------------------------------------------------------
    def refine_completely(self, cell):
        rc = lib().dccrgx_refine_completely(self.h, int(cell))
        if rc == ENOTFOUND:
            return False
        check(rc)
        return True

    def unrefine_completely(self, cell):
        """unrefine_completely (dccrg.hpp:2560): False for a cell that is not
        a local leaf or whose sibling has children."""
        rc = lib().dccrgx_unrefine_completely(self.h, int(cell))
        if rc == ENOTFOUND:
            return False
        check(rc)
        return True

    def dont_unrefine(self, cell):
        rc = lib().dccrgx_dont_unrefine(self.h, int(cell))
        if rc == ENOTFOUND:
            return False
        check(rc)
        return True

    def dont_refine(self, cell):
        rc = lib().dccrgx_dont_refine(self.h, int(cell))
        if rc == ENOTFOUND:
            return False
        check(rc)
        return True

    def get_removed_cells(self, sorted=False):
        """Cells removed by the last stop_refining whose parent is local
        (get_removed_cells, dccrg.hpp:3497)."""
        ids = self._u64_query(lib().dccrgx_get_removed_cells)
        return np.sort(ids) if sorted else ids

    def stop_refining(self):
        """Executes the collected refines and unrefines (collective); returns
        the local cells created by refinement."""
        n = C.c_size_t()
        check(lib().dccrgx_stop_refining(self.h, None, 0, C.byref(n)))
        return self._u64_query(lib().dccrgx_get_new_cells)

    def set_cells(self, ids, owners):
        """Replace the global leaf set + partition (identical on every rank)."""
        ids = np.ascontiguousarray(ids, np.uint64)
        owners = np.ascontiguousarray(owners, np.int32)
        check(lib().dccrgx_set_cells(self.h, _ptr(ids), _ptr(owners), ids.size))
        return self

    # ---- partition ------------------------------------------------------------
    def pin(self, cell, process):
        rc = lib().dccrgx_pin(self.h, int(cell), int(process))
        if rc == ENOTFOUND:
            return False
        check(rc)
        return True

    def unpin(self, cell):
        check(lib().dccrgx_unpin(self.h, int(cell)))
        return True

    def balance_load(self, use_zoltan=True):
        """balance_load (dccrg.hpp:1024): the native RCB partitioner (unless
        use_zoltan is False or the method is "NONE"), then the pins; collective."""
        check(lib().dccrgx_balance_load(self.h, 1 if use_zoltan else 0))
        return self

    def make_new_partition(self):
        """The partitioner's decision alone (no migration): (local cells
        ascending, their new processes); collective."""
        n = C.c_size_t()
        rc = lib().dccrgx_make_new_partition(self.h, None, None, 0, C.byref(n))
        if rc != ERANGE:
            check(rc)
        cells = np.empty(n.value, np.uint64)
        procs = np.empty(n.value, np.int32)
        check(lib().dccrgx_make_new_partition(self.h, _ptr(cells), _ptr(procs), n.value, C.byref(n)))
        return cells, procs

    def set_load_balancing_method(self, method):
        check(lib().dccrgx_set_load_balancing_method(self.h, method.encode()))
        return self

    def get_load_balancing_method(self):
        buf = C.create_string_buffer(64)
        check(lib().dccrgx_get_load_balancing_method(self.h, buf, 64))
        return buf.value.decode()

    def set_cell_weight(self, cell, weight):
        rc = lib().dccrgx_set_cell_weight(self.h, int(cell), float(weight))
        if rc == ENOTFOUND:
            return False
        check(rc)
        return True

    def get_cell_weight(self, cell):
        return float(lib().dccrgx_get_cell_weight(self.h, int(cell)))

    def balance_load_to(self, cells, new_processes):
        """Repartition with this rank's export list (local cells and their new
        process, a partitioner's export list); collective, payloads migrate."""
        ids = np.ascontiguousarray(cells, np.uint64)
        own = np.ascontiguousarray(new_processes, np.int32)
        check(lib().dccrgx_balance_load_to(self.h, _ptr(ids), _ptr(own), ids.size))
        return self

    # split form (initialize_balance_load 3746 / continue 3899 / finish 3942)
    def initialize_balance_load(self, cells=(), new_processes=(), use_zoltan=False):
        ids = np.ascontiguousarray(cells, np.uint64)
        own = np.ascontiguousarray(new_processes, np.int32)
        check(lib().dccrgx_initialize_balance_load(self.h, 1 if use_zoltan else 0, _ptr(ids), _ptr(own), ids.size))

    def continue_balance_load(self):
        check(lib().dccrgx_continue_balance_load(self.h))

    def finish_balance_load(self):
        check(lib().dccrgx_finish_balance_load(self.h))

    def migration_message_size(self, peer):
        a, b = C.c_size_t(), C.c_size_t()
        check(lib().dccrgx_migration_message_size(self.h, int(peer), C.byref(a), C.byref(b)))
        return a.value, b.value

    def migration_pack(self, peer):
        n, _ = self.migration_message_size(peer)
        buf = np.empty(max(n, 1), np.uint8)
        check(lib().dccrgx_migration_pack(self.h, int(peer), _ptr(buf), n))
        return buf[:n]

    def migration_place(self, peer, data):
        a = np.ascontiguousarray(data, np.uint8)
        check(lib().dccrgx_migration_place(self.h, int(peer), _ptr(a), a.size))

    def get_cell_process(self):
        """(ids, owners) of the leaves this rank knows - its own and its ghost
        leaves - ascending id (get_cell_process, dccrg.hpp:6848, lists every
        leaf of the grid)."""
        n = C.c_size_t()
        check(lib().dccrgx_get_cell_process(self.h, None, None, 0, C.byref(n)))
        ids = np.empty(n.value, np.uint64)
        own = np.empty(n.value, np.int32)
        check(lib().dccrgx_get_cell_process(self.h, _ptr(ids), _ptr(own), ids.size, C.byref(n)))
        return ids, own

    # ---- grid files (save_grid_data 1089, load_grid_data 1742) ---------------------
    def save_grid_data(self, path, offset=0, header=b""):
        hb = bytes(header)
        buf = C.create_string_buffer(hb, len(hb)) if hb else None
        check(lib().dccrgx_save_grid_data(self.h, str(path).encode(), int(offset), buf, len(hb)))
        return True

    def load_grid_data(self, path, offset=0, header_bytes=0):
        """Initializes this grid from a file written by save_grid_data (call
        instead of initialize, after registering the same transferred fields;
        a variable-size field, at most one, takes the rest of each record)."""
        check(lib().dccrgx_load_grid_data(self.h, str(path).encode(), int(offset), int(header_bytes)))
        return self

    def start_loading_grid_data(self, path, offset=0, header_bytes=0):
        """start_loading_grid_data (dccrg.hpp:1795): the grid and its cells
        from the file, no payload; then continue_loading_grid_data per part
        of the records, then finish_loading_grid_data."""
        check(lib().dccrgx_start_loading_grid_data(self.h, str(path).encode(), int(offset), int(header_bytes)))
        return self

    def continue_loading_grid_data(self, field, counts=None):
        """continue_loading_grid_data (2112): the next bytes of every local
        cell's record into `field` - a fixed-size field its window, a
        variable-size one `counts[s]` elements for local slot s."""
        if isinstance(field, VariableField):
            b = np.ascontiguousarray(np.asarray(counts, np.uint64) * np.uint64(field.dtype.itemsize))
            if b.size != self.n_local:
                raise ValueError("one element count per local cell")
            check(lib().dccrgx_continue_loading_grid_data(self.h, field.id, _ptr(b)))
        else:
            check(lib().dccrgx_continue_loading_grid_data(self.h, field.id, None))
        return self

    def grid_file_bytes_left(self):
        out = np.empty(self.n_local, np.uint64)
        check(lib().dccrgx_grid_file_bytes_left(self.h, _ptr(out)))
        return out

    def finish_loading_grid_data(self):  # 2380
        check(lib().dccrgx_finish_loading_grid_data(self.h))
        return self

    # ---- fields ---------------------------------------------------------------
    def add_field(self, name, dtype, transfer=True):
        fid = C.c_int()
        dt = np.dtype(dtype)
        check(lib().dccrgx_add_field(self.h, name.encode(), dt.itemsize, int(transfer), C.byref(fid)))
        f = Field(self, fid.value, name, dt, transfer)
        self.fields[name] = f
        return f

    def add_variable_field(self, name, dtype, transfer=True):
        """A payload whose size differs per cell (tests/variable_data_size)."""
        fid = C.c_int()
        check(lib().dccrgx_add_variable_field(self.h, name.encode(), int(transfer), C.byref(fid)))
        f = VariableField(self, fid.value, name, dtype, transfer)
        self.fields[name] = f
        return f

    def set_send_single_cells(self, on):  # 6677
        check(lib().dccrgx_set_send_single_cells(self.h, int(bool(on))))
        return self

    def get_send_single_cells(self):  # 6684
        v = C.c_int()
        check(lib().dccrgx_get_send_single_cells(self.h, C.byref(v)))
        return bool(v.value)

    # ---- halo -------------------------------------------------------------------
    def update_copies_of_remote_neighbors(self, hood=None):
        if hood is not None and hood != DEFAULT_HOOD:
            check(lib().dccrgx_update_copies_of_remote_neighbors_hood(self.h, int(hood)))
            return True
        check(lib().dccrgx_update_copies_of_remote_neighbors(self.h))
        return True

    def start_remote_neighbor_copy_updates(self):
        check(lib().dccrgx_start_remote_neighbor_copy_updates(self.h))
        return True

    def wait_remote_neighbor_copy_update_receives(self):
        check(lib().dccrgx_wait_remote_neighbor_copy_update_receives(self.h))
        return True

    def wait_remote_neighbor_copy_update_sends(self):
        check(lib().dccrgx_wait_remote_neighbor_copy_update_sends(self.h))
        return True

    def wait_remote_neighbor_copy_updates(self):
        check(lib().dccrgx_wait_remote_neighbor_copy_updates(self.h))
        return True

    # explicit halo transport: the wire message of one peer
    def halo_message_size(self, peer, hood=DEFAULT_HOOD):
        a, b = C.c_size_t(), C.c_size_t()
        check(lib().dccrgx_halo_message_size(self.h, int(hood), int(peer), C.byref(a), C.byref(b)))
        return a.value, b.value

    def halo_pack(self, peer, hood=DEFAULT_HOOD):
        n, _ = self.halo_message_size(peer, hood)
        buf = np.empty(max(n, 1), np.uint8)
        check(lib().dccrgx_halo_pack(self.h, int(hood), int(peer), _ptr(buf), n))
        return buf[:n]

    def halo_place(self, peer, data, hood=DEFAULT_HOOD):
        a = np.ascontiguousarray(data, np.uint8)
        check(lib().dccrgx_halo_place(self.h, int(hood), int(peer), _ptr(a), a.size))

    # ---- built-in sweeps ------------------------------------------------------------
    def gol_step(self, state: Field, region="all"):
        check(lib().dccrgx_gol_step(self.h, state.id, REGION[region]))

    def gol_commit(self, state: Field):
        check(lib().dccrgx_gol_commit(self.h, state.id))

    def gol_amr_collect(self, state: Field, lst: Field, region="all"):
        """First loop of get_live_neighbors (tests/game_of_life/solve.hpp:46-110)."""
        check(lib().dccrgx_gol_amr(self.h, 0, state.id, lst.id, REGION[region]))

    def gol_amr_spread(self, state: Field, lst: Field, region="all"):
        """Spread among siblings + rule (tests/game_of_life/solve.hpp:113-167)."""
        check(lib().dccrgx_gol_amr(self.h, 1, state.id, lst.id, REGION[region]))

    def get_live_neighbors(self, state: Field, lst: Field):
        """One turn of the refined game emulating the unrefined one, as
        tests/game_of_life/solve.hpp:37-170 (collect, halo of the transferred
        fields, spread + rule; every local list error_cell at the end, as the
        reference leaves it).  `lst` is a 64-byte field (8 x uint64)."""
        check(lib().dccrgx_get_live_neighbors(self.h, state.id, lst.id))

    @staticmethod
    def _fids(fields):
        assert len(fields) == 7
        return (C.c_int * 7)(*[f.id for f in fields])

    def advection_step(self, fields, dt, region="all"):
        check(lib().dccrgx_advection_step(self.h, self._fids(fields), float(dt), REGION[region]))

    def advection_commit(self, density: Field):
        check(lib().dccrgx_advection_commit(self.h, density.id))

    def advection_initialize(self, fields):
        check(lib().dccrgx_advection_initialize(self.h, self._fids(fields)))

    def advection_max_time_step(self, fields):
        v = C.c_double()
        check(lib().dccrgx_advection_max_time_step(self.h, self._fids(fields), C.byref(v)))
        return self.allreduce(v.value, "min")

    def advection_max_time_step_device(self, fields, out):
        """max_time_step reduced over all ranks into device memory `out` (a
        float64 torch tensor on the GPU, or a device address), queued on the
        compute stream: no host round trip over RCCL."""
        check(lib().dccrgx_advection_max_time_step_device(self.h, self._fids(fields), _dev_ptr(out)))

    def advection_layout(self):
        """Tile layout of the advection sweep and its algorithmic HBM bytes per
        sweep over all local cells (see include/dccrgx.h)."""
        out = (C.c_uint64 * 12)()
        check(lib().dccrgx_advection_layout(self.h, out))
        keys = ("tile", "tiles", "ext_total", "ext_max", "finer_faces", "face_entries", "alg_bytes",
                "alg_bytes_core", "regular_tiles", "regular_cells", "ext_regular", "bytes_needed")
        return dict(zip(keys, (int(v) for v in out)))

    def advection_check_adaptation(self, density, diff_increase, diff_threshold=0.25, unrefine_sensitivity=0.5):
        """check_for_adaptation (tests/advection/adapter.hpp:47-178) + the
        requests of adapt_grid; returns (refines, dont_unrefines, unrefines)."""
        c = np.zeros(3, np.uint64)
        check(lib().dccrgx_advection_check_adaptation(self.h, density.id, float(diff_increase), float(diff_threshold),
                                                      float(unrefine_sensitivity), _ptr(c)))
        return tuple(int(x) for x in c)

    def advection_adapt(self, fields):
        """adapt_grid (adapter.hpp:232-309), collective; returns (created, removed)."""
        out = np.zeros(2, np.uint64)
        check(lib().dccrgx_advection_adapt(self.h, self._fids(fields), _ptr(out)))
        return int(out[0]), int(out[1])

    def advection_refine_candidates(self, density, diff_increase, diff_threshold):
        return self._u64_query(lib().dccrgx_advection_refine_candidates, density.id, float(diff_increase),
                               float(diff_threshold))

    # ---- collectives / sync -------------------------------------------------------
    def allreduce(self, value, op="sum"):
        v = C.c_double(float(value))
        check(lib().dccrgx_allreduce_f64(self.h, C.byref(v), 1, {"sum": 0, "min": 1, "max": 2}[op]))
        return v.value

    def allreduce_device(self, src, dst=None, op="sum"):
        """MPI_Allreduce of `count` device doubles (torch tensors or device
        addresses; dst defaults to src), stream-ordered on the compute stream,
        combined in rank order (bitwise allreduce()'s result)."""
        n = int(src.numel()) if hasattr(src, "numel") else None
        if n is None:
            raise TypeError("allreduce_device needs a torch tensor (its element count)")
        d = src if dst is None else dst
        check(lib().dccrgx_allreduce_f64_device(self.h, _dev_ptr(src), _dev_ptr(d), n,
                                                {"sum": 0, "min": 1, "max": 2}[op]))

    def transport(self):
        """(kind, communicator ranks) the library holds: kind "none" (a
        detached view), "rccl" (ranks = ncclCommCount) or "host"."""
        k, n = C.c_int(), C.c_int()
        check(lib().dccrgx_get_transport(self.h, C.byref(k), C.byref(n)))
        return ("none", "rccl", "host")[k.value], n.value

    def barrier(self):
        check(lib().dccrgx_barrier(self.h))

    def synchronize(self):
        check(lib().dccrgx_synchronize(self.h))

    def kernel_timing(self, enable=-1):
        ms, cnt = C.c_double(), C.c_int64()
        check(lib().dccrgx_kernel_timing(self.h, int(enable), C.byref(ms), C.byref(cnt)))
        return ms.value, cnt.value
