"""Variable-size payload fields on one rank (tests/variable_data_size: a
Cell_Data whose get_mpi_datatype describes a different number of bytes per
cell): sizes, resize semantics (std::vector::resize: the leading values
kept, new ones zero), byte round trips, refusals of the fixed-field calls,
payloads kept across a rebuild.  The multi-process transport of these
fields is tests/test_gpu_transport.py::test_variable_size_payloads."""
import ctypes as C

import numpy as np
import pytest

import dccrg_amd
from dccrg_amd._lib import check

pytestmark = pytest.mark.gpu


def _grid(length=(4, 3, 2), R=1):
    g = dccrg_amd.Dccrg(0, 1, 0).set_initial_length(length).set_maximum_refinement_level(R)
    g.set_neighborhood_length(1).initialize()
    return g


def test_set_get_resize(gpu):
    g = _grid()
    v = g.add_variable_field("vars", np.float64)
    n = g.n_local
    assert np.all(v.sizes(0, n) == 0)
    vals = [np.arange(i % 4, dtype=np.float64) + 10 * i for i in range(n)]
    v.set(vals)
    assert np.array_equal(v.sizes(0, n), np.array([8 * (i % 4) for i in range(n)], np.uint64))
    assert all(np.array_equal(a, b) for a, b in zip(v.get(0, n), vals))
    # resize: shrink keeps the leading values, growth appends zeros
    counts = [(i * 3) % 5 for i in range(n)]
    v.resize(counts)
    for i, a in enumerate(v.get(0, n)):
        k = min(counts[i], vals[i].size)
        assert a.size == counts[i]
        assert np.array_equal(a[:k], vals[i][:k]) and np.all(a[k:] == 0)
    # a slot range in the middle
    v.set([np.array([1.5, 2.5])], slot0=3)
    assert np.array_equal(v.get(3, 1)[0], [1.5, 2.5])
    g.close()


def test_fixed_field_calls_refuse_a_variable_field(gpu):
    g = _grid()
    v = g.add_variable_field("vars", np.int32)
    with pytest.raises(dccrg_amd.DccrgError, match="variable-size"):
        dccrg_amd.Field(g, v.id, "vars", np.int32, True).get(0, 1)
    with pytest.raises(dccrg_amd.DccrgError, match="byte count"):
        raw = np.zeros(4, np.uint8)
        check(dccrg_amd.lib().dccrgx_variable_field_upload(g.h, v.id, 0, 1, raw.ctypes.data_as(C.c_void_p), raw.nbytes))
    g.close()


def test_payloads_survive_refinement(gpu):
    """Cells that stay keep their values across stop_refining (a full
    rebuild); the new children start empty (default-constructed in the
    reference, dccrg.hpp:10228-10255)."""
    g = _grid((4, 4, 1), 1)
    v = g.add_variable_field("vars", np.int32)
    sl = g.slot_ids()[: g.n_local]
    v.set([np.full(int(c) % 3 + 1, int(c), np.int32) for c in sl])
    g.refine_completely(int(sl[0]))
    new = g.stop_refining()
    now = g.slot_ids()[: g.n_local]
    got = v.get(0, g.n_local)
    for c, a in zip(now, got):
        if int(c) in set(new.tolist()):
            assert a.size == 0
        else:
            assert np.array_equal(a, np.full(int(c) % 3 + 1, int(c), np.int32))
    g.close()
