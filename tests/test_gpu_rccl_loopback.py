"""The RCCL branch of the byte mover (comm.hip move_bytes: ncclGroupStart,
ncclSend / ncclRecv per message, ncclGroupEnd) executed on one GPU: a grid
created with an RCCL bootstrap id at size 1 owns a one-rank communicator, and
dccrgx_comm_loopback sends a field's slots to this rank itself and receives
them straight into other slots of the same field - the direct receive into
field slots that every halo of a full-window field uses (grid.hip halo_start).
Multi-rank RCCL needs one GPU per rank; the driver's N > 1 bench runs it."""
import numpy as np
import pytest

import dccrg_amd

pytestmark = pytest.mark.gpu


def test_rccl_self_send_recv(gpu):
    g = dccrg_amd.Dccrg(0, 1, 0, dccrg_amd.Dccrg.unique_id())
    g.set_initial_length((8, 8, 4)).set_neighborhood_length(1).initialize()
    n = g.n_slots
    assert n == 256
    f = g.add_field("payload", np.float64)
    vals = np.random.default_rng(3).standard_normal(n)
    f.set(vals)
    # the first 100 slots into slots 128..227, through ncclSend / ncclRecv
    g.comm_loopback(f, 0, 100, 128)
    got = f.get()
    exp = vals.copy()
    exp[128:228] = vals[:100]
    assert np.array_equal(got, exp)
    # byte-sized elements, an odd count
    h = g.add_field("bytes", np.uint8)
    b = np.arange(n, dtype=np.uint8)
    h.set(b)
    g.comm_loopback(h, 7, 33, 200)
    eb = b.copy()
    eb[200:233] = b[7:40]
    assert np.array_equal(h.get(), eb)
    # overlapping ranges and a grid without the RCCL transport are refused
    with pytest.raises(dccrg_amd.DccrgError, match="overlapping"):
        g.comm_loopback(f, 0, 100, 50)
    d = dccrg_amd.Dccrg(0, 1, 0).set_initial_length((2, 2, 2)).initialize()
    fd = d.add_field("x", np.float64)
    with pytest.raises(dccrg_amd.DccrgError, match="RCCL"):
        d.comm_loopback(fd, 0, 1, 4)
    g.close()
    d.close()


def test_rccl_self_send_recv_single_cells(gpu):
    """send_single_cells on: one ncclSend / ncclRecv pair per element, 9000
    of them, posted in rounds of at most 4096 per group (comm.hip
    kPiecesPerGroup); the bytes land as with one message."""
    g = dccrg_amd.Dccrg(0, 1, 0, dccrg_amd.Dccrg.unique_id())
    g.set_initial_length((32, 32, 20)).set_neighborhood_length(1).initialize()
    n = g.n_slots
    assert n == 20480
    f = g.add_field("payload", np.float64)
    vals = np.random.default_rng(5).standard_normal(n)
    f.set(vals)
    g.set_send_single_cells(True)
    g.comm_loopback(f, 11, 9000, 10000)
    exp = vals.copy()
    exp[10000:19000] = vals[11:9011]
    assert np.array_equal(f.get(), exp)
    g.set_send_single_cells(False)
    g.close()
