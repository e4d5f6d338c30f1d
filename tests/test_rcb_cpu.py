"""The sequential restatement of the native partitioner's rule
(oracle/rcb.py, the checker of dccrg_amd/csrc/partition.hip): CPU properties.
Parity against Zoltan's RCB is unpinned (Zoltan is absent)."""
import numpy as np

from oracle import oracle as O
from oracle import rcb as RCB


def _uniform(length):
    m = O.Mapping(length, 0)
    ids = np.arange(1, int(np.prod(length)) + 1, dtype=np.uint64)
    return ids, RCB.centers2(m, ids)


def test_uniform_slabs_are_exact():
    ids, c2 = _uniform((4, 4, 16))
    own = RCB.rcb(ids, c2, None, 4)
    # longest axis z: four z slabs of 4 planes, in process order
    z = (c2[:, 2] - 1) // 2
    assert np.array_equal(own, z // 4)


def test_balanced_and_boxes():
    ids, c2 = _uniform((6, 5, 7))
    for P in (2, 3, 5, 7):
        own = RCB.rcb(ids, c2, None, P)
        cnt = np.bincount(own, minlength=P)
        assert cnt.max() - cnt.min() <= P, cnt
        assert set(own.tolist()) == set(range(P))


def test_weights_shift_the_cut():
    ids, c2 = _uniform((8, 1, 1))
    w = np.ones(ids.size)
    w[:2] = 3.0  # the two low-x cells weigh 6 of 12
    own = RCB.rcb(ids, c2, w, 2)
    assert own.tolist() == [0, 0, 1, 1, 1, 1, 1, 1]


def test_independent_of_input_order():
    ids, c2 = _uniform((5, 4, 3))
    rng = np.random.default_rng(3)
    p = rng.permutation(ids.size)
    a = RCB.rcb(ids, c2, None, 3)
    b = RCB.rcb(ids[p], c2[p], None, 3)
    assert np.array_equal(a[p], b)
