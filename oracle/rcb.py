"""Test infrastructure only (the checker, never the product): a sequential
restatement of the native repartitioner's rule (dccrg_amd/csrc/partition.hip),
which stands in for the reference's default Zoltan "RCB" partition
(dccrg.hpp:7082, make_new_partition 8349-8376, inputs 11682-11783).  Zoltan is
absent here, so this rule is the repo's own: parity unpinned against Zoltan.

Rule: processes [lo, hi) holding a set of cells split into [lo, lo + P1) and
[lo + P1, hi), P1 = (hi - lo) // 2.  The cut axis is the longest side of the
bounding box of the set's centers (ties x, y, z).  Cells are ordered by
(center along the axis, id); the lower half takes the longest prefix whose
weight is <= floor(W * P1 / (hi - lo)).  Centers are 2 x minimum index +
length in indices, weights fixed point round(w * 2^16)."""
import numpy as np

WEIGHT_ONE = 65536


def centers2(mapping, ids):
    """Integer centers (2 x min index + length in indices) from an
    oracle.Mapping."""
    b = mapping.batch(np.asarray(ids, np.uint64))
    idx = np.asarray(b["indices"], np.int64)
    ln = np.asarray(b["length"], np.int64)
    return 2 * idx + ln[:, None]


def rcb(ids, c2, weights, P):
    """New process of every cell (same order as ids).  weights: floats or
    None (all 1)."""
    ids = np.asarray(ids, np.uint64)
    n = ids.size
    w = (np.full(n, WEIGHT_ONE, dtype=object) if weights is None
         else np.array([int(round(float(x) * WEIGHT_ONE)) for x in weights], dtype=object))
    owner = np.zeros(n, np.int32)

    def split(sel, lo, hi):
        if hi - lo < 2 or sel.size == 0:
            owner[sel] = lo
            return
        cc = c2[sel]
        ext = cc.max(axis=0) - cc.min(axis=0)
        axis = int(np.argmax(ext))  # first maximum: x before y before z
        order = np.lexsort((ids[sel], cc[:, axis]))
        s = sel[order]
        gp = hi - lo
        p1 = gp // 2
        W = int(sum(w[s]))
        target = W * p1 // gp
        cum = np.cumsum(w[s])
        k = 0
        while k < s.size and int(cum[k]) <= target:
            k += 1
        split(s[:k], lo, lo + p1)
        split(s[k:], lo + p1, hi)

    split(np.arange(n), 0, P)
    return owner
