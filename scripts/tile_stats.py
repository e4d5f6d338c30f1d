"""Offline restatement of the advection tile layout (tile_build.hip) for a
leaf set, to study how a mesh splits into regular / general tiles without a
GPU.  Usage: python scripts/tile_stats.py leaves.npy base R [T]

The leaves come from the oracle (e.g. O.Grid(...).adv_prerefine(); cells()).
Slots: Morton order of the min corner (mesh.hip k_morton_sort); tiles: the
greedy aligned cuts of cut_run; regular: classify_tiles_kernel's rule (an
aligned 8^3 box of one level whose every side is absent or one aligned
same-level box stored contiguously)."""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from oracle import oracle as O  # noqa: E402


def spread3(v):
    v = v.astype(np.uint64)
    out = np.zeros_like(v)
    for b in range(21):
        out |= ((v >> np.uint64(b)) & np.uint64(1)) << np.uint64(3 * b)
    return out


def layout(ids, base, R, T=512):
    M = O.Mapping(base, R)
    mb = M.batch(ids)
    lvl, ind, clen = mb["level"], mb["indices"], mb["length"].astype(np.int64)
    key = spread3(ind[:, 0]) | (spread3(ind[:, 1]) << np.uint64(1)) | (spread3(ind[:, 2]) << np.uint64(2))
    order = np.argsort(key, kind="stable")
    lvl, ind, clen, key = lvl[order], ind[order].astype(np.int64), clen[order], key[order]
    n = ids.size
    k = ind[:, 0] | ind[:, 1] | ind[:, 2]
    # alignment = trailing zeros of x | y | z (align_kernel)
    tz = np.zeros(n, np.int64)
    kk = k.copy()
    alive = k != 0
    for b in range(40):
        z = alive & ((kk & 1) == 0)
        tz += z
        alive = z
        kk = kk >> 1
    al = np.where(k == 0, 63, tz)
    # cut_run
    lo = max(1, T // 4)
    starts = []
    a = 0
    while a < n:
        starts.append(a)
        if n - a <= T:
            break
        w = al[a + lo: a + T + 1]
        j = len(w) - 1 - int(np.argmax(w[::-1]))
        a = a + lo + j
    starts = np.array(starts + [n])
    return dict(lvl=lvl, ind=ind, clen=clen, key=key, starts=starts)


def classify(L, base, R):
    lvl, ind, clen, key, starts = L["lvl"], L["ind"], L["clen"], L["key"], L["starts"]
    glen = np.array(base, np.int64) * (1 << R)
    # leaf lookup: (level, min corner) -> slot
    code = (lvl.astype(np.int64) << 60) | (key.astype(np.int64) & ((1 << 60) - 1))
    srt = np.argsort(code)
    code_s = code[srt]

    def find(lv, x, y, z):
        kk = spread3(np.array([x])) | (spread3(np.array([y])) << np.uint64(1)) | (spread3(np.array([z])) << np.uint64(2))
        c = (np.int64(lv) << 60) | np.int64(kk[0])
        i = np.searchsorted(code_s, c)
        return int(srt[i]) if i < code_s.size and code_s[i] == c else -1

    nt = starts.size - 1
    reason = np.zeros(nt, np.int32)  # 1 regular, 0x10 not 512, 0x20 not a box, 0x30 irregular side
    per = (True, True, False)
    for t in range(nt):
        ts, te = starts[t], starts[t + 1]
        if te - ts != 512:
            reason[t] = 0x10
            continue
        lv = lvl[ts]
        ln = clen[ts]
        c = ind[ts]
        if np.any(lvl[ts:te] != lv) or np.any(c % (8 * ln)) or np.any(ind[ts:te] < c) or np.any(ind[ts:te] >= c + 8 * ln):
            reason[t] = 0x20
            continue
        ok = True
        for d in range(6):
            ax, plus = d >> 1, d & 1
            nb = c.copy()
            nb[ax] += 8 * ln if plus else -8 * ln
            if nb[ax] < 0 or nb[ax] >= glen[ax]:
                if not per[ax]:
                    continue
                nb[ax] %= glen[ax]
            s0 = find(lv, *nb)
            if s0 < 0 or s0 + 512 > lvl.size or np.any(lvl[s0:s0 + 512] != lv) or \
                    np.any(ind[s0:s0 + 512] < nb) or np.any(ind[s0:s0 + 512] >= nb + 8 * ln):
                ok = False
                break
        reason[t] = 1 if ok else 0x30
    return reason


def main():
    ids = np.load(sys.argv[1])
    base = tuple(int(v) for v in sys.argv[2].split(","))
    R = int(sys.argv[3])
    T = int(sys.argv[4]) if len(sys.argv) > 4 else 512
    L = layout(ids, base, R, T)
    reason = classify(L, base, R)
    sz = np.diff(L["starts"])
    print("cells", ids.size, "tiles", sz.size, "levels", np.bincount(L["lvl"]))
    for r in (1, 0x10, 0x20, 0x30):
        m = reason == r
        print(f"reason {r:#x}: tiles {m.sum()} cells {sz[m].sum()}")
    m = reason == 0x10
    print("non-512 tile size histogram (bins of 64):", np.histogram(sz[m], bins=np.arange(0, 577, 64))[0])
    # level mix of general tiles
    gen = reason != 1
    mixed = 0
    for t in np.nonzero(gen)[0]:
        a, b = L["starts"][t], L["starts"][t + 1]
        if np.unique(L["lvl"][a:b]).size > 1:
            mixed += 1
    print("general tiles with mixed levels:", mixed)
    np.savez("/tmp/tile_layout.npz", starts=L["starts"], reason=reason, lvl=L["lvl"], ind=L["ind"])
    st = L["starts"]
    for r in (1, 0x30):
        t = np.nonzero(reason == r)[0]
        print(f"reason {r:#x}: boxes by level", np.bincount(L["lvl"][st[t]], minlength=R + 1))


if __name__ == "__main__":
    main()
