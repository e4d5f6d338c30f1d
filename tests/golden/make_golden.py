"""Generate the golden fixtures under tests/golden/ (run here, where
/root/reference exists; the fixtures travel, the reference does not).

1. mapping_ref.json — outputs of the reference's own Mapping and
   Cartesian_Geometry (dccrg_mapping.hpp, dccrg_cartesian_geometry.hpp compiled
   unmodified into oracle/_ref/ref_probe) for random ids / index queries.
2. kat_*.json — the known answers the reference's own tests assert,
   transcribed as data:
     kat_face_cache.json   tests/get_neighbors_/test1.cpp:37-638
     kat_face_counts.json  tests/get_face_neighbors/test1.cpp:37-260
     kat_hood_counts.json  tests/user_neighborhood/neighbor_list_length.cpp:61-308
     kat_gol.json          tests/game_of_life/game_of_life_test.cpp:54-232 +
                           tests/game_of_life/initialize.hpp:28-93, and
                           examples/simple_game_of_life.cpp (blinker)

Usage: python tests/golden/make_golden.py
"""
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
PROBE = os.path.join(ROOT, "oracle", "_ref", "ref_probe")


def run_probe(length, R, start, l0, ids, queries):
    inp = [" ".join(map(str, list(length) + [R] + list(start) + list(l0)))]
    inp.append(str(len(ids)) + " " + " ".join(str(int(i)) for i in ids))
    inp.append(str(len(queries)) + " " + " ".join(" ".join(str(int(v)) for v in q) for q in queries))
    out = subprocess.run([PROBE], input="\n".join(inp) + "\n", capture_output=True, text=True, check=True).stdout
    lines = out.strip().split("\n")
    recs = []
    for ln in lines[: len(ids)]:
        f = ln.split()
        recs.append(dict(id=int(f[0]), level=int(f[1]), indices=[int(x) for x in f[2:5]], length=int(f[5]),
                         parent=int(f[6]), child=int(f[7]), level0_parent=int(f[8]),
                         siblings=[int(x) for x in f[9:17]],
                         center=[float(x) for x in f[17:20]], cell_length=[float(x) for x in f[20:23]]))
    qres = [int(x) for x in lines[len(ids): len(ids) + len(queries)]]
    last, maxpos = (int(x) for x in lines[-1].split())
    return recs, qres, last, maxpos


def mapping_fixture():
    rng = np.random.default_rng(20241024)
    grids = [
        ((1, 1, 1), 0, (0, 0, 0), (1, 1, 1)),
        ((3, 1, 1), 3, (0, 0, 0), (1, 1, 1)),
        ((5, 7, 3), 2, (-1.0, 0.5, 2.0), (0.1, 0.2, 0.3)),
        ((7, 5, 3), 4, (0, 0, 0), (1.0 / 7, 1.0 / 5, 1.0 / 3)),
        ((16, 16, 16), 2, (0, 0, 0), (1.0 / 16, 1.0 / 16, 1.0 / 16)),
        ((128, 128, 128), 2, (0, 0, 0), (1.0 / 128, 1.0 / 128, 1.0 / 128)),
        ((1024, 1024, 64), 0, (0, 0, 0), (1, 1, 1)),
        ((2, 3, 5), 10, (0, 0, 0), (1, 1, 1)),
    ]
    out = []
    for length, R, start, l0 in grids:
        g = int(np.prod(length))
        last = sum(g * 8 ** i for i in range(R + 1))
        ids = [0, 1, 2, g, g + 1, last, last + 1]
        ids += [int(x) for x in rng.integers(1, last + 1, size=200)]
        queries = []
        for _ in range(200):
            lvl = int(rng.integers(-1, R + 2))
            idx = [int(rng.integers(0, length[d] * 2 ** R + 2)) for d in range(3)]
            queries.append(idx + [lvl])
        recs, qres, lastc, maxpos = run_probe(length, R, start, l0, ids, queries)
        assert lastc == last
        out.append(dict(length=list(length), max_ref_lvl=R, start=list(start), level_0_cell_length=list(l0),
                        last_cell=lastc, max_possible_level=maxpos, ids=recs,
                        queries=[dict(indices=q[:3], level=q[3], cell=c) for q, c in zip(queries, qres)]))
    return out


ERR = 0


def cid(length, R, x, y, z, lvl):
    """Mapping::get_cell_from_indices restated for fixture construction only
    (cross-checked against the probe output above by tests)."""
    if lvl < 0 or lvl > R:
        return 0
    g = length[0] * length[1] * length[2]
    c = 1 + sum(g * 8 ** i for i in range(lvl))
    sh = 2 ** (R - lvl)
    lx, ly = length[0] * 2 ** lvl, length[1] * 2 ** lvl
    return c + x // sh + (y // sh) * lx + (z // sh) * lx * ly


def face_cache_fixture():
    """tests/get_neighbors_/test1.cpp — expected neighbors_[cell] for every leaf."""
    cases = []
    for L in (0, 1, 2, 3):
        # 1x1x1, every periodicity combination tested (37-150)
        for per, exp in [((0, 0, 0), [ERR] * 6), ((1, 1, 1), [1] * 6), ((0, 1, 1), [ERR, ERR, 1, 1, 1, 1]),
                         ((1, 0, 1), [1, 1, ERR, ERR, 1, 1]), ((1, 1, 0), [1, 1, 1, 1, ERR, ERR])]:
            cases.append(dict(length=[1, 1, 1], R=0, periodic=list(per), hood=L, refine=[], expected={"1": exp}))
        # 3x1x1 / 1x3x1 / 1x1x3 non-periodic (152-300)
        cases.append(dict(length=[3, 1, 1], R=0, periodic=[0, 0, 0], hood=L, refine=[],
                          expected={"1": [ERR, 2, ERR, ERR, ERR, ERR], "2": [1, 3, ERR, ERR, ERR, ERR],
                                    "3": [2, ERR, ERR, ERR, ERR, ERR]}))
        cases.append(dict(length=[1, 3, 1], R=0, periodic=[0, 0, 0], hood=L, refine=[],
                          expected={"1": [ERR, ERR, ERR, 2, ERR, ERR], "2": [ERR, ERR, 1, 3, ERR, ERR],
                                    "3": [ERR, ERR, 2, ERR, ERR, ERR]}))
        cases.append(dict(length=[1, 1, 3], R=0, periodic=[0, 0, 0], hood=L, refine=[],
                          expected={"1": [ERR, ERR, ERR, ERR, ERR, 2], "2": [ERR, ERR, ERR, ERR, 1, 3],
                                    "3": [ERR, ERR, ERR, ERR, 2, ERR]}))
        # refined 1x1x1, non-periodic (303-370) and periodic (372-460)
        ln = (1, 1, 1)
        gc = lambda x, y, z: cid(ln, 1, x, y, z, 1)
        exp_np, exp_p = {}, {}
        for cell in range(2, 10):
            i = cell - 2
            x, y, z = i & 1, (i >> 1) & 1, (i >> 2) & 1
            r = [ERR] * 6
            other = [gc(1 - x, y, z), gc(x, 1 - y, z), gc(x, y, 1 - z)]
            for d, (coord, o) in enumerate(zip((x, y, z), other)):
                if coord == 0:
                    r[2 * d + 1] = o
                else:
                    r[2 * d] = o
            exp_np[str(cell)] = r
            exp_p[str(cell)] = [other[0], other[0], other[1], other[1], other[2], other[2]]
        cases.append(dict(length=[1, 1, 1], R=1, periodic=[0, 0, 0], hood=L, refine=[1], expected=exp_np))
        cases.append(dict(length=[1, 1, 1], R=1, periodic=[1, 1, 1], hood=L, refine=[1], expected=exp_p))
        # 2x1x1 with cell 1 refined (463-546)
        ln = (2, 1, 1)

        def ge(x, y, z):  # get_existing_cell({x,y,z}, 0, 1): level 1 inside cell 1, else level 0
            return cid(ln, 1, x, y, z, 1) if x < 2 else cid(ln, 1, x, y, z, 0)

        exp = {"2": [ge(1, 0, 0), ERR, ERR, ERR, ERR, ERR],
               "3": [ERR, ge(1, 0, 0), ERR, ge(0, 1, 0), ERR, ge(0, 0, 1)],
               "4": [ge(0, 0, 0), ge(2, 0, 0), ERR, ge(1, 1, 0), ERR, ge(1, 0, 1)],
               "7": [ERR, ge(1, 1, 0), ge(0, 0, 0), ERR, ERR, ge(0, 1, 1)],
               "8": [ge(0, 1, 0), ge(2, 1, 0), ge(1, 0, 0), ERR, ERR, ge(1, 1, 1)],
               "11": [ERR, ge(1, 0, 1), ERR, ge(0, 1, 1), ge(0, 0, 0), ERR],
               "12": [ge(0, 0, 1), ge(2, 0, 1), ERR, ge(1, 1, 1), ge(1, 0, 0), ERR],
               "15": [ERR, ge(1, 1, 1), ge(0, 0, 1), ERR, ge(0, 1, 0), ERR],
               "16": [ge(0, 1, 1), ge(2, 1, 1), ge(1, 0, 1), ERR, ge(1, 1, 0), ERR]}
        cases.append(dict(length=[2, 1, 1], R=1, periodic=[0, 0, 0], hood=L, refine=[1], expected=exp))
        # 1x2x1 with cell 1 refined (548-636)
        ln = (1, 2, 1)

        def ge2(x, y, z):
            return cid(ln, 1, x, y, z, 1) if y < 2 else cid(ln, 1, x, y, z, 0)

        exp = {"2": [ERR, ERR, ge2(0, 1, 0), ERR, ERR, ERR],
               "3": [ERR, ge2(1, 0, 0), ERR, ge2(0, 1, 0), ERR, ge2(0, 0, 1)],
               "4": [ge2(0, 0, 0), ERR, ERR, ge2(1, 1, 0), ERR, ge2(1, 0, 1)],
               "5": [ERR, ge2(1, 1, 0), ge2(0, 0, 0), ge2(0, 2, 0), ERR, ge2(0, 1, 1)],
               "6": [ge2(0, 1, 0), ERR, ge2(1, 0, 0), ge2(1, 2, 0), ERR, ge2(1, 1, 1)],
               "11": [ERR, ge2(1, 0, 1), ERR, ge2(0, 1, 1), ge2(0, 0, 0), ERR],
               "12": [ge2(0, 0, 1), ERR, ERR, ge2(1, 1, 1), ge2(1, 0, 0), ERR],
               "13": [ERR, ge2(1, 1, 1), ge2(0, 0, 1), ge2(0, 2, 1), ge2(0, 1, 0), ERR],
               "14": [ge2(0, 1, 1), ERR, ge2(1, 0, 1), ge2(1, 2, 1), ge2(1, 1, 0), ERR]}
        cases.append(dict(length=[1, 2, 1], R=1, periodic=[0, 0, 0], hood=L, refine=[1], expected=exp))
    return cases


def face_count_fixture():
    """tests/get_face_neighbors/test1.cpp — number (and ids) of face neighbors, 1 process."""
    cases = []
    for L in (0, 1, 2, 3):
        for per, n in [((0, 0, 0), 0), ((1, 1, 1), 6), ((0, 1, 1), 4), ((1, 0, 1), 4), ((1, 1, 0), 4)]:
            cases.append(dict(length=[1, 1, 1], R=0, periodic=list(per), hood=L, refine=[], counts={"1": n},
                              first={}))
        for ln in ([2, 1, 1], [1, 2, 1], [1, 1, 2]):
            cases.append(dict(length=ln, R=0, periodic=[0, 0, 0], hood=L, refine=[], counts={"1": 1, "2": 1},
                              first={"1": 2, "2": 1}))
        cases.append(dict(length=[1, 1, 1], R=1, periodic=[0, 0, 0], hood=L, refine=[1],
                          counts={str(c): 3 for c in range(2, 10)}, first={}))
    return cases


def hood_count_fixture():
    """tests/user_neighborhood/neighbor_list_length.cpp — iterator list lengths
    on a 10x10x10 periodic grid with neighborhood length 2 (default hood) and
    user neighborhoods."""
    hoods = [
        dict(name="default", hood=None, n_of=124, n_to=124),
        dict(name="id1", hood=[[-2, -2, -2]], n_of=1, n_to=1),
        dict(name="id2", hood=[[-1, -1, -1], [2, 2, 2]], n_of=2, n_to=2),
        dict(name="id-3", hood=[[i, j, 0] for i in range(-2, 3) for j in range(-2, 3) if (i, j) != (0, 0)],
             n_of=24, n_to=24),
        dict(name="id-4", hood=[[0, j, k] for j in range(-2, 3) for k in range(-2, 3) if (j, k) != (0, 0)],
             n_of=24, n_to=24),
    ]
    return dict(length=[10, 10, 10], R=0, periodic=[1, 1, 1], hood_len=2, hoods=hoods)


def gol_fixture():
    n = 15

    def live(grid_size):  # tests/game_of_life/initialize.hpp:28-93
        s = set()
        b = 198
        s |= {b, b + 1, b + 2}
        t = 188
        s |= {t, t + 1, t + 2, t + 1 + grid_size, t + 2 + grid_size, t + 3 + grid_size}
        be = 137
        s |= {be, be + 1, be - grid_size, be + 1 - grid_size, be + 2 - 2 * grid_size, be + 3 - 2 * grid_size,
              be + 2 - 3 * grid_size, be + 3 - 3 * grid_size}
        g = 143
        s |= {g + 1, g + 2 - grid_size, g - 2 * grid_size, g + 1 - 2 * grid_size, g + 2 - 2 * grid_size}
        bl = 47
        s |= {bl, bl + 1, bl - grid_size, bl + 1 - grid_size}
        bh = 51
        s |= {bh - grid_size, bh + 1, bh + 2, bh + 1 - 2 * grid_size, bh + 2 - 2 * grid_size, bh + 3 - grid_size}
        return sorted(s)

    kat = dict(
        length=[n, n, 1], R=0, periodic=[0, 0, 0], hood_len=1, steps=25, initial_live=live(n),
        always_alive=[22, 23, 32, 33, 36, 39, 47, 48, 52, 53, 94, 95, 110, 122, 137, 138, 188, 199, 206],
        alive_even=[109, 123, 189, 190, 198, 200, 204, 205],
        alive_odd=[174, 184, 214, 220],
        glider={"20": [43, 44, 45, 60, 74], "21": [29, 44, 45, 58, 60], "22": [29, 30, 43, 45, 60],
                "23": [29, 30, 45, 59], "24": [29, 30, 45]},
    )
    # examples/simple_game_of_life.cpp: 10x10x1, hood 1, blinker 54/55/56
    blinker = dict(length=[10, 10, 1], R=0, periodic=[0, 0, 0], hood_len=1, steps=100, initial_live=[54, 55, 56],
                   always_alive=[55], alive_after_even_turn=[45, 65], dead_after_even_turn=[54, 56])
    return dict(game_of_life_test=kat, simple_game_of_life=blinker)


WRITE_PROBE = os.path.join(ROOT, "oracle", "_ref", "ref_write_probe")

GRID_FILE_CASES = [
    # length, R, hood, periodic, start, level-0 cell length
    ([4, 3, 2], 2, 1, [1, 0, 1], [0.5, -1.0, 2.0], [0.25, 0.125, 1.5]),
    ([128, 128, 128], 2, 0, [1, 1, 0], [0.0, 0.0, 0.0], [1 / 128, 1 / 128, 1 / 128]),
    ([10, 10, 10], 0, 2, [1, 1, 1], [-3.0, 0.0, 7.5], [0.1, 0.2, 0.3]),
]


def grid_file_fixture():
    """The internal-grid-data block of save_grid_data (dccrg.hpp:1196-1258)
    written by the reference's own Mapping / Topology / Cartesian_Geometry
    writers (oracle/ref_write_probe.cpp)."""
    out = []
    for length, R, hood, per, start, l0 in GRID_FILE_CASES:
        path = os.path.join("/tmp", f"dccrgx_probe_{os.getpid()}.bin")
        line = " ".join(str(v) for v in [*length, R, hood, *per] + [repr(float(v)) for v in [*start, *l0]] + [path])
        sizes = subprocess.run([WRITE_PROBE], input=line + "\n", capture_output=True, text=True,
                               check=True).stdout.split()
        data = open(path, "rb").read()
        os.remove(path)
        out.append(dict(length=length, R=R, hood=hood, periodic=per, start=start, l0=l0,
                        sizes=[int(v) for v in sizes], block_hex=data.hex()))
    return out


def main():
    if not os.path.exists(PROBE):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    with open(os.path.join(HERE, "mapping_ref.json"), "w") as f:
        json.dump(mapping_fixture(), f)
    with open(os.path.join(HERE, "kat_face_cache.json"), "w") as f:
        json.dump(face_cache_fixture(), f, indent=0)
    with open(os.path.join(HERE, "kat_face_counts.json"), "w") as f:
        json.dump(face_count_fixture(), f, indent=0)
    with open(os.path.join(HERE, "kat_hood_counts.json"), "w") as f:
        json.dump(hood_count_fixture(), f, indent=0)
    with open(os.path.join(HERE, "kat_gol.json"), "w") as f:
        json.dump(gol_fixture(), f, indent=0)
    with open(os.path.join(HERE, "grid_file_ref.json"), "w") as f:
        json.dump(grid_file_fixture(), f, indent=0)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    sys.exit(main())
