"""ORACLE — TEST INFRASTRUCTURE ONLY: the CPU baseline leg of bench.py.

One process of the CPU baseline: times the oracle restatement of the
reference's stencil loop (oracle/dccrg_oracle.cpp: the same AoS + hashed
neighbor lookups as the reference's per-rank loop) on a bounded sample of a
bench workload and prints one JSON line {"cells", "steps", "seconds"}.
bench.py starts one such process per host core it uses (the reference's
MPI ranks, one per core, each owning its own subdomain) and sums their
cell-updates/s.

    python -m oracle.cpu_bench --workload advection --seconds 10
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oracle import oracle as O  # noqa: E402


def alive_rule(ids):
    z = (ids ^ np.uint64(0x5DEECE66D)) + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    z = z ^ (z >> np.uint64(31))
    return (z < np.uint64(int(0.2 * 2 ** 64))).astype(np.uint32)


def advection(seconds):
    """64 x 64 x 8 base, R = 2, the reference's pre-refinement (config 3's
    mesh recipe on a 1/64 base: ~172 K cells, a working set of tens of MB per
    process, beyond a core's L2 and its share of L3), fused flux + apply steps."""
    o = O.Grid((64, 64, 8), 2, (True, True, False), 0, 1)
    o.set_geometry((0, 0, 0), (1 / 64, 1 / 64, 1 / 64))
    o.adv_prerefine(0.025, 0.25)
    ids, _ = o.cells()
    dt = o.adv_max_time_step()
    o.adv_steps(1, 0.5 * dt)
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        o.adv_steps(5, 0.5 * dt)
        steps += 5
    return ids.size, steps, time.perf_counter() - t0, "64x64x8 base, R=2, pre-refined"


def gol(seconds):
    """64 x 64 x 16 game of life, 26-point stencil, non-periodic (config 2's
    rule on a smaller grid)."""
    o = O.Grid((64, 64, 16), 0, (False, False, False), 1, 1)
    ids, _ = o.cells()
    o.gol_set(ids, alive_rule(ids))
    o.gol_steps(1)
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        o.gol_steps(1)
        steps += 1
    return ids.size, steps, time.perf_counter() - t0, "64x64x16, neighborhood 1"


def gol_amr(seconds):
    """get_live_neighbors (tests/game_of_life/solve.hpp) on 128 x 128 x 1
    level-0 cells, a seeded quarter refined once."""
    n = 128
    o = O.Grid((n, n, 1), 1, (False, False, False), 1, 1)
    rng = np.random.default_rng(7)
    ids0, _ = o.cells()
    live0 = rng.random(n * n) < 0.3
    for c in rng.choice(ids0, size=n * n // 4, replace=False):
        o.refine_completely(int(c))
    o.stop_refining()
    ids, _ = o.cells()
    par = o.mapping.batch(ids)["level0_parent"].astype(np.int64) - 1
    o.gola_set(ids, live0[par].astype(np.uint32))
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        o.gola_steps(1)
        steps += 1
    return ids.size, steps, time.perf_counter() - t0, "128x128x1 level-0, quarter refined"


def poisson(seconds):
    """poisson3d.cpp on a 32^3 base refined twice at the center, batches of
    20 BiCG iterations (min = max)."""
    n = 32
    L0 = (2 * math.pi / n, math.pi / n, 8 * math.pi / n)
    o = O.Grid((n, n, n), 2, (True, True, True), 0, 1)
    o.set_geometry((0, 0, 0), L0)
    for _ in range(2):  # poisson3d.cpp:174-192
        ids, _ = o.cells()
        c, L = o.geometry(ids)
        mn, mx = c - L / 2, c + L / 2
        sel = ((mn[:, 0] < 1.01 * math.pi) & (mx[:, 0] > 0.99 * math.pi) & (mn[:, 1] < 0.51 * math.pi)
               & (mx[:, 1] > 0.49 * math.pi) & (mn[:, 2] < 4.01 * math.pi) & (mx[:, 2] > 3.99 * math.pi))
        for cell in ids[sel]:
            o.refine_completely(int(cell))
        o.stop_refining()
    ids, _ = o.cells()
    c, _ = o.geometry(ids)
    rhs = -(81.0 / 16.0) * np.sin(c[:, 0]) * np.cos(2 * c[:, 1]) * np.sin(c[:, 2] / 4)
    its, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        o.po_set(ids, rhs, np.zeros(ids.size), np.zeros(ids.size, np.int32))
        it, _ = o.po_solve(20, 20)
        its += it
    return ids.size, its, time.perf_counter() - t0, "32^3 base refined twice at the center, setup included"


WORKLOADS = {"advection": advection, "gol": gol, "scalability": gol, "gol_amr": gol_amr, "poisson": poisson}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workload", choices=sorted(WORKLOADS), required=True)
    p.add_argument("--seconds", type=float, default=10.0)
    a = p.parse_args()
    cells, steps, el, sample = WORKLOADS[a.workload](a.seconds)
    print(json.dumps({"cells": cells, "steps": steps, "seconds": el, "sample": sample}), flush=True)


if __name__ == "__main__":
    main()
