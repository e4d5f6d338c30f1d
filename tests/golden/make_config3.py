"""Golden fixture of BASELINE config 3 at full size from the oracle (test
infrastructure): the 128^3-base, R = 2 advection mesh after the reference's
pre-refinement (tests/advection/2d.cpp:260-285), and the density after
3 and after 100 steps of 0.5 * max_time_step (solve.hpp:44-333) at a sample
of cells, with the total mass sum(rho * lx * ly * lz) (math.fsum) at steps
0 and 100.

Writes tests/golden/config3_adv.json: the leaf count per level, the SHA-256
of the ascending leaf ids (little-endian uint64), dt, and for every 499th leaf
(ascending id) plus the first and last leaf of each level the oracle's
density after the 3 and the 100 steps.  tests/test_gpu_config_full.py
compares the product at full size with it.  Takes ~6 minutes and ~9 GB of
host memory.

    python tests/golden/make_config3.py
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

BASE, R, STEPS, STEPS_LONG, STRIDE = (128, 128, 128), 2, 3, 100, 499


def main():
    t0 = time.time()
    o = O.Grid(BASE, R, (True, True, False), 0, 1)
    o.set_geometry((0, 0, 0), tuple(1.0 / b for b in BASE))
    o.adv_prerefine(0.025, 0.25)
    ids, _ = o.cells()
    ids = np.sort(ids)
    lvl = O.Mapping(BASE, R).batch(ids)["level"]
    dt = o.adv_max_time_step()
    o.adv_initialize()

    def mass():
        import math

        a = o.adv_get(ids)
        return math.fsum((a[:, 0] * (a[:, 6] * a[:, 7] * a[:, 8])).tolist())

    m0 = mass()
    o.adv_steps(STEPS, 0.5 * dt)
    pick = set(range(0, ids.size, STRIDE))
    for L in range(R + 1):
        w = np.nonzero(lvl == L)[0]
        if w.size:
            pick.update((int(w[0]), int(w[-1])))
    pick = np.array(sorted(pick))
    rho = o.adv_get(ids[pick])[:, 0]
    o.adv_steps(STEPS_LONG - STEPS, 0.5 * dt)
    rho_long = o.adv_get(ids[pick])[:, 0]
    m_long = mass()
    out = {
        "what": "oracle (oracle/dccrg_oracle.cpp) on BASELINE config 3: base 128^3, max_ref_lvl 2, periodic x,y, "
                "cell length 1/128, pre-refined (relative_diff 0.025/R, diff_threshold 0.25), then 3 steps of "
                "0.5 * max_time_step; density at sampled leaves",
        "base": list(BASE), "max_ref_lvl": R, "steps": STEPS,
        "n_cells": int(ids.size), "cells_per_level": np.bincount(lvl, minlength=R + 1).tolist(),
        "ids_sha256": hashlib.sha256(ids.astype("<u8").tobytes()).hexdigest(),
        "dt": float(dt), "max_abs_rho_sample": float(np.max(np.abs(rho))),
        "sample_ids": ids[pick].tolist(), "sample_rho": rho.tolist(),
        "steps_long": STEPS_LONG, "sample_rho_long": rho_long.tolist(),
        "mass_0": m0, "mass_long": m_long,
        "seconds": time.time() - t0,
    }
    with open(os.path.join(ROOT, "tests", "golden", "config3_adv.json"), "w") as f:
        json.dump(out, f)
    print(out["n_cells"], out["cells_per_level"], len(out["sample_ids"]), m0, m_long, f"{out['seconds']:.0f} s")


if __name__ == "__main__":
    main()
