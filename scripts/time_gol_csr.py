"""Time the CSR game-of-life sweep (gol_csr_kernel: refined meshes and
partitions the structured kernel cannot take) on a 2048 x 2048 x 1 grid with
a seeded quarter of the level-0 cells refined (the gol_amr bench mesh),
neighborhood 1.  Prints one JSON line: ms per sweep (HIP events around the
launches) and the SURVEY §8(d) CSR bytes rate (8 B + 4 B per entry + 4 B)."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
import dccrg_amd  # noqa: E402


def main(steps=50):
    n = 2048
    g = dccrg_amd.Dccrg(0, 1, 0).set_initial_length((n, n, 1)).set_neighborhood_length(1)
    g.set_maximum_refinement_level(1).initialize()
    rng = np.random.default_rng(7)
    for c in rng.choice(np.arange(1, n * n + 1, dtype=np.uint64), size=n * n // 4, replace=False):
        g.refine_completely(int(c))
    g.stop_refining()
    st = g.add_field("is_alive", np.uint32)
    st.set((rng.random(g.n_local) < 0.3).astype(np.uint32))
    for _ in range(3):
        g.gol_step(st)
        g.gol_commit(st)
    g.synchronize()
    g.kernel_timing(1)
    t0 = time.perf_counter()
    for _ in range(steps):
        g.gol_step(st)
        g.gol_commit(st)
    g.synchronize()
    el = time.perf_counter() - t0
    kms, kn = g.kernel_timing(0)
    nl = g.n_local
    k = g.neighbor_entries("iterator") / nl
    b = (8 + 4 * k + 4) * nl
    print(json.dumps({"what": "gol_csr sweep, refined 2048^2 level-0 grid", "cells": nl, "entries_per_cell": k,
                      "ms_per_step": el / steps * 1e3, "kernel_ms": kms / steps,
                      "GB_per_s": b / (kms / steps / 1e3) / 1e9 if kms else None}))
    g.close()


if __name__ == "__main__":
    main()
