"""Fixture tests/golden/poisson1d_ref.npz: the reference's own serial 1-D
Poisson solutions (tests/poisson/reference_poisson_solve.hpp, compiled
unmodified into oracle/_ref/ref_poisson_probe by `make -C oracle ref`) for
the cases of tests/poisson/poisson1d.cpp:150-160 - n = 8 ... 32768 cells of
length 2 pi / n, rhs = sin((i + 0.5) dx), solution 0 in the last cell.
Arrays "n<cells>" (the solution) and "rhs<cells>" (the rhs after solve()
offset it to a zero total, which poisson1d.cpp:225-236 hands to the grids);
float64, cell index order.  Run here, where
/root/reference exists; the fixture travels, the reference does not.

Usage: python tests/golden/make_poisson_ref.py
"""
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
PROBE = os.path.join(ROOT, "oracle", "_ref", "ref_poisson_probe")


def main():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "_ref/ref_poisson_probe"], check=True)
    out = subprocess.run([PROBE], capture_output=True, text=True, check=True).stdout.split()
    arrays, i = {}, 0
    while i < len(out):
        n = int(out[i])
        v = np.array([float(x) for x in out[i + 1: i + 1 + 2 * n]], np.float64).reshape(n, 2)
        arrays[f"n{n}"] = v[:, 0].copy()
        arrays[f"rhs{n}"] = v[:, 1].copy()
        i += 1 + 2 * n
    np.savez_compressed(os.path.join(HERE, "poisson1d_ref.npz"), **arrays)
    print({k: v.size for k, v in arrays.items() if k.startswith('n')})


if __name__ == "__main__":
    main()
