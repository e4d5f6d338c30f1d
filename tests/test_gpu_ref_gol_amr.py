"""Refined game of life pinned to the reference's own code.

examples/bin/ref_game_of_life_amr is a repo-owned main in the shape of
tests/game_of_life/unrefined2d.cpp that includes the reference's
tests/game_of_life/{cell,initialize,refine,solve}.hpp unmodified and runs
through the drop-in facade (built by __graft_entry__.build_examples()): every
turn the reference's Refine::refine (random refines / unrefines), a balance,
the halo, and its get_live_neighbors (solve.hpp:37-170), checked inside the
program against an unrefined game.  It dumps, per turn and rank, the mesh and
each cell's state before and after get_live_neighbors.  Here every turn is
replayed on the device: the same leaves (dccrgx_set_cells), the same input
states, one turn of the product's refined game (collect, halo, spread +
rule kernels of gol_amr.hip) - the output states must equal the reference
code's bit for bit.  At 1 and 2 MPI ranks (two ranks: a partitioned mesh
and the facade's halo in the reference run; the replay is one rank)."""
import os
import subprocess

import numpy as np
import pytest

import dccrg_amd

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "examples", "bin", "ref_game_of_life_amr")
MPIEXEC = "/opt/conda/bin/mpiexec"
LIST = np.dtype((np.uint64, 8))
MAGIC = 0x676f6c616d723031


def _load(prefix, step, P):
    recs = []
    for r in range(P):
        raw = open(f"{prefix}.{step}.{r}", "rb").read()
        magic, n = np.frombuffer(raw, "<u8", 2)
        assert magic == MAGIC
        recs.append(np.frombuffer(raw, "<u8", 3 * int(n), 16).reshape(-1, 3))
    a = np.concatenate(recs)
    return a[np.argsort(a[:, 0])]


@pytest.mark.parametrize("direction,P", [("z", 1), ("x", 1), ("z", 2), ("y", 2)])
def test_refined_game_matches_reference_solve(gpu, tmp_path, direction, P):
    if not os.path.exists(BIN):
        pytest.fail(f"{BIN} missing: run __graft_entry__.build() first")
    steps = 25
    prefix = str(tmp_path / "gol")
    r = subprocess.run([MPIEXEC, "-n", str(P), BIN, direction, str(steps), prefix], capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0 and "PASSED" in r.stdout, (r.stdout + r.stderr)[-3000:]
    length = [15, 15, 15]
    length["xyz".index(direction)] = 1
    refined_turns = 0
    for step in range(steps):
        rec = _load(prefix, step, P)
        ids, pre, post = rec[:, 0].copy(), rec[:, 1], rec[:, 2]
        g = dccrg_amd.Dccrg(0, 1, 0).set_initial_length(tuple(length)).set_maximum_refinement_level(1)
        g.set_neighborhood_length(1).initialize()
        g.set_cells(ids, np.zeros(ids.size, np.int32))
        st = g.add_field("is_alive", np.uint32)
        ls = g.add_field("gol_list", LIST)
        slots = g.slot_ids()[: g.n_local]
        assert np.array_equal(np.sort(slots), ids)
        order = np.searchsorted(ids, slots)
        st.set(pre[order].astype(np.uint32))
        g.get_live_neighbors(st, ls)
        got = st.get(0, g.n_local)
        assert np.array_equal(got, post[order].astype(np.uint32)), f"turn {step}: {int((got != post[order]).sum())} cells"
        refined_turns += int(ids.size > 225)
        g.close()
    assert refined_turns >= steps // 2  # the mesh really is refined on most turns
