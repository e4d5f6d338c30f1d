"""One rank of tests/poisson/poisson1d.cpp's n = 4096 grid over the host
transport (the case test_gpu_transport.py::test_poisson1d_reference_distributed
failed at twice in round 5), for a HIP API / kernel / copy trace per rank:
RANK / WORLD_SIZE / MASTER_* from the environment (scripts/trace_poisson1d.sh
starts the ranks, each under its own rocprofv3).  Prints the rank's 2-norms
against the reference solver's solution."""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import torch  # noqa: E402,F401  (one HIP runtime: torch's)
import torch.distributed as dist  # noqa: E402

import dccrg_amd  # noqa: E402
from poisson_cases import POISSON1D_SOLVER, offset_last, p_norm, poisson1d_reference  # noqa: E402


def main():
    n = int(os.environ.get("N", "4096"))
    reps = int(os.environ.get("REPS", "3"))
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    ref, rhs = poisson1d_reference(n)
    h = 2 * math.pi / n
    norms = []
    for _ in range(reps):
        for d in range(3):
            length, L0 = [1, 1, 1], [1.0, 1.0, 1.0]
            length[d], L0[d] = n, h
            g = dccrg_amd.Dccrg.from_torch_distributed(device=0, transport="host")
            g.set_initial_length(tuple(length)).set_maximum_refinement_level(0).set_periodic(True, True, True)
            g.set_neighborhood_length(0).initialize()
            g.set_geometry((0, 0, 0), tuple(L0))
            for c in g.local_cells():
                g.pin(int(c), int(c) % world)
            g.balance_load(False)
            g.unpin_all_cells()
            slots = g.slot_ids()[: g.n_local]
            rf = g.add_field("rhs", np.float64, False)
            sf = g.add_field("solution", np.float64, False)
            rf.set(rhs[slots.astype(np.int64) - 1])
            sf.set(np.zeros(slots.size))
            dccrg_amd.Poisson_Solve(*POISSON1D_SOLVER).solve(slots, g)
            parts = [None] * world
            dist.all_gather_object(parts, dict(zip(slots.tolist(), sf.get(0, slots.size).tolist())))
            d_all = {}
            for part in parts:
                d_all.update(part)
            norms.append(p_norm(offset_last(np.array([d_all[i] for i in range(1, n + 1)])), ref))
            g.close()
    if rank == 0:
        print({"n": n, "world": world, "norms": norms, "max": max(norms)}, flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
