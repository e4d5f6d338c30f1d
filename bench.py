"""Benchmark: BASELINE.json metric — cell-updates/s (node) for 3-D advection
with halo exchange, and the % of HBM roofline of the advection sweep kernel.

Workload (BASELINE config 3, tests/advection): level-0 base 128 x 128 x
(128 * N) with cubic cells of length 1/128, maximum refinement level 2
(512^3-equivalent per GPU), neighborhood length 0 (face neighbors), periodic
in x and y, non-periodic in z, the reference's initial condition (hump +
rotating velocity, tests/advection/initialize.hpp) and its pre-refinement
criterion (adapter.hpp check_for_adaptation, refine side).  The mesh is then
frozen; one step = halo update of the density (RCCL, N > 1) overlapped with
the inner-cell sweep, then the outer-cell sweep, fused flux + apply.  Weak
scaling: every GPU owns one 128^3-base slab (block partition of level-0 ids,
children inherit the owner).

    python bench.py [--gpus N --steps K --warmup W]   (N > 1 via torch.distributed.run)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

NAMES = ("density", "vx", "vy", "vz", "lx", "ly", "lz")
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--base", type=int, default=128, help="level-0 cells per dimension per GPU")
    p.add_argument("--max-ref-lvl", type=int, default=2)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=15.0)
    p.add_argument("--workload", choices=["advection", "gol", "gol_amr", "poisson"], default="advection",
                   help="advection = BASELINE metric (default); gol = config 2 game of life line; "
                        "poisson = config 4 BiCG line")
    return p.parse_args()


def gol_main(a, dccrgx_mod, torch):
    """BASELINE config 2: game of life 1024 x 1024 x 64, 26-point stencil,
    uint32 state, 1 GPU (algorithmic 8 B per cell-update)."""
    nx, ny, nz = 1024, 1024, 64
    g = dccrgx_mod.Dccrg(0, 1, 0).set_initial_length((nx, ny, nz)).set_neighborhood_length(1)
    g.set_maximum_refinement_level(0).initialize()
    st = g.add_field("is_alive", np.uint32)
    ids = np.arange(1, nx * ny * nz + 1, dtype=np.uint64)
    z = (ids ^ np.uint64(0x5DEECE66D)) + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    z = z ^ (z >> np.uint64(31))
    st.set((z < np.uint64(int(0.2 * 2 ** 64))).astype(np.uint32))
    for _ in range(a.warmup):
        g.gol_step(st)
        g.gol_commit(st)
    g.synchronize()
    torch.cuda.synchronize()
    g.kernel_timing(1)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        g.gol_step(st)
        g.gol_commit(st)
    g.synchronize()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    kms, kn = g.kernel_timing(0)
    n = nx * ny * nz
    ach = 8.0 * n * a.steps / (kms / 1e3) / 1e9
    print(json.dumps({
        "metric": "cell-updates/s, game of life 3D (BASELINE config 2)", "value": n * a.steps / el,
        "unit": "cell-updates/s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": el / a.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u32", "data": "synthetic: seeded alive(id) rule, p=0.2",
        "config": {"workload": "game of life 1024x1024x64, neighborhood 1, non-periodic (config 2)"},
        "roofline": {"bound": "hbm", "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": ach / PEAK_HBM_GBS,
                     "traffic": None, "kernel": "gol_structured_kernel", "alg_bytes_per_step": 8 * n,
                     "kernel_ms_per_step": kms / a.steps},
        "cpu_baseline": None if a.no_cpu_baseline else gol_cpu_baseline(a.cpu_seconds)}), flush=True)
    g.close()


def gol_amr_main(a, dccrgx_mod, torch):
    """the refined game emulating the level-0 game
    (tests/game_of_life/solve.hpp get_live_neighbors, as unrefined2d.cpp
    plays it) on a 2048 x 2048 x 1 level-0 grid, max refinement level 1, a
    seeded quarter of the level-0 cells refined (children inherit the state),
    p = 0.3 live.  One step = collect + spread over every leaf (1 GPU: the
    halo between them is a no-op).  Algorithmic bytes per leaf and step:
    level-0 parent per slot decoded per phase (2 x (8 B id read + 8 B
    written)); collect: own parent 8 B, row pointers 8 B, per neighbor entry
    slot 4 B + parent 8 B + state 4 B, list 64 B written; spread: own parent
    and id 16 B, row pointers 8 B, own list 64 B, and for a level-1 leaf per
    neighbor entry slot 4 B + parent 8 B and its 7 siblings' lists 7 x 64 B,
    state 4 B written."""
    n = 2048
    g = dccrgx_mod.Dccrg(0, 1, 0).set_initial_length((n, n, 1)).set_neighborhood_length(1)
    g.set_maximum_refinement_level(1).initialize()
    rng = np.random.default_rng(7)
    lvl0 = np.arange(1, n * n + 1, dtype=np.uint64)
    live0 = rng.random(n * n) < 0.3
    t_setup = time.perf_counter()
    for c in rng.choice(lvl0, size=n * n // 4, replace=False):
        g.refine_completely(int(c))
    g.stop_refining()
    setup_s = time.perf_counter() - t_setup
    st = g.add_field("is_alive", np.uint32)
    ls = g.add_field("gol_list", np.dtype((np.uint64, 8)))
    slots = g.slot_ids()[: g.n_local]
    lvl = (slots > np.uint64(n * n)).astype(np.int64)
    # level-0 parent of a level-1 leaf (2 x 2 x 2 children per parent, x fastest)
    c1 = slots.astype(np.int64) - 1 - n * n
    x1, y1 = c1 % (2 * n), (c1 // (2 * n)) % (2 * n)
    par = np.where(lvl == 0, slots.astype(np.int64) - 1, (y1 // 2) * n + x1 // 2)
    st.set(live0[par].astype(np.uint32))
    for _ in range(a.warmup):
        g.get_live_neighbors(st, ls)
    g.synchronize()
    torch.cuda.synchronize()
    g.kernel_timing(1)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        g.get_live_neighbors(st, ls)
    g.synchronize()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    kms, kn = g.kernel_timing(0)
    nl = g.n_local
    kbar = g.neighbor_entries("of") / nl
    f1 = float(np.mean(lvl == 1))  # fraction of level-1 leaves
    per_cell = (2 * 16) + (8 + 8 + kbar * 16 + 64) + (16 + 8 + 64 + f1 * (kbar * 12 + 7 * 64) + 4)
    ach = per_cell * nl * a.steps / (kms / 1e3) / 1e9 if kms > 0 else None
    print(json.dumps({
        "metric": "cell-updates/s, refined game of life emulating the level-0 game (SURVEY a14)",
        "value": nl * a.steps / el, "unit": "cell-updates/s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": el / a.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u32/u64", "data": "synthetic: seeded level-0 states (p=0.3), a seeded quarter of the cells refined",
        "config": {"workload": "get_live_neighbors, 2048x2048x1 level-0, max_ref_lvl 1, neighborhood 1",
                   "leaves": nl, "neighbor_entries_per_leaf": kbar, "setup_s": setup_s},
        "roofline": {"bound": "hbm", "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": ach / PEAK_HBM_GBS if ach else None, "traffic": None,
                     "kernel": "gol_amr_collect_kernel + gol_amr_spread_kernel", "alg_bytes_per_cell": per_cell,
                     "kernel_ms_per_step": kms / a.steps, "launches_per_step": kn / a.steps},
        "cpu_baseline": None if a.no_cpu_baseline else gol_amr_cpu_baseline(a.cpu_seconds)}), flush=True)
    g.close()


def gol_amr_cpu_baseline(seconds):
    """The oracle's get_live_neighbors (one core) on a 128 x 128 x 1 sample of
    the same workload."""
    from oracle import oracle as O

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
    el = time.perf_counter() - t0
    return dict(value=ids.size * steps / el, unit="cell-updates/s", cores=1, kind="port",
                sample=f"oracle restatement, 128x128x1 level-0, quarter refined ({ids.size} leaves), {steps} steps, "
                       f"{el:.1f} s on 1 host core")


def poisson_main(a, dccrgx_mod, torch, rank, world, uid):
    """BASELINE config 4: Poisson BiCG (tests/poisson/poisson3d.cpp) on a
    128^3-base grid per GPU (cell lengths 2pi/128, pi/128, 8pi/128), periodic,
    refined twice around (pi, pi/2, 4pi); one step = one BiCG iteration over
    every solve cell (min = max = steps iterations, as SURVEY §8(d))."""
    import math

    n = a.base
    L0 = (2 * math.pi / n, math.pi / n, 8 * math.pi / n)
    g = dccrgx_mod.Dccrg(rank, world, int(os.environ.get("LOCAL_RANK", rank)), uid)
    g.set_initial_length((n, n, n * world)).set_neighborhood_length(0).set_maximum_refinement_level(2)
    g.set_periodic(True, True, True).initialize()
    g.set_geometry((0, 0, 0), L0)
    t_setup = time.perf_counter()
    for _ in range(2):  # poisson3d.cpp:174-192
        ids = g.local_cells()
        c, L = g.geometry(ids)
        mn, mx = c - L / 2, c + L / 2
        sel = ((mn[:, 0] < 1.01 * math.pi) & (mx[:, 0] > 0.99 * math.pi) & (mn[:, 1] < 0.51 * math.pi)
               & (mx[:, 1] > 0.49 * math.pi) & (mn[:, 2] < 4.01 * math.pi) & (mx[:, 2] > 3.99 * math.pi))
        for cell in ids[sel]:
            g.refine_completely(int(cell))
        g.stop_refining()
    ids = g.local_cells()
    slots = g.slot_ids()[: g.n_local]
    c, _ = g.geometry(slots)
    rhs = g.add_field("rhs", np.float64, False)
    sol = g.add_field("solution", np.float64, False)
    rhs.set(-(81.0 / 16.0) * np.sin(c[:, 0]) * np.cos(2 * c[:, 1]) * np.sin(c[:, 2] / 4))
    sol.set(np.zeros(slots.size))
    solver = dccrgx_mod.Poisson_Solve(a.warmup, a.warmup)
    solver.solve(ids, g)  # cache_system_info + warm-up iterations
    setup_s = time.perf_counter() - t_setup
    sol.set(np.zeros(slots.size))
    solver = dccrgx_mod.Poisson_Solve(a.steps, a.steps)
    g.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    g.kernel_timing(1)
    t0 = time.perf_counter()
    it, res = solver.solve(ids, g, cache_is_up_to_date=True)
    g.synchronize()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    kms, kn = g.kernel_timing(0)
    n_solve = ids.size
    stats = torch.tensor([el, float(n_solve), kms], dtype=torch.float64, device="cuda")
    if world > 1:
        import torch.distributed as dist
        mx_ = stats.clone()
        dist.all_reduce(mx_, op=dist.ReduceOp.MAX)
        sm = stats.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        el, total = float(mx_[0]), int(sm[1])
    else:
        total = n_solve
    # algorithmic bytes per solve cell and iteration: SURVEY §8(d) 3-phase
    # minimum 272 B + the face table read by phases A and B (2 x 6 x int32)
    per_cell = 272 + 48
    ach = per_cell * n_solve * it / (kms / 1e3) / 1e9 if kms > 0 else None
    if rank == 0:
        print(json.dumps({
            "metric": "cell-updates/s, Poisson BiCG iterations (BASELINE config 4)", "value": total * it / el,
            "unit": "cell-updates/s", "n_gpus": world, "steps": it, "warmup": a.warmup,
            "ms_per_step": el / it * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f64", "data": "synthetic: poisson3d.cpp rhs on its center-refined mesh",
            "config": {"workload": f"poisson3d BiCG, base {n}x{n}x{n * world}, periodic, refined twice at the "
                                   f"center, min = max = {a.steps} iterations",
                       "solve_cells_rank0": n_solve, "setup_s": setup_s, "parallelism": f"domain decomposition x{world}"},
            "roofline": {"bound": "hbm", "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": ach / PEAK_HBM_GBS if ach else None, "traffic": None,
                         "kernel": "po_phase_a + po_phase_b + po_phase_c", "alg_bytes_per_cell_iteration": per_cell,
                         "kernel_ms_per_step": kms / it, "launches_per_step": kn / it, "residual_min": res},
            "cpu_baseline": None if (a.no_cpu_baseline or world > 1) else poisson_cpu_baseline(a.cpu_seconds)}),
            flush=True)
    g.close()


def build_grid(dccrg_amd, rank, size, base, R, uid):
    nx, ny, nz = base, base, base * size
    g = dccrg_amd.Dccrg(rank, size, int(os.environ.get("LOCAL_RANK", rank)), uid)
    g.set_initial_length((nx, ny, nz)).set_neighborhood_length(0).set_maximum_refinement_level(R)
    g.set_periodic(True, True, False).initialize()
    g.set_geometry((0.0, 0.0, 0.0), (1.0 / nx, 1.0 / ny, 1.0 / nx))
    f = [g.add_field(n, np.float64, n == "density") for n in NAMES]
    # pre-refinement (tests/advection/2d.cpp:260-285), refine side
    for _ in range(R):
        g.advection_initialize(f)
        for c in g.advection_refine_candidates(f[0], 0.025 / R, 0.25):
            g.refine_completely(int(c))
        g.stop_refining()
    g.advection_initialize(f)
    return g, f


def poisson_cpu_baseline(seconds):
    """The oracle's Poisson_Solve (one core) on a 32^3 sample of config 4
    (same cell lengths, periodic, refined twice at the center, same rhs):
    batches of 20 iterations (min = max) until ~`seconds`."""
    import math

    from oracle import oracle as O

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
    el = time.perf_counter() - t0
    return dict(value=ids.size * its / el, unit="cell-updates/s", cores=1, kind="port",
                sample=f"oracle restatement, 32^3 base refined twice at the center ({ids.size} cells), "
                       f"{its} BiCG iterations incl. setup, {el:.1f} s on 1 host core")


def gol_cpu_baseline(seconds):
    """The oracle's game of life (CPU restatement of the reference's loop over
    cell.neighbors_of, one core) on a 64 x 64 x 16 sample of config 2 (same
    26-point stencil, non-periodic, same alive(id) rule)."""
    from oracle import oracle as O

    n = (64, 64, 16)
    o = O.Grid(n, 0, (False, False, False), 1, 1)
    ids, _ = o.cells()
    z = (ids ^ np.uint64(0x5DEECE66D)) + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    z = z ^ (z >> np.uint64(31))
    o.gol_set(ids, (z < np.uint64(int(0.2 * 2 ** 64))).astype(np.uint32))
    o.gol_steps(1)
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        o.gol_steps(1)
        steps += 1
    el = time.perf_counter() - t0
    return dict(value=ids.size * steps / el, unit="cell-updates/s", cores=1, kind="port",
                sample=f"oracle restatement, 64x64x16 game of life ({ids.size} cells), {steps} steps, "
                       f"{el:.1f} s on 1 host core")


def cpu_baseline(seconds):
    """The oracle (CPU restatement, one core) on a bounded sample of the same
    workload: 32 x 32 x 4 base, R = 2, same pre-refinement, time steps until
    ~`seconds` of CPU time."""
    from oracle import oracle as O

    base = (32, 32, 4)
    o = O.Grid(base, 2, (True, True, False), 0, 1)
    o.set_geometry((0, 0, 0), (1 / 32, 1 / 32, 1 / 32))
    o.adv_prerefine(0.025, 0.25)
    ids, _ = o.cells()
    dt = o.adv_max_time_step()
    o.adv_steps(1, 0.5 * dt)
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        o.adv_steps(5, 0.5 * dt)
        steps += 5
    el = time.perf_counter() - t0
    return dict(value=ids.size * steps / el, unit="cell-updates/s", cores=1, kind="port",
                sample=f"oracle restatement, 32x32x4 base R=2 pre-refined ({ids.size} cells), {steps} steps, "
                       f"{el:.1f} s on 1 host core")


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    import dccrg_amd

    if a.workload == "gol":
        return gol_main(a, dccrg_amd, torch)
    if a.workload == "gol_amr":
        return gol_amr_main(a, dccrg_amd, torch)
    uid = None
    if world > 1:
        obj = [dccrg_amd.Dccrg.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        uid = obj[0]
    if a.workload == "poisson":
        return poisson_main(a, dccrg_amd, torch, rank, world, uid)

    t_setup = time.perf_counter()
    g, f = build_grid(dccrg_amd, rank, world, a.base, a.max_ref_lvl, uid)
    setup_s = time.perf_counter() - t_setup
    dt = 0.5 * g.advection_max_time_step(f)  # cfl 0.5 (2d.cpp:121-123)
    c = g.counts
    n_local = c["inner"] + c["outer"]
    variant = int(os.environ.get("DCCRGX_ADV_VARIANT", "11"))
    layout = g.advection_layout()
    n_fine = layout["finer_faces"]

    def step():
        g.start_remote_neighbor_copy_updates()
        g.advection_step(f, dt, "inner")
        g.wait_remote_neighbor_copy_update_receives()
        g.advection_step(f, dt, "outer")
        g.wait_remote_neighbor_copy_update_sends()
        g.advection_commit(f[0])

    for _ in range(a.warmup):
        step()
    g.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    g.kernel_timing(1)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    g.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    kern_ms, kern_n = g.kernel_timing(0)

    # halo break-out (N > 1): the same exchange alone, K times back to back
    # (pack + grouped RCCL send/recv of the density into the halo slots)
    halo_el = 0.0
    if world > 1:
        g.synchronize()
        dist.barrier()
        th = time.perf_counter()
        for _ in range(a.steps):
            g.update_copies_of_remote_neighbors()
        g.synchronize()
        dist.barrier()
        halo_el = time.perf_counter() - th
    n_send = g.get_number_of_update_send_cells()
    n_peers = len(g.get_peers())

    # device neighbor build (find_neighbors_of / _to for every
    # local cell, initialize_neighbors): the full neighbors_of / neighbors_to /
    # iterator CSR of the frozen mesh, built once here (the sweep itself
    # uses the face tables); output bytes = 8 B id + 12 B offset + 4 B slot per
    # neighbors_of entry, 8 B per neighbors_to entry, 4 B per iterator entry
    g.synchronize()
    tb = time.perf_counter()
    n_of = g.neighbor_entries("of")
    g.synchronize()
    build_s = time.perf_counter() - tb
    n_to = g.neighbor_entries("to")
    n_it = g.neighbor_entries("iterator")

    stats = torch.tensor([el, float(n_local), float(c["recv"]), kern_ms, halo_el, float(n_send)],
                         dtype=torch.float64, device="cuda")
    if world > 1:
        mx = stats.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = stats.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        el_max, total_cells = float(mx[0]), int(sm[1])
    else:
        el_max, total_cells = el, n_local

    # algorithmic bytes of one sweep, as SURVEY §8(d) fixes them: per cell
    # read density, vx, vy, vz, lx, ly, lz + write density = 64 B, plus the
    # face structure as a CSR (4 B per face-neighbor entry + 4 B row pointer);
    # the 64 B core alone is reported beside it
    alg_core = layout["alg_bytes_core"]
    alg_bytes_step = layout["alg_bytes"]
    kern_s = kern_ms / 1e3
    achieved = alg_bytes_step * a.steps / kern_s / 1e9 if kern_s > 0 else None
    launches_per_step = kern_n / a.steps if a.steps else 0

    # HBM bytes per step of the sweep kernels from the committed PMC passes
    # (FETCH_SIZE x 2 + WRITE_SIZE, summed over the regular-tile and the
    # general tile kernel, scripts/traffic.py); only valid for the same mesh,
    # so it is dropped for any other cell count
    traffic = None
    tf = os.path.join(ROOT, "profiles", "advection_traffic.json")
    if os.path.exists(tf):
        try:
            t = json.load(open(tf))
            if t.get("cells") == n_local and t.get("alg_bytes_per_step") == alg_bytes_step and world == 1:
                traffic = t.get("hbm_bytes_per_step")
        except (OSError, ValueError):
            traffic = None

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(a.cpu_seconds)

    if rank == 0:
        value = total_cells * a.steps / el_max
        line = {
            "metric": "cell-updates/s (node) for 3D advection w/ halo exchange; % of HBM roofline",
            "value": value,
            "unit": "cell-updates/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": el_max / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: reference initial condition (tests/advection/initialize.hpp), pre-refined mesh",
            "config": {
                "workload": "advection3d (BASELINE config 3): base 128x128x128 per GPU, max_ref_lvl 2, "
                            "face neighbors, periodic x,y, frozen mesh",
                "base": [a.base, a.base, a.base * world],
                "max_ref_lvl": a.max_ref_lvl,
                "cells_total": total_cells,
                "cells_rank0": n_local,
                "halo_cells_rank0": c["recv"],
                "partition": "block (level-0 z-slabs, children inherit)",
                "parallelism": f"domain decomposition x{world}",
                "setup_s": setup_s,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": PEAK_HBM_GBS,
                "unit": "GB/s",
                "frac": (achieved / PEAK_HBM_GBS) if achieved else None,
                "traffic": traffic,
                "kernel": "advection_regular_pp_kernel + advection_tiles_pp_kernel" if variant == 11
                          else f"advection_kernel variant {variant}",
                "layout": layout,
                "alg_bytes_per_step": alg_bytes_step,
                "alg_bytes_core_per_step": alg_core,
                "frac_core_64B": (alg_core * a.steps / kern_s / 1e9 / PEAK_HBM_GBS) if kern_s > 0 else None,
                "finer_faces": n_fine,
                "kernel_ms_per_step": kern_ms / a.steps if a.steps else None,
                "launches_per_step": launches_per_step,
            },
            "cpu_baseline": cpu,
            "neighbor_build": {
                "what": "neighbors_of + neighbors_to + iterator CSR of all local cells (device kernels)",
                "seconds": build_s, "cells_per_s": n_local / build_s if build_s > 0 else None,
                "entries_of": n_of, "entries_to": n_to,
                "output_GB_per_s": (24 * n_of + 8 * n_to + 4 * n_it) / build_s / 1e9 if build_s > 0 else None,
            },
        }
        if world > 1:
            # rank with the most halo traffic; xGMI: one link per peer pair,
            # ~153 GB/s per link and direction (BASELINE north star)
            halo_ms = float(mx[4]) / a.steps * 1e3
            send_bytes = float(mx[5]) * 8.0
            per_link = send_bytes / max(n_peers, 1) / (halo_ms / 1e3) / 1e9 if halo_ms > 0 else None
            line["halo"] = {
                "ms_per_exchange": halo_ms,
                "frac_of_step": halo_ms / line["ms_per_step"] if line["ms_per_step"] else None,
                "payload_bytes_per_cell": 8,
                "send_bytes_max_rank": send_bytes,
                "peers_rank0": n_peers,
                "xgmi": {"achieved": per_link, "peak": 153.0, "unit": "GB/s per link per direction",
                         "frac": per_link / 153.0 if per_link else None},
            }
        print(json.dumps(line), flush=True)
    g.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
