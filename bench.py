"""Benchmark: BASELINE.json metric - cell-updates/s (node) for 3-D advection
with halo exchange, and the % of HBM roofline of the advection sweep.

Default workload (BASELINE config 3, tests/advection): level-0 base 128 x
128 x (128 * N) with cubic cells of length 1/128, maximum refinement level 2
(512^3-equivalent per GPU), neighborhood length 0 (face neighbors), periodic
in x and y, non-periodic in z, the reference's initial condition (hump +
rotating velocity, tests/advection/initialize.hpp) and its pre-refinement
criterion (adapter.hpp check_for_adaptation, refine side).  The mesh is then
frozen; one step = halo update of the density (RCCL, N > 1) overlapped with
the inner-cell sweep, then the outer-cell sweep, fused flux + apply.  Weak
scaling: every GPU owns one 128^3-base slab (block partition of level-0 ids,
children inherit the owner).

Other lines (--workload): gol (config 2), gol_amr, poisson
(config 4), scalability (config 5: 1024 x 1024 x 128 per GPU, halo exchange
of 1-B and 4-B payloads, game of life on the 4-B state, one half-shift
repartition).

    python bench.py [--gpus N --steps K --warmup W]

With --gpus N > 1 and no WORLD_SIZE in the environment, this process is only
a launcher: it starts N rank processes of this script (RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set, one GPU each), touches
no GPU itself, relays their output (rank 0 prints the JSON line) and exits
non-zero if any rank fails - the reference's scalability harness launches its
own ranks per process count the same way (tests/scalability/run_tests.py:
27-30, 185-198).  Under an external launcher (torch.distributed.run) WORLD_SIZE
must equal --gpus.
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

NAMES = ("density", "vx", "vy", "vz", "lx", "ly", "lz")
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
XGMI_LINK_GBS = 153.0  # one xGMI link, one direction
CPU_SHARE = 16         # host cores of one GPU's share on the bench box


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--base", type=int, default=None,
                   help="level-0 cells per dimension per GPU (default 128; poisson 384)")
    p.add_argument("--max-ref-lvl", type=int, default=2)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--workload", choices=["advection", "advection_adapt", "gol", "gol_amr", "poisson",
                                          "scalability"],
                   default="advection",
                   help="advection = BASELINE metric (default); gol = config 2; gol_amr = SURVEY a14; "
                        "poisson = config 4; scalability = config 5; advection_adapt = SURVEY f1")
    return p.parse_args(argv)


# ---------------------------------------------------------------------------- rank launcher
def free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def rank_commands(n, argv, port, base_env=None, child=None):
    """(argv, env) of every rank process: this script with the same
    arguments, one GPU per rank (LOCAL_RANK = RANK on one node)."""
    base = dict(os.environ if base_env is None else base_env)
    cmd = list(child) if child is not None else [sys.executable, "-u", os.path.abspath(__file__)]
    out = []
    for r in range(n):
        env = dict(base)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        out.append((cmd + list(argv), env))
    return out


def launch(n, argv, child=None, poll_s=0.2):
    """Start n ranks, wait for all of them; when one fails the others are
    stopped (they would wait forever in a collective).  Returns the exit code:
    0 when every rank exited 0, else the first failing rank's code (1 if that
    was a signal).  Ranks inherit stdout / stderr, so rank 0's JSON line is
    this process's output."""
    procs = [subprocess.Popen(c, env=e, cwd=ROOT) for c, e in rank_commands(n, argv, free_port(), child=child)]
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0] if bad[0] > 0 else 1
                sys.stderr.write(f"bench launcher: a rank exited with {bad[0]}; stopping the others\n")
                break
            if all(c == 0 for c in codes):
                return 0
            time.sleep(poll_s)
    except KeyboardInterrupt:
        rc = 130
    for p in procs:
        if p.poll() is None:
            p.terminate()
    for p in procs:
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    return rc


def world_check(a, env=None):
    """None: run as a rank (or alone); 'launch': spawn --gpus ranks; else an
    error message (WORLD_SIZE set by a launcher and different from --gpus)."""
    env = os.environ if env is None else env
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return "launch" if a.gpus > 1 else None
    if int(ws) != a.gpus:
        return f"WORLD_SIZE={ws} from the launcher but --gpus {a.gpus}: pass --gpus {ws}"
    return None


# ---------------------------------------------------------------------------- CPU baseline
def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(workload, seconds):
    """The oracle (CPU restatement of the reference's loop, AoS + hashed
    lookups) timed on the host: one process per core of this GPU's share
    (the reference's one MPI rank per core), each on its own copy of a
    bounded sample of the workload (oracle/cpu_bench.py); value = the sum of
    their cell-updates/s."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    cores = max(1, min(avail, CPU_SHARE))
    cmd = [sys.executable, "-m", "oracle.cpu_bench", "--workload", workload, "--seconds", str(seconds)]
    procs = [subprocess.Popen(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for _ in range(cores)]
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=seconds * 10 + 120)
        if p.returncode != 0:
            raise RuntimeError(f"cpu baseline worker failed: {e[-500:]}")
        outs.append(json.loads(o.strip().splitlines()[-1]))
    total = sum(r["cells"] * r["steps"] / r["seconds"] for r in outs)
    per_core = [r["cells"] * r["steps"] / r["seconds"] for r in outs]
    nproc = os.cpu_count() or cores
    return dict(value=total, unit="cell-updates/s", cores=cores, kind="port",
                sample=f"oracle restatement ({outs[0]['sample']}, {outs[0]['cells']} cells) x {cores} processes, "
                       f"~{seconds:.0f} s each; per core {min(per_core):.3g}-{max(per_core):.3g} cell-updates/s",
                cores_note=f"measured on {cores} cores, running at once: this GPU's share of the host (the GPU box "
                           f"allots {CPU_SHARE} cores per GPU and caps worker pools there; {nproc} are visible); "
                           "each process is one MPI rank of the reference's layout on its own subdomain",
                per_core_mean=total / cores, nproc=nproc, affinity=avail, cpu_model=cpu_model())


def measured_traffic(workload, cells, alg_bytes, world):
    """HBM bytes per step of the workload's kernels from the committed PMC
    passes (profiles/<workload>_traffic.json: FETCH_SIZE x 2 + WRITE_SIZE,
    scripts/traffic.py); only valid for the same mesh and byte accounting,
    so it is dropped for any other cell count."""
    tf = os.path.join(ROOT, "profiles", f"{workload}_traffic.json")
    if world != 1 or not os.path.exists(tf):
        return None
    try:
        t = json.load(open(tf))
    except (OSError, ValueError):
        return None
    if t.get("cells") == cells and abs(t.get("alg_bytes_per_step", -1) - alg_bytes) <= 1e-6 * alg_bytes:
        return t.get("hbm_bytes_per_step")
    return None


def alive_rule(ids):
    z = (ids ^ np.uint64(0x5DEECE66D)) + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    z = z ^ (z >> np.uint64(31))
    return (z < np.uint64(int(0.2 * 2 ** 64))).astype(np.uint32)


def line_base(metric, value, world, a, ms, dtype, data, config, scaling="weak", g=None):
    line = {"metric": metric, "value": value, "unit": "cell-updates/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": scaling, "vs_baseline": None,
            "dtype": dtype, "data": data, "config": config}
    if g is not None:
        kind, ranks = g.transport()
        line["transport"] = {"kind": kind, "comm_ranks": ranks}
    return line


# Rehearsal of the N > 1 path on one GPU (DCCRG_BENCH_TRANSPORT=host): every
# rank on cuda:0, a gloo group, and the library's host exchange instead of
# RCCL (which needs one GPU per rank).  Same timing, reductions and JSON; the
# numbers measure the host transport, not xGMI.
HOST_TRANSPORT = "host"


def make_grid(mod, rank, world, uid):
    if uid == HOST_TRANSPORT:
        g = mod.Dccrg(rank, world, 0, exchange=mod.grid.TorchExchange())
    else:
        g = mod.Dccrg(rank, world, int(os.environ.get("LOCAL_RANK", rank)), uid)
    if world > 1:
        kind, ranks = g.transport()
        if ranks != world:  # the library's communicator must span every rank
            raise RuntimeError(f"rank {rank}: the grid's {kind} communicator has {ranks} ranks, expected {world}")
    return g


def reduce_stats(torch, dist, world, vals):
    """(max over ranks, sum over ranks) of a list of floats."""
    dev = "cpu" if world > 1 and dist.get_backend() == "gloo" else "cuda"
    t = torch.tensor(vals, dtype=torch.float64, device=dev)
    if world == 1:
        return [float(x) for x in t], [float(x) for x in t]
    mx, sm = t.clone(), t.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    dist.all_reduce(sm, op=dist.ReduceOp.SUM)
    return [float(x) for x in mx], [float(x) for x in sm]


def timed(g, torch, dist, world, fn, steps):
    g.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    g.kernel_timing(1)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    g.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    kms, kn = g.kernel_timing(0)
    return el, kms, kn


# ---------------------------------------------------------------------------- game of life (config 2)
def gol_main(a, dccrgx_mod, torch, dist, rank, world, uid):
    """BASELINE config 2: game of life 1024 x 1024 x 64 (x N, z slabs),
    26-point stencil, uint32 state (algorithmic 8 B per cell-update)."""
    nx, ny, nz = 1024, 1024, 64 * world
    g = make_grid(dccrgx_mod, rank, world, uid)
    g.set_initial_length((nx, ny, nz)).set_neighborhood_length(1).set_maximum_refinement_level(0).initialize()
    st = g.add_field("is_alive", np.uint32)
    st.set(alive_rule(g.slot_ids()[: g.n_local]))

    def step():
        g.start_remote_neighbor_copy_updates()
        g.gol_step(st, "inner")
        g.wait_remote_neighbor_copy_update_receives()
        g.gol_step(st, "outer")
        g.wait_remote_neighbor_copy_update_sends()
        g.gol_commit(st)

    for _ in range(a.warmup):
        step()
    el, kms, kn = timed(g, torch, dist, world, step, a.steps)
    n = g.n_local
    mx, sm = reduce_stats(torch, dist, world, [el, float(n), kms])
    ach = 8.0 * n * a.steps / (kms / 1e3) / 1e9
    if rank == 0:
        line = line_base("cell-updates/s, game of life 3D (BASELINE config 2)", sm[1] * a.steps / mx[0], world, a,
                         mx[0] / a.steps * 1e3, "u32", "synthetic: seeded alive(id) rule, p=0.2",
                         {"workload": f"game of life {nx}x{ny}x{nz}, neighborhood 1, non-periodic (config 2"
                                      f"{', z slabs' if world > 1 else ''})", "cells_rank0": n}, g=g)
        line["roofline"] = {"bound": "hbm", "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                            "frac": ach / PEAK_HBM_GBS, "traffic": measured_traffic("gol", n, 8 * n, world),
                            "kernel": "gol_structured_yr<2, 2> (gol_structured_v3 with two rows per wave)",
                            "alg_bytes_per_step": 8 * n, "kernel_ms_per_step": kms / a.steps}
        line["cpu_baseline"] = None if (a.no_cpu_baseline or world > 1) else cpu_baseline("gol", a.cpu_seconds)
        print(json.dumps(line), flush=True)
    g.close()


# ---------------------------------------------------------------------------- refined game of life (a14)
def gol_amr_main(a, dccrgx_mod, torch, dist, rank, world, uid):
    """the refined game emulating the level-0 game
    (tests/game_of_life/solve.hpp get_live_neighbors, as unrefined2d.cpp
    plays it) on a 2048 x 2048 x 1 level-0 grid per GPU, max refinement level
    1, a seeded quarter of the level-0 cells refined (children inherit the
    state), p = 0.3 live.

    One process: one step = collect + spread over every leaf, which on one
    process is the level-0 game (gol_amr.hip): the roofline bytes are the
    ones its two passes move (below).  N > 1: one partitioned grid of
    2048 x 2048 N (the block partition: a 2048 x 2048 slab per rank, each
    rank refining a seeded quarter of its own cells), and one step is the
    reference's turn across processes (unrefined2d.cpp:186-218): the copies
    of remote neighbors refreshed, then get_live_neighbors (geometric collect,
    its own halo of the collected lists, spread + rule); the roofline bytes
    are SURVEY §8(d)'s CSR/AMR figure."""
    n = 2048
    if world > 1:
        return gol_amr_partitioned(a, dccrgx_mod, torch, dist, rank, world, uid, n)
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
    st.set(live0[level0_index(slots, n, n)].astype(np.uint32))
    for _ in range(a.warmup):
        g.get_live_neighbors(st, ls)
    el, kms, kn = timed(g, torch, dist, world, lambda: g.get_live_neighbors(st, ls), a.steps)
    nl = g.n_local
    total = nl
    kbar = g.neighbor_entries("of") / nl
    # roofline: the bytes the turn's kernels must move over the turn's kernel
    # time, so `achieved` / `frac` are a share of HBM bandwidth.  The grid is
    # one process, so the turn is the level-0 game (gol_amr.hip lg_table_kernel
    # + lg_game_kernel, one row per level-0 cell): per leaf its state read by
    # the table pass and read + written by the game pass (12 B), per level-0
    # cell the row's slot, octant byte and packed level-0 coordinates read by
    # both passes (2 x 9 B) and its table byte written once and read once
    # (2 B).  SURVEY §8(d)'s fixed CSR/AMR figure (8 B + 4 B per neighbor entry
    # + 4 B row pointer) counts neighbor-entry reads this path does not make;
    # it is reported beside it as model_throughput_GBs / frac_model, a
    # throughput figure, not bandwidth.
    per_cell = 8 + 4 * kbar + 4
    moved_step = 12 * nl + 20 * n * n
    kern = "lg_table_kernel + lg_game_kernel"
    moved_model = "level-0 game: 12 B per leaf (state) + 20 B per level-0 cell (row, octant, coordinates, table)"
    moved = moved_step / nl
    ach = moved_step * a.steps / (kms / 1e3) / 1e9 if kms > 0 else None
    model = per_cell * nl * a.steps / (kms / 1e3) / 1e9 if kms > 0 else None
    line = line_base("cell-updates/s, refined game of life emulating the level-0 game (SURVEY a14)",
                     total * a.steps / el, world, a, el / a.steps * 1e3, "u32",
                     "synthetic: seeded level-0 states (p=0.3), a seeded quarter of the cells refined",
                     {"workload": "get_live_neighbors, 2048x2048x1 level-0, max_ref_lvl 1, neighborhood 1",
                      "cells_rank0": nl, "neighbor_entries_per_leaf": kbar, "setup_s": setup_s}, g=g)
    line["roofline"] = {"bound": "hbm", "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                        "frac": ach / PEAK_HBM_GBS if ach else None,
                        "traffic": measured_traffic("gol_amr", nl, moved_step, 1),
                        "kernel": kern,
                        "alg_bytes_per_leaf": moved, "alg_bytes_per_step": moved_step,
                        "alg_bytes_model": moved_model,
                        "model_bytes_per_leaf": per_cell, "model": "SURVEY 8(d) GoL CSR/AMR: 8 + 4 k + 4",
                        "model_throughput_GBs": model, "frac_model": model / PEAK_HBM_GBS if model else None,
                        "kernel_ms_per_step": kms / a.steps, "launches_per_step": kn / a.steps}
    line["cpu_baseline"] = None if a.no_cpu_baseline else cpu_baseline("gol_amr", a.cpu_seconds)
    print(json.dumps(line), flush=True)
    g.close()


def level0_index(ids, nx, ny):
    """0-based level-0 parent index (raster) of level-0 / level-1 leaves of
    an nx x ny x 1 grid with max refinement level 1."""
    ids = ids.astype(np.int64)
    n0 = nx * ny
    lvl = ids > n0
    c1 = ids - 1 - n0
    x1, y1 = c1 % (2 * nx), (c1 // (2 * nx)) % (2 * ny)
    return np.where(lvl, (y1 // 2) * nx + x1 // 2, ids - 1)


def gol_amr_partitioned(a, dccrgx_mod, torch, dist, rank, world, uid, n):
    """The refined game at N > 1 on one partitioned grid (gol_amr_main)."""
    nx, ny = n, n * world
    g = make_grid(dccrgx_mod, rank, world, uid)
    g.set_initial_length((nx, ny, 1)).set_neighborhood_length(1).set_maximum_refinement_level(1).initialize()
    live0 = np.random.default_rng(7).random(nx * ny) < 0.3
    t_setup = time.perf_counter()
    loc = g.local_cells()
    for c in np.random.default_rng(7 + rank).choice(loc, size=loc.size // 4, replace=False):
        g.refine_completely(int(c))
    g.stop_refining()
    setup_s = time.perf_counter() - t_setup
    st = g.add_field("is_alive", np.uint32)
    ls = g.add_field("gol_list", np.dtype((np.uint64, 8)))
    slots = g.slot_ids()[: g.n_local]
    st.set(live0[level0_index(slots, nx, ny)].astype(np.uint32))

    def step():
        # unrefined2d.cpp:186-218: the copies of remote neighbors refreshed,
        # then the turn (its own halo of the collected lists inside)
        g.update_copies_of_remote_neighbors()
        g.get_live_neighbors(st, ls)

    for _ in range(a.warmup):
        step()
    el, kms, kn = timed(g, torch, dist, world, step, a.steps)
    nl = g.n_local
    kbar = g.neighbor_entries("of") / nl
    per_cell = 8 + 4 * kbar + 4
    mx, sm = reduce_stats(torch, dist, world, [el, float(nl), kms, float(g.get_number_of_update_send_cells())])
    if rank == 0:
        line = line_base("cell-updates/s, refined game of life emulating the level-0 game (SURVEY a14)",
                         sm[1] * a.steps / mx[0], world, a, mx[0] / a.steps * 1e3, "u32",
                         "synthetic: seeded level-0 states (p=0.3), a seeded quarter of every rank's cells refined",
                         {"workload": f"get_live_neighbors, {nx}x{ny}x1 level-0 (block partition, a {nx}x{n} slab "
                                      "per rank), max_ref_lvl 1, neighborhood 1; step = state halo + turn",
                          "cells_rank0": nl, "cells_total": int(sm[1]), "neighbor_entries_per_leaf": kbar,
                          "setup_s": setup_s, "parallelism": f"domain decomposition x{world}"}, g=g)
        ach = per_cell * nl * a.steps / (mx[2] / 1e3) / 1e9 if mx[2] > 0 else None
        line["roofline"] = {"bound": "hbm", "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                            "frac": ach / PEAK_HBM_GBS if ach else None, "traffic": None,
                            "kernel": "gol_amr geometric collect + spread (+ exact collect when a family disagrees)",
                            "alg_bytes_per_leaf": per_cell, "model": "SURVEY 8(d) GoL CSR/AMR: 8 + 4 k + 4",
                            "kernel_ms_per_step_max_rank": mx[2] / a.steps, "launches_per_step": kn / a.steps}
        line["halo"] = {"send_cells_max_rank": mx[3]}
        line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    g.close()


# ---------------------------------------------------------------------------- Poisson (config 4)
def poisson_main(a, dccrgx_mod, torch, dist, rank, world, uid):
    """BASELINE config 4: Poisson BiCG (tests/poisson/poisson3d.cpp) on a
    384^3-base grid per GPU (cell lengths 2pi/n, pi/n, 8pi/n), periodic,
    refined twice around (pi, pi/2, 4pi); one step = one BiCG iteration over
    every solve cell (min = max = steps iterations, as SURVEY §8(d)).  The
    timed kernels of an iteration run from its first phase to its last, the
    two global reductions included.  At 384^3 (56.6 M cells) every solver
    vector is 453 MB, so no phase finds its operands in the 256 MiB Infinity
    Cache beyond what the previous phase just wrote."""
    import math

    n = a.base
    L0 = (2 * math.pi / n, math.pi / n, 8 * math.pi / n)
    g = make_grid(dccrgx_mod, rank, world, uid)
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
    res = {}
    el, kms, kn = timed(g, torch, dist, world, lambda: res.update(r=solver.solve(ids, g, cache_is_up_to_date=True)), 1)
    it, resid = res["r"]
    n_solve = ids.size
    mx, sm = reduce_stats(torch, dist, world, [el, float(n_solve), kms])
    # SURVEY §8(d) 3-phase minimum (34 fp64 accesses) + the 24-B face table read by
    # phases A and B; split per kernel in scripts/roofline_summary.py (A 112, B 160, C 48)
    per_cell = 272 + 48
    ach = per_cell * n_solve * it / (kms / 1e3) / 1e9 if kms > 0 else None
    if rank == 0:
        line = line_base("cell-updates/s, Poisson BiCG iterations (BASELINE config 4)", sm[1] * it / mx[0], world, a,
                         mx[0] / it * 1e3, "f64", "synthetic: poisson3d.cpp rhs on its center-refined mesh",
                         {"workload": f"poisson3d BiCG, base {n}x{n}x{n * world}, periodic, refined twice at the "
                                      f"center, min = max = {a.steps} iterations",
                          "cells_rank0": n_solve, "setup_s": setup_s,
                          "parallelism": f"domain decomposition x{world}"}, g=g)
        line["steps"] = it
        line["roofline"] = {"bound": "hbm", "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                            "frac": ach / PEAK_HBM_GBS if ach else None,
                            "traffic": measured_traffic("poisson", n_solve, per_cell * n_solve, world),
                            "alg_bytes_per_step": per_cell * n_solve,
                            "kernel": "po_phase_a + po_reduce + po_phase_b + po_reduce + po_phase_c",
                            "alg_bytes_per_cell_iteration": per_cell, "kernel_ms_per_step": kms / it,
                            "timed_intervals_per_step": kn / it, "residual_min": resid}
        line["cpu_baseline"] = None if (a.no_cpu_baseline or world > 1) else cpu_baseline("poisson", a.cpu_seconds)
        print(json.dumps(line), flush=True)
    g.close()


# ---------------------------------------------------------------------------- scalability (config 5)
def scalability_main(a, dccrgx_mod, torch, dist, rank, world, uid):
    """BASELINE config 5 (tests/scalability/scalability.cpp): a uniform
    1024 x 1024 x (128 N) grid, neighborhood 1, block partition (z slabs,
    134 M cells per GPU).  One step = the reference's loop with its 'solve'
    being the game of life on the 4-B payload: start the halo update, sweep
    the inner cells, wait, sweep the outer cells.  Reported beside it: the
    halo exchange alone for 1-B and 4-B payloads (the reference's data_size)
    and one repartition from the block partition to the block partition
    shifted by half a rank (every rank exports its first half to the
    previous rank; at N = 1 nothing moves and the time is the rebuild)."""
    nx, ny, nzr = 1024, 1024, 128
    g = make_grid(dccrgx_mod, rank, world, uid)
    g.set_initial_length((nx, ny, nzr * world)).set_neighborhood_length(1).set_maximum_refinement_level(0)
    g.initialize()
    st = g.add_field("is_alive", np.uint32)
    b1 = g.add_field("data_1B", np.uint8, False)
    st.set(alive_rule(g.slot_ids()[: g.n_local]))

    def step():
        g.start_remote_neighbor_copy_updates()
        g.gol_step(st, "inner")
        g.wait_remote_neighbor_copy_update_receives()
        g.gol_step(st, "outer")
        g.wait_remote_neighbor_copy_update_sends()
        g.gol_commit(st)

    for _ in range(a.warmup):
        step()
    el, kms, kn = timed(g, torch, dist, world, step, a.steps)
    n = g.n_local

    def halo_time(fields_on):
        for f in (st, b1):
            f.set_transfer(f in fields_on)
        e, _, _ = timed(g, torch, dist, world, g.update_copies_of_remote_neighbors, a.steps)
        return e / a.steps

    h4 = halo_time([st])
    h1 = halo_time([b1])
    st.set_transfer(True)
    b1.set_transfer(False)
    n_send = g.get_number_of_update_send_cells()
    peers = len(g.get_peers())
    # one repartition: the first half of every rank's cells to the previous rank
    loc = g.local_cells()
    half = loc[: loc.size // 2]
    dest = np.full(half.size, (rank - 1) % world, np.int32)
    g.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    g.balance_load_to(half, dest)
    g.synchronize()
    if world > 1:
        dist.barrier()
    rep = time.perf_counter() - t0
    moved = int(half.size) if world > 1 else 0
    mx, sm = reduce_stats(torch, dist, world, [el, float(n), kms, h4, h1, rep, float(n_send), float(moved)])
    if rank == 0:
        line = line_base("cell-updates/s, scalability (BASELINE config 5): game of life + halo on 134M cells/GPU",
                         sm[1] * a.steps / mx[0], world, a, mx[0] / a.steps * 1e3, "u32",
                         "synthetic: seeded alive(id) rule, p=0.2",
                         {"workload": f"tests/scalability 1024x1024x{nzr * world} uniform, neighborhood 1, "
                                      "block partition (z slabs), game of life on the 4-B payload",
                          "cells_total": int(sm[1]), "cells_rank0": int(n),
                          "parallelism": f"domain decomposition x{world}"}, g=g)
        ach = 8.0 * n * a.steps / (kms / 1e3) / 1e9 if kms > 0 else None
        line["roofline"] = {"bound": "hbm", "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                            "frac": ach / PEAK_HBM_GBS if ach else None,
                            "traffic": measured_traffic("scalability", n, 8 * n, world),
                            "kernel": "gol_structured_yr<2, 2> (plane boxes)", "alg_bytes_per_step": 8 * n,
                            "kernel_ms_per_step": kms / a.steps}
        halo = {"ms_per_exchange_4B": mx[3] * 1e3, "ms_per_exchange_1B": mx[4] * 1e3,
                "send_cells_max_rank": mx[6], "peers_rank0": peers}
        if world > 1 and mx[3] > 0:
            per_link = mx[6] * 4 / max(peers, 1) / mx[3] / 1e9
            halo["xgmi_4B"] = {"achieved": per_link, "peak": XGMI_LINK_GBS, "unit": "GB/s per link per direction",
                               "frac": per_link / XGMI_LINK_GBS}
        line["halo"] = halo
        line["repartition"] = {"seconds": mx[5], "cells_moved_total": sm[7],
                               "what": "balance_load_to: first half of every rank's cells to the previous rank "
                                       "(payload migration + distributed ghost refresh + full rebuild)"}
        line["cpu_baseline"] = None if (a.no_cpu_baseline or world > 1) else cpu_baseline("scalability",
                                                                                          a.cpu_seconds)
        print(json.dumps(line), flush=True)
    g.close()


# ---------------------------------------------------------------------------- adaptive advection
def advection_adapt_main(a, dccrg_amd, torch, dist, rank, world, uid):
    """tests/advection/2d.cpp with its defaults adapt_n = 1 and balance_n = 25
    on BASELINE config 3's grid: every step = halo + inner / outer sweep,
    check_for_adaptation on the pre-step densities, apply, adapt_grid
    (refines, unrefines, merged parents' mean density, velocity / length
    reset, all-field halo), a new dt; every 25th step a balance_load (the
    native RCB) with an all-field halo.  value = cell-updates (local cells
    summed over steps and ranks) / wall time; the sweep kernels' roofline on
    the 64-B core bytes is reported beside it."""
    t_setup = time.perf_counter()
    g, f = build_grid(dccrg_amd, rank, world, a.base, a.max_ref_lvl, uid)
    setup_s = time.perf_counter() - t_setup
    R = a.max_ref_lvl
    cells0 = g.n_local

    def step(state):
        dt = 0.5 * g.advection_max_time_step(f)
        if world > 1:
            dt = g.allreduce(dt, "min")
        state["cells"] += g.n_local
        g.start_remote_neighbor_copy_updates()
        g.advection_step(f, dt, "inner")
        g.wait_remote_neighbor_copy_update_receives()
        g.advection_step(f, dt, "outer")
        g.wait_remote_neighbor_copy_update_sends()
        t0 = time.perf_counter()
        g.advection_check_adaptation(f[0], 0.025 / R, 0.25, 0.5)
        t1 = time.perf_counter()
        g.advection_commit(f[0])
        c, r = g.advection_adapt(f)
        g.synchronize()
        t2 = time.perf_counter()
        state["t_check"] += t1 - t0
        state["t_adapt"] += t2 - t1
        state["created"] += c
        state["removed"] += r
        state["step"] += 1
        if state["step"] % 25 == 0 and world > 1:
            g.balance_load()
            for ff in f:
                ff.set_transfer(True)
            g.update_copies_of_remote_neighbors()
            for ff in f[1:]:
                ff.set_transfer(False)

    st = {"cells": 0, "created": 0, "removed": 0, "step": 0, "t_check": 0.0, "t_adapt": 0.0}
    for _ in range(a.warmup):
        step(st)
    reset = getattr(dccrg_amd.lib(), "dccrgx_phase_reset", None)  # phase-timing analysis builds only
    if reset is not None:
        reset()
    st.update(cells=0, created=0, removed=0, t_check=0.0, t_adapt=0.0)
    el, kms, kn = timed(g, torch, dist, world, lambda: step(st), a.steps)
    mx, sm = reduce_stats(torch, dist, world, [el, float(st["cells"]), kms, float(st["created"]),
                                               float(st["removed"]), float(g.n_local)])
    if rank == 0:
        line = line_base("cell-updates/s, 3D advection with grid adaptation every step (SURVEY f1)",
                         sm[1] / mx[0], world, a, mx[0] / a.steps * 1e3, "f64",
                         "synthetic: reference initial condition (tests/advection/initialize.hpp), adapt_n = 1",
                         {"workload": "advection3d, base 128x128x128 per GPU, max_ref_lvl 2, face neighbors, "
                                      "adapt every step (check_for_adaptation + adapt_grid), balance every 25",
                          "cells_rank0_first": cells0, "cells_rank0_last": g.n_local, "setup_s": setup_s,
                          "parallelism": f"domain decomposition x{world}"}, g=g)
        ach = 64.0 * sm[1] / world / (kms / 1e3) / 1e9 if kms > 0 else None
        line["roofline"] = {"bound": "hbm", "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                            "frac": ach / PEAK_HBM_GBS if ach else None, "traffic": None,
                            "kernel": "advection sweeps (64-B core bytes per cell-update)",
                            "kernel_ms_per_step": kms / a.steps, "sweep_share_of_step": kms / (mx[0] * 1e3)}
        line["adaptation"] = {"created_total": sm[3], "removed_total": sm[4],
                              "ms_check_per_step_rank0": st["t_check"] / a.steps * 1e3,
                              "ms_adapt_per_step_rank0": st["t_adapt"] / a.steps * 1e3}
        line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    g.close()


# ---------------------------------------------------------------------------- advection (config 3, headline)
def build_grid(dccrg_amd, rank, size, base, R, uid):
    nx, ny, nz = base, base, base * size
    g = make_grid(dccrg_amd, rank, size, uid)
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


def advection_main(a, dccrg_amd, torch, dist, rank, world, uid):
    t_setup = time.perf_counter()
    g, f = build_grid(dccrg_amd, rank, world, a.base, a.max_ref_lvl, uid)
    setup_s = time.perf_counter() - t_setup
    dt = 0.5 * g.advection_max_time_step(f)  # cfl 0.5 (2d.cpp:121-123)
    c = g.counts
    n_local = c["inner"] + c["outer"]
    layout = g.advection_layout()

    def step():
        g.start_remote_neighbor_copy_updates()
        g.advection_step(f, dt, "inner")
        g.wait_remote_neighbor_copy_update_receives()
        g.advection_step(f, dt, "outer")
        g.wait_remote_neighbor_copy_update_sends()
        g.advection_commit(f[0])

    for _ in range(a.warmup):
        step()
    el, kern_ms, kern_n = timed(g, torch, dist, world, step, a.steps)

    # halo break-out (N > 1): the same exchange alone, K times back to back
    # (pack + grouped RCCL send/recv of the density into the halo slots)
    halo_el = 0.0
    if world > 1:
        halo_el, _, _ = timed(g, torch, dist, world, g.update_copies_of_remote_neighbors, a.steps)
    n_send = g.get_number_of_update_send_cells()
    n_peers = len(g.get_peers())

    # device neighbor build (find_neighbors_of / _to for every
    # local cell, initialize_neighbors): the full neighbors_of / neighbors_to /
    # iterator CSR of the frozen mesh, built once here (the sweep itself uses
    # the face tables); output bytes = 8 B id + 12 B offset + 4 B slot per
    # neighbors_of entry, 8 B per neighbors_to entry, 4 B per iterator entry
    g.synchronize()
    tb = time.perf_counter()
    n_of = g.neighbor_entries("of")
    g.synchronize()
    build_s = time.perf_counter() - tb
    n_to = g.neighbor_entries("to")
    n_it = g.neighbor_entries("iterator")

    mx, sm = reduce_stats(torch, dist, world, [el, float(n_local), float(c["recv"]), kern_ms, halo_el, float(n_send)])
    el_max, total_cells = mx[0], int(sm[1])

    # algorithmic bytes of one sweep, as SURVEY §8(d) fixes them: per cell
    # read density, vx, vy, vz, lx, ly, lz + write density = 64 B, plus the
    # face structure as a CSR (4 B per face-neighbor entry + 4 B row pointer);
    # the 64 B core alone is reported beside it
    alg_core = layout["alg_bytes_core"]
    alg_bytes_step = layout["alg_bytes"]
    kern_s = kern_ms / 1e3
    achieved = alg_bytes_step * a.steps / kern_s / 1e9 if kern_s > 0 else None

    traffic = measured_traffic("advection", n_local, alg_bytes_step, world)

    if rank == 0:
        line = line_base("cell-updates/s (node) for 3D advection w/ halo exchange; % of HBM roofline",
                         total_cells * a.steps / el_max, world, a, el_max / a.steps * 1e3, "f64",
                         "synthetic: reference initial condition (tests/advection/initialize.hpp), pre-refined mesh",
                         {"workload": "advection3d (BASELINE config 3): base 128x128x128 per GPU, max_ref_lvl 2, "
                                      "face neighbors, periodic x,y, frozen mesh",
                          "base": [a.base, a.base, a.base * world], "max_ref_lvl": a.max_ref_lvl,
                          "cells_total": total_cells, "cells_rank0": n_local, "halo_cells_rank0": c["recv"],
                          "partition": "block (level-0 z-slabs, children inherit)",
                          "parallelism": f"domain decomposition x{world}", "setup_s": setup_s}, g=g)
        line["roofline"] = {
            "bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": (achieved / PEAK_HBM_GBS) if achieved else None, "traffic": traffic,
            "kernel": "advection_regular_pp_kernel + advection_tiles_pp_kernel", "layout": layout,
            "alg_bytes_per_step": alg_bytes_step, "alg_bytes_core_per_step": alg_core,
            "frac_core_64B": (alg_core * a.steps / kern_s / 1e9 / PEAK_HBM_GBS) if kern_s > 0 else None,
            # the bytes the two kernels need, each value read once (layout
            # bytes_needed: core + face codes + per out-of-tile neighbor its
            # density and 24-B record + list entries + finer faces + tile
            # records), beside SURVEY's CSR-inclusive count
            "bytes_needed_per_step": layout["bytes_needed"],
            "frac_bytes_needed": (layout["bytes_needed"] * a.steps / kern_s / 1e9 / PEAK_HBM_GBS) if kern_s > 0
            else None,
            "kernel_ms_per_step": kern_ms / a.steps if a.steps else None,
            "timed_intervals_per_step": kern_n / a.steps if a.steps else 0}
        line["cpu_baseline"] = None if (a.no_cpu_baseline or world > 1) else cpu_baseline("advection", a.cpu_seconds)
        line["neighbor_build"] = {
            "what": "neighbors_of + neighbors_to + iterator CSR of all local cells (device kernels)",
            "seconds": build_s, "cells_per_s": n_local / build_s if build_s > 0 else None,
            "entries_of": n_of, "entries_to": n_to,
            "output_GB_per_s": (24 * n_of + 8 * n_to + 4 * n_it) / build_s / 1e9 if build_s > 0 else None}
        if world > 1:
            # rank with the most halo traffic; xGMI: one link per peer pair,
            # ~153 GB/s per link and direction
            halo_ms = mx[4] / a.steps * 1e3
            send_bytes = mx[5] * 8.0
            per_link = send_bytes / max(n_peers, 1) / (halo_ms / 1e3) / 1e9 if halo_ms > 0 else None
            line["halo"] = {
                "ms_per_exchange": halo_ms, "frac_of_step": halo_ms / line["ms_per_step"],
                "payload_bytes_per_cell": 8, "send_bytes_max_rank": send_bytes, "peers_rank0": n_peers,
                "xgmi": {"achieved": per_link, "peak": XGMI_LINK_GBS, "unit": "GB/s per link per direction",
                         "frac": per_link / XGMI_LINK_GBS if per_link else None}}
        print(json.dumps(line), flush=True)
    g.close()


def main():
    a = parse()
    wc = world_check(a)
    if wc == "launch":
        # before any torch / HIP call: this process never touches the GPU
        sys.exit(launch(a.gpus, sys.argv[1:]))
    if wc is not None:
        sys.stderr.write(f"bench.py: {wc}\n")
        sys.exit(2)
    if a.base is None:
        # Poisson at 256^3 per GPU: one phase's working set (~1.5 GB) is far
        # above the 256 MiB Infinity Cache, so its rate is an HBM rate
        a.base = 384 if a.workload == "poisson" else 128
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    host = world > 1 and os.environ.get("DCCRG_BENCH_TRANSPORT") == HOST_TRANSPORT
    torch.cuda.set_device(0 if host else local)
    if host:
        dist.init_process_group("gloo")
    elif world > 1:
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    import dccrg_amd

    uid = HOST_TRANSPORT if host else None
    if world > 1 and not host:
        obj = [dccrg_amd.Dccrg.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        uid = obj[0]
    fn = {"advection": advection_main, "advection_adapt": advection_adapt_main, "gol": gol_main,
          "gol_amr": gol_amr_main, "poisson": poisson_main,
          "scalability": scalability_main}[a.workload]
    fn(a, dccrg_amd, torch, dist, rank, world, uid)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
