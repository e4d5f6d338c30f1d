"""3-D advection (tests/advection/solve.hpp) on refined grids vs the oracle.

Tolerance (fp64): per cell |rho_gpu - rho_oracle| <= 1e-12 * max|rho_oracle|.
The flux through a face is evaluated with the reference's expression and
operand order on both sides (no contraction), so the only difference is the
order in which a cell's face fluxes are summed (gather here, hash-ordered
scatter in the reference)."""
import os

import numpy as np
import pytest

import dccrg_amd
from oracle import oracle as O

pytestmark = pytest.mark.gpu

NAMES = ("density", "vx", "vy", "vz", "lx", "ly", "lz")
TOL = 1e-12


def gpu_grid(base, R, periodic=(True, True, False)):
    g = dccrg_amd.Dccrg(0, 1, 0).set_initial_length(base).set_neighborhood_length(0)
    g.set_maximum_refinement_level(R).set_periodic(*periodic).initialize()
    g.set_geometry((0, 0, 0), tuple(1.0 / b for b in base))
    f = [g.add_field(n, np.float64, n == "density") for n in NAMES]
    return g, f


def prerefine(g, f, R, relative_diff=0.025, diff_threshold=0.25):
    """tests/advection/2d.cpp:260-285 (refine side of check_for_adaptation)."""
    for _ in range(R):
        g.advection_initialize(f)
        for c in g.advection_refine_candidates(f[0], relative_diff / R, diff_threshold):
            g.refine_completely(int(c))
        g.stop_refining()
    g.advection_initialize(f)


@pytest.mark.parametrize("base,R", [((16, 16, 2), 2), ((12, 12, 3), 2), ((20, 20, 1), 1)])
def test_prerefined_mesh_matches_oracle(gpu, base, R):
    g, f = gpu_grid(base, R)
    prerefine(g, f, R)
    o = O.Grid(base, R, (True, True, False), 0, 1)
    o.set_geometry((0, 0, 0), tuple(1.0 / b for b in base))
    o.adv_prerefine(0.025, 0.25)
    oi, _ = o.cells()
    assert np.array_equal(np.sort(g.local_cells()), oi)
    assert oi.size > np.prod(base)  # refinement happened
    g.close()


@pytest.mark.parametrize("base,R,steps", [((16, 16, 2), 2, 30), ((24, 24, 2), 2, 100), ((10, 10, 4), 1, 20)])
def test_steps_match_oracle(gpu, base, R, steps):
    g, f = gpu_grid(base, R)
    prerefine(g, f, R)
    ids = g.slot_ids()[: g.n_local]
    o = O.Grid(base, R, (True, True, False), 0, 1)
    o.set_geometry((0, 0, 0), tuple(1.0 / b for b in base))
    o.set_cells(ids, np.zeros(ids.size, np.int32))
    o.adv_initialize()
    # initial state is bitwise the reference's (host evaluation, same expressions)
    init = o.adv_get(ids)
    for k, (col) in enumerate((0, 1, 2, 3, 6, 7, 8)):
        assert np.array_equal(f[k].get(0, ids.size), init[:, col]), NAMES[k]
    dt = g.advection_max_time_step(f)
    assert dt == o.adv_max_time_step()
    for _ in range(steps):
        g.advection_step(f, 0.5 * dt)
        g.advection_commit(f[0])
    o.adv_steps(steps, 0.5 * dt)
    exp = o.adv_get(ids)[:, 0]
    got = f[0].get(0, ids.size)
    scale = np.max(np.abs(exp))
    assert np.max(np.abs(got - exp)) <= TOL * scale
    g.close()


def test_mass_conservation_large(gpu):
    """Full-size property: x,y periodic, z non-periodic with vz = 0, so the
    total mass sum(rho * volume) is conserved by every step to rounding."""
    base, R = (64, 64, 16), 2
    g, f = gpu_grid(base, R)
    prerefine(g, f, R)
    n = g.n_local
    vol = f[4].get(0, n) * f[5].get(0, n) * f[6].get(0, n)
    m0 = np.sum(f[0].get(0, n) * vol)
    dt = g.advection_max_time_step(f)
    for _ in range(50):
        g.advection_step(f, 0.5 * dt)
        g.advection_commit(f[0])
    m1 = np.sum(f[0].get(0, n) * vol)
    assert abs(m1 - m0) <= 1e-11 * abs(m0)
    g.close()


def test_inner_outer_split_equals_all(gpu):
    """Sweeping inner then outer regions gives bitwise the same result as
    one sweep over all local cells (single rank: outer is empty)."""
    g, f = gpu_grid((12, 12, 2), 2)
    prerefine(g, f, 2)
    dt = g.advection_max_time_step(f)
    g.advection_step(f, dt, "inner")
    g.advection_step(f, dt, "outer")
    g.advection_commit(f[0])
    a = f[0].get(0, g.n_local)
    g.close()
    g, f = gpu_grid((12, 12, 2), 2)
    prerefine(g, f, 2)
    g.advection_step(f, dt, "all")
    g.advection_commit(f[0])
    b = f[0].get(0, g.n_local)
    assert np.array_equal(a, b)
    g.close()


@pytest.mark.parametrize("base,R", [((32, 32, 8), 2), ((12, 12, 3), 2), ((10, 10, 4), 1)])
def test_face_table_sweep_bitwise_equals_tiles(gpu, base, R):
    """The first step on a freshly built mesh sweeps the fixed-width face
    table (advection_ell_kernel) instead of building tiles; the tiles come
    with the second step.  A grid whose tiles are built up front
    (advection_layout) gives bitwise the same densities at every step."""
    out = []
    for tiles_first in (True, False):
        g, f = gpu_grid(base, R)
        prerefine(g, f, R)
        if tiles_first:
            lay = g.advection_layout()
            assert lay["tiles"] > 0
        dt = g.advection_max_time_step(f)
        rho = []
        for _ in range(3):
            g.advection_step(f, 0.5 * dt)
            g.advection_commit(f[0])
            rho.append(f[0].get(0, g.n_local))
        out.append(rho)
        g.close()
    for a, b in zip(*out):
        assert np.array_equal(a, b)


def test_face_table_second_pass_same_table(gpu, monkeypatch):
    """The face table numbers its finer faces in (row, direction) order by a
    scan of per-wave counts (k_face_table's default); the sorted form
    (DCCRGX_FACE_KEYS=sort) gives the keys room for a quarter of the rows
    first and runs the pass again with room for all of them when that was too
    little: forced here with room for one key.  The densities of three table
    sweeps (which read the table, finer faces included) are bitwise the same
    for all three builds."""
    out = []
    for keys, cap in ((None, None), ("sort", None), ("sort", "1")):
        if keys is None:
            monkeypatch.delenv("DCCRGX_FACE_KEYS", raising=False)
        else:
            monkeypatch.setenv("DCCRGX_FACE_KEYS", keys)
        if cap is None:
            monkeypatch.delenv("DCCRGX_FACE_KEY_CAP", raising=False)
        else:
            monkeypatch.setenv("DCCRGX_FACE_KEY_CAP", cap)
        g, f = gpu_grid((16, 16, 8), 2)
        prerefine(g, f, 2)
        dt = g.advection_max_time_step(f)
        rho = []
        for _ in range(3):
            g.advection_step(f, 0.5 * dt)
            g.advection_commit(f[0])
            rho.append(f[0].get(0, g.n_local))
        out.append(rho)
        g.close()
    monkeypatch.delenv("DCCRGX_FACE_KEY_CAP", raising=False)
    monkeypatch.delenv("DCCRGX_FACE_KEYS", raising=False)
    for a, b, c in zip(*out):
        assert np.array_equal(a, b) and np.array_equal(a, c)


def _run_parity_grid(base=(32, 32, 8), R=2, steps=100):
    g, f = gpu_grid(base, R)
    prerefine(g, f, R)
    lay = g.advection_layout()
    dt = g.advection_max_time_step(f)
    ids = g.slot_ids()[: g.n_local]
    for _ in range(steps):
        g.advection_step(f, 0.5 * dt)
        g.advection_commit(f[0])
    return g, f, lay, dt, ids


def test_parity_grid_exercises_both_tile_kernels(gpu):
    """SURVEY §8(d)'s oracle parity grid (32 x 32 x 8 base, R = 2, periodic
    x and y, 100 steps): the layout must contain regular tiles (swept by
    advection_regular_pp_kernel without face rows) and general tiles
    (advection_tiles_pp_kernel), and every cell must match the oracle within
    1e-12 x max|rho| - so both kernels are checked against the oracle."""
    base, R, steps = (32, 32, 8), 2, 100
    g, f, lay, dt, ids = _run_parity_grid(base, R, steps)
    assert lay["regular_tiles"] > 0, lay
    assert lay["tiles"] > lay["regular_tiles"], lay
    assert lay["finer_faces"] > 0, lay
    o = O.Grid(base, R, (True, True, False), 0, 1)
    o.set_geometry((0, 0, 0), tuple(1.0 / b for b in base))
    o.adv_prerefine(0.025, 0.25)
    oi, _ = o.cells()
    assert np.array_equal(np.sort(ids), oi)
    assert dt == o.adv_max_time_step()
    o.adv_initialize()
    o.adv_steps(steps, 0.5 * dt)
    exp = o.adv_get(ids)[:, 0]
    got = f[0].get(0, ids.size)
    scale = np.max(np.abs(exp))
    assert np.max(np.abs(got - exp)) <= TOL * scale
    # the cells the regular kernel swept are among those checked: a regular
    # tile is 512 consecutive slots of one level-R box
    assert lay["regular_cells"] == 512 * lay["regular_tiles"] and lay["regular_cells"] < ids.size
    g.close()


def test_tile_build_paths_bitwise(gpu, monkeypatch):
    """The tile ext lists are built per tile in LDS (tile_build.hip
    tile_ext_kernel) unless a tile has more distinct out-of-tile neighbors
    than its LDS holds; then by one global sort (the fallback).  Forced to the
    fallback (DCCRGX_TILE_GLOBAL=1), the parity grid must give the same layout
    and the same densities bit for bit after 20 steps."""
    base, R, steps = (32, 32, 8), 2, 20
    g1, f1, lay1, _, ids1 = _run_parity_grid(base, R, steps)
    rho1 = f1[0].get(0, ids1.size)
    g1.close()
    monkeypatch.setenv("DCCRGX_TILE_GLOBAL", "1")
    g2, f2, lay2, _, ids2 = _run_parity_grid(base, R, steps)
    rho2 = f2[0].get(0, ids2.size)
    g2.close()
    assert np.array_equal(ids1, ids2)
    for k in ("tiles", "ext_total", "ext_max", "finer_faces", "regular_tiles"):
        assert lay1[k] == lay2[k], k
    assert np.array_equal(rho1, rho2)


def test_parity_grid_four_rank_slabs_bitwise(gpu):
    """The parity grid, 16 level-0 cells deep, split into 4 z-slabs (block
    partition of the level-0 cells, children inherit, execute_refines
    10228-10237) on detached views, the density halo moved by the library's
    pack / place: every cell bitwise equals the one-rank run after 30 steps;
    the ranks' inner runs contain regular tiles."""
    from test_gpu_multirank import emulated_exchange

    base, R, P, steps = (32, 32, 16), 2, 4, 30
    ref, rf, lay, dt, ids = _run_parity_grid(base, R, 0)
    leaves = np.sort(ids)
    n0 = int(np.prod(base))
    plane = base[0] * base[1]
    l0p = np.array([ref.get_cell_from_indices(ref.get_indices(int(c)), 0) for c in leaves], np.int64)
    owners = ((l0p - 1) // plane // (base[2] // P)).astype(np.int32)
    assert np.array_equal(owners, ((l0p - 1) * P // n0).astype(np.int32))
    gs, n_regular = [], 0
    for r in range(P):
        g = dccrg_amd.Dccrg(r, P, 0).set_initial_length(base).set_neighborhood_length(0)
        g.set_maximum_refinement_level(R).set_periodic(True, True, False).initialize()
        g.set_geometry((0, 0, 0), tuple(1.0 / b for b in base))
        for n in NAMES:
            g.add_field(n, np.float64, n == "density")
        g.set_cells(leaves, owners)
        g.advection_initialize([g.fields[n] for n in NAMES])
        n_regular += g.advection_layout()["regular_tiles"]
        gs.append(g)
    assert n_regular > 0
    for _ in range(steps):
        emulated_exchange(gs, ["density"])
        for g in gs:
            f = [g.fields[n] for n in NAMES]
            g.advection_step(f, 0.5 * dt, "inner")
            g.advection_step(f, 0.5 * dt, "outer")
            g.advection_commit(f[0])
        ref.advection_step(rf, 0.5 * dt)
        ref.advection_commit(rf[0])
    final = dict(zip(ref.slot_ids()[: ref.n_local].tolist(), rf[0].get(0, ref.n_local).tolist()))
    for g in gs:
        assert g.counts["outer"] > 0
        sl = g.slot_ids()[: g.n_local]
        assert np.array_equal(g.fields["density"].get(0, g.n_local), np.array([final[int(c)] for c in sl]))
    for g in gs + [ref]:
        g.close()


@pytest.mark.parametrize("base,R", [((32, 32, 8), 2), ((24, 16, 6), 2), ((40, 24, 4), 1)])
def test_tile_cut_matches_restatement(gpu, base, R):
    """The device tile cut (tile_build.hip device_cut: greedy best-aligned
    cuts by pointer jumping) and the regular / general classification equal
    the host restatement scripts/tile_stats.py on the same leaf set."""
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
    import tile_stats

    g, f = gpu_grid(base, R)
    prerefine(g, f, R)
    lay = g.advection_layout()
    leaves = np.sort(g.local_cells())
    L = tile_stats.layout(leaves, base, R, 512)
    reason = tile_stats.classify(L, base, R)
    assert lay["tiles"] == reason.size
    assert lay["regular_tiles"] == int(np.sum(reason == 1))
    assert lay["regular_cells"] == 512 * lay["regular_tiles"]
    g.close()


def _steps_with(base, R, steps, external=(), edit=None):
    """`steps` sweeps on a fresh pre-refined grid (tiles from the second
    step on); `external`: fields whose device pointer is taken first (the
    sweeps then read the fields, not the neighbor records); `edit(f, k)` runs
    before step k."""
    g, f = gpu_grid(base, R)
    prerefine(g, f, R)
    for k in external:
        f[k].device_ptr()
    dt = g.advection_max_time_step(f)
    out = []
    for k in range(steps):
        if edit is not None:
            edit(f, k)
        g.advection_step(f, 0.5 * dt)
        g.advection_commit(f[0])
        out.append(f[0].get(0, g.n_local))
    g.close()
    return out


@pytest.fixture
def nbrec_on(monkeypatch):
    """The neighbor records are an opt-in experiment (DCCRGX_NBREC=1; it lost
    its paired A/B) kept for reproducing it: parity with it on."""
    monkeypatch.setenv("DCCRGX_NBREC", "1")
    yield
    monkeypatch.delenv("DCCRGX_NBREC", raising=False)


@pytest.mark.parametrize("base,R", [((32, 32, 8), 2), ((12, 12, 3), 2), ((10, 10, 4), 1)])
def test_neighbor_records_bitwise_equal_fields(gpu, nbrec_on, base, R):
    """The tile sweeps read an out-of-tile neighbor's length, face area and
    velocity from its per-axis record (NbRecords, sweep_kernels.hip) instead
    of the fields; staged as (l_a, area, 1.0) every flux forms the same
    products, so the densities are bitwise those of the field reads (here
    forced by handing out a velocity field's device pointer)."""
    a = _steps_with(base, R, 4)
    b = _steps_with(base, R, 4, external=(1,))
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("k_field", [1, 2, 3, 4, 5, 6])
def test_neighbor_records_follow_field_writes(gpu, nbrec_on, k_field):
    """A write of any velocity or length field between steps (here an
    upload) invalidates the records: the next sweep rebuilds them, so the
    densities stay bitwise those of the field reads."""
    def edit(f, k):
        if k == 3:
            v = f[k_field].get()
            f[k_field].set(v * 0.5 + 0.01 if k_field <= 3 else v * 1.25)
    a = _steps_with((16, 16, 4), 2, 6, edit=edit)
    b = _steps_with((16, 16, 4), 2, 6, external=(k_field,), edit=edit)
    c = _steps_with((16, 16, 4), 2, 6)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    assert not np.array_equal(a[-1], c[-1])  # the edit mattered
