"""BASELINE config 3 at its full per-GPU size (the bench's headline mesh:
128^3 base, max_ref_lvl 2, periodic x and y, 8.87 M leaves).

* The product's pre-refined leaf set equals the oracle's (count per level and
  the SHA-256 of the ascending ids, tests/golden/config3_adv.json, written by
  tests/golden/make_config3.py from oracle/dccrg_oracle.cpp), dt is bitwise
  the oracle's, and after 3 steps the density at ~17.8 K sampled leaves of
  every level is within 1e-12 x max|rho| of the oracle's.
* After 100 steps the same samples are within 1e-12 x
  max|rho| of the oracle's and the total mass sum(rho * volume) is within
  1e-13 (relative) of the initial mass and of the oracle's.
* The same mesh split into 4 z-slabs (block partition of the level-0 cells,
  children inherit, dccrg.hpp:7981-8013 / 10228-10237) on detached views with
  the density halo moved by the library's pack / place: every cell bitwise
  equals the one-rank run after 3 steps."""
import hashlib
import json
import os

import numpy as np
import pytest

import dccrg_amd
from test_gpu_advection import NAMES, TOL, gpu_grid, prerefine

pytestmark = pytest.mark.gpu

BASE, R, STEPS = (128, 128, 128), 2, 3


@pytest.fixture(scope="module")
def golden(golden_dir):
    with open(os.path.join(golden_dir, "config3_adv.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def one_rank(gpu):
    g, f = gpu_grid(BASE, R)
    prerefine(g, f, R)
    yield g, f
    g.close()


def test_config3_mesh_dt_and_steps_match_oracle(one_rank, golden):
    g, f = one_rank
    assert golden["base"] == list(BASE) and golden["max_ref_lvl"] == R and golden["steps"] == STEPS
    ids = np.sort(g.local_cells())
    assert ids.size == golden["n_cells"]
    lvl = g.mapping_batch(ids)["level"]
    assert np.bincount(lvl, minlength=R + 1).tolist() == golden["cells_per_level"]
    assert hashlib.sha256(ids.astype("<u8").tobytes()).hexdigest() == golden["ids_sha256"]
    lay = g.advection_layout()
    # the tile cut and classification equal the host restatement
    # (scripts/tile_stats.py on the oracle's leaf set: 18800 tiles, 9408 regular)
    assert (lay["tiles"], lay["regular_tiles"]) == (18800, 9408), lay
    dt = g.advection_max_time_step(f)
    assert dt == golden["dt"]
    for _ in range(STEPS):
        g.advection_step(f, 0.5 * dt)
        g.advection_commit(f[0])
    sl = g.slot_ids()[: g.n_local]
    rho = f[0].get(0, g.n_local)
    order = np.argsort(sl)
    want = np.array(golden["sample_ids"], np.uint64)
    pos = np.searchsorted(sl[order], want)
    assert np.array_equal(sl[order][pos], want)
    got = rho[order][pos]
    exp = np.array(golden["sample_rho"])
    assert np.max(np.abs(got - exp)) <= TOL * np.max(np.abs(exp))
    # the whole field stays finite
    assert np.all(np.isfinite(rho))


def test_config3_four_slabs_bitwise(gpu):
    from test_gpu_multirank import emulated_exchange

    P = 4
    ref, rf = gpu_grid(BASE, R)
    prerefine(ref, rf, R)
    dt = ref.advection_max_time_step(rf)
    leaves = np.sort(ref.local_cells())
    mb = ref.mapping_batch(leaves)
    l0p = mb["level0_parent"].astype(np.int64)
    n0 = int(np.prod(BASE))
    owners = ((l0p - 1) * P // n0).astype(np.int32)
    del mb, l0p
    gs, n_regular = [], 0
    for r in range(P):
        g = dccrg_amd.Dccrg(r, P, 0).set_initial_length(BASE).set_neighborhood_length(0)
        g.set_maximum_refinement_level(R).set_periodic(True, True, False).initialize()
        g.set_geometry((0, 0, 0), tuple(1.0 / b for b in BASE))
        for n in NAMES:
            g.add_field(n, np.float64, n == "density")
        g.set_cells(leaves, owners)
        g.advection_initialize([g.fields[n] for n in NAMES])
        n_regular += g.advection_layout()["regular_tiles"]
        gs.append(g)
    assert n_regular > 0
    assert sum(g.n_local for g in gs) == leaves.size
    for _ in range(STEPS):
        emulated_exchange(gs, ["density"])
        for g in gs:
            f = [g.fields[n] for n in NAMES]
            g.advection_step(f, 0.5 * dt, "inner")
            g.advection_step(f, 0.5 * dt, "outer")
            g.advection_commit(f[0])
        ref.advection_step(rf, 0.5 * dt)
        ref.advection_commit(rf[0])
    rsl = ref.slot_ids()[: ref.n_local]
    order = np.argsort(rsl)
    rsl, rrho = rsl[order], rf[0].get(0, ref.n_local)[order]
    for g in gs:
        assert g.counts["outer"] > 0
        sl = g.slot_ids()[: g.n_local]
        pos = np.searchsorted(rsl, sl)
        assert np.array_equal(rsl[pos], sl)
        assert np.array_equal(g.fields["density"].get(0, g.n_local), rrho[pos])
    for g in gs + [ref]:
        g.close()


def _mass(rho, lx, ly, lz):
    import math

    return math.fsum((rho * (lx * ly * lz)).tolist())


def test_config3_hundred_steps_and_mass(gpu, golden):
    """SURVEY §8(d) config 3's parity depth: 100 steps at full size."""
    long = golden.get("steps_long")
    assert long == 100, "regenerate tests/golden/config3_adv.json (make_config3.py)"
    g, f = gpu_grid(BASE, R)
    prerefine(g, f, R)
    dt = g.advection_max_time_step(f)
    assert dt == golden["dt"]
    n = g.n_local
    lx, ly, lz = (f[k].get(0, n) for k in (4, 5, 6))
    m0 = _mass(f[0].get(0, n), lx, ly, lz)
    assert m0 == pytest.approx(golden["mass_0"], rel=1e-15)
    for _ in range(long):
        g.advection_step(f, 0.5 * dt)
        g.advection_commit(f[0])
    sl = g.slot_ids()[:n]
    rho = f[0].get(0, n)
    m1 = _mass(rho, lx, ly, lz)
    assert abs(m1 - m0) <= 1e-13 * m0, (m0, m1)
    assert abs(m1 - golden["mass_long"]) <= 1e-13 * m0, (m1, golden["mass_long"])
    order = np.argsort(sl)
    want = np.array(golden["sample_ids"], np.uint64)
    pos = np.searchsorted(sl[order], want)
    assert np.array_equal(sl[order][pos], want)
    exp = np.array(golden["sample_rho_long"])
    assert np.max(np.abs(rho[order][pos] - exp)) <= TOL * np.max(np.abs(exp))
    g.close()
