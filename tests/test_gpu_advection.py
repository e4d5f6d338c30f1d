"""3-D advection (tests/advection/solve.hpp) on refined grids vs the oracle.

Tolerance (fp64): per cell |rho_gpu - rho_oracle| <= 1e-12 * max|rho_oracle|.
The flux through a face is evaluated with the reference's expression and
operand order on both sides (no contraction), so the only difference is the
order in which a cell's face fluxes are summed (gather here, hash-ordered
scatter in the reference)."""
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


def _variant_rho(base=(64, 64, 16), R=2, steps=10):
    """Density after `steps` sweeps of the large refined case (regular and
    general tiles both present) under the current DCCRGX_ADV_* schedule."""
    g, f = gpu_grid(base, R)
    prerefine(g, f, R)
    dt = g.advection_max_time_step(f)
    for _ in range(steps):
        g.advection_step(f, 0.5 * dt)
        g.advection_commit(f[0])
    rho = f[0].get(0, g.n_local)
    g.close()
    return rho


@pytest.mark.parametrize("env", ["DCCRGX_ADV_DEPTH=2", "DCCRGX_ADV_DYN=1", "DCCRGX_ADV_DYN=1 DCCRGX_ADV_2S=1"])
def test_schedule_variants_bitwise(gpu, tmp_path, env):
    """The A/B schedules of the persistent tile sweeps (two tiles of loads in
    flight instead of one, per-XCD tile tickets, the general sweep on a second
    stream) change only which block sweeps which tile and when: every cell's
    result is bitwise the default's.  The knobs are read once per process, so
    the variant runs in a child process."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / "rho.npy"
    code = ("import sys, numpy as np, torch; sys.path[:0] = [%r, %r]; "
            "from test_gpu_advection import _variant_rho; np.save(%r, _variant_rho())"
            % (root, os.path.join(root, "tests"), str(out)))
    child_env = dict(os.environ)
    for kv in env.split():
        k, v = kv.split("=")
        child_env[k] = v
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=child_env, capture_output=True, text=True,
                       timeout=100)
    assert r.returncode == 0, r.stderr[-2000:]
    assert np.array_equal(np.load(str(out)), _variant_rho())
