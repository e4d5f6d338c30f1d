"""Headline parity pinned to the reference's own advection code.

examples/bin/ref_advection is the repo's 2d.cpp-style main compiled against
the facade with the reference's tests/advection/{cell,initialize,solve,
adapter}.hpp included unmodified (__graft_entry__.build_examples()): the
reference's initialize(), check_for_adaptation / adapt_grid (pre-refinement
to the maximum level, 2d.cpp:258-292), max_time_step and calculate_fluxes /
apply_fluxes (solve.hpp:44-279) run on the host over the facade's iterators
and halo.  It dumps every local cell after pre-refinement and after K frozen
steps at 1 and 2 MPI ranks (2 ranks: balance_load() at the start as
2d.cpp:254, the facade's halo between the inner and outer flux passes).

The device path (dccrgx_advection_* through dccrg_amd.Dccrg) must then give,
on SURVEY §8(d)'s oracle parity grid (32^3 base, R = 2, x and y periodic):
  * the same leaf set after its own pre-refinement (exact),
  * the same initial fields and time step (bitwise),
  * densities after K = 100 steps within 1e-12 x max|rho| of the
    reference's,
  * the total mass sum(rho * volume) after K steps within 1e-13 (relative)
    of the initial one, on the device and in the reference's run (no flux
    leaves through the non-periodic z boundary, every face's flux enters one
    side and leaves the other),
with both sweep kernels exercised (regular tiles > 0, general tiles > 0).
The oracle's restatement is checked against the same dumps."""
import os
import subprocess

import numpy as np
import pytest

import dccrg_amd
from oracle import oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "examples", "bin", "ref_advection")
MPIEXEC = "/opt/conda/bin/mpiexec"
BASE, R, STEPS = (32, 32, 32), 2, 100  # parity after 100 steps
NAMES = ("density", "vx", "vy", "vz", "lx", "ly", "lz")
COLS = (0, 1, 2, 3, 6, 7, 8)  # Cell::data index of each field (cell.hpp:33-44)
TOL = 1e-12
REC = np.dtype([("id", "<u8"), ("data", "<f8", (9,))])
MAGIC = 0x6164766563746E31


def load(prefix, stage, P):
    ids, data, dts = [], [], []
    for r in range(P):
        with open(f"{prefix}.{stage}.{r}", "rb") as f:
            magic, n = np.frombuffer(f.read(16), "<u8")
            assert int(magic) == MAGIC
            dts.append(float(np.frombuffer(f.read(8), "<f8")[0]))
            rec = np.frombuffer(f.read(), REC)
        assert rec.size == int(n)
        ids.append(rec["id"])
        data.append(rec["data"])
    assert len(set(dts)) == 1  # one global time step (MPI_Allreduce MIN)
    ids, data = np.concatenate(ids), np.concatenate(data)
    order = np.argsort(ids)
    ids, data = ids[order], data[order]
    assert np.all(np.diff(ids.astype(np.int64)) > 0)  # every cell exactly once
    return ids, data, dts[0]


@pytest.fixture(scope="module")
def ref_runs(tmp_path_factory):
    if not os.path.exists(EXE):
        pytest.fail(f"{EXE} missing: run __graft_entry__.build() where /root/reference exists")
    d = tmp_path_factory.mktemp("ref_advection")
    runs = {}
    for P in (1, 2):
        prefix = str(d / f"p{P}")
        cmd = [MPIEXEC, "-n", str(P), EXE, *map(str, BASE), str(R), str(STEPS), prefix, "1" if P > 1 else "0"]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        assert "ref_advection cells" in r.stdout
        runs[P] = (load(prefix, "prerefined", P), load(prefix, "final", P))
    return runs


def device_run(steps):
    g = dccrg_amd.Dccrg(0, 1, 0).set_initial_length(BASE).set_neighborhood_length(0)
    g.set_maximum_refinement_level(R).set_periodic(True, True, False).initialize()
    g.set_geometry((0, 0, 0), tuple(1.0 / b for b in BASE))
    f = [g.add_field(n, np.float64, n == "density") for n in NAMES]
    for _ in range(R):  # 2d.cpp:266-289 through the device adaptation
        g.advection_initialize(f)
        for c in g.advection_refine_candidates(f[0], 0.025 / R, 0.25):
            g.refine_completely(int(c))
        g.stop_refining()
    g.advection_initialize(f)
    ids = g.slot_ids()[: g.n_local]
    init = np.stack([fi.get(0, ids.size) for fi in f], 1)
    dt = g.advection_max_time_step(f)
    lay = g.advection_layout()
    for _ in range(steps):
        g.advection_step(f, 0.5 * dt)
        g.advection_commit(f[0])
    rho = f[0].get(0, ids.size)
    g.close()
    order = np.argsort(ids)
    return ids[order], init[order], dt, rho[order], lay


@pytest.fixture(scope="module")
def dev(gpu):
    return device_run(STEPS)


@pytest.mark.parametrize("P", [1, 2])
def test_prerefined_state_matches_reference(ref_runs, dev, P):
    (ids, data, dt), _ = ref_runs[P]
    dids, dinit, ddt, _, _ = dev
    assert ids.size > np.prod(BASE)  # the reference's adapter refined
    assert np.array_equal(dids, ids)
    for k, c in enumerate(COLS):
        assert np.array_equal(dinit[:, k], data[:, c]), NAMES[k]
    assert ddt == dt


@pytest.mark.parametrize("P", [1, 2])
def test_steps_match_reference(ref_runs, dev, P):
    _, (ids, data, dt) = ref_runs[P]
    dids, _, ddt, rho, lay = dev
    assert lay["regular_tiles"] > 0 and lay["tiles"] > lay["regular_tiles"], lay
    assert np.array_equal(dids, ids) and ddt == dt
    exp = data[:, 0]
    assert np.max(np.abs(rho - exp)) <= TOL * np.max(np.abs(exp))
    # the reference's fluxes are zeroed by apply_fluxes (solve.hpp:276-277)
    assert np.all(data[:, 4] == 0)


def test_oracle_matches_reference(ref_runs):
    """The CPU restatement (oracle/dccrg_oracle.cpp adv_*) against the
    reference's own solver on the same mesh and time step."""
    (ids, data, dt), (_, fin, _) = ref_runs[1]
    o = O.Grid(BASE, R, (True, True, False), 0, 1)
    o.set_geometry((0, 0, 0), tuple(1.0 / b for b in BASE))
    o.set_cells(ids, np.zeros(ids.size, np.int32))
    o.adv_initialize()
    init = o.adv_get(ids)
    assert np.array_equal(init[:, list(COLS)], data[:, list(COLS)])
    assert o.adv_max_time_step() == dt
    o.adv_steps(STEPS, 0.5 * dt)
    exp = fin[:, 0]
    assert np.max(np.abs(o.adv_get(ids)[:, 0] - exp)) <= TOL * np.max(np.abs(exp))


def _mass(rho, lx, ly, lz):
    import math

    return math.fsum((rho * (lx * ly * lz)).tolist())


MASS_TOL = 1e-13


def test_total_mass_conserved_device(dev):
    _, init, _, rho, _ = dev
    m0 = _mass(init[:, 0], init[:, 4], init[:, 5], init[:, 6])
    m1 = _mass(rho, init[:, 4], init[:, 5], init[:, 6])
    assert m0 > 0
    assert abs(m1 - m0) <= MASS_TOL * m0, (m0, m1)


@pytest.mark.parametrize("P", [1, 2])
def test_total_mass_conserved_reference_and_device_agree(ref_runs, dev, P):
    (ids, data, _), (_, fin, _) = ref_runs[P]
    m0 = _mass(data[:, 0], data[:, 6], data[:, 7], data[:, 8])
    m1 = _mass(fin[:, 0], data[:, 6], data[:, 7], data[:, 8])
    assert abs(m1 - m0) <= MASS_TOL * m0, (m0, m1)
    _, init, _, rho, _ = dev
    md = _mass(rho, init[:, 4], init[:, 5], init[:, 6])
    assert abs(md - m1) <= MASS_TOL * m0, (md, m1)
