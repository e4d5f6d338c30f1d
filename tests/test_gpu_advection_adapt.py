"""Advection with grid adaptation every step (tests/advection/2d.cpp with
adapt_n = 1: check_for_adaptation before apply_fluxes, adapt_grid after it,
adapter.hpp:47-309) through the product - refinement, unrefinement,
dont_unrefine, the merged parents' mean density, the velocity / length reset
and the all-field halo - against the oracle's restatement: the leaf set equals
the oracle's after every step, dt agrees bitwise, densities within
1e-12 x max|rho| at the end."""
import numpy as np
import pytest

from oracle import oracle as O
from test_gpu_advection import gpu_grid, prerefine

pytestmark = pytest.mark.gpu

TOL = 1e-12


def product_step(g, f, dt, di):
    g.start_remote_neighbor_copy_updates()
    g.advection_step(f, dt, "inner")
    g.wait_remote_neighbor_copy_update_receives()
    g.advection_step(f, dt, "outer")
    g.wait_remote_neighbor_copy_update_sends()
    g.advection_check_adaptation(f[0], di)
    g.advection_commit(f[0])
    return g.advection_adapt(f)


@pytest.mark.parametrize("base,R,steps", [((16, 16, 1), 2, 40), ((10, 10, 3), 2, 15)])
def test_adaptive_advection_matches_oracle(gpu, base, R, steps):
    g, f = gpu_grid(base, R)
    prerefine(g, f, R)
    o = O.Grid(base, R, (True, True, False), 0, 1)
    o.set_geometry((0, 0, 0), tuple(1.0 / b for b in base))
    o.adv_prerefine(0.025, 0.25)
    assert np.array_equal(g.local_cells(), o.cells()[0])
    di = 0.025 / R
    created = removed = 0
    for step in range(steps):
        dt = 0.5 * g.advection_max_time_step(f)
        assert dt == 0.5 * o.adv_max_time_step(), step
        c, r = product_step(g, f, dt, di)
        o.adv_check(di)
        o.adv_steps(1, dt)
        oc, orm = o.adv_adapt()
        assert (c, r) == (oc, orm), step
        created += c
        removed += r
        assert np.array_equal(g.local_cells(), o.cells()[0]), step
    assert created > 0 and removed > 0
    ids = g.slot_ids()[: g.n_local]
    exp = o.adv_get(ids)
    got = f[0].get(0, g.n_local)
    assert np.max(np.abs(got - exp[:, 0])) <= TOL * np.max(np.abs(exp[:, 0]))
    for k, col in ((1, 1), (2, 2), (4, 6), (5, 7), (6, 8)):
        assert np.array_equal(f[k].get(0, g.n_local), exp[:, col])  # velocities and lengths bitwise
    g.close()


def test_check_with_pending_unrefine_matches_device_decisions(gpu):
    """check_for_adaptation decides on the device unless unrefine requests
    are already pending; then it walks the slots on the host.  Two identical
    grids step together, the second with an unrefine request of one level-2
    family issued before every check: whatever the check decides for that
    family (keep: its dont_unrefine mark cancels the request; unrefine: the
    same family twice), both grids must adapt identically - so the host walk
    and the device decisions agree."""
    base, R, steps = (16, 16, 1), 2, 12
    grids = []
    for _ in range(2):
        g, f = gpu_grid(base, R)
        prerefine(g, f, R)
        grids.append((g, f))
    di = 0.025 / R
    issued = 0
    for step in range(steps):
        dt = 0.5 * grids[0][0].advection_max_time_step(grids[0][1])
        out = []
        for k, (g, f) in enumerate(grids):
            g.advection_step(f, dt)
            if k == 1:
                cells = g.local_cells()
                lvl2 = [int(c) for c in cells[::97] if g.get_refinement_level(int(c)) == R]
                if lvl2:
                    g.unrefine_completely(lvl2[0])
                    issued += 1
            g.advection_check_adaptation(f[0], di)
            g.advection_commit(f[0])
            out.append(g.advection_adapt(f))
        assert out[0] == out[1], step
        assert np.array_equal(grids[0][0].local_cells(), grids[1][0].local_cells()), step
        assert np.array_equal(grids[0][1][0].get(0, grids[0][0].n_local), grids[1][1][0].get(0, grids[1][0].n_local))
    assert issued > 0
    for g, _ in grids:
        g.close()


@pytest.mark.parametrize("base,split", [((16, 16, 1), True), ((10, 10, 3), False)])
def test_sweep_bands_match_bands_kernel(gpu, monkeypatch, base, split):
    """The face-table sweep also writes check_for_adaptation's bands (with the
    last check's parameters) and the check then takes them instead of running
    its own bands kernel.  Two identical grids step together, the second with
    that cache switched off (DCCRGX_BAND_CACHE=0: the sweep computes no bands):
    every step's created / removed counts, leaf set and densities must be
    bitwise the same.  Sweeps as inner + outer runs or as one whole-grid run."""
    R, steps = 2, 12
    grids = []
    for _ in range(2):
        g, f = gpu_grid(base, R)
        prerefine(g, f, R)
        grids.append((g, f))
    di = 0.025 / R
    for step in range(steps):
        dt = 0.5 * grids[0][0].advection_max_time_step(grids[0][1])
        out = []
        for k, (g, f) in enumerate(grids):
            if k == 1:
                monkeypatch.setenv("DCCRGX_BAND_CACHE", "0")
            else:
                monkeypatch.delenv("DCCRGX_BAND_CACHE", raising=False)
            if split:
                g.advection_step(f, dt, "inner")
                g.advection_step(f, dt, "outer")
            else:
                g.advection_step(f, dt)
            g.advection_check_adaptation(f[0], di)
            g.advection_commit(f[0])
            out.append(g.advection_adapt(f))
        assert out[0] == out[1], step
        assert np.array_equal(grids[0][0].local_cells(), grids[1][0].local_cells()), step
        assert np.array_equal(grids[0][1][0].get(0, grids[0][0].n_local), grids[1][1][0].get(0, grids[1][0].n_local))
    monkeypatch.delenv("DCCRGX_BAND_CACHE", raising=False)
    for g, _ in grids:
        g.close()


def test_kept_children_order_without_sort(gpu, monkeypatch):
    """On one process the merged families' children (the removed store)
    are put in ascending order by ranks within the eight octant streams
    instead of a sort (k_kept_children, all_local).  Against the sorted form
    (DCCRGX_KEPT_SORT=1) on a twin grid: the removed cells in the same order
    (ascending), the merged parents' densities bitwise, every step."""
    base, R, steps = (10, 10, 3), 2, 10
    grids = []
    for _ in range(2):
        g, f = gpu_grid(base, R)
        prerefine(g, f, R)
        grids.append((g, f))
    di = 0.025 / R
    merged = 0
    for step in range(steps):
        dt = 0.5 * grids[0][0].advection_max_time_step(grids[0][1])
        out, rem = [], []
        for k, (g, f) in enumerate(grids):
            if k == 1:
                monkeypatch.setenv("DCCRGX_KEPT_SORT", "1")
            else:
                monkeypatch.delenv("DCCRGX_KEPT_SORT", raising=False)
            out.append(product_step(g, f, dt, di))
            rem.append(g.get_removed_cells())
        monkeypatch.delenv("DCCRGX_KEPT_SORT", raising=False)
        assert out[0] == out[1], step
        assert np.array_equal(rem[0], rem[1]), step
        assert np.all(np.diff(rem[0].astype(np.int64)) > 0), step
        merged += len(rem[0])
        assert np.array_equal(grids[0][1][0].get(0, grids[0][0].n_local), grids[1][1][0].get(0, grids[1][0].n_local))
    assert merged > 0
    for g, _ in grids:
        g.close()
