"""Multi-rank structures on one GPU: detached per-rank views (no transport)
vs the oracle's per-rank views (update_remote_neighbor_info 8992-9095,
recalculate_neighbor_update_send_receive_lists 8590-8752), plus an emulated
halo exchange that moves field payloads between the views in wire order
and runs the inner/outer split sweeps — results must equal one rank's."""
import numpy as np
import pytest

import dccrg_amd
from helpers import make_pair

pytestmark = pytest.mark.gpu


def views(length, R, periodic, hood, nprocs, rounds=0, frac=0.1, seed=0):
    out = []
    o = None
    for r in range(nprocs):
        g, o = make_pair(length, R, periodic, hood, rounds, frac, seed, nprocs=nprocs, rank=r)
        out.append(g)
    return out, o


CASES = [((10, 6, 5), 0, (False, False, False), 1, 2, 0), ((10, 6, 5), 0, (True, True, True), 1, 3, 0),
         ((8, 8, 4), 0, (False, True, False), 2, 4, 0), ((7, 5, 3), 0, (True, False, True), 0, 5, 0),
         ((6, 6, 6), 2, (False, False, False), 1, 3, 2), ((6, 6, 4), 2, (True, True, False), 0, 4, 2)]


@pytest.mark.parametrize("length,R,periodic,hood,P,rounds", CASES)
def test_rank_views_match_oracle(gpu, length, R, periodic, hood, P, rounds):
    gs, o = views(length, R, periodic, hood, P, rounds, 0.15, 7)
    for r, g in enumerate(gs):
        assert np.array_equal(g.local_cells(), o.rank_cells(r, "local"))
        assert np.array_equal(g.inner_cells(), o.rank_cells(r, "inner"))
        assert np.array_equal(g.outer_cells(), o.rank_cells(r, "outer"))
        assert np.array_equal(g.remote_cells(), o.rank_cells(r, "remote_bdy"))
        for p in range(P):
            if p == r:
                continue
            assert np.array_equal(g.get_cells_to_send(p), o.cells_to_send(r, p)), (r, p)
            assert np.array_equal(g.get_cells_to_receive(p), o.cells_to_receive(r, p)), (r, p)
            # wire consistency: what r sends to p is what p expects from r
            assert np.array_equal(g.get_cells_to_send(p), gs[p].get_cells_to_receive(r))
    for g in gs:
        g.close()


def emulated_exchange(gs, fields=None):
    """update_copies_of_remote_neighbors between detached views of one
    process: the library packs each peer's wire message (transferred fields,
    cells_to_send in ascending id, start_user_data_sends 10802-10997) and
    the receiver's library places it into its halo copies.  `fields`, when
    given, must be exactly the transferred fields (checked)."""
    for g in gs:
        if fields is not None:
            assert sorted(n for n, f in g.fields.items() if f.transfer) == sorted(fields)
    msgs = {}
    for r, g in enumerate(gs):
        for p in g.get_peers():
            sb, rb = g.halo_message_size(p)
            assert (sb, rb) == tuple(reversed(gs[p].halo_message_size(r)))  # both ends agree on the sizes
            msgs[(r, p)] = g.halo_pack(p)
    for (r, p), m in msgs.items():
        gs[p].halo_place(r, m)


def test_multirank_gol_equals_single_rank(gpu):
    length, P, steps = (12, 10, 8), 3, 5
    gs, o = views(length, 0, (True, False, True), 1, P)
    ref, _ = make_pair(length, 0, (True, False, True), 1)
    rng = np.random.default_rng(1)
    ids_all = ref.slot_ids()
    a0 = (rng.random(ids_all.size) < 0.3).astype(np.uint32)
    val = dict(zip(ids_all.tolist(), a0.tolist()))
    rs = ref.add_field("is_alive", np.uint32)
    rs.set(a0)
    for g in gs:
        st = g.add_field("is_alive", np.uint32)
        sl = g.slot_ids()[: g.n_local]
        st.set(np.array([val[int(c)] for c in sl], np.uint32))
    for _ in range(steps):
        emulated_exchange(gs, ["is_alive"])
        for g in gs:
            g.gol_step(g.fields["is_alive"], "inner")
            g.gol_step(g.fields["is_alive"], "outer")
            g.gol_commit(g.fields["is_alive"])
        ref.gol_step(rs)
        ref.gol_commit(rs)
    final = dict(zip(ids_all.tolist(), rs.get().tolist()))
    for g in gs:
        sl = g.slot_ids()[: g.n_local]
        got = g.fields["is_alive"].get(0, g.n_local)
        assert np.array_equal(got, np.array([final[int(c)] for c in sl], np.uint32))
    for g in gs + [ref]:
        g.close()


def test_multirank_advection_equals_single_rank(gpu):
    from test_gpu_advection import NAMES, gpu_grid, prerefine

    base, R, P, steps = (12, 12, 4), 2, 3, 10
    ref, rf = gpu_grid(base, R)
    prerefine(ref, rf, R)
    leaves = np.sort(ref.local_cells())
    # block partition of level-0 parents, children follow (execute_refines 10228-10237)
    m = dccrg_amd.Dccrg(0, 1, 0).set_initial_length(base).set_maximum_refinement_level(R).initialize()
    n0 = int(np.prod(base))
    l0p = np.array([m.get_cell_from_indices(m.get_indices(int(c)), 0) for c in leaves], np.int64)
    owners = ((l0p - 1) * P // n0).astype(np.int32)
    m.close()
    gs = []
    for r in range(P):
        g = dccrg_amd.Dccrg(r, P, 0).set_initial_length(base).set_neighborhood_length(0)
        g.set_maximum_refinement_level(R).set_periodic(True, True, False).initialize()
        g.set_geometry((0, 0, 0), tuple(1.0 / b for b in base))
        for n in NAMES:
            g.add_field(n, np.float64, n == "density")
        g.set_cells(leaves, owners)
        g.advection_initialize([g.fields[n] for n in NAMES])
        gs.append(g)
    dt = ref.advection_max_time_step(rf)
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
        got = g.fields["density"].get(0, g.n_local)
        exp = np.array([final[int(c)] for c in sl])
        # identical face sets and operand order: bitwise equal
        assert np.array_equal(got, exp)
    for g in gs + [ref]:
        g.close()


@pytest.mark.parametrize("length,periodic,P", [((256, 6, 9), (True, False, True), 3),
                                               ((256, 4, 12), (False, True, False), 4),
                                               ((512, 3, 8), (True, True, True), 2)])
def test_slab_gol_structured_equals_single_rank(gpu, length, periodic, P):
    """z-slab partitions of a uniform grid whose x length is a multiple of 256
    run the structured 26-point kernel per plane box (inner planes, then each
    outer plane with its halo plane as z-1 / z+1, gol_slab_plan): bit-exact
    against the one-rank game."""
    steps = 5
    gs, _ = views(length, 0, periodic, 1, P)
    ref, _ = make_pair(length, 0, periodic, 1)
    rng = np.random.default_rng(11)
    ids_all = ref.slot_ids()
    a0 = (rng.random(ids_all.size) < 0.3).astype(np.uint32)
    val = dict(zip(ids_all.tolist(), a0.tolist()))
    rs = ref.add_field("is_alive", np.uint32)
    rs.set(a0)
    for g in gs:
        st = g.add_field("is_alive", np.uint32)
        st.set(np.array([val[int(c)] for c in g.slot_ids()[: g.n_local]], np.uint32))
        assert g.n_local % (length[0] * length[1]) == 0
    for _ in range(steps):
        emulated_exchange(gs, ["is_alive"])
        for g in gs:
            g.gol_step(g.fields["is_alive"], "inner")
            g.gol_step(g.fields["is_alive"], "outer")
            g.gol_commit(g.fields["is_alive"])
        ref.gol_step(rs)
        ref.gol_commit(rs)
    final = dict(zip(ids_all.tolist(), rs.get().tolist()))
    for g in gs:
        sl = g.slot_ids()[: g.n_local]
        assert np.array_equal(g.fields["is_alive"].get(0, g.n_local), np.array([final[int(c)] for c in sl]))
    for g in gs + [ref]:
        g.close()


def test_get_cells_criteria_match_neighbor_types(gpu):
    """get_cells(criteria, exact_match) (dccrg.hpp:651-739 with
    is_neighbor_type_match 2946-3053) on 3 detached views of a refined grid:
    the library's answer equals the neighbor types computed here from the
    rank's neighbors_of / neighbors_to lists and its local set, for the
    reference's documented criteria (598-630)."""
    from dccrg_amd.grid import (HAS_LOCAL_NEIGHBOR_BOTH, HAS_LOCAL_NEIGHBOR_OF, HAS_LOCAL_NEIGHBOR_TO,
                                HAS_NO_NEIGHBOR, HAS_REMOTE_NEIGHBOR_BOTH, HAS_REMOTE_NEIGHBOR_OF,
                                HAS_REMOTE_NEIGHBOR_TO)

    gs, _ = views((8, 6, 5), 1, (True, False, False), 1, 3, rounds=1, frac=0.2, seed=3)
    cases = [([], False),
             ([HAS_NO_NEIGHBOR, HAS_LOCAL_NEIGHBOR_OF, HAS_LOCAL_NEIGHBOR_TO, HAS_LOCAL_NEIGHBOR_BOTH], True),
             ([HAS_REMOTE_NEIGHBOR_BOTH], False), ([HAS_REMOTE_NEIGHBOR_OF], False),
             ([HAS_LOCAL_NEIGHBOR_TO | HAS_REMOTE_NEIGHBOR_TO], True),
             ([HAS_LOCAL_NEIGHBOR_BOTH | HAS_REMOTE_NEIGHBOR_BOTH], True)]
    for g in gs:
        local = set(g.local_cells().tolist())
        slots = g.slot_ids()[: g.n_local]
        optr, oids, _ = g.csr("of")
        tptr, tids, _ = g.csr("to")
        types = {}
        for s, c in enumerate(slots.tolist()):
            t = 0
            for i in oids[optr[s]:optr[s + 1]].tolist():
                t |= HAS_LOCAL_NEIGHBOR_OF if i in local else HAS_REMOTE_NEIGHBOR_OF
            for i in tids[tptr[s]:tptr[s + 1]].tolist():
                t |= HAS_LOCAL_NEIGHBOR_TO if i in local else HAS_REMOTE_NEIGHBOR_TO
            types[c] = t
        for crit, exact in cases:
            if not crit:
                exp = sorted(types)
            elif exact:
                exp = sorted(c for c, t in types.items() if t in crit)
            else:
                m = 0
                for x in crit:
                    m |= x
                exp = sorted(c for c, t in types.items() if t & m)
            assert g.get_cells(crit, exact).tolist() == exp, (crit, exact)
        # the inner / outer split is the reference's process-boundary split
        assert g.get_cells([HAS_REMOTE_NEIGHBOR_BOTH], False).tolist() == g.outer_cells().tolist()
    for g in gs:
        g.close()
