"""Shared helpers: build the same mesh in the product (dccrg_amd) and the
oracle, and compare their neighbor structures."""
import numpy as np


def random_refines(ids, levels, R, rng, frac):
    cand = ids[levels < R]
    if cand.size == 0:
        return []
    k = max(1, int(frac * cand.size))
    return sorted(int(c) for c in rng.choice(cand, size=min(k, cand.size), replace=False))


def make_pair(length, R=0, periodic=(False, False, False), hood=1, rounds=0, frac=0.1, seed=0, nprocs=1,
              rank=0, device=0):
    """Product grid (detached view of `rank` when nprocs > 1) + oracle grid with
    identical refinement history.  Returns (grid, oracle)."""
    import dccrg_amd
    from oracle import oracle as O

    o = O.Grid(length, R, periodic, hood, nprocs)
    rng = np.random.default_rng(seed)
    for _ in range(rounds):
        ids, _ = o.cells()
        lv = o.mapping.batch(ids)["level"]
        for c in random_refines(ids, lv, R, rng, frac):
            o.refine_completely(c)
        o.stop_refining()
    g = dccrg_amd.Dccrg(rank, nprocs, device)
    g.set_initial_length(length).set_maximum_refinement_level(R).set_periodic(*periodic)
    g.set_neighborhood_length(hood).initialize()
    if rounds:
        ids, own = o.cells()
        g.set_cells(ids, own)
    return g, o


def make_pair_refined_by_product(length, R, periodic, hood, rounds, frac, seed):
    """Refinement driven through the product's refine_completely/stop_refining
    (induce_refines closure on the host), mirrored on the oracle."""
    import dccrg_amd
    from oracle import oracle as O

    o = O.Grid(length, R, periodic, hood, 1)
    g = dccrg_amd.Dccrg(0, 1, 0)
    g.set_initial_length(length).set_maximum_refinement_level(R).set_periodic(*periodic)
    g.set_neighborhood_length(hood).initialize()
    rng = np.random.default_rng(seed)
    for _ in range(rounds):
        ids = g.local_cells()
        lv = np.array([g.get_refinement_level(int(c)) for c in ids])
        req = random_refines(ids, lv, R, rng, frac)
        for c in req:
            assert g.refine_completely(c)
            o.refine_completely(c)
        g.stop_refining()
        o.stop_refining()
    return g, o


def compare_neighbors(g, o, check_iterator=True):
    """Every local row of the device CSRs against the oracle's lists."""
    slots = g.slot_ids()
    nl = g.n_local
    ptr, ids, offs = g.csr("of")
    tptr, tids, _ = g.csr("to")
    fptr, fids, fdirs = g.csr("face")
    iptr, iids, ioffs = g.csr("iterator") if check_iterator else (None, None, None)
    for s in range(nl):
        c = int(slots[s])
        eid, eoff = o.neighbors_of(c)
        gid = ids[ptr[s]:ptr[s + 1]]
        goff = offs[ptr[s]:ptr[s + 1]]
        assert np.array_equal(gid, eid), (c, gid, eid)
        assert np.array_equal(goff, eoff), (c, goff, eoff)
        tid, _ = o.neighbors_to(c)
        assert np.array_equal(tids[tptr[s]:tptr[s + 1]], tid), (c, tids[tptr[s]:tptr[s + 1]], tid)
        fid, fd = o.face_neighbors_of(c)
        assert np.array_equal(fids[fptr[s]:fptr[s + 1]], fid), (c, fids[fptr[s]:fptr[s + 1]], fid)
        assert np.array_equal(fdirs[fptr[s]:fptr[s + 1]], fd), c
        if check_iterator:
            # update_cell_pointers 11451-11500: only-of, then both, each in
            # (id, offset) order - the exact sequence with offsets
            iid, ioff = o.iterator_neighbors_of(c)
            assert np.array_equal(iids[iptr[s]:iptr[s + 1]], iid), (c, iids[iptr[s]:iptr[s + 1]], iid)
            assert np.array_equal(ioffs[iptr[s]:iptr[s + 1]], ioff), c
    return nl
