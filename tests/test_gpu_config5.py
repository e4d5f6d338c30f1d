"""BASELINE config 5 at its full per-GPU size (tests/scalability/
scalability.cpp; SURVEY §8 ★: no O(N_global) state per rank) across 2 real
processes sharing the one GPU over the library's host exchange (the
transport of tests/test_gpu_transport.py)."""
import numpy as np
import pytest

from test_gpu_transport import _grid, _play, _run_group, alive_rule

pytestmark = pytest.mark.gpu


def _gol_slab_numpy(nx, ny, nz, z0, z1):
    """Independent checker: one 26-point game-of-life step (non-periodic, the
    alive(id) initial state) of planes [z0, z1) of an nx x ny x nz grid,
    as uint32 next states shaped (z1 - z0, ny, nx)."""
    zs = np.arange(max(z0 - 1, 0), min(z1 + 1, nz))
    a = np.zeros((z1 - z0 + 2, ny + 2, nx + 2), np.uint8)
    for k, z in enumerate(zs):
        ids = np.uint64(1 + int(z) * nx * ny) + np.arange(nx * ny, dtype=np.uint64)
        a[int(z) - z0 + 1, 1:-1, 1:-1] = alive_rule(ids).reshape(ny, nx)
    s = a[:, :, :-2] + a[:, :, 1:-1] + a[:, :, 2:]
    s = s[:, :-2] + s[:, 1:-1] + s[:, 2:]
    s = s[:-2] + s[1:-1] + s[2:]
    cur = a[1:-1, 1:-1, 1:-1]
    cnt = s - cur
    return np.where(cnt == 3, 1, np.where(cnt == 2, cur, 0)).astype(np.uint32)


def sc_config5(rank, world):
    """BASELINE config 5 at full size (tests/scalability/scalability.cpp,
    SURVEY ★): 1024 x 1024 x 128 cells per rank (z slabs of the block
    partition, neighborhood 1, non-periodic), the bench's half-shift
    repartition (every rank's first half of its cells to the previous rank,
    balance_load 3746-4147) moving 67 M cells per rank through the library,
    then: the local sets are the shifted slabs, each rank knows exactly its
    own cells plus one ghost plane per side with their true owners and no
    other cell (no O(N_global) state), its send lists are the two boundary
    planes, and one halo + game-of-life step from the migrated payload equals
    an independent numpy game on the same initial state."""
    import sys
    import time

    t0 = time.perf_counter()

    def note(what):  # progress on stderr (seen with pytest -s)
        print(f"[config5 rank {rank}] {time.perf_counter() - t0:7.1f} s {what}", file=sys.stderr, flush=True)

    nx, ny, nzr = 1024, 1024, 128
    nz, plane = nzr * world, nx * ny
    g = _grid((nx, ny, nz), 0, (False, False, False), 1)
    note("initialized")
    st = g.add_field("is_alive", np.uint32)
    sl = g.slot_ids()[: g.n_local]
    st.set(alive_rule(sl))
    del sl
    loc = g.local_cells()
    half = loc[: loc.size // 2]
    note("state set")
    g.balance_load_to(half, np.full(half.size, (rank - 1) % world, np.int32))
    note("repartitioned")
    del loc, half
    res = {}
    # owner of plane z after the shift: the first half of slab r went to r - 1
    def owner(z):
        r = z // nzr
        return (r - 1) % world if (z % nzr) < nzr // 2 else r
    mine = [z for z in range(nz) if owner(z) == rank]
    runs = []  # maximal runs of owned planes
    for z in mine:
        if runs and runs[-1][1] == z:
            runs[-1][1] = z + 1
        else:
            runs.append([z, z + 1])
    exp_local = np.concatenate([np.arange(1 + a * plane, 1 + b * plane, dtype=np.uint64) for a, b in runs])
    res["local"] = bool(np.array_equal(g.local_cells(), exp_local))
    del exp_local
    kid, kown = g.get_cell_process()
    note("local checked, known downloaded")
    kz = ((kid - np.uint64(1)) // np.uint64(plane)).astype(np.int64)
    known_planes = sorted({z for a, b in runs for z in range(max(a - 1, 0), min(b + 1, nz))})
    exp_n = len(known_planes) * plane
    per_plane = np.bincount(kz, minlength=nz)
    res["known"] = bool(kid.size == exp_n and np.all(kid[1:] > kid[:-1])
                        and np.nonzero(per_plane)[0].tolist() == known_planes
                        and bool(np.all(per_plane[known_planes] == plane))
                        and np.array_equal(kown, np.array([owner(z) for z in range(nz)], np.int32)[kz]))
    del kid, kown, kz
    ghost_planes = [z for z in known_planes if owner(z) != rank]
    res["send_planes"] = g.get_number_of_update_send_cells() == len(ghost_planes) * plane
    note("known checked")
    _play(g, st, 1)
    note("played")
    sl = g.slot_ids()[: g.n_local]
    got = st.get(0, g.n_local)
    ok = True
    for a, b in runs:
        sel = (sl >= np.uint64(1 + a * plane)) & (sl < np.uint64(1 + b * plane))
        exp = _gol_slab_numpy(nx, ny, nz, a, b).ravel()
        ok = ok and bool(np.array_equal(got[sel], exp[(sl[sel] - np.uint64(1 + a * plane)).astype(np.int64)]))
    res["game"] = ok
    note("game checked")
    res["cells"] = int(g.n_local)
    g.close()
    return res


@pytest.mark.timeout(900)
def test_config5_full_size_two_ranks(gpu, tmp_path):
    res = _run_group(2, tmp_path, ["sc_config5"], module="test_gpu_config5")
    assert "sc_config5" in res
    for rank, (kind, out) in sorted(res["sc_config5"].items()):
        assert kind == "ok", f"rank {rank}:\n{out}"
        for k in ("local", "known", "send_planes", "game"):
            assert out[k], f"rank {rank}: {k} ({out})"
    assert sum(o["cells"] for _, o in res["sc_config5"].values()) == 2 * 1024 * 1024 * 128
