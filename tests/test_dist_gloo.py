"""N > 1 path on CPU: two processes over torch.distributed (gloo).

1. The bootstrap bench.py / Dccrg.from_torch_distributed use: rank 0 creates
   the 128-byte RCCL unique id and broadcasts it; every rank holds the same id.
2. The halo wire protocol of update_copies_of_remote_neighbors
   (dccrg.hpp:10587-10997, one message per peer in ascending id order) between
   two real processes on the oracle's per-rank views: each rank sends the
   payloads of cells_to_send[peer] in list order, the receiver places them at
   cells_to_receive[peer] in list order; a distributed game of life run this
   way equals the single-process game bit for bit.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import dccrg_amd
        from oracle import oracle as O

        # 1. bootstrap id broadcast
        obj = [dccrg_amd.Dccrg.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        ids_all = [None] * world
        dist.all_gather_object(ids_all, obj[0])
        assert len(obj[0]) == 128 and all(x == ids_all[0] for x in ids_all)

        # 2. halo protocol on the oracle's per-rank views
        length, steps = (9, 7, 5), 6
        o = O.Grid(length, 0, (True, False, True), 1, world)
        cells, _ = o.cells()
        rng = np.random.default_rng(4)
        a0 = (rng.random(cells.size) < 0.3).astype(np.uint32)
        local = o.rank_cells(rank, "local")
        state = {int(c): int(a0[i]) for i, c in enumerate(cells) if int(c) in set(local.tolist())}
        peers = [p for p in range(world) if p != rank]
        nbrs = {int(c): [int(x) for x in o.iterator_neighbors_of(int(c))[0]] for c in local}
        for _ in range(steps):
            halo = {}
            reqs = []
            recv_bufs = {}
            for p in peers:
                send = o.cells_to_send(rank, p)
                recv = o.cells_to_receive(rank, p)
                sb = torch.tensor([state[int(c)] for c in send], dtype=torch.int64)
                rb = torch.empty(len(recv), dtype=torch.int64)
                recv_bufs[p] = (recv, rb)
                if sb.numel():
                    reqs.append(dist.isend(sb, p))
                if rb.numel():
                    reqs.append(dist.irecv(rb, p))
            for r in reqs:
                r.wait()
            for p, (recv, rb) in recv_bufs.items():
                for c, v in zip(recv.tolist(), rb.tolist()):
                    halo[int(c)] = int(v)
            view = dict(state)
            view.update(halo)
            new = {}
            for c in local:
                c = int(c)
                k = sum(1 for n in nbrs[c] if view[n] > 0)
                new[c] = 1 if k == 3 else (state[c] if k == 2 else 0)
            state = new
        gathered = [None] * world
        dist.all_gather_object(gathered, state)
        if rank == 0:
            full = {}
            for g in gathered:
                full.update(g)
            o1 = O.Grid(length, 0, (True, False, True), 1, 1)
            o1.gol_set(cells, a0)
            o1.gol_steps(steps)
            exp = o1.gol_get(cells)
            got = np.array([full[int(c)] for c in cells], np.uint32)
            q.put(("ok", bool(np.array_equal(got, exp))))
    except Exception as e:  # pragma: no cover
        q.put(("error", repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_bootstrap_and_halo_protocol(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    kind, val = q.get(timeout=5)
    assert kind == "ok" and val is True
