"""CPU, world_size 2 over gloo: the torch.distributed bring-up of the multi-GPU path
(shadow_amd/dist.py) and bench.py's timing protocol (barrier, max over ranks).  The RCCL
unique id is created by the native library on rank 0 (no GPU needed for that) and must reach
every rank intact; the row-block split must be the library's (routing.hip make_plan); and the
distributed FW schedule itself (shadow_amd.dist.line_fw) runs on 2-4 gloo ranks."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from shadow_amd import dist as sd
        uid = sd.share_unique_id()
        ids = [None] * world
        dist.all_gather_object(ids, uid)
        # timing protocol of bench.py: max over ranks of the per-rank elapsed time
        t = torch.tensor([0.5 + rank], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        q.put((rank, len(uid), all(x == ids[0] for x in ids), float(t.item()), sd.split_rows(79, world)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_unique_id_shared_over_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, n, same, tmax, split in res:
        assert n == 128 and same
        assert tmax == 0.5 + (world - 1)
        assert split == [(0, 39), (39, 79)]


def _plain_fw(W):
    D = W.copy()
    for k in range(D.shape[0]):
        D = np.minimum(D, D[:, k:k + 1] + D[k:k + 1, :])
    return D


def _sym_weights(V, seed):
    rng = np.random.default_rng(seed)
    W = rng.integers(1, 1000, size=(V, V)).astype(np.int64)
    W = np.minimum(W, W.T)  # symmetric, like an undirected GML graph's W
    np.fill_diagonal(W, 0)
    return W


def _line_worker(rank, world, port, q, V, T, seed):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from shadow_amd import dist as sd

        def allgatherv(buf, offs, lens):
            segs = [None] * world
            dist.all_gather_object(segs, buf[offs[rank]:offs[rank] + lens[rank]].copy())
            for r in range(world):
                if r != rank:
                    buf[offs[r]:offs[r] + lens[r]] = segs[r]

        D = sd.line_fw(_sym_weights(V, seed), T, world, rank, allgatherv)
        q.put((rank, D))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,V,T", [(2, 160, 16), (3, 192, 16), (4, 96, 8), (8, 80, 8)])
def test_line_fw_schedule_over_gloo(world, V, T):
    """The distributed symmetric FW schedule of routing.hip fw_line_sym (tile (I, J) on rank (I + J) mod G,
    one line-buffer allgather per pivot, redundant pivot closure, final tile exchange), restated in
    numpy (shadow_amd.dist.line_fw) and run on `world` gloo ranks: every rank ends with the plain
    FW closure, bit for bit (8 ranks on 10 row blocks: lines of 1-2 tiles per rank)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_line_worker, args=(r, world, port, q, V, T, 7 + world)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _plain_fw(_sym_weights(V, 7 + world))
    for rank, D in res:
        assert np.array_equal(D, ref), f"rank {rank}"


def test_ownership_and_line_slots():
    """The ownership the library computes: symmetric FW tile (I, J) -> rank (I + J) mod G balances
    every pivot's bulk and every line; a line's slots are owner-major with one contiguous segment
    per rank (kernels.hip.h LineMap); sources split by position; general FW rows by row blocks."""
    from shadow_amd import dist as sd
    nb = 79
    for G in (1, 2, 3, 4, 8):
        tiles = [0] * G
        for I in range(nb):
            for J in range(I, nb):
                tiles[sd.tile_owner(I, J, G)] += 1
        assert max(tiles) - min(tiles) <= nb // G + 1
        lm = sd.LineMap(nb, G)
        for L in (0, 1, 40, 78):
            slots = [lm.slot(j, L) for j in range(nb)]
            assert sorted(slots) == list(range(nb))
            for r in range(G):
                seg = sorted(lm.slot(j, L) for j in range(nb) if lm.owner(j, L) == r)
                assert seg == list(range(lm.base(r, L), lm.base(r, L) + lm.count(r, L)))
                assert lm.count(r, L) <= nb // G + 1
        assert sd.source_split(10000, G) == [(10000 * r // G, 10000 * (r + 1) // G) for r in range(G)]
    assert sd.split_rows(79, 2) == [(0, 39), (39, 79)]
