"""CPU, world_size 2 over gloo: the torch.distributed bring-up of the multi-GPU path
(shadow_amd/dist.py) and bench.py's timing protocol (barrier, max over ranks).  The RCCL
unique id is created by the native library on rank 0 (no GPU needed for that) and must reach
every rank intact; the row-block split must be the library's (routing.hip make_plan)."""
import os
import socket

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
