"""Bring-up probe: two ranks on ONE GPU through the library's RCCL communicator (gloo carries
the unique id).  RCCL may refuse two ranks on one device; either outcome is printed.  With the
communicator up, a 2-rank dense build and a 2-rank sparse build are compared bit for bit with
the single-GPU build.  usage: python -m torch.distributed.run --nproc-per-node 2 tools/rccl_two_ranks.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402

from shadow_amd import Router, synth  # noqa: E402
from shadow_amd import _native as N  # noqa: E402
from shadow_amd import dist as sd  # noqa: E402

dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
uid = sd.share_unique_id()
r = Router(0)
try:
    r.init_comm(world, rank, uid)
    print(f"[rank {rank}] RCCL communicator up: {r.comm_size()}", flush=True)
except Exception as e:  # noqa: BLE001
    print(f"[rank {rank}] RCCL init refused: {e}", flush=True)
    sys.exit(0)
for name, g, algo in [("dense", synth.atlas_like(700, seed=3), N.SRG_ALGO_DENSE),
                      ("sparse", synth.barabasi_albert(3000, 4, seed=5), N.SRG_ALGO_SPARSE)]:
    nodes = list(range(g.num_vertices))
    r.set_option(N.SRG_OPT_ALGORITHM, algo)
    got = r.compute_shortest_paths(g, nodes)
    ref_r = Router(0)
    ref_r.set_option(N.SRG_OPT_ALGORITHM, algo)
    ref = ref_r.compute_shortest_paths(g, nodes)
    ok = np.array_equal(got.latency_ns, ref.latency_ns) and np.array_equal(
        got.packet_loss.view(np.uint32), ref.packet_loss.view(np.uint32))
    print(f"[rank {rank}] {name}: 2-rank RCCL build == single-GPU build: {ok} ({got.stats['local_sources']} local sources)",
          flush=True)
dist.destroy_process_group()
