"""Multi-GPU bring-up over torch.distributed (one process per GPU).

torch.distributed is plumbing here: it launches the ranks and carries the 128-byte RCCL unique
id from rank 0 to every rank.  The collectives of the routing build itself (pivot-panel
broadcasts, essential-edge bitmask and output-row exchange) are issued by the native library
on its own RCCL communicator (shadow_amd/csrc/comm.cpp), over xGMI.
"""
import torch.distributed as dist

from .graph import Router


def share_unique_id(group=None, make_id=None):
    """Rank 0 creates the unique id, every rank returns the same 128 bytes."""
    make_id = make_id or Router.comm_unique_id
    obj = [make_id() if dist.get_rank(group) == 0 else None]
    dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    return obj[0]


def split_rows(num_blocks, nranks):
    """FW row blocks per rank, exactly as the library splits them (routing.hip make_plan):
    rank r owns blocks [r*nb//G, (r+1)*nb//G)."""
    return [(r * num_blocks // nranks, (r + 1) * num_blocks // nranks) for r in range(nranks)]


def init_router(device, group=None):
    """A Router on `device` attached to an RCCL communicator spanning the process group."""
    router = Router(device)
    ws = dist.get_world_size(group)
    if ws > 1:
        uid = share_unique_id(group)
        router.init_comm(ws, dist.get_rank(group), uid)
    return router
