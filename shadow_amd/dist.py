"""Multi-GPU bring-up over torch.distributed (one process per GPU), and a numpy
statement of the distributed FW schedule.

torch.distributed is plumbing here: it launches the ranks and carries the 128-byte RCCL unique
id from rank 0 to every rank.  The collectives of the routing build itself (line-buffer
allgathers, packed-triangle exchange, output rows) are issued by the native library on its own
RCCL communicator (shadow_amd/csrc/comm.hip), over xGMI.

`line_fw` restates, in numpy, the schedule routing.hip fw_line_sym runs on the GPUs (skewed tile
ownership, owner-major line slots, per-pivot line exchange, redundant closure, write-backs,
final tile exchange) over any
allgatherv -- tests/test_dist_cpu.py runs it on gloo ranks against a plain FW, so the protocol
is exercised on CPU with world size > 1.  It is a specification of the schedule, not a product
path: the library never calls it.
"""
import numpy as np
import torch.distributed as dist

from .graph import Router


def share_unique_id(group=None, make_id=None):
    """Rank 0 creates the unique id, every rank returns the same 128 bytes."""
    make_id = make_id or Router.comm_unique_id
    obj = [make_id() if dist.get_rank(group) == 0 else None]
    dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    return obj[0]


def split_rows(num_blocks, nranks):
    """Row blocks of the general (non-symmetric) FW: [r*nb//G, (r+1)*nb//G) (routing.hip make_plan)."""
    return [(r * num_blocks // nranks, (r + 1) * num_blocks // nranks) for r in range(nranks)]


def tile_owner(I, J, nranks):
    """Symmetric FW: the stored tile (I, J), I <= J, belongs to rank (I + J) mod G."""
    return (I + J) % nranks


class LineMap:
    """kernels.hip.h LineMap: owner-major slots of a line buffer, so that each rank's tiles of
    line L (tile j = (min(j, L), max(j, L)), owner (j + L) mod G) are one contiguous segment."""

    def __init__(self, nb, nranks):
        self.nb, self.G = nb, nranks

    def j0(self, r, L):
        return (r - L) % self.G

    def count(self, r, L):
        a = self.j0(r, L)
        return (self.nb - 1 - a) // self.G + 1 if a < self.nb else 0

    def base(self, r, L):
        return sum(self.count(q, L) for q in range(r))

    def owner(self, j, L):
        return (j + L) % self.G

    def slot(self, j, L):
        r = self.owner(j, L)
        return self.base(r, L) + (j - self.j0(r, L)) // self.G


def source_split(n, nranks):
    """Sources per rank: positions [n r / G, n (r+1) / G) of `nodes` (its output rows)."""
    return [(n * r // nranks, n * (r + 1) // nranks) for r in range(nranks)]


def _tile(D, T, I, J):
    return D[I * T:(I + 1) * T, J * T:(J + 1) * T]


def _minplus(A, B):
    return (A[:, :, None] + B[None, :, :]).min(axis=1)


def _close(P):
    P = P.copy()
    for k in range(P.shape[0]):
        P = np.minimum(P, P[:, k:k + 1] + P[k:k + 1, :])
    return P


def line_fw(D, T, nranks, rank, allgatherv):
    """The symmetric line-buffer FW of routing.hip fw_line_sym, on rank `rank` of `nranks`.

    D: this rank's copy of the initial symmetric distance matrix (V = nb*T, int64, 0 diagonal);
    every rank starts from the same D.  allgatherv(buf, offs, lens) fills the other ranks'
    [offs[r], offs[r] + lens[r]) segments of the 1-D array `buf` from their copies.  Returns this
    rank's D after the final tile exchange (the whole closed matrix)."""
    D = D.copy()
    V = D.shape[0]
    nb = V // T
    lm = LineMap(nb, nranks)
    own = lambda I, J: tile_owner(I, J, nranks) == rank  # noqa: E731

    def stored(j, L):  # stored tile (min, max) of line L
        return min(j, L), max(j, L)

    def product(C, lb, P, I, J):  # C = min(C, D[I][P] (x) D[P][J]) through line P's buffer
        A = lb[lm.slot(I, P)] if I <= P else lb[lm.slot(I, P)].T
        B = lb[lm.slot(J, P)] if J >= P else lb[lm.slot(J, P)].T
        return np.minimum(C, _minplus(A, B))

    def close_and_line(lb, L):  # steps 3 and 4: redundant closure, line L w.r.t. L, own tiles back
        p = lm.slot(L, L)
        lb[p] = _close(lb[p])
        if own(L, L):
            _tile(D, T, L, L)[:] = lb[p]
        for j in range(nb):
            if j == L:
                continue
            I, J = stored(j, L)
            lb[lm.slot(j, L)] = product(lb[lm.slot(j, L)], lb, L, I, J)
            if own(I, J):
                _tile(D, T, I, J)[:] = lb[lm.slot(j, L)]

    # line 0: every rank holds the same initial D
    lb = np.zeros((nb, T, T), dtype=D.dtype)
    for j in range(nb):
        lb[lm.slot(j, 0)] = _tile(D, T, *stored(j, 0))
    close_and_line(lb, 0)
    for kb in range(nb):
        k1 = kb + 1
        if k1 < nb:
            nxt = np.zeros_like(lb)
            for m in range(lm.count(rank, k1)):  # step 1: own tiles of line k1 w.r.t. kb
                j = lm.j0(rank, k1) + nranks * m
                I, J = stored(j, k1)
                if j == kb:  # (kb, k1) is final in line kb
                    nxt[lm.slot(j, k1)] = lb[lm.slot(k1, kb)]
                    continue
                _tile(D, T, I, J)[:] = product(_tile(D, T, I, J), lb, kb, I, J)
                nxt[lm.slot(j, k1)] = _tile(D, T, I, J)
            flat = nxt.reshape(-1)  # step 2
            allgatherv(flat, [lm.base(r, k1) * T * T for r in range(nranks)],
                       [lm.count(r, k1) * T * T for r in range(nranks)])
            nxt = flat.reshape(nb, T, T)
            close_and_line(nxt, k1)  # steps 3, 4
        # bulk of kb: own stored tiles off lines kb and k1, through line kb
        for I in range(nb):
            for J in range(I, nb):
                if own(I, J) and not ({I, J} & {kb, k1}):
                    _tile(D, T, I, J)[:] = product(_tile(D, T, I, J), lb, kb, I, J)
        if k1 < nb:
            lb = nxt
    # every rank ends with the whole D: own tiles packed owner-major, all-gathered, unpacked + mirror
    tri = [(I, J) for I in range(nb) for J in range(I, nb)]
    order = sorted(range(len(tri)), key=lambda t: (tile_owner(*tri[t], nranks), t))
    slot = {t: i for i, t in enumerate(order)}
    P = np.zeros((len(tri), T, T), dtype=D.dtype)
    for t, (I, J) in enumerate(tri):
        if own(I, J):
            P[slot[t]] = _tile(D, T, I, J)
    first = [sum(1 for t in range(len(tri)) if tile_owner(*tri[t], nranks) < r) for r in range(nranks + 1)]
    flat = P.reshape(-1)
    allgatherv(flat, [first[r] * T * T for r in range(nranks)], [(first[r + 1] - first[r]) * T * T for r in range(nranks)])
    P = flat.reshape(len(tri), T, T)
    for t, (I, J) in enumerate(tri):
        _tile(D, T, I, J)[:] = P[slot[t]]
        _tile(D, T, J, I)[:] = P[slot[t]].T
    return D


def init_router(device, group=None):
    """A Router on `device` attached to an RCCL communicator spanning the process group."""
    router = Router(device)
    ws = dist.get_world_size(group)
    if ws > 1:
        uid = share_unique_id(group)
        router.init_comm(ws, dist.get_rank(group), uid)
    return router
