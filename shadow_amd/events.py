"""Stretch row f4: one scheduling round's cross-host packet-event batch on the GPU.

Host-side mirror of the reference's per-packet path, batched (srg_order_packet_events_device,
include/shadow_routing.h):
  Worker::send_packet      src/main/core/worker.rs:391-424  latency lookup, deliver time raised
                                                            to the round end, runahead / next
                                                            event bookkeeping
  push_packet_to_host      worker.rs:644-654                one EventQueue per destination host
  EventQueue / Event order event_queue.rs:38-49, event.rs:84-155
  min next event           manager.rs:459-464
The latency table is the dense routing table (RoutingInfo's backing store), e.g. the
`latency_ns` matrix of a PathTable, kept in HBM.  torch tensors are only HBM containers here.
"""
import ctypes

import numpy as np
import torch

from . import _native as N
from .graph import NetGraphError, _raise

FIELDS_U32 = ("src_node", "dst_node", "src_host", "dst_host")
FIELDS_U64 = ("send_time_ns", "src_event_id")


class EventOrderError(NetGraphError):
    """Two events with no relative order: the reference's PanickingOrd unwrap panic."""


def _i32(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32).view(np.int32)).to(dev)


def _i64(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(dev)


class DeviceEventBatch:
    """An event batch resident in HBM (uint32/uint64 data held in int32/int64 tensors)."""

    def __init__(self, batch, num_hosts, round_end_ns, device="cuda:0"):
        dev = torch.device(device)
        self.n = len(batch["send_time_ns"])
        self.num_hosts = int(num_hosts)
        self.round_end_ns = int(round_end_ns)
        self.t = {k: _i32(batch[k], dev) for k in FIELDS_U32}
        self.t.update({k: _i64(batch[k], dev) for k in FIELDS_U64})

    def as_struct(self):
        p = {k: v.data_ptr() for k, v in self.t.items()}
        return N.EventBatch(self.n, p["src_node"], p["dst_node"], p["src_host"], p["dst_host"], p["send_time_ns"],
                            p["src_event_id"], self.num_hosts, 0, self.round_end_ns)


def order_packet_events_device(router, dbatch, table_t, out_deliver_t, out_order_t, out_host_off_t, stream=None):
    """table_t int64 [tn, tn]; outputs int64[n], int32[n], int64[num_hosts + 1] on the GPU."""
    assert table_t.dtype == torch.int64 and table_t.dim() == 2 and table_t.shape[0] == table_t.shape[1]
    assert out_deliver_t.numel() == dbatch.n and out_order_t.numel() == dbatch.n
    assert out_host_off_t.numel() == dbatch.num_hosts + 1
    res = N.EventResult()
    err = ctypes.create_string_buffer(1024)
    b = dbatch.as_struct()
    s = stream if stream is not None else torch.cuda.current_stream(table_t.device)
    rc = N.lib().srg_order_packet_events_device(
        router._h, ctypes.byref(b), table_t.data_ptr(), table_t.shape[0], out_deliver_t.data_ptr(),
        out_order_t.data_ptr(), out_host_off_t.data_ptr(), ctypes.c_void_p(s.cuda_stream), ctypes.byref(res), err,
        len(err))
    if rc == N.SRG_ERR_EVENT_ORDER:
        raise EventOrderError(rc, err.value.decode(errors="replace"))
    if rc != N.SRG_OK:
        _raise(rc, err.value.decode(errors="replace"))
    return res.as_dict()


def order_packet_events(router, batch, table, num_hosts, round_end_ns, device=None):
    """Host arrays in, host arrays out: (deliver u64[n], order u32[n], host_offsets u64[H+1], result)."""
    dev = torch.device(device or f"cuda:{router.device}")
    db = DeviceEventBatch(batch, num_hosts, round_end_ns, dev)
    tab = _i64(np.asarray(table), dev)
    n = db.n
    deliver = torch.empty(max(n, 1), dtype=torch.int64, device=dev)[:n]
    order = torch.empty(max(n, 1), dtype=torch.int32, device=dev)[:n]
    off = torch.empty(db.num_hosts + 1, dtype=torch.int64, device=dev)
    res = order_packet_events_device(router, db, tab, deliver, order, off)
    torch.cuda.synchronize(dev)
    return (deliver.cpu().numpy().view(np.uint64), order.cpu().numpy().view(np.uint32),
            off.cpu().numpy().view(np.uint64), res)


def synthetic_round(n, num_hosts, table_n, seed=7, t0=10**12, runahead=5_000_000):
    """n events, send times uniform in one round window [t0, t0 + runahead),
    src/dst hosts uniform, per-source monotone event ids, hosts mapped to table rows."""
    rng = np.random.default_rng(seed)
    src_host = rng.integers(0, num_hosts, n, dtype=np.uint32)
    dst_host = rng.integers(0, num_hosts, n, dtype=np.uint32)
    host_node = rng.integers(0, table_n, num_hosts, dtype=np.uint32)
    send = (t0 + rng.integers(0, runahead, n, dtype=np.uint64)).astype(np.uint64)
    # per-source monotone counters (Host::get_new_event_id) in send order
    order = np.lexsort((send, src_host))
    eid = np.empty(n, dtype=np.uint64)
    starts = np.r_[0, np.flatnonzero(np.diff(src_host[order])) + 1]
    counts = np.diff(np.r_[starts, n])
    eid[order] = (np.arange(n) - np.repeat(starts, counts)).astype(np.uint64) + 1
    return dict(src_node=host_node[src_host], dst_node=host_node[dst_host], src_host=src_host, dst_host=dst_host,
                send_time_ns=send, src_event_id=eid), t0 + runahead
