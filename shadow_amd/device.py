"""Device-resident entry point: inputs and outputs already in HBM (torch tensors as plumbing).

Calls srg_compute_shortest_paths_device (include/shadow_routing.h) on the tensors' device
pointers and torch's current HIP stream.  This is what bench.py times.
"""
import ctypes

import numpy as np
import torch

from . import _native as N
from .graph import Router, _raise


class DeviceGraph:
    """An Edges list copied to HBM once (uint32/uint64 data held in int32/int64 tensors)."""

    def __init__(self, edges, device="cuda:0"):
        dev = torch.device(device)
        self.num_vertices = edges.num_vertices
        self.directed = edges.directed
        self.num_edges = edges.num_edges
        self.src = torch.from_numpy(edges.src.view(np.int32)).to(dev)
        self.dst = torch.from_numpy(edges.dst.view(np.int32)).to(dev)
        self.lat = torch.from_numpy(edges.latency_ns.view(np.int64)).to(dev)
        self.loss = torch.from_numpy(edges.packet_loss).to(dev)
        self.ids = None if edges.node_ids is None else torch.from_numpy(edges.node_ids.view(np.int32)).to(dev)

    def as_struct(self):
        return N.EdgeList(self.num_vertices, int(self.directed), self.num_edges, self.src.data_ptr(),
                          self.dst.data_ptr(), self.lat.data_ptr(), self.loss.data_ptr(),
                          None if self.ids is None else self.ids.data_ptr())


def compute_shortest_paths_device(router, dgraph, nodes_t, out_lat_t, out_loss_t, stream=None):
    """nodes_t int32[n] (NodeIndex), out_lat_t int64[n,n], out_loss_t float32[n,n] on the GPU."""
    n = nodes_t.numel()
    assert out_lat_t.numel() == n * n and out_loss_t.numel() == n * n
    assert out_lat_t.dtype == torch.int64 and out_loss_t.dtype == torch.float32 and nodes_t.dtype == torch.int32
    assert nodes_t.is_contiguous() and out_lat_t.is_contiguous() and out_loss_t.is_contiguous()
    st = N.Stats()
    err = ctypes.create_string_buffer(1024)
    el = dgraph.as_struct()
    s = stream if stream is not None else torch.cuda.current_stream(nodes_t.device)
    rc = N.lib().srg_compute_shortest_paths_device(
        router._h, ctypes.byref(el), nodes_t.data_ptr(), n, out_lat_t.data_ptr(), out_loss_t.data_ptr(),
        ctypes.c_void_p(s.cuda_stream), ctypes.byref(st), err, len(err))
    if rc != N.SRG_OK:
        _raise(rc, err.value.decode(errors="replace"))
    return st.as_dict()


def set_profiling(router, enable):
    router.set_option(N.SRG_OPT_PROFILING, 1 if enable else 0)


__all__ = ["DeviceGraph", "Router", "compute_shortest_paths_device", "set_profiling"]
