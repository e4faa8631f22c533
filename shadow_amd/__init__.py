"""shadow_amd — MI355X-native routing-table builder for the Shadow network simulator.

One hot path, rebuilt for gfx950: NetworkGraph::compute_shortest_paths -> RoutingInfo
(src/main/network/graph/mod.rs:183-228) as hand-written HIP kernels behind the C ABI in
include/shadow_routing.h.  See DESIGN.md.
"""
from .graph import (Edges, HipError, LocalGroup, MultiRouter, NetGraphError, NetworkGraph, PathProperties, PathTable,
                    Router, RoutingInfo, RoutingPanic, generate_routing_info)

__all__ = ["Edges", "HipError", "LocalGroup", "MultiRouter", "NetGraphError", "NetworkGraph", "PathProperties", "PathTable", "Router",
           "RoutingInfo", "RoutingPanic", "generate_routing_info"]
