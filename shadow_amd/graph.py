"""Host-side mirror of Shadow's network-graph interface for the routing path.

Same names, argument meaning and error behaviour as the reference:
  PathProperties                 src/main/network/graph/mod.rs:296-340
  NetworkGraph.parse             mod.rs:134-181    (GML ingest, native C++ parser)
  NetworkGraph.node_id_to_index  mod.rs:126-128
  NetworkGraph.node_index_to_id  mod.rs:130-132
  NetworkGraph.compute_shortest_paths   mod.rs:183-228  (HIP, gfx950 — no CPU fallback)
  NetworkGraph.get_direct_paths  mod.rs:230-252  (HIP)
  RoutingInfo                    mod.rs:428-477            (native dense table, srg_routing_info)
  generate_routing_info          src/main/core/sim_config.rs:425-462  (srg_routing_info_build)

The reference returns HashMap<(NodeIndex, NodeIndex), PathProperties>; here the result is a
dense PathTable (row-major by position in `nodes`) that behaves like that map
(`table[(src, dst)]`, `len`, `items()`, `to_dict()`), because building 10^8 Python dict
entries would dwarf the GPU computation.
"""
import ctypes
import threading

import numpy as np

from . import _native as N


class NetGraphError(Exception):
    """Box<dyn Error> returned by NetworkGraph methods (mod.rs:18)."""

    def __init__(self, code, message):
        super().__init__(message)
        self.code = code
        self.message = message


class RoutingPanic(NetGraphError):
    """The reference panics here (assert_eq! at mod.rs:219: an unreachable used pair)."""


class HipError(RuntimeError):
    """No usable HIP device / runtime failure.  The routing builder never falls back to CPU."""

    def __init__(self, code, message):
        super().__init__(message)
        self.code = code


def _raise(code, msg):
    if code == N.SRG_ERR_UNREACHABLE:
        raise RoutingPanic(code, msg)
    if code in (N.SRG_ERR_HIP, N.SRG_ERR_OOM, N.SRG_ERR_RCCL, N.SRG_ERR_INTERNAL):
        raise HipError(code, msg)
    raise NetGraphError(code, msg)


class PathProperties:
    """Network characteristics for a path (mod.rs:296-340).

    Ordering is lexicographic (latency_ns, then packet_loss); `+` composes two paths with
    loss = 1 - (1-a)*(1-b) in float32, each operation rounded separately (no FMA)."""

    __slots__ = ("latency_ns", "packet_loss")

    def __init__(self, latency_ns=0, packet_loss=0.0):
        self.latency_ns = int(latency_ns)
        self.packet_loss = float(np.float32(packet_loss))

    def _key(self):
        return (self.latency_ns, self.packet_loss)

    def __lt__(self, o):
        return self._key() < o._key()

    def __le__(self, o):
        return self._key() <= o._key()

    def __gt__(self, o):
        return self._key() > o._key()

    def __ge__(self, o):
        return self._key() >= o._key()

    def __eq__(self, o):
        return isinstance(o, PathProperties) and self._key() == o._key()

    def __hash__(self):
        return hash(self._key())

    def __add__(self, o):
        f = np.float32
        one = f(1.0)
        loss = one - (one - f(self.packet_loss)) * (one - f(o.packet_loss))
        return PathProperties((self.latency_ns + o.latency_ns) & 0xFFFFFFFFFFFFFFFF, loss)

    def __repr__(self):
        return f"PathProperties(latency_ns={self.latency_ns}, packet_loss={self.packet_loss!r})"


class PathTable:
    """Dense result of compute_shortest_paths / get_direct_paths for `nodes` (NodeIndex)."""

    def __init__(self, nodes, latency_ns, packet_loss, stats=None):
        self.nodes = np.asarray(nodes, dtype=np.uint32)
        self.latency_ns = latency_ns
        self.packet_loss = packet_loss
        self.stats = stats
        self._pos = {int(v): i for i, v in enumerate(self.nodes)}

    def __len__(self):
        return len(self.nodes) ** 2

    def __contains__(self, key):
        a, b = key
        return a in self._pos and b in self._pos

    def __getitem__(self, key):
        a, b = key
        i, j = self._pos[a], self._pos[b]
        return PathProperties(int(self.latency_ns[i, j]), self.packet_loss[i, j])

    def get(self, key, default=None):
        return self[key] if key in self else default

    def items(self):
        for i, a in enumerate(self.nodes):
            for j, b in enumerate(self.nodes):
                yield (int(a), int(b)), PathProperties(int(self.latency_ns[i, j]), self.packet_loss[i, j])

    def to_dict(self):
        return dict(self.items())


class Router:
    """One srg_ctx (device workspace) per HIP device; thread-safe (the C side serialises)."""

    _default = {}
    _lock = threading.Lock()

    def __init__(self, device=0):
        L = N.lib()
        h = ctypes.c_void_p()
        err = ctypes.create_string_buffer(1024)
        rc = L.srg_create(ctypes.byref(h), int(device), err, len(err))
        if rc != N.SRG_OK:
            _raise(rc, err.value.decode(errors="replace"))
        self._h = h
        self.device = device

    @classmethod
    def default(cls, device=0):
        with cls._lock:
            r = cls._default.get(device)
            if r is None:
                r = cls._default[device] = Router(device)
            return r

    def set_option(self, option, value):
        rc = N.lib().srg_set_option(self._h, int(option), float(value))
        if rc != N.SRG_OK:
            _raise(rc, f"srg_set_option({option}, {value}) failed")

    def get_option(self, option):
        v = ctypes.c_double()
        rc = N.lib().srg_get_option(self._h, int(option), ctypes.byref(v))
        if rc != N.SRG_OK:
            _raise(rc, f"srg_get_option({option}) failed")
        return v.value

    def close(self):
        if getattr(self, "_h", None):
            N.lib().srg_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _run(self, fn, edges, nodes, out_lat=None, out_loss=None):
        nodes = np.ascontiguousarray(nodes, dtype=np.uint32)
        n = len(nodes)
        if out_lat is None:
            out_lat = np.zeros((n, n), dtype=np.uint64)
        if out_loss is None:
            out_loss = np.zeros((n, n), dtype=np.float32)
        assert out_lat.dtype == np.uint64 and out_lat.size == n * n and out_lat.flags.c_contiguous
        assert out_loss.dtype == np.float32 and out_loss.size == n * n and out_loss.flags.c_contiguous
        st = N.Stats()
        err = ctypes.create_string_buffer(1024)
        el = edges.as_struct()
        rc = fn(self._h, ctypes.byref(el), nodes.ctypes.data, n, out_lat.ctypes.data, out_loss.ctypes.data,
                ctypes.byref(st), err, len(err))
        if rc != N.SRG_OK:
            _raise(rc, err.value.decode(errors="replace"))
        return PathTable(nodes, out_lat, out_loss, st.as_dict())

    def compute_shortest_paths(self, edges, nodes, out_lat=None, out_loss=None):
        """Host entry (srg_compute_shortest_paths): host edge list in, host n x n table out.
        out_lat (u64) / out_loss (f32) may be caller-provided n x n arrays (reused buffers)."""
        return self._run(N.lib().srg_compute_shortest_paths, edges, nodes, out_lat, out_loss)

    # ---- multi-GPU (include/shadow_routing.h srg_comm_*) ----------------------------------
    @staticmethod
    def comm_unique_id():
        """128-byte RCCL unique id (rank 0 creates it; share it with every rank)."""
        buf = ctypes.create_string_buffer(N.SRG_UNIQUE_ID_BYTES)
        err = ctypes.create_string_buffer(1024)
        rc = N.lib().srg_comm_unique_id(buf, err, len(err))
        if rc != N.SRG_OK:
            _raise(rc, err.value.decode(errors="replace"))
        return buf.raw

    def init_comm(self, nranks, rank, unique_id):
        """Attach an RCCL communicator: later calls run SPMD across `nranks` GPUs."""
        assert len(unique_id) == N.SRG_UNIQUE_ID_BYTES
        err = ctypes.create_string_buffer(1024)
        rc = N.lib().srg_comm_init(self._h, int(nranks), int(rank), bytes(unique_id), err, len(err))
        if rc != N.SRG_OK:
            _raise(rc, err.value.decode(errors="replace"))

    def init_comm_local(self, group, rank):
        """Attach rank `rank` of an in-process LocalGroup (ranks are threads of this process)."""
        err = ctypes.create_string_buffer(1024)
        rc = N.lib().srg_comm_init_local(self._h, group._h, int(rank), err, len(err))
        if rc != N.SRG_OK:
            _raise(rc, err.value.decode(errors="replace"))

    def comm_size(self):
        nr, rk = ctypes.c_int(), ctypes.c_int()
        N.lib().srg_comm_size(self._h, ctypes.byref(nr), ctypes.byref(rk))
        return nr.value, rk.value

    def get_direct_paths(self, edges, nodes):
        return self._run(N.lib().srg_get_direct_paths, edges, nodes)


class MultiRouter:
    """srg_multi: ONE call site driving several GPUs of this process (Shadow's one-process model).

    compute_shortest_paths has Router.compute_shortest_paths' arguments and result: the whole
    n x n table lands in the caller's arrays, each GPU writing its own sources' rows."""

    def __init__(self, devices):
        devices = [int(d) for d in devices]
        arr = (ctypes.c_int * len(devices))(*devices)
        h = ctypes.c_void_p()
        err = ctypes.create_string_buffer(1024)
        rc = N.lib().srg_multi_create(ctypes.byref(h), arr, len(devices), err, len(err))
        if rc != N.SRG_OK:
            _raise(rc, err.value.decode(errors="replace"))
        self._h = h
        self.devices = devices

    def __len__(self):
        return int(N.lib().srg_multi_size(self._h))

    def set_option(self, option, value):
        rc = N.lib().srg_multi_set_option(self._h, int(option), float(value))
        if rc != N.SRG_OK:
            _raise(rc, f"srg_multi_set_option({option}, {value}) failed")

    def close(self):
        if getattr(self, "_h", None):
            N.lib().srg_multi_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def compute_shortest_paths(self, edges, nodes, out_lat=None, out_loss=None):
        return Router._run(self, N.lib().srg_multi_compute_shortest_paths, edges, nodes, out_lat, out_loss)


class LocalGroup:
    """srg_local_group: N ranks inside one process (threads), e.g. several ranks on one GPU."""

    def __init__(self, nranks):
        h = ctypes.c_void_p()
        rc = N.lib().srg_local_group_create(int(nranks), ctypes.byref(h))
        if rc != N.SRG_OK:
            _raise(rc, "srg_local_group_create failed")
        self._h = h
        self.nranks = nranks

    def close(self):
        if getattr(self, "_h", None):
            N.lib().srg_local_group_release(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Edges:
    """Edge list in petgraph raw_edges() order (the C-ABI's srg_edge_list, host memory)."""

    def __init__(self, num_vertices, src, dst, latency_ns, packet_loss, directed=False, node_ids=None):
        self.num_vertices = int(num_vertices)
        self.directed = bool(directed)
        self.src = np.ascontiguousarray(src, dtype=np.uint32)
        self.dst = np.ascontiguousarray(dst, dtype=np.uint32)
        self.latency_ns = np.ascontiguousarray(latency_ns, dtype=np.uint64)
        self.packet_loss = np.ascontiguousarray(packet_loss, dtype=np.float32)
        self.node_ids = None if node_ids is None else np.ascontiguousarray(node_ids, dtype=np.uint32)
        assert len(self.src) == len(self.dst) == len(self.latency_ns) == len(self.packet_loss)

    @property
    def num_edges(self):
        return len(self.src)

    def as_struct(self):
        return N.EdgeList(self.num_vertices, int(self.directed), self.num_edges, self.src.ctypes.data,
                          self.dst.ctypes.data, self.latency_ns.ctypes.data, self.packet_loss.ctypes.data,
                          None if self.node_ids is None else self.node_ids.ctypes.data)

    def as_tuple(self):
        """(V, directed, src, dst, lat, loss, node_ids) -- the oracle's graph argument."""
        return (self.num_vertices, self.directed, self.src, self.dst, self.latency_ns, self.packet_loss,
                self.node_ids)


class NetworkGraph:
    """A network graph: the parsed GML graph plus GML-id <-> NodeIndex maps (mod.rs:113-181)."""

    def __init__(self, edges, bandwidth_down=None, bandwidth_up=None):
        self.edges = edges
        ids = edges.node_ids if edges.node_ids is not None else np.arange(edges.num_vertices, dtype=np.uint32)
        self._ids = ids
        self._id_to_index = {}
        for i, gid in enumerate(ids.tolist()):
            self._id_to_index[gid] = i  # later duplicates win (HashMap::insert, mod.rs:161)
        self.bandwidth_down = bandwidth_down
        self.bandwidth_up = bandwidth_up

    @staticmethod
    def parse(graph_text):
        """NetworkGraph::parse (mod.rs:134-181) via the native GML parser."""
        L = N.lib()
        data = graph_text.encode("utf-8") if isinstance(graph_text, str) else bytes(graph_text)
        h = ctypes.c_void_p()
        err = ctypes.create_string_buffer(2048)
        rc = L.srg_graph_parse_gml(data, len(data), ctypes.byref(h), err, len(err))
        if rc != N.SRG_OK:
            _raise(rc, err.value.decode(errors="replace"))
        try:
            el = N.EdgeList()
            L.srg_graph_edge_list(h, ctypes.byref(el))
            V, E = el.num_vertices, el.num_edges

            def arr(ptr, ctype, count, dtype):
                if count == 0:
                    return np.zeros(0, dtype=dtype)
                return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctype)), shape=(count,)).copy()

            edges = Edges(V, arr(el.src, ctypes.c_uint32, E, np.uint32), arr(el.dst, ctypes.c_uint32, E, np.uint32),
                          arr(el.latency_ns, ctypes.c_uint64, E, np.uint64),
                          arr(el.packet_loss, ctypes.c_float, E, np.float32), bool(el.directed),
                          arr(el.node_ids, ctypes.c_uint32, V, np.uint32))
            d, u = np.zeros(V, np.uint64), np.zeros(V, np.uint64)
            hd, hu = np.zeros(V, np.int32), np.zeros(V, np.int32)
            if V:
                L.srg_graph_node_bandwidths(h, d.ctypes.data, hd.ctypes.data, u.ctypes.data, hu.ctypes.data)
            down = [int(x) if k else None for x, k in zip(d.tolist(), hd.tolist())]
            up = [int(x) if k else None for x, k in zip(u.tolist(), hu.tolist())]
            chunks = int(L.srg_graph_parse_chunks(h))
        finally:
            L.srg_graph_free(h)
        g = NetworkGraph(edges, down, up)
        g.parse_chunks = chunks
        return g

    @property
    def directed(self):
        return self.edges.directed

    def num_nodes(self):
        return self.edges.num_vertices

    def node_id_to_index(self, gml_id):
        return self._id_to_index.get(gml_id)

    def node_index_to_id(self, index):
        if 0 <= index < self.edges.num_vertices:
            return int(self._ids[index])
        return None

    def compute_shortest_paths(self, nodes, router=None):
        """NetworkGraph::compute_shortest_paths (mod.rs:183-228) on the GPU."""
        return (router or Router.default()).compute_shortest_paths(self.edges, nodes)

    def get_direct_paths(self, nodes, router=None):
        """NetworkGraph::get_direct_paths (mod.rs:230-252) on the GPU."""
        return (router or Router.default()).get_direct_paths(self.edges, nodes)


class RoutingInfo:
    """RoutingInfo<u32> (mod.rs:428-477) backed by the native dense table (srg_routing_info):
    path(start, end) by GML id, packet counters with saturating_add, get_smallest_latency_ns."""

    def __init__(self, handle, stats=None):
        self._h = handle
        self.stats = stats

    def close(self):
        if getattr(self, "_h", None):
            N.lib().srg_routing_info_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def path(self, start, end):
        lat, loss = ctypes.c_uint64(), ctypes.c_float()
        if not N.lib().srg_routing_info_path(self._h, int(start), int(end), ctypes.byref(lat), ctypes.byref(loss)):
            return None
        return PathProperties(lat.value, loss.value)

    def increment_packet_count(self, start, end):
        N.lib().srg_routing_info_increment_packet_count(self._h, int(start), int(end))

    def packet_count(self, start, end):
        return int(N.lib().srg_routing_info_packet_count(self._h, int(start), int(end)))

    def get_smallest_latency_ns(self):
        v = ctypes.c_uint64()
        if not N.lib().srg_routing_info_smallest_latency_ns(self._h, ctypes.byref(v)):
            return None
        return int(v.value)

    def tables(self):
        """(latency_ns u64 [n, n], packet_loss f32 [n, n], gml_ids u32 [n]) -- zero-copy views of the
        native tables.  Each array keeps this RoutingInfo alive (its numpy base holds a reference),
        so the native memory outlives every view even when the RoutingInfo itself is dropped."""
        lp, fp, ip, n = N._u64p(), N._f32p(), N._u32p(), ctypes.c_uint32()
        N.lib().srg_routing_info_tables(self._h, ctypes.byref(lp), ctypes.byref(fp), ctypes.byref(ip), ctypes.byref(n))
        n = n.value
        if n == 0:
            return (np.zeros((0, 0), np.uint64), np.zeros((0, 0), np.float32), np.zeros(0, np.uint32))

        def view(ptr, ctype, shape):
            buf = (ctype * int(np.prod(shape))).from_address(ctypes.addressof(ptr.contents))
            buf._owner = self  # the ctypes array holds the owner; numpy's base chain holds the array
            return np.ctypeslib.as_array(buf).reshape(shape)

        return (view(lp, ctypes.c_uint64, (n, n)), view(fp, ctypes.c_float, (n, n)), view(ip, ctypes.c_uint32, (n,)))

    def __len__(self):
        return int(N.lib().srg_routing_info_num_nodes(self._h)) ** 2


def generate_routing_info(graph, nodes, use_shortest_paths=True, router=None):
    """sim_config.rs:425-462 through srg_routing_info_build (srg_routing_info_build_multi for a
    MultiRouter): GML ids -> NodeIndex, shortest or direct paths on the GPU(s), a dense RoutingInfo
    keyed by GML id (no n^2 HashMap)."""
    router = router or Router.default()
    ids = np.ascontiguousarray(list(nodes), dtype=np.uint32)
    edges = graph.edges if isinstance(graph, NetworkGraph) else graph
    if edges.node_ids is None and isinstance(graph, NetworkGraph):
        edges = Edges(edges.num_vertices, edges.src, edges.dst, edges.latency_ns, edges.packet_loss, edges.directed,
                      graph._ids)
    el = edges.as_struct()
    h = ctypes.c_void_p()
    st = N.Stats()
    err = ctypes.create_string_buffer(2048)
    build = N.lib().srg_routing_info_build_multi if isinstance(router, MultiRouter) else N.lib().srg_routing_info_build
    rc = build(router._h, ctypes.byref(el), ids.ctypes.data, len(ids), 1 if use_shortest_paths else 0, ctypes.byref(h),
               ctypes.byref(st), err, len(err))
    if rc != N.SRG_OK:
        _raise(rc, err.value.decode(errors="replace"))
    return RoutingInfo(h, st.as_dict())
