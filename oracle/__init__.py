"""CPU oracle for the routing-table path — TEST / BENCH INFRASTRUCTURE ONLY.

Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
checker or the timed CPU baseline; the product (shadow_amd) never imports this package.

ctypes wrapper over oracle/liboracle.so (oracle/oracle.cpp, a C++ restatement of
src/main/network/graph/mod.rs:183-340 + petgraph 0.6.5 dijkstra).  Parity of the
restatement is pinned by the reference's own KATs (mod.rs:515-647, replayed in
tests/test_oracle.py) and by tests/golden/ fixtures built with an independent numpy-f32
Dijkstra (tests/golden/make_golden.py).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_f32p = ctypes.POINTER(ctypes.c_float)


def build():
    src = os.path.join(_HERE, "oracle.cpp")
    if not os.path.exists(_LIB_PATH) or os.path.getmtime(src) > os.path.getmtime(_LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_compute_shortest_paths.restype = ctypes.c_int
        L.oracle_compute_shortest_paths.argtypes = [
            ctypes.c_uint32, ctypes.c_int, ctypes.c_uint64, _u32p, _u32p, _u64p, _f32p, _u32p,
            _u32p, ctypes.c_uint32, _u32p, ctypes.c_uint32, _u64p, _f32p, ctypes.c_int, ctypes.c_int,
            ctypes.c_char_p, ctypes.c_size_t]
        L.oracle_get_direct_paths.restype = ctypes.c_int
        L.oracle_get_direct_paths.argtypes = [
            ctypes.c_uint32, ctypes.c_int, ctypes.c_uint64, _u32p, _u32p, _u64p, _f32p, _u32p,
            _u32p, ctypes.c_uint32, _u64p, _f32p, ctypes.c_char_p, ctypes.c_size_t]
        L.oracle_path_add.restype = None
        L.oracle_path_add.argtypes = [ctypes.c_uint64, ctypes.c_float, ctypes.c_uint64, ctypes.c_float,
                                      _u64p, _f32p]
        L.oracle_time_sources.restype = ctypes.c_double
        L.oracle_time_sources.argtypes = [
            ctypes.c_uint32, ctypes.c_int, ctypes.c_uint64, _u32p, _u32p, _u64p, _f32p, _u32p,
            ctypes.c_uint32, _u32p, ctypes.c_uint32, ctypes.c_int, _u64p]
        L.oracle_time_sources_mode.restype = ctypes.c_double
        L.oracle_time_sources_mode.argtypes = [
            ctypes.c_uint32, ctypes.c_int, ctypes.c_uint64, _u32p, _u32p, _u64p, _f32p, _u32p,
            ctypes.c_uint32, _u32p, ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
            _u64p]
        L.oracle_hw_threads.restype = ctypes.c_int
        L.oracle_order_packet_events.restype = ctypes.c_int
        L.oracle_order_packet_events.argtypes = [
            ctypes.c_uint64, _u32p, _u32p, _u32p, _u32p, _u64p, _u64p, _u64p, ctypes.c_uint32, ctypes.c_uint32,
            ctypes.c_uint64, _u64p, _u32p, _u64p, _u64p, _u64p]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t) if a is not None else None


class OracleError(Exception):
    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code
        self.msg = msg


def _graph_arrays(g):
    V, directed, src, dst, lat, loss, ids = g
    src = np.ascontiguousarray(src, dtype=np.uint32)
    dst = np.ascontiguousarray(dst, dtype=np.uint32)
    lat = np.ascontiguousarray(lat, dtype=np.uint64)
    loss = np.ascontiguousarray(loss, dtype=np.float32)
    ids = None if ids is None else np.ascontiguousarray(ids, dtype=np.uint32)
    return int(V), int(bool(directed)), src, dst, lat, loss, ids


def compute_shortest_paths(graph, nodes, rows=None, mode=1, nthreads=0):
    """graph = (V, directed, src, dst, lat_ns, loss, node_ids|None); nodes = NodeIndex list.
    Returns (lat u64 [R x n], loss f32 [R x n]) with R = n (or len(rows)), ordered by position
    in `nodes`.  mode 0 = reference-equivalent plumbing, 1 = fast dense membership."""
    V, d, src, dst, lat, loss, ids = _graph_arrays(graph)
    nodes = np.ascontiguousarray(nodes, dtype=np.uint32)
    n = len(nodes)
    rws = None if rows is None else np.ascontiguousarray(rows, dtype=np.uint32)
    R = n if rws is None else len(rws)
    out_lat = np.zeros((R, n), dtype=np.uint64)
    out_loss = np.zeros((R, n), dtype=np.float32)
    err = ctypes.create_string_buffer(512)
    rc = lib().oracle_compute_shortest_paths(
        V, d, len(src), _p(src, _u32p), _p(dst, _u32p), _p(lat, _u64p), _p(loss, _f32p),
        _p(ids, _u32p), _p(nodes, _u32p), n, _p(rws, _u32p), R, _p(out_lat, _u64p),
        _p(out_loss, _f32p), mode, nthreads, err, len(err))
    if rc:
        raise OracleError(rc, err.value.decode())
    return out_lat, out_loss


def get_direct_paths(graph, nodes):
    V, d, src, dst, lat, loss, ids = _graph_arrays(graph)
    nodes = np.ascontiguousarray(nodes, dtype=np.uint32)
    n = len(nodes)
    out_lat = np.zeros((n, n), dtype=np.uint64)
    out_loss = np.zeros((n, n), dtype=np.float32)
    err = ctypes.create_string_buffer(512)
    rc = lib().oracle_get_direct_paths(
        V, d, len(src), _p(src, _u32p), _p(dst, _u32p), _p(lat, _u64p), _p(loss, _f32p),
        _p(ids, _u32p), _p(nodes, _u32p), n, _p(out_lat, _u64p), _p(out_loss, _f32p), err, len(err))
    if rc:
        raise OracleError(rc, err.value.decode())
    return out_lat, out_loss


def path_add(a, b):
    """PathProperties + PathProperties (mod.rs:322-331); a, b = (latency_ns, packet_loss)."""
    lo = ctypes.c_uint64()
    fo = ctypes.c_float()
    lib().oracle_path_add(a[0], a[1], b[0], b[1], ctypes.byref(lo), ctypes.byref(fo))
    return lo.value, fo.value


def time_sources(graph, nodes, sample, nthreads=0):
    """Reference-equivalent CPU pipeline over a sample of source positions; returns seconds."""
    V, d, src, dst, lat, loss, _ = _graph_arrays(graph)
    nodes = np.ascontiguousarray(nodes, dtype=np.uint32)
    sample = np.ascontiguousarray(sample, dtype=np.uint32)
    cs = ctypes.c_uint64()
    return lib().oracle_time_sources(
        V, d, len(src), _p(src, _u32p), _p(dst, _u32p), _p(lat, _u64p), _p(loss, _f32p),
        _p(nodes, _u32p), len(nodes), _p(sample, _u32p), len(sample), nthreads, ctypes.byref(cs))


def time_sources_mode(graph, nodes, sample, nthreads=0, mode=0):
    """CPU-baseline timer: mode 0 reference-equivalent, 1 CPU-best heap Dijkstra (sparse), 2 CPU-best
    dense-matrix Dijkstra.  Returns (seconds for the sample, one-time setup seconds)."""
    V, d, src, dst, lat, loss, _ = _graph_arrays(graph)
    nodes = np.ascontiguousarray(nodes, dtype=np.uint32)
    sample = np.ascontiguousarray(sample, dtype=np.uint32)
    cs = ctypes.c_uint64()
    setup = ctypes.c_double()
    t = lib().oracle_time_sources_mode(
        V, d, len(src), _p(src, _u32p), _p(dst, _u32p), _p(lat, _u64p), _p(loss, _f32p),
        _p(nodes, _u32p), len(nodes), _p(sample, _u32p), len(sample), nthreads, mode, ctypes.byref(setup),
        ctypes.byref(cs))
    return t, setup.value


def hw_threads():
    return lib().oracle_hw_threads()


def order_packet_events(batch, table, num_hosts, round_end):
    """Stretch C5 restatement (worker.rs:391-424, event.rs:84-155, manager.rs:459-464).
    batch: dict of numpy arrays src_node, dst_node, src_host, dst_host (u32), send_time_ns,
    src_event_id (u64); table: u64 [tn x tn] routing latencies.  Returns (deliver, order,
    host_off, min_next, min_lat) or raises OracleError (3 = unordered events, the panic)."""
    a = {k: np.ascontiguousarray(batch[k], dtype=np.uint32) for k in ("src_node", "dst_node", "src_host", "dst_host")}
    send = np.ascontiguousarray(batch["send_time_ns"], dtype=np.uint64)
    eid = np.ascontiguousarray(batch["src_event_id"], dtype=np.uint64)
    table = np.ascontiguousarray(table, dtype=np.uint64)
    n = len(send)
    deliver = np.zeros(n, dtype=np.uint64)
    order = np.zeros(n, dtype=np.uint32)
    host_off = np.zeros(num_hosts + 1, dtype=np.uint64)
    mn, ml = ctypes.c_uint64(), ctypes.c_uint64()
    rc = lib().oracle_order_packet_events(
        n, _p(a["src_node"], _u32p), _p(a["dst_node"], _u32p), _p(a["src_host"], _u32p), _p(a["dst_host"], _u32p),
        _p(send, _u64p), _p(eid, _u64p), _p(table, _u64p), table.shape[0], num_hosts, round_end,
        _p(deliver, _u64p), _p(order, _u32p), _p(host_off, _u64p), ctypes.byref(mn), ctypes.byref(ml))
    if rc:
        raise OracleError(rc, {1: "index out of range", 2: "time overflow",
                               3: "events with no relative order (PanickingOrd panic)"}[rc])
    return deliver, order, host_off, mn.value, ml.value
