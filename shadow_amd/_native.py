"""ctypes binding of libshadow_routing.so (C ABI: include/shadow_routing.h).

The library is built in-tree by shadow_amd/build.py.  There is no CPU fallback anywhere in
the product: if the library is missing, importing the routing entry points raises, and on a
machine without a HIP device srg_create() returns SRG_ERR_HIP, which surfaces as HipError.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libshadow_routing.so")

SRG_OK = 0
SRG_ERR_ARG = 1
SRG_ERR_NO_EDGE = 2
SRG_ERR_MULTI_EDGE = 3
SRG_ERR_UNREACHABLE = 4
SRG_ERR_LATENCY_RANGE = 5
SRG_ERR_HIP = 6
SRG_ERR_OOM = 7
SRG_ERR_PARSE = 8
SRG_ERR_RCCL = 9
SRG_ERR_INTERNAL = 10
SRG_ERR_EVENT_ORDER = 11

SRG_PATH_DENSE_U32 = 0
SRG_PATH_DENSE_U64 = 1
SRG_PATH_DIRECT = 2
SRG_PATH_SPARSE_U32 = 3
SRG_PATH_SPARSE_U64 = 4

SRG_OPT_PROFILING = 1
SRG_OPT_SPARSE_THRESHOLD = 2
SRG_OPT_GATHER_OUTPUT = 3
SRG_OPT_ALGORITHM = 4
SRG_OPT_SPARSE_LOCALITY = 5
SRG_OPT_SIMULATE_RANK = 6
SRG_OPT_FW_TILE = 7
SRG_OPT_SPARSE_DELTA_DIV = 12
SRG_OPT_SPARSE_GLOBAL_BITMAPS = 14
SRG_OPT_FW_SYMMETRIC = 17
SRG_OPT_D2H_MODE = 20
SRG_OPT_LOSS_CHUNKS = 21
SRG_OPT_SCAN_GROUPS = 22
SRG_OPT_H2D_CODEC = 25
SRG_OPT_EDGE_SHARD = 29
SRG_OPT_LATE_LOSS = 30
SRG_OPT_FW_LINE_SPLIT = 31
SRG_OPT_FW_STEP = 32
SRG_OPT_FW_OVERLAP = 33
SRG_OPT_TEST_FAULT = 34
SRG_OPT_TABLE_POOL_BYTES = 35
SRG_OPT_TABLE_POOL_IDLE_BYTES = 36
SRG_OPT_CREATE_MS_RUNTIME = 37
SRG_OPT_CREATE_MS_LIBRARY = 38
SRG_OPT_FW_XCD_ORDER = 39
SRG_ALGO_AUTO = 0
SRG_ALGO_DENSE = 1
SRG_ALGO_SPARSE = 2
SRG_UNIQUE_ID_BYTES = 128

SRG_SCAN_NONE = 0
SRG_SCAN_SPARSE = 1
SRG_SCAN_DENSE = 2

_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_f32p = ctypes.POINTER(ctypes.c_float)


class EdgeList(ctypes.Structure):
    _fields_ = [
        ("num_vertices", ctypes.c_uint32),
        ("directed", ctypes.c_uint32),
        ("num_edges", ctypes.c_uint64),
        ("src", ctypes.c_void_p),
        ("dst", ctypes.c_void_p),
        ("latency_ns", ctypes.c_void_p),
        ("packet_loss", ctypes.c_void_p),
        ("node_ids", ctypes.c_void_p),
    ]


class EventBatch(ctypes.Structure):
    _fields_ = [
        ("num_events", ctypes.c_uint64),
        ("src_node", ctypes.c_void_p),
        ("dst_node", ctypes.c_void_p),
        ("src_host", ctypes.c_void_p),
        ("dst_host", ctypes.c_void_p),
        ("send_time_ns", ctypes.c_void_p),
        ("src_event_id", ctypes.c_void_p),
        ("num_hosts", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32),
        ("round_end_ns", ctypes.c_uint64),
    ]


class EventResult(ctypes.Structure):
    _fields_ = [
        ("min_next_event_ns", ctypes.c_uint64),
        ("min_used_latency_ns", ctypes.c_uint64),
        ("key_bits", ctypes.c_uint32),
        ("radix_passes", ctypes.c_uint32),
        ("ms_total", ctypes.c_double),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class Stats(ctypes.Structure):
    _fields_ = [
        ("ms_total", ctypes.c_double),
        ("ms_h2d", ctypes.c_double),
        ("ms_build", ctypes.c_double),
        ("ms_fw", ctypes.c_double),
        ("ms_scan", ctypes.c_double),
        ("ms_loss", ctypes.c_double),
        ("ms_extract", ctypes.c_double),
        ("ms_d2h", ctypes.c_double),
        ("path_kind", ctypes.c_int32),
        ("loss_rounds", ctypes.c_int32),
        ("multi_pred_pairs", ctypes.c_uint64),
        ("relaxations", ctypes.c_uint64),
        ("essential_edges", ctypes.c_uint64),
        ("scan_kind", ctypes.c_int32),
        ("table_keys", ctypes.c_int32),
        ("prof_launches", ctypes.c_uint64),
        ("prof_kernel_ms", ctypes.c_double),
        ("prof_relaxations", ctypes.c_uint64),
        ("ms_exchange", ctypes.c_double),
        ("nranks", ctypes.c_int32),
        ("rank", ctypes.c_int32),
        ("local_sources", ctypes.c_uint64),
        ("ms_host_register", ctypes.c_double),
        ("d2h_overlapped_bytes", ctypes.c_uint64),
        ("min_latency_ns", ctypes.c_uint64),
        ("latency_unit_ns", ctypes.c_uint64),
        ("fw_overlap_pivots", ctypes.c_int32),
        ("fw_overlap_kept", ctypes.c_int32),
        ("d2h_key_rows", ctypes.c_int32),
        ("reserved0", ctypes.c_int32),
        ("ms_key_widen", ctypes.c_double),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


# every function declared in include/shadow_routing.h (checked by tests/test_abi.py)
EXPORTS = [
    "srg_create", "srg_destroy", "srg_set_option", "srg_compute_shortest_paths", "srg_compute_shortest_paths_device",
    "srg_get_direct_paths", "srg_graph_parse_gml", "srg_graph_free", "srg_graph_edge_list",
    "srg_graph_num_vertices", "srg_graph_num_edges", "srg_graph_directed", "srg_graph_node_index",
    "srg_graph_node_id", "srg_graph_node_bandwidth", "srg_graph_node_bandwidths", "srg_graph_parse_chunks",
    "srg_version", "srg_comm_unique_id", "srg_comm_init",
    "srg_local_group_create", "srg_local_group_release", "srg_comm_init_local", "srg_comm_size",
    "srg_order_packet_events_device", "srg_routing_info_build", "srg_routing_info_free", "srg_routing_info_num_nodes",
    "srg_routing_info_path", "srg_routing_info_increment_packet_count", "srg_routing_info_packet_count",
    "srg_routing_info_smallest_latency_ns", "srg_routing_info_tables",
    "srg_multi_create", "srg_multi_destroy", "srg_multi_size", "srg_multi_set_option", "srg_multi_compute_shortest_paths",
    "srg_multi_get_direct_paths", "srg_routing_info_build_multi", "srg_get_option",
]

_lib = None


def lib():
    """Load the native library; raises (never falls back) when it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: torch ships its own libamdhip64 (soname libamdhip64.so.7).
    # Loading torch first makes the dynamic linker reuse that runtime for our library too;
    # loading ours first would pull /opt/rocm's copy and torch's HIP init would then fail.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python shadow_amd/build.py` "
            "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    # SRG_LIB_PATH: load another build of the library (A/B of two builds in one tree; diagnostics)
    L = ctypes.CDLL(os.environ.get("SRG_LIB_PATH") or LIB_PATH)
    c = ctypes
    L.srg_create.restype = c.c_int
    L.srg_create.argtypes = [c.POINTER(c.c_void_p), c.c_int, c.c_char_p, c.c_size_t]
    L.srg_set_option.restype = c.c_int
    L.srg_set_option.argtypes = [c.c_void_p, c.c_int, c.c_double]
    L.srg_destroy.restype = None
    L.srg_destroy.argtypes = [c.c_void_p]
    host_sig = [c.c_void_p, c.POINTER(EdgeList), c.c_void_p, c.c_uint32, c.c_void_p, c.c_void_p,
                c.POINTER(Stats), c.c_char_p, c.c_size_t]
    L.srg_compute_shortest_paths.restype = c.c_int
    L.srg_compute_shortest_paths.argtypes = host_sig
    L.srg_get_direct_paths.restype = c.c_int
    L.srg_get_direct_paths.argtypes = host_sig
    L.srg_compute_shortest_paths_device.restype = c.c_int
    L.srg_compute_shortest_paths_device.argtypes = [
        c.c_void_p, c.POINTER(EdgeList), c.c_void_p, c.c_uint32, c.c_void_p, c.c_void_p, c.c_void_p,
        c.POINTER(Stats), c.c_char_p, c.c_size_t]
    L.srg_graph_parse_gml.restype = c.c_int
    L.srg_graph_parse_gml.argtypes = [c.c_char_p, c.c_size_t, c.POINTER(c.c_void_p), c.c_char_p, c.c_size_t]
    L.srg_graph_free.restype = None
    L.srg_graph_free.argtypes = [c.c_void_p]
    L.srg_graph_edge_list.restype = None
    L.srg_graph_edge_list.argtypes = [c.c_void_p, c.POINTER(EdgeList)]
    L.srg_graph_num_vertices.restype = c.c_uint32
    L.srg_graph_num_vertices.argtypes = [c.c_void_p]
    L.srg_graph_num_edges.restype = c.c_uint64
    L.srg_graph_num_edges.argtypes = [c.c_void_p]
    L.srg_graph_directed.restype = c.c_int
    L.srg_graph_directed.argtypes = [c.c_void_p]
    L.srg_graph_node_index.restype = c.c_int
    L.srg_graph_node_index.argtypes = [c.c_void_p, c.c_uint32, _u32p]
    L.srg_graph_node_id.restype = c.c_uint32
    L.srg_graph_node_id.argtypes = [c.c_void_p, c.c_uint32]
    L.srg_graph_node_bandwidth.restype = None
    L.srg_graph_node_bandwidth.argtypes = [c.c_void_p, c.c_uint32, _u64p, c.POINTER(c.c_int), _u64p,
                                           c.POINTER(c.c_int)]
    L.srg_graph_node_bandwidths.restype = None
    L.srg_graph_node_bandwidths.argtypes = [c.c_void_p, c.c_void_p, c.c_void_p, c.c_void_p, c.c_void_p]
    L.srg_graph_parse_chunks.restype = c.c_uint32
    L.srg_graph_parse_chunks.argtypes = [c.c_void_p]
    L.srg_version.restype = c.c_char_p
    L.srg_version.argtypes = []
    L.srg_comm_unique_id.restype = c.c_int
    L.srg_comm_unique_id.argtypes = [c.c_char_p, c.c_char_p, c.c_size_t]
    L.srg_comm_init.restype = c.c_int
    L.srg_comm_init.argtypes = [c.c_void_p, c.c_int, c.c_int, c.c_char_p, c.c_char_p, c.c_size_t]
    L.srg_local_group_create.restype = c.c_int
    L.srg_local_group_create.argtypes = [c.c_int, c.POINTER(c.c_void_p)]
    L.srg_local_group_release.restype = None
    L.srg_local_group_release.argtypes = [c.c_void_p]
    L.srg_comm_init_local.restype = c.c_int
    L.srg_comm_init_local.argtypes = [c.c_void_p, c.c_void_p, c.c_int, c.c_char_p, c.c_size_t]
    L.srg_order_packet_events_device.restype = c.c_int
    L.srg_order_packet_events_device.argtypes = [
        c.c_void_p, c.POINTER(EventBatch), c.c_void_p, c.c_uint32, c.c_void_p, c.c_void_p, c.c_void_p, c.c_void_p,
        c.POINTER(EventResult), c.c_char_p, c.c_size_t]
    L.srg_routing_info_build.restype = c.c_int
    L.srg_routing_info_build.argtypes = [c.c_void_p, c.POINTER(EdgeList), c.c_void_p, c.c_uint32, c.c_int,
                                         c.POINTER(c.c_void_p), c.POINTER(Stats), c.c_char_p, c.c_size_t]
    L.srg_routing_info_free.restype = None
    L.srg_routing_info_free.argtypes = [c.c_void_p]
    L.srg_routing_info_num_nodes.restype = c.c_uint32
    L.srg_routing_info_num_nodes.argtypes = [c.c_void_p]
    L.srg_routing_info_path.restype = c.c_int
    L.srg_routing_info_path.argtypes = [c.c_void_p, c.c_uint32, c.c_uint32, _u64p, _f32p]
    L.srg_routing_info_increment_packet_count.restype = None
    L.srg_routing_info_increment_packet_count.argtypes = [c.c_void_p, c.c_uint32, c.c_uint32]
    L.srg_routing_info_packet_count.restype = c.c_uint64
    L.srg_routing_info_packet_count.argtypes = [c.c_void_p, c.c_uint32, c.c_uint32]
    L.srg_routing_info_smallest_latency_ns.restype = c.c_int
    L.srg_routing_info_smallest_latency_ns.argtypes = [c.c_void_p, _u64p]
    L.srg_routing_info_tables.restype = None
    L.srg_routing_info_tables.argtypes = [c.c_void_p, c.POINTER(_u64p), c.POINTER(_f32p), c.POINTER(_u32p),
                                          c.POINTER(c.c_uint32)]
    L.srg_multi_create.restype = c.c_int
    L.srg_multi_create.argtypes = [c.POINTER(c.c_void_p), c.c_void_p, c.c_int, c.c_char_p, c.c_size_t]
    L.srg_multi_destroy.restype = None
    L.srg_multi_destroy.argtypes = [c.c_void_p]
    L.srg_multi_size.restype = c.c_int
    L.srg_multi_size.argtypes = [c.c_void_p]
    L.srg_multi_set_option.restype = c.c_int
    L.srg_multi_set_option.argtypes = [c.c_void_p, c.c_int, c.c_double]
    L.srg_multi_compute_shortest_paths.restype = c.c_int
    L.srg_multi_compute_shortest_paths.argtypes = host_sig
    L.srg_multi_get_direct_paths.restype = c.c_int
    L.srg_multi_get_direct_paths.argtypes = host_sig
    L.srg_routing_info_build_multi.restype = c.c_int
    L.srg_routing_info_build_multi.argtypes = [c.c_void_p, c.POINTER(EdgeList), c.c_void_p, c.c_uint32, c.c_int,
                                               c.POINTER(c.c_void_p), c.POINTER(Stats), c.c_char_p, c.c_size_t]
    L.srg_get_option.restype = c.c_int
    L.srg_get_option.argtypes = [c.c_void_p, c.c_int, c.POINTER(c.c_double)]
    L.srg_comm_size.restype = c.c_int
    L.srg_comm_size.argtypes = [c.c_void_p, c.POINTER(c.c_int), c.POINTER(c.c_int)]
    _lib = L
    return L
