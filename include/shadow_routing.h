/*
 * shadow_routing.h — C ABI of the MI355X routing-table builder for Shadow.
 *
 * Drop-in boundary for ONE reference path: Shadow's all-pairs routing-table build
 *   NetworkGraph::compute_shortest_paths(&self, nodes: &[NodeIndex])
 *       -> Result<HashMap<(NodeIndex, NodeIndex), PathProperties>, NetGraphError>
 *   (/root/reference/src/main/network/graph/mod.rs:183-228)
 * and its use_shortest_path=false sibling
 *   NetworkGraph::get_direct_paths  (mod.rs:230-252, get_edge_weight mod.rs:254-293)
 * plus the ingest step in front of it
 *   NetworkGraph::parse              (mod.rs:134-181, gml-parser/src/parser.rs:44-281,
 *                                     ShadowNode/ShadowEdge mod.rs:28-111, units.rs:377-439)
 *
 * Plain C types only (no torch, no C++ types).  Every function is noexcept: errors are
 * integer status codes plus a message written to a caller buffer, formatted like the
 * reference's error strings so the Rust wrapper can forward them verbatim.
 *
 * Output layout: dense row-major num_nodes x num_nodes, indexed by POSITION in `nodes`
 * (out[i*num_nodes + j] = path nodes[i] -> nodes[j]).  The reference returns a HashMap
 * keyed by (NodeIndex, NodeIndex); the Rust-side binding in INTEGRATION.md rebuilds that
 * map (or, per SURVEY f1, keeps the dense arrays).  PathProperties is split SoA:
 * latency_ns (u64) + packet_loss (f32), because the Rust struct is not repr(C).
 */
#ifndef SHADOW_ROUTING_H
#define SHADOW_ROUTING_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------------------- */
#define SRG_OK 0
#define SRG_ERR_ARG 1           /* bad argument (null pointer, index out of range, duplicate node) */
#define SRG_ERR_NO_EDGE 2       /* "No edge connecting node {src_id} to {dst_id}"       mod.rs:266-268 */
#define SRG_ERR_MULTI_EDGE 3    /* "More than one edge connecting node {a} to {b}"      mod.rs:269-274 */
#define SRG_ERR_UNREACHABLE 4   /* assert_eq!(paths.len(), nodes.len().pow(2)) panics   mod.rs:219 */
#define SRG_ERR_LATENCY_RANGE 5 /* latency.convert(Nano).unwrap() overflow (mod.rs:336), or a used
                                   pair with no path below 2^62 units on a graph whose worst-case
                                   path sum reaches 2^62 units (unit = srg_stats.latency_unit_ns, the
                                   gcd of the non-self-loop latencies).  The u64 keys hold distances
                                   below 2^62 units only (an edge of >= 2^62 units counts as absent),
                                   so such a pair may be unreachable OR have a shortest path in
                                   [2^62, 2^64) ns that the reference would return (e.g. one edge of
                                   2^63 + 1 ns) -- a documented deviation; a graph whose used pairs
                                   all have paths below 2^62 units succeeds whatever its latencies */
#define SRG_ERR_HIP 6           /* HIP runtime failure (no device, launch failure) */
#define SRG_ERR_OOM 7           /* device allocation failed */
#define SRG_ERR_PARSE 8         /* GML / attribute error from NetworkGraph::parse (mod.rs:134-181) */
#define SRG_ERR_RCCL 9          /* collective failure (multi-GPU) */
#define SRG_ERR_INTERNAL 10     /* invariant violated inside the builder (a bug) */

/* ---- graph as the Rust side would marshal it from petgraph ------------------------- */
/* One entry per petgraph edge, in graph.raw_edges() order (== GML edge order).
 * src/dst are NodeIndex values (dense 0..num_vertices-1, GML node order, mod.rs:157-162).
 * Self-loops and parallel edges are allowed exactly as in the reference.                */
typedef struct srg_edge_list {
    uint32_t num_vertices;
    uint32_t directed;          /* 1 = petgraph::Directed, 0 = Undirected (GML default 0) */
    uint64_t num_edges;
    const uint32_t* src;        /* [num_edges] */
    const uint32_t* dst;        /* [num_edges] */
    const uint64_t* latency_ns; /* [num_edges] latency.convert(Nano) (mod.rs:336) */
    const float* packet_loss;   /* [num_edges] raw f32 in [0,1] (mod.rs:95-103) */
    const uint32_t* node_ids;   /* [num_vertices] GML id per NodeIndex, for error text; may be NULL */
} srg_edge_list;

/* Timing / path report for one call (all fields written when the pointer is non-NULL). */
typedef struct srg_stats {
    double ms_total;            /* entry -> return wall time */
    double ms_h2d;              /* host -> device copies (host entry points only) */
    double ms_build;            /* dense weight-matrix build + validation kernels */
    double ms_fw;               /* blocked Floyd-Warshall (dense) / batched Bellman-Ford (sparse) */
    double ms_scan;             /* essential-edge extraction + tight-predecessor scan */
    double ms_loss;             /* left-fold loss rounds over the tight DAG */
    double ms_extract;          /* used x used sub-matrix + diagonal self-loop overwrite */
    double ms_d2h;              /* device -> host copies (host entry points only) */
    int32_t path_kind;          /* SRG_PATH_* below */
    int32_t loss_rounds;        /* max fold rounds over rows (DAG depth + 1) */
    uint64_t multi_pred_pairs;  /* (s,t) pairs with >1 tight predecessor (slow path) */
    uint64_t relaxations;       /* min-plus relaxations issued by the FW kernels */
    uint64_t essential_edges;   /* edges with W[u][t] == D[u][t] (candidates for tightness) */
    int32_t scan_kind;          /* SRG_SCAN_* below */
    int32_t table_keys;         /* srg_routing_info_build: 1 = the table kept the build's u32 latency keys
                                   (latency = key x latency_unit_ns; 0.4 GB less D2H and host memory at C3),
                                   0 = u64 ns (u64-key builds, several ranks, direct paths) */
    /* filled only when profiling is enabled (SRG_OPT_PROFILING): HIP events recorded on the
     * launch stream around every launch of the dominant kernel (FW phase-3 product).      */
    uint64_t prof_launches;     /* profiled launches */
    double prof_kernel_ms;      /* sum of their event-measured durations */
    uint64_t prof_relaxations;  /* relaxations those launches performed */
    /* multi-rank (srg_comm_init*): this rank's view */
    double ms_exchange;         /* output row exchange (all ranks end with every row) */
    int32_t nranks;             /* ranks in the communicator (1 = single GPU) */
    int32_t rank;               /* this rank */
    uint64_t local_sources;     /* used sources routed by this rank */
    /* host entry: the caller's output arrays are page-locked concurrently with H2D + FW, then
     * finished rows leave while later kernels run; ms_d2h above is only the exposed tail.   */
    double ms_host_register;    /* page-locking time (hidden; -1 = not used / failed)      */
    uint64_t d2h_overlapped_bytes; /* output bytes copied to the host while kernels ran    */
    uint64_t min_latency_ns;    /* host entry: min latency over all n^2 outputs, diagonal included
                                   (RoutingInfo::get_smallest_latency_ns, mod.rs:474-476);
                                   UINT64_MAX when n = 0                                       */
    uint64_t latency_unit_ns;   /* shortest paths: the gcd of the non-self-loop edge latencies; the
                                   kernels count latency in these units (exact: every path sum is a
                                   multiple), outputs are back in ns.  1 = nanosecond keys        */
    int32_t fw_overlap_pivots;  /* host entry: FW pivots enqueued while the edge list was still crossing
                                   PCIe (SRG_OPT_FW_OVERLAP; 0 = none)                              */
    int32_t fw_overlap_kept;    /* host entry: 1 = the FW that ran beside the H2D produced the table
                                   (its certification passed), 0 = the build ran FW after the H2D   */
    int32_t d2h_key_rows;       /* host entry, u64 output: 1 = the latency rows crossed PCIe as the build's
                                   u32 keys (4 B instead of 8 per pair) and were widened on the host  */
    int32_t reserved0;
    double ms_key_widen;        /* its widening + key-copy wall time on the helper thread (overlapped
                                   with the loss pass; the part after the kernels is in ms_d2h)     */
} srg_stats;

#define SRG_PATH_DENSE_U32 0    /* dense FW, u32 saturating latency keys (exact, certified) */
#define SRG_PATH_DENSE_U64 1    /* dense FW, u64 latency keys */
#define SRG_PATH_DIRECT 2       /* get_direct_paths */
#define SRG_PATH_SPARSE_U32 3   /* sparse: batched lexicographic Bellman-Ford, u32 latency keys */
#define SRG_PATH_SPARSE_U64 4   /* sparse, u64 latency keys (used paths past 2^32-1 latency units) */

#define SRG_SCAN_NONE 0         /* no used sources */
#define SRG_SCAN_SPARSE 1       /* tight scan over the essential edges (default) */
#define SRG_SCAN_DENSE 2        /* tight scan over all (s,u,t) triples (essential-dense graphs) */

typedef struct srg_ctx srg_ctx; /* opaque: owns device workspace; one HIP device */

/* Create a context bound to HIP device `device` (one process per GPU).  Besides the HIP runtime's
 * device initialisation it warms what the first host-entry call would otherwise pay on the routing
 * path: the kernels' code object on the device, each stream's first dispatch, the H2D codec's worker
 * pool and page-locked rings, the first H2D / D2H / SDMA copies (SRG_CREATE_WARM=0 in the environment
 * skips that, for A/B).  Shadow creates its context before parsing the GML, so this
 * runs off the routing path.  Replaces nothing in the reference: the context is the device state that
 * compute_shortest_paths (mod.rs:183-228) needs and Rust's CPU path does not have. */
int srg_create(srg_ctx** out, int device, char* errbuf, size_t errlen);
void srg_destroy(srg_ctx* ctx);


/* Context options.
 *   SRG_OPT_PROFILING         1 = HIP-event timing of every dominant-kernel launch (stats.prof_*)
 *   SRG_OPT_SPARSE_THRESHOLD  essential-edge density (E_ess / V^2) up to which the sparse
 *                             tight scan is used (default 0.35; 0 forces the dense scan)      */
#define SRG_OPT_PROFILING 1
#define SRG_OPT_SPARSE_THRESHOLD 2
#define SRG_OPT_GATHER_OUTPUT 3   /* multi-rank: 1 (default) = every rank ends with all rows;
                                     0 = each rank fills only the rows of the sources it owns (the host
                                     entry then copies only those rows to the caller, and
                                     stats.min_latency_ns is over those rows) */
#define SRG_OPT_ALGORITHM 4       /* SRG_ALGO_*: how compute_shortest_paths routes */
#define SRG_ALGO_AUTO 0           /* sparse when V >= 2048 and arcs * 32 < V^2, else dense */
#define SRG_ALGO_DENSE 1          /* blocked FW + tight-DAG loss pass */
#define SRG_ALGO_SPARSE 2         /* batched lexicographic Bellman-Ford over CSR */
#define SRG_OPT_SPARSE_LOCALITY 5 /* sparse: 1 (default) = batch sources in BFS order, 0 = in `nodes` order */
#define SRG_OPT_SIMULATE_RANK 6   /* TIMING AID ONLY: value = nranks*1000 + rank runs this rank's share
                                     with every collective elided -- outputs are NOT valid; 0 detaches */
#define SRG_OPT_FW_TILE 7         /* dense u32 FW tile: 0 = auto (128), 64, 128 */
/* 8 (SRG_OPT_FW_PACKED) and 18 (SRG_OPT_CHAIN_PRIO) were A/B switches, removed in round 4: the u32 FW
 * always runs the pair-packed tile and the chain kernels always raise their priority. */
/* 10 (SPARSE_GROUP), 11 (SPARSE_WGS_PER_CU) and 13 (SPARSE_DELTA_ALL) were A/B switches of the sparse
 * kernel, removed in round 4: 8 rows in flight, two workgroups per CU, any-lane bucket test. */
#define SRG_OPT_SPARSE_DELTA_DIV 12  /* sparse: delta-stepping bucket width = max edge latency / value;
                                        0 = a single bucket (plain Bellman-Ford); default 1 */
#define SRG_OPT_SPARSE_GLOBAL_BITMAPS 14 /* sparse: 1 = keep the per-batch vertex bitmaps in global memory
                                        (automatic when 5V/8 bytes do not fit the LDS budget) */
#define SRG_OPT_FW_SYMMETRIC 17     /* dense: 1 (default) = for an undirected graph, update only the FW tiles
                                       I <= J (D stays symmetric; u32 keys on 128-tiles, u64 keys on 64-tiles,
                                       one rank or many) and mirror at the end; 0 = the general FW */
#define SRG_OPT_D2H_MODE 20         /* host entry: how finished rows are shipped into the page-locked caller
                                     * arrays while kernels run: 1 (default) = an SDMA engine, 0 =
                                     * hipMemcpyAsync (a full-chip blit kernel: slows the overlapped kernels) */
#define SRG_OPT_LOSS_CHUNKS 21       /* dense: k_loss_rows launches (row chunks); 0 (default) = 8 when the host
                                     * entry ships rows early, else 1 */
#define SRG_OPT_SCAN_GROUPS 22       /* host entry: source-block groups the tight scan is
                                     * launched in, each group's loss rows folded and shipped while
                                     * later groups scan; 0 (default) = 3, 1 = scan, then loss */
#define SRG_OPT_H2D_CODEC 25         /* host entry: 1 (default) = the edge list crosses PCIe narrowed (u16
                                     * endpoints, u32 latencies; 12 instead of 20 B per edge) when every
                                     * endpoint < 65536 and latency < 2^32, widened on the device; 0 = plain */
#define SRG_OPT_EDGE_SHARD 29        /* host entry, multi-rank: 1 = each rank ships 1/N of the edge list over
                                     * its own PCIe link and the ranks exchange the slices over the GPU
                                     * links (allgatherv); 0 = every rank ships the whole list; -1 (default)
                                     * = 1 when the group has >= 4 ranks */
#define SRG_OPT_LATE_LOSS 30         /* host entry: 1 (default) = the edge losses cross PCIe after the endpoints
                                     * and latencies, on their own stream beside the W build and FW (which
                                     * need no loss); 0 = with them */
#define SRG_OPT_FW_LINE_SPLIT 31     /* symmetric FW: sub-tiles per dimension of the critical chain's line
                                     * launches, 1 (whole 128-tiles) / 2 / 4; 0 (default) = by the bulk a
                                     * pivot leaves this rank: >= 2048 tiles 1, >= 1024 tiles 2, else 4
                                     * (C3: 1 on one rank, 2 on two, 4 on more; C1/C2: 4) */
#define SRG_OPT_FW_STEP 32           /* symmetric FW schedule.  -1 (default) = the bulk and the next pivot's chain
                                     * on two streams; between ranks the chain exchanges its line segments
                                     * device-side (stores into the peers' line buffers + arrival words) for
                                     * simulated ranks and in-process ranks on distinct devices, else with
                                     * the communicator's allgather.  0 = two streams, always the allgather.
                                     * 2 = two streams, device-side exchange also for ranks sharing a GPU
                                     * (each rank's chain stream needs a hardware queue of its own).
                                     * 1 = one fused launch per pivot (chain on the launch's first
                                     * workgroups, exchange inside it; measured slower) */
#define SRG_OPT_FW_OVERLAP 33        /* host entry, one rank: 1 (default) = FW starts while the edge list is still
                                     * crossing PCIe (an undirected list ordered by source row with every edge
                                     * (s, d), s <= d -- a GML complete graph: each block-row of W is split and
                                     * caught up on the pivots already run as soon as its edges have landed);
                                     * 0 = FW after the whole list (any list falls back to that by itself) */
#define SRG_OPT_TEST_FAULT 34         /* TEST BUILD ONLY: compiled in only with -DSRG_TEST_HOOKS (the test library
                                     * libshadow_routing_testhooks.so); the product library refuses any value
                                     * but 0 with SRG_ERR_ARG.  1 = overwrite the closed FW matrix
                                     * with zeros after FW (a lost synchronisation's result: the build must fail
                                     * with SRG_ERR_INTERNAL, not return it); 2 = nonzero FW sync words and zero
                                     * line buffers before each symmetric FW (a recycled allocation: the build
                                     * must still be exact); 0 (default) = off */
#define SRG_OPT_TABLE_POOL_BYTES 35  /* RoutingInfo tables (srg_routing_info_build, one rank) come from a pool of
                                     * page-locked host tables on the context; freeing a RoutingInfo returns
                                     * them, so the next build skips the prefault + page-locking.  Bytes of idle
                                     * tables the pool keeps (default: no byte cap, only the most recently freed
                                     * table pair; setting a byte cap replaces that count cap; 0 = free them at
                                     * once).  Idle tables stay page-locked (not reclaimable by the OS) until
                                     * reused, trimmed or srg_destroy */
#define SRG_OPT_TABLE_POOL_IDLE_BYTES 36  /* read-only: bytes of idle tables the pool holds now */
#define SRG_OPT_CREATE_MS_RUNTIME 37  /* read-only: srg_create's HIP-runtime part (device count, device context,
                                      * the first stream, where the runtime initialises the device: the first
                                      * context of a process pays the runtime's initialisation) */
#define SRG_OPT_CREATE_MS_LIBRARY 38  /* read-only: srg_create's own part (three more streams, mailbox, SDMA
                                      * agents, events, the warm-up) */
#define SRG_OPT_FW_XCD_ORDER 39      /* symmetric FW bulk launch order: 1 (default) = the tiles dealt to the 8 XCDs as
                                     * Z-order runs, one list per pivot (each XCD a compact block of the triangle,
                                     * its line-buffer operands L2-resident: C3 bulk HBM traffic 1.38x -> 1.12x of
                                     * the C tiles); 0 = triangle order (consecutive tiles round-robin) */
int srg_set_option(srg_ctx* ctx, int option, double value);
/* current value of an option (SRG_OK), or SRG_ERR_ARG for an unknown option */
int srg_get_option(srg_ctx* ctx, int option, double* value);

/* Replaces NetworkGraph::compute_shortest_paths (mod.rs:183-228).
 * Host pointers in, host pointers out.  out_* are caller-allocated num_nodes^2.
 * Diagonal = raw self-loop weight (mod.rs:210-217); errors in `nodes` order.           */
int srg_compute_shortest_paths(srg_ctx* ctx, const srg_edge_list* graph,
                               const uint32_t* nodes, uint32_t num_nodes,
                               uint64_t* out_latency_ns, float* out_packet_loss,
                               srg_stats* stats, char* errbuf, size_t errlen);

/* Same computation with every array already resident in device memory (HBM):
 * graph->src/dst/latency_ns/packet_loss/node_ids, nodes and out_* are device pointers;
 * `hip_stream` is a hipStream_t (NULL = default stream).  Returns after the stream work
 * is complete.  (The benchmark's headline times the HOST entry above, as Shadow calls it;
 * this entry is reported beside it as the inputs-resident-in-HBM figure.)              */
int srg_compute_shortest_paths_device(srg_ctx* ctx, const srg_edge_list* graph_dev,
                                      const uint32_t* nodes_dev, uint32_t num_nodes,
                                      uint64_t* out_latency_ns_dev, float* out_packet_loss_dev,
                                      void* hip_stream, srg_stats* stats,
                                      char* errbuf, size_t errlen);

/* Replaces NetworkGraph::get_direct_paths (mod.rs:230-252): every used pair <- the single
 * edge src->dst (undirected: either orientation), error unless exactly one exists.     */
int srg_get_direct_paths(srg_ctx* ctx, const srg_edge_list* graph,
                         const uint32_t* nodes, uint32_t num_nodes,
                         uint64_t* out_latency_ns, float* out_packet_loss,
                         srg_stats* stats, char* errbuf, size_t errlen);

/* ---- RoutingInfo, dense-backed ------------------------------------------
 * Replaces generate_routing_info (src/main/core/sim_config.rs:425-462) and RoutingInfo<u32>
 * (mod.rs:428-477).  The reference builds two n^2-entry HashMaps (mod.rs:190-208 and
 * sim_config.rs:448-450); here the table is the dense n x n SoA the GPU wrote plus a GML-id ->
 * position index, so building it costs one host-entry call (srg_compute_shortest_paths).     */
typedef struct srg_routing_info srg_routing_info;
/* gml_ids[num_ids]: the used nodes' GML ids (ip_assignment.get_nodes(), any order); they are
 * resolved with graph->node_ids (node_id_to_index, mod.rs:126-128; NULL = id == index).
 * use_shortest_paths = network.use_shortest_path (configuration.rs:286-292).  Errors carry the
 * reference's context prefix ("Failed to compute shortest paths between graph nodes: ...").   */
int srg_routing_info_build(srg_ctx* ctx, const srg_edge_list* graph, const uint32_t* gml_ids, uint32_t num_ids,
                           int use_shortest_paths, srg_routing_info** out, srg_stats* stats,
                           char* errbuf, size_t errlen);
/* The same, built by every GPU of an srg_multi (declared below). */
struct srg_multi;
int srg_routing_info_build_multi(struct srg_multi* m, const srg_edge_list* graph, const uint32_t* gml_ids,
                                 uint32_t num_ids, int use_shortest_paths, srg_routing_info** out, srg_stats* stats,
                                 char* errbuf, size_t errlen);
void srg_routing_info_free(srg_routing_info* ri);
uint32_t srg_routing_info_num_nodes(const srg_routing_info* ri);
/* RoutingInfo::path (mod.rs:444-446): 1 and the path's properties, or 0 (None).              */
int srg_routing_info_path(const srg_routing_info* ri, uint32_t start_id, uint32_t end_id,
                          uint64_t* latency_ns, float* packet_loss);
/* RoutingInfo::increment_packet_count (mod.rs:449-456): saturating, thread-safe.              */
void srg_routing_info_increment_packet_count(srg_routing_info* ri, uint32_t start_id, uint32_t end_id);
uint64_t srg_routing_info_packet_count(srg_routing_info* ri, uint32_t start_id, uint32_t end_id);
/* RoutingInfo::get_smallest_latency_ns (mod.rs:474-476): 1 and the min over all entries
 * (diagonal included), or 0 (None, empty table).                                               */
int srg_routing_info_smallest_latency_ns(const srg_routing_info* ri, uint64_t* out);
/* Borrowed dense tables (row-major by position) and the GML id of each position.             */
void srg_routing_info_tables(const srg_routing_info* ri, const uint64_t** latency_ns, const float** packet_loss,
                             const uint32_t** gml_ids, uint32_t* n);

/* ---- ingest: GML text -> graph (NetworkGraph::parse, mod.rs:134-181) --------------- */
typedef struct srg_graph srg_graph;  /* opaque host-side parsed graph */

int srg_graph_parse_gml(const char* text, size_t len, srg_graph** out,
                        char* errbuf, size_t errlen);
void srg_graph_free(srg_graph* g);
/* Borrowed view of the edge list (valid until srg_graph_free). */
void srg_graph_edge_list(const srg_graph* g, srg_edge_list* out);
uint32_t srg_graph_num_vertices(const srg_graph* g);
uint64_t srg_graph_num_edges(const srg_graph* g);
int srg_graph_directed(const srg_graph* g);
/* node_id_to_index (mod.rs:126-128): SRG_OK or SRG_ERR_ARG if the id is unknown. */
int srg_graph_node_index(const srg_graph* g, uint32_t gml_id, uint32_t* out_index);
/* node_index_to_id (mod.rs:130-132). */
uint32_t srg_graph_node_id(const srg_graph* g, uint32_t index);
/* ShadowNode bandwidths in bit/s (mod.rs:34-57); has_* = 0 when the key was absent.   */
void srg_graph_node_bandwidth(const srg_graph* g, uint32_t index,
                              uint64_t* down_bits, int* has_down,
                              uint64_t* up_bits, int* has_up);
/* All nodes at once: arrays of srg_graph_num_vertices entries (any pointer may be NULL).      */
void srg_graph_node_bandwidths(const srg_graph* g, uint64_t* down_bits, int* has_down,
                               uint64_t* up_bits, int* has_up);
/* Diagnostics: how many text chunks the last parse of `g` used (1 = one sequential pass).    */
uint32_t srg_graph_parse_chunks(const srg_graph* g);

/* ---- multi-GPU: one process (or thread) per GPU, SPMD -------------------------------
 * After srg_comm_init*, every rank calls srg_compute_shortest_paths[_device] with the SAME
 * graph and nodes.  Undirected graphs: the symmetric FW's stored tiles (I, J), I <= J, are dealt
 * to rank (I + J) mod G and each pivot's line buffer (the pivot's row panel = its column panel)
 * is exchanged once per pivot (allgather; SRG_OPT_FW_STEP = 2: device-side stores); directed
 * graphs: row blocks with a per-pivot broadcast of the row panel.  Each rank routes the used
 * sources at positions [n r / G, n (r+1) / G) of `nodes`; output rows are exchanged
 * (SRG_OPT_GATHER_OUTPUT).  The reference has no multi-process path (rayon threads only,
 * mod.rs:190-208): this is new, MI355X-side design.                         */
#define SRG_UNIQUE_ID_BYTES 128
/* RCCL (over xGMI): rank 0 creates the id, the caller shares it (e.g. torch.distributed). */
int srg_comm_unique_id(unsigned char id[SRG_UNIQUE_ID_BYTES], char* errbuf, size_t errlen);
int srg_comm_init(srg_ctx* ctx, int nranks, int rank, const unsigned char id[SRG_UNIQUE_ID_BYTES],
                  char* errbuf, size_t errlen);
/* In-process group: several contexts of ONE process (threads; may share one GPU). */
typedef struct srg_local_group srg_local_group;
int srg_local_group_create(int nranks, srg_local_group** out);
void srg_local_group_release(srg_local_group* g);
int srg_comm_init_local(srg_ctx* ctx, srg_local_group* g, int rank, char* errbuf, size_t errlen);
int srg_comm_size(srg_ctx* ctx, int* nranks, int* rank);

/* ---- several GPUs behind ONE call (Shadow's one-process model) ------------------------
 * Shadow builds RoutingInfo once, in one process (sim_config.rs:137-141 -> manager.rs:301-324),
 * so the drop-in for a multi-GPU node is one object driving N devices: one context per device in
 * an in-process group (collectives are pull kernels over xGMI, peer access enabled), one worker
 * thread per rank.  srg_multi_compute_shortest_paths has exactly srg_compute_shortest_paths'
 * arguments and results: the whole n x n table lands in the caller's two arrays, every GPU
 * shipping its own sources' rows over its own PCIe link.  stats: wall times of the slowest
 * rank, counts summed over ranks, nranks = N.  A device may be listed more than once (several
 * ranks sharing one GPU: how the one-GPU test box exercises this path).                     */
typedef struct srg_multi srg_multi;
int srg_multi_create(srg_multi** out, const int* devices, int num_devices, char* errbuf, size_t errlen);
void srg_multi_destroy(srg_multi* m);
int srg_multi_size(const srg_multi* m);
/* srg_set_option on every rank (SRG_OPT_GATHER_OUTPUT and SRG_OPT_SIMULATE_RANK are fixed: ERR_ARG) */
int srg_multi_set_option(srg_multi* m, int option, double value);
int srg_multi_compute_shortest_paths(srg_multi* m, const srg_edge_list* graph, const uint32_t* nodes,
                                     uint32_t num_nodes, uint64_t* out_latency_ns, float* out_packet_loss,
                                     srg_stats* stats, char* errbuf, size_t errlen);
/* get_direct_paths (use_shortest_path = false) on the first device: an n^2 gather, no SSSP work */
int srg_multi_get_direct_paths(srg_multi* m, const srg_edge_list* graph, const uint32_t* nodes, uint32_t num_nodes,
                               uint64_t* out_latency_ns, float* out_packet_loss, srg_stats* stats, char* errbuf,
                               size_t errlen);

/* ---- stretch: one round's cross-host packet-event batch ---------------
 * Replaces, for a whole batch at once, the per-packet tail of Worker::send_packet
 * (src/main/core/worker.rs:391-424: latency lookup in RoutingInfo, deliver time raised to the
 * round end, lowest used latency for the dynamic runahead runahead.rs:61-116, next event time)
 * and the per-destination EventQueue ordering (worker.rs:644-654, event_queue.rs:38-49,
 * Event::partial_cmp event.rs:84-155: time, then src_host_id, then src_host_event_id), plus the
 * round's minimum next-event time (manager.rs:459-464).  The latency table is the dense
 * num_nodes x num_nodes output of srg_compute_shortest_paths (rows = sending node position).
 * Outputs: deliver_ns[i] per event; order = event indices grouped by destination host
 * (increasing HostId), each host's events in its queue's pop order; host_offsets[h] ..
 * host_offsets[h+1] = host h's slice.  The packet-drop draw (worker.rs:374-389) consumes each
 * host's RNG stream in program order and is not part of the batch.                          */
#define SRG_ERR_EVENT_ORDER 11  /* two events with no relative order: PanickingOrd unwrap panic
                                   (event.rs:141-147, event_queue.rs:87-90) */
typedef struct srg_event_batch {
    uint64_t num_events;
    const uint32_t* src_node;      /* [n] row of the latency table (sender's node position)   */
    const uint32_t* dst_node;      /* [n] column of the latency table                          */
    const uint32_t* src_host;      /* [n] HostId of the sender                                 */
    const uint32_t* dst_host;      /* [n] HostId of the receiver, < num_hosts                  */
    const uint64_t* send_time_ns;  /* [n] Worker::current_time at the send (EmulatedTime ns)   */
    const uint64_t* src_event_id;  /* [n] src_host.get_new_event_id()                          */
    uint32_t num_hosts;
    uint32_t reserved;
    uint64_t round_end_ns;         /* Worker::round_end_time                                   */
} srg_event_batch;

typedef struct srg_event_result {
    uint64_t min_next_event_ns;    /* min deliver time (UINT64_MAX when empty)                 */
    uint64_t min_used_latency_ns;  /* min latency used (UINT64_MAX when empty)                 */
    uint32_t key_bits;             /* composite sort-key width actually used                   */
    uint32_t radix_passes;         /* 8-bit LSD passes run                                     */
    double ms_total;
} srg_event_result;

/* Device pointers throughout (batch arrays, table, outputs); `hip_stream` as above.          */
int srg_order_packet_events_device(srg_ctx* ctx, const srg_event_batch* batch_dev,
                                   const uint64_t* latency_table_dev, uint32_t table_n,
                                   uint64_t* out_deliver_ns_dev, uint32_t* out_order_dev,
                                   uint64_t* out_host_offsets_dev, void* hip_stream,
                                   srg_event_result* result, char* errbuf, size_t errlen);

/* Library build/version string. */
const char* srg_version(void);

#ifdef __cplusplus
}
#endif
#endif /* SHADOW_ROUTING_H */
