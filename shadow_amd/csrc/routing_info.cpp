// routing_info.cpp — dense-backed RoutingInfo behind the C ABI.
//
// Replaces, on Shadow's side of the boundary:
//   generate_routing_info   src/main/core/sim_config.rs:425-462  (GML ids -> NodeIndex, shortest or
//                           direct paths, results keyed back by GML id)
//   RoutingInfo<u32>        src/main/network/graph/mod.rs:428-477 (path lookup, packet counters,
//                           get_smallest_latency_ns)
// The reference materialises two HashMaps of n^2 entries (mod.rs:190-208 and sim_config.rs:448-450:
// 2 x 10^8 inserts at C3).  Here the table stays the dense n x n SoA the GPU wrote (row-major by
// position of the id in the caller's list) plus a GML-id -> position index, so the build is the
// host entry (H2D + kernels + overlapped D2H) and nothing else.  A single-context RoutingInfo owns
// its tables from the context's pinned-table pool (srg_internal_table_get): freeing it returns them
// still page-locked, so the next build skips the prefault + page-locking.  Host-only C++: no HIP
// calls here.
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/shadow_routing.h"
#include "internal.h"

namespace {

constexpr uint32_t NO_POS = 0xFFFFFFFFu;

void put_err(char* buf, size_t len, const std::string& m) {
    if (buf && len) std::snprintf(buf, len, "%s", m.c_str());
}

// per-path packet counters (mod.rs:432, 449-456): RwLock<HashMap> in the reference, here 64
// lock-striped maps so that concurrent senders on different paths rarely share a lock
struct Counters {
    static constexpr int SHARDS = 64;
    struct Shard {
        std::mutex mu;
        std::unordered_map<uint64_t, uint64_t> m;
    } shard[SHARDS];
    static uint64_t key(uint32_t a, uint32_t b) { return (uint64_t)a << 32 | b; }
    Shard& of(uint64_t k) { return shard[(k * 0x9E3779B97F4A7C15ull) >> 58]; }
};

// an n x n host table: from the context's pool (single context), else plain heap memory
struct HostTable {
    srg_table* pooled = nullptr;
    std::unique_ptr<unsigned char[]> own;
    void* p = nullptr;
    HostTable() = default;
    HostTable(const HostTable&) = delete;
    HostTable& operator=(const HostTable&) = delete;
    void alloc(srg_ctx* ctx, size_t bytes) {
        reset();
        if (ctx) {
            pooled = srg_internal_table_get(ctx, bytes, &p);
            if (!pooled) throw std::bad_alloc();
        } else {
            own.reset(new unsigned char[std::max<size_t>(bytes, 1)]);
            p = own.get();
        }
    }
    void reset() {
        if (pooled) srg_internal_table_put(pooled);
        pooled = nullptr;
        own.reset();
        p = nullptr;
    }
    ~HostTable() { reset(); }
};

}  // namespace

struct srg_routing_info {
    uint32_t n = 0;
    std::vector<uint32_t> ids;       // GML id per position
    // [n x n] tables, left uninitialised (every entry is written by the build; no 1.2 GB memset).
    // Latencies are kept either as the build's certified u32 keys (key = latency / unit, exact; the
    // diagonal's raw self-loop latencies in diag) -- 0.4 GB less D2H and host memory at C3 -- or,
    // when the build needed u64 keys or ran on several ranks, as u64 ns in lat.
    HostTable t_lat, t_key, t_loss;
    uint64_t* lat = nullptr;
    uint32_t* key = nullptr;
    std::vector<uint64_t> diag;
    uint64_t unit = 1;
    float* loss = nullptr;
    std::unique_ptr<uint64_t[]> lat_wide;  // tables(): the u64 view of a key table, built on first use
    std::once_flag widened;
    uint64_t min_lat = UINT64_MAX;
    // GML id -> position: a direct table when the ids are dense enough, else a hash map
    std::vector<uint32_t> pos_direct;
    std::unordered_map<uint32_t, uint32_t> pos_hash;
    Counters counters;

    uint32_t pos(uint32_t id) const {
        if (!pos_direct.empty()) return id < pos_direct.size() ? pos_direct[id] : NO_POS;
        auto f = pos_hash.find(id);
        return f == pos_hash.end() ? NO_POS : f->second;
    }
};

namespace {

// compute(nodes, n, out_lat, out_loss, tab_lat, tab_loss, stats, errbuf, errlen): one of the host
// entry points (tab_*: the tables' pool handles, null for heap tables)
using Compute = std::function<int(const uint32_t*, uint32_t, uint64_t*, float*, srg_table*, srg_table*, srg_stats*,
                                  char*, size_t)>;
// compute_keys(nodes, n, out_key, out_diag, out_loss, unit, tab_key, tab_loss, stats, errbuf, errlen):
// the key-table entry
using ComputeKeys = std::function<int(const uint32_t*, uint32_t, uint32_t*, uint64_t*, float*, uint64_t*, srg_table*,
                                      srg_table*, srg_stats*, char*, size_t)>;

// ctx: the context whose pool holds the tables (null: heap tables)
int build_routing_info(srg_ctx* ctx, const Compute& compute, const ComputeKeys& compute_keys, const srg_edge_list* graph,
                       const uint32_t* gml_ids, uint32_t num_ids, int use_shortest_paths, srg_routing_info** out,
                       srg_stats* stats, char* errbuf, size_t errlen) {
    *out = nullptr;
    try {
        // node_id_to_index (mod.rs:126-128): GML id -> NodeIndex, later duplicate ids win (:161)
        const uint32_t V = graph->num_vertices;
        std::unordered_map<uint32_t, uint32_t> id_to_index;
        id_to_index.reserve(V);
        for (uint32_t v = 0; v < V; ++v) id_to_index[graph->node_ids ? graph->node_ids[v] : v] = v;
        std::vector<uint32_t> nodes(num_ids);
        for (uint32_t i = 0; i < num_ids; ++i) {
            auto f = id_to_index.find(gml_ids[i]);
            if (f == id_to_index.end()) {  // graph.node_id_to_index(*x).unwrap() panics (sim_config.rs:433)
                put_err(errbuf, errlen,
                        "called `Option::unwrap()` on a `None` value (GML node id " + std::to_string(gml_ids[i]) +
                            " is not in the graph)");
                return SRG_ERR_ARG;
            }
            nodes[i] = f->second;
        }
        auto* ri = new srg_routing_info();
        std::unique_ptr<srg_routing_info> hold(ri);
        ri->n = num_ids;
        ri->ids.assign(gml_ids, gml_ids + num_ids);
        const size_t nn = (size_t)num_ids * num_ids;
        ri->t_loss.alloc(ctx, nn * 4);
        ri->loss = (float*)ri->t_loss.p;
        srg_stats local{};
        srg_stats* st = stats ? stats : &local;
        int rc = SRG_INTERNAL_NEED_U64;
        if (compute_keys) {
            ri->t_key.alloc(ctx, nn * 4);
            ri->key = (uint32_t*)ri->t_key.p;
            ri->diag.resize(num_ids);
            rc = compute_keys(nodes.data(), num_ids, ri->key, ri->diag.data(), ri->loss, &ri->unit, ri->t_key.pooled,
                              ri->t_loss.pooled, st, errbuf, errlen);
            if (rc == SRG_INTERNAL_NEED_U64) {
                ri->t_key.reset();
                ri->key = nullptr;
                ri->diag.clear();
                ri->unit = 1;
            }
        }
        if (rc == SRG_INTERNAL_NEED_U64) {
            ri->t_lat.alloc(ctx, nn * 8);
            ri->lat = (uint64_t*)ri->t_lat.p;
            rc = compute(nodes.data(), num_ids, ri->lat, ri->loss, ri->t_lat.pooled, ri->t_loss.pooled, st, errbuf, errlen);
        }
        hold.release();
        if (rc != SRG_OK) {
            delete ri;
            // .context("Failed to compute shortest paths between graph nodes") (sim_config.rs:446-447)
            if (errbuf && errlen) {
                const std::string inner = errbuf;
                put_err(errbuf, errlen,
                        std::string(use_shortest_paths ? "Failed to compute shortest paths between graph nodes: "
                                                       : "Failed to get the direct paths between graph nodes: ") +
                            inner);
            }
            return rc;
        }
        ri->min_lat = st->min_latency_ns;
        if (!use_shortest_paths) ri->min_lat = nn ? *std::min_element(ri->lat, ri->lat + nn) : UINT64_MAX;
        if (stats) stats->table_keys = ri->key ? 1 : 0;
        uint32_t max_id = 0;
        for (uint32_t id : ri->ids) max_id = std::max(max_id, id);
        if (num_ids && (uint64_t)max_id < std::max<uint64_t>(1u << 20, 16ull * num_ids)) {
            ri->pos_direct.assign((size_t)max_id + 1, NO_POS);
            for (uint32_t i = 0; i < num_ids; ++i) {
                if (ri->pos_direct[ri->ids[i]] != NO_POS) {
                    delete ri;
                    put_err(errbuf, errlen, "duplicate GML id in the node list");
                    return SRG_ERR_ARG;
                }
                ri->pos_direct[ri->ids[i]] = i;
            }
        } else {
            for (uint32_t i = 0; i < num_ids; ++i)
                if (!ri->pos_hash.emplace(ri->ids[i], i).second) {
                    delete ri;
                    put_err(errbuf, errlen, "duplicate GML id in the node list");
                    return SRG_ERR_ARG;
                }
        }
        *out = ri;
        return SRG_OK;
    } catch (const std::bad_alloc&) {
        put_err(errbuf, errlen, "out of host memory");
        return SRG_ERR_OOM;
    } catch (...) {
        put_err(errbuf, errlen, "internal error");
        return SRG_ERR_INTERNAL;
    }
}

}  // namespace

extern "C" {

int srg_routing_info_build(srg_ctx* ctx, const srg_edge_list* graph, const uint32_t* gml_ids, uint32_t num_ids,
                           int use_shortest_paths, srg_routing_info** out, srg_stats* stats, char* errbuf,
                           size_t errlen) {
    if (!ctx || !graph || !out || (num_ids && !gml_ids)) {
        put_err(errbuf, errlen, "null argument");
        return SRG_ERR_ARG;
    }
    *out = nullptr;
    // RoutingInfo::path is total over the node set (mod.rs:444-446): a rank of a multi-rank
    // context that fills only its own rows cannot build one
    int nr = 1, rk = 0;
    double gather = 1.0;
    if (srg_comm_size(ctx, &nr, &rk) == SRG_OK && nr > 1 && srg_get_option(ctx, SRG_OPT_GATHER_OUTPUT, &gather) == SRG_OK &&
        gather == 0.0) {
        put_err(errbuf, errlen,
                "srg_routing_info_build needs the whole table: this rank fills only its own rows "
                "(SRG_OPT_GATHER_OUTPUT 0); use srg_routing_info_build_multi or SRG_OPT_GATHER_OUTPUT 1");
        return SRG_ERR_ARG;
    }
    // one rank: the tables come from the context's pool (a rank of a group writes its shared table
    // through the group's page-locking instead)
    srg_ctx* pool_ctx = nr == 1 ? ctx : nullptr;
    Compute f = [&](const uint32_t* nodes, uint32_t n, uint64_t* lat, float* loss, srg_table* tl, srg_table* ts,
                    srg_stats* st, char* eb, size_t el) {
        if (tl && ts)
            return srg_internal_compute_table(ctx, graph, nodes, n, use_shortest_paths, lat, nullptr, nullptr, loss,
                                              nullptr, tl, ts, st, eb, el);
        return use_shortest_paths ? srg_compute_shortest_paths(ctx, graph, nodes, n, lat, loss, st, eb, el)
                                  : srg_get_direct_paths(ctx, graph, nodes, n, lat, loss, st, eb, el);
    };
    // one rank, shortest paths: the table stays in the build's u32 keys
    ComputeKeys fk = nullptr;
    if (use_shortest_paths && nr == 1)
        fk = [&](const uint32_t* nodes, uint32_t n, uint32_t* key, uint64_t* diag, float* loss, uint64_t* unit,
                 srg_table* tk, srg_table* ts, srg_stats* st, char* eb, size_t el) {
            return srg_internal_compute_table(ctx, graph, nodes, n, 1, nullptr, key, diag, loss, unit, tk, ts, st, eb,
                                              el);
        };
    return build_routing_info(pool_ctx, f, fk, graph, gml_ids, num_ids, use_shortest_paths, out, stats, errbuf, errlen);
}

int srg_routing_info_build_multi(srg_multi* m, const srg_edge_list* graph, const uint32_t* gml_ids, uint32_t num_ids,
                                 int use_shortest_paths, srg_routing_info** out, srg_stats* stats, char* errbuf,
                                 size_t errlen) {
    if (!m || !graph || !out || (num_ids && !gml_ids)) {
        put_err(errbuf, errlen, "null argument");
        return SRG_ERR_ARG;
    }
    Compute f = [&](const uint32_t* nodes, uint32_t n, uint64_t* lat, float* loss, srg_table*, srg_table*, srg_stats* st,
                    char* eb, size_t el) {
        return use_shortest_paths ? srg_multi_compute_shortest_paths(m, graph, nodes, n, lat, loss, st, eb, el)
                                  : srg_multi_get_direct_paths(m, graph, nodes, n, lat, loss, st, eb, el);
    };
    return build_routing_info(nullptr, f, nullptr, graph, gml_ids, num_ids, use_shortest_paths, out, stats, errbuf, errlen);
}

void srg_routing_info_free(srg_routing_info* ri) { delete ri; }

uint32_t srg_routing_info_num_nodes(const srg_routing_info* ri) { return ri ? ri->n : 0; }

int srg_routing_info_path(const srg_routing_info* ri, uint32_t start, uint32_t end, uint64_t* latency_ns,
                          float* packet_loss) {
    if (!ri) return 0;
    const uint32_t a = ri->pos(start), b = ri->pos(end);
    if (a == NO_POS || b == NO_POS) return 0;  // paths.get(&(start, end)) == None
    const size_t k = (size_t)a * ri->n + b;
    if (latency_ns) *latency_ns = !ri->key ? ri->lat[k] : a == b ? ri->diag[a] : (uint64_t)ri->key[k] * ri->unit;
    if (packet_loss) *packet_loss = ri->loss[k];
    return 1;
}

void srg_routing_info_increment_packet_count(srg_routing_info* ri, uint32_t start, uint32_t end) {
    if (!ri) return;
    const uint64_t k = Counters::key(start, end);
    auto& s = ri->counters.of(k);
    std::lock_guard<std::mutex> lk(s.mu);
    uint64_t& c = s.m[k];
    if (c != UINT64_MAX) ++c;  // saturating_add(1)
}

uint64_t srg_routing_info_packet_count(srg_routing_info* ri, uint32_t start, uint32_t end) {
    if (!ri) return 0;
    const uint64_t k = Counters::key(start, end);
    auto& s = ri->counters.of(k);
    std::lock_guard<std::mutex> lk(s.mu);
    auto f = s.m.find(k);
    return f == s.m.end() ? 0 : f->second;
}

int srg_routing_info_smallest_latency_ns(const srg_routing_info* ri, uint64_t* out) {
    if (!ri || ri->n == 0) return 0;  // an empty map: None
    if (out) *out = ri->min_lat;
    return 1;
}

void srg_routing_info_tables(const srg_routing_info* ri, const uint64_t** latency_ns, const float** packet_loss,
                             const uint32_t** gml_ids, uint32_t* n) {
    if (latency_ns && ri && ri->key) {  // a key table: its u64 view, widened once (exact: key * unit)
        auto* m = const_cast<srg_routing_info*>(ri);
        std::call_once(m->widened, [m] {
            const size_t nn = (size_t)m->n * m->n;
            m->lat_wide.reset(new uint64_t[std::max<size_t>(nn, 1)]);
            m->lat = m->lat_wide.get();
            for (uint32_t a = 0; a < m->n; ++a) {
                const uint32_t* kr = m->key + (size_t)a * m->n;
                uint64_t* lr = m->lat + (size_t)a * m->n;
                for (uint32_t b = 0; b < m->n; ++b) lr[b] = (uint64_t)kr[b] * m->unit;
                lr[a] = m->diag[a];
            }
        });
    }
    if (latency_ns) *latency_ns = ri ? ri->lat : nullptr;
    if (packet_loss) *packet_loss = ri ? ri->loss : nullptr;
    if (gml_ids) *gml_ids = ri ? ri->ids.data() : nullptr;
    if (n) *n = ri ? ri->n : 0;
}

}  // extern "C"
