// oracle/oracle.cpp — CPU restatement of Shadow's routing-table build.
//
// TEST / BENCH INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg load this library, and only as the checker / the timed CPU baseline.
// The product (shadow_amd/, libshadow_routing.so) never links, loads or calls it.
//
// What it restates (reference snapshot /root/reference, Shadow v3.2.0):
//   * PathProperties            src/main/network/graph/mod.rs:296-331
//       ordering: latency_ns (u64) first, then packet_loss.partial_cmp   (:305-313)
//       add:      lat = a+b ; loss = 1 - (1-a)*(1-b), four separately rounded f32 ops (:322-331)
//   * petgraph 0.6.5 algo::dijkstra (third-party crate, NOT vendored in the reference;
//     pinned in src/Cargo.lock "petgraph 0.6.5"; called at mod.rs:195,198).  Restated from
//     its published algorithm: HashMap scores, visit map, BinaryHeap<MinScored>, push
//     (K::default(), start); pop; skip visited; for each edge of graph.edges(node): skip
//     visited targets; next = node_score + cost(edge); insert if vacant, replace+push only
//     if next < old (strict); mark node visited after its edge loop.
//   * petgraph Graph adjacency: per-node singly linked lists, edges prepended on add_edge;
//     Undirected::edges(a) = outgoing list, then incoming list minus self-loops, with the
//     incoming part reported with target() = the other endpoint.
//   * compute_shortest_paths    mod.rs:183-228 (per-source Dijkstra, `nodes.contains`
//     filter :203, per-source HashMap, rayon flat_map/collect merge :190-208, diagonal
//     overwritten with the raw single self-loop :210-217, assert n^2 entries :219)
//   * get_edge_weight           mod.rs:254-293 (edges_connecting; exactly one edge)
//   * get_direct_paths          mod.rs:230-252
//
// Parity pins: the reference's own KATs (mod.rs:515-647) are replayed against this file in
// tests/test_oracle.py; latencies are cross-checked against networkx; the f32 loss fold
// against an independent numpy-float32 Dijkstra in tests/golden/make_golden.py.
//
// Built with -ffp-contract=off (Rust never contracts `1 - x*y` into an FMA) and SSE math.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <queue>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

struct PP {                 // PathProperties (mod.rs:297-303)
    uint64_t lat;
    float loss;
};

// PartialOrd for PathProperties (mod.rs:305-313); loss is never NaN (validated in [0,1]).
inline bool pp_less(const PP& a, const PP& b) {
    if (a.lat != b.lat) return a.lat < b.lat;
    return a.loss < b.loss;
}

// Add for PathProperties (mod.rs:322-331).  volatile forces each f32 op to round.
inline PP pp_add(const PP& a, const PP& b) {
    volatile float one_minus_a = 1.0f - a.loss;
    volatile float one_minus_b = 1.0f - b.loss;
    volatile float prod = one_minus_a * one_minus_b;
    volatile float res = 1.0f - prod;
    return PP{a.lat + b.lat, res};
}

// petgraph::graph::Graph restated: edges in a Vec, per-node list heads [out, in].
struct Graph {
    uint32_t V = 0;
    bool directed = false;
    std::vector<uint32_t> esrc, edst;
    std::vector<PP> ew;
    std::vector<uint32_t> enext_out, enext_in;  // next edge in the source's out list / target's in list
    std::vector<uint32_t> head_out, head_in;    // per node
    std::vector<uint32_t> node_id;              // GML ids (error text)
    static constexpr uint32_t END = 0xFFFFFFFFu;

    void build(uint32_t nv, int dir, uint64_t E, const uint32_t* s, const uint32_t* d,
               const uint64_t* lat, const float* loss, const uint32_t* ids) {
        V = nv;
        directed = dir != 0;
        esrc.assign(s, s + E);
        edst.assign(d, d + E);
        ew.resize(E);
        for (uint64_t e = 0; e < E; ++e) ew[e] = PP{lat[e], loss[e]};
        head_out.assign(V, END);
        head_in.assign(V, END);
        enext_out.assign(E, END);
        enext_in.assign(E, END);
        // Graph::add_edge prepends to both lists (petgraph graph_impl add_edge).
        for (uint64_t e = 0; e < E; ++e) {
            enext_out[e] = head_out[s[e]];
            head_out[s[e]] = (uint32_t)e;
            enext_in[e] = head_in[d[e]];
            head_in[d[e]] = (uint32_t)e;
        }
        node_id.resize(V);
        for (uint32_t v = 0; v < V; ++v) node_id[v] = ids ? ids[v] : v;
    }

    // graph.edges(a): calls f(target, weight) in petgraph's iteration order.
    template <class F>
    void for_each_edge(uint32_t a, F&& f) const {
        for (uint32_t e = head_out[a]; e != END; e = enext_out[e]) f(edst[e], ew[e]);
        if (!directed) {
            for (uint32_t e = head_in[a]; e != END; e = enext_in[e]) {
                if (esrc[e] == a) continue;  // self-loop already yielded by the out list
                f(esrc[e], ew[e]);
            }
        }
    }

    // edges_connecting(a, b) count + first weight (mod.rs:265-266, 279-280).
    uint32_t count_connecting(uint32_t a, uint32_t b, PP* first) const {
        uint32_t c = 0;
        for_each_edge(a, [&](uint32_t t, const PP& w) {
            if (t == b) {
                if (c == 0 && first) *first = w;
                ++c;
            }
        });
        return c;
    }
};

struct HeapItem {           // MinScored<PathProperties, NodeIndex>
    PP score;
    uint32_t node;
};
struct HeapCmp {            // BinaryHeap is a max-heap; MinScored reverses the order
    bool operator()(const HeapItem& a, const HeapItem& b) const { return pp_less(b.score, a.score); }
};

// petgraph::algo::dijkstra with HashMap scores (reference-equivalent data structures).
void dijkstra_hash(const Graph& g, uint32_t start, std::unordered_map<uint32_t, PP>& scores,
                   std::vector<uint64_t>& visited) {
    scores.clear();
    visited.assign((g.V + 63) / 64, 0);
    std::priority_queue<HeapItem, std::vector<HeapItem>, HeapCmp> heap;
    const PP zero{0, 0.0f};
    scores.emplace(start, zero);
    heap.push({zero, start});
    while (!heap.empty()) {
        HeapItem it = heap.top();
        heap.pop();
        const uint32_t node = it.node;
        if (visited[node >> 6] >> (node & 63) & 1) continue;
        g.for_each_edge(node, [&](uint32_t next, const PP& w) {
            if (visited[next >> 6] >> (next & 63) & 1) return;
            PP ns = pp_add(it.score, w);
            auto f = scores.find(next);
            if (f != scores.end()) {
                if (pp_less(ns, f->second)) {
                    f->second = ns;
                    heap.push({ns, next});
                }
            } else {
                scores.emplace(next, ns);
                heap.push({ns, next});
            }
        });
        visited[node >> 6] |= 1ull << (node & 63);
    }
}

// Same algorithm with a dense score vector (identical semantics; used for fast checks).
void dijkstra_dense(const Graph& g, uint32_t start, std::vector<PP>& score, std::vector<uint8_t>& seen,
                    std::vector<uint8_t>& visited) {
    score.resize(g.V);
    seen.assign(g.V, 0);
    visited.assign(g.V, 0);
    std::priority_queue<HeapItem, std::vector<HeapItem>, HeapCmp> heap;
    const PP zero{0, 0.0f};
    score[start] = zero;
    seen[start] = 1;
    heap.push({zero, start});
    while (!heap.empty()) {
        HeapItem it = heap.top();
        heap.pop();
        const uint32_t node = it.node;
        if (visited[node]) continue;
        g.for_each_edge(node, [&](uint32_t next, const PP& w) {
            if (visited[next]) return;
            PP ns = pp_add(it.score, w);
            if (seen[next]) {
                if (pp_less(ns, score[next])) {
                    score[next] = ns;
                    heap.push({ns, next});
                }
            } else {
                seen[next] = 1;
                score[next] = ns;
                heap.push({ns, next});
            }
        });
        visited[node] = 1;
    }
}

// Dense-matrix Dijkstra for complete / near-complete graphs (mode 2, a fast CHECKER for the
// full-size configs).  Parallel edges are collapsed to their lexicographic-min (latency, loss)
// -- PathProperties ordering, mod.rs:305-313 -- which cannot change any score: the fold
// 1-(1-L)(1-p) is monotone in p.  Each step finalises the unvisited vertex with the
// lexicographically smallest score (linear scan, no heap), then relaxes its row with the
// same strict-< rule as petgraph.  The lexicographic score of every vertex is the unique
// fixpoint lexmin over its latency-tight predecessors (positive latencies), so this equals
// the heap Dijkstra bit for bit; tests/test_oracle.py pins mode 2 against mode 1.
struct DenseW {
    uint32_t V = 0;
    std::vector<uint64_t> lat;   // UINT64_MAX = no edge
    std::vector<float> loss;
    void build(const Graph& g) {
        V = g.V;
        lat.assign((size_t)V * V, UINT64_MAX);
        loss.assign((size_t)V * V, 0.0f);
        auto put = [&](uint32_t a, uint32_t b, const PP& w) {
            const size_t k = (size_t)a * V + b;
            if (lat[k] == UINT64_MAX || pp_less(w, PP{lat[k], loss[k]})) {
                lat[k] = w.lat;
                loss[k] = w.loss;
            }
        };
        for (size_t e = 0; e < g.esrc.size(); ++e) {
            const uint32_t s = g.esrc[e], t = g.edst[e];
            if (s == t) continue;  // a self-loop never improves a score (positive latency)
            put(s, t, g.ew[e]);
            if (!g.directed) put(t, s, g.ew[e]);
        }
    }
};

void dijkstra_matrix(const DenseW& w, uint32_t start, std::vector<PP>& score, std::vector<uint8_t>& seen,
                     std::vector<uint8_t>& visited) {
    const uint32_t V = w.V;
    score.assign(V, PP{UINT64_MAX, 1.0f});
    seen.assign(V, 0);
    visited.assign(V, 0);
    score[start] = PP{0, 0.0f};
    seen[start] = 1;
    for (;;) {
        uint32_t best = UINT32_MAX;
        for (uint32_t v = 0; v < V; ++v)
            if (seen[v] && !visited[v] && (best == UINT32_MAX || pp_less(score[v], score[best]))) best = v;
        if (best == UINT32_MAX) break;
        visited[best] = 1;
        const PP sb = score[best];
        const uint64_t* lrow = &w.lat[(size_t)best * V];
        const float* prow = &w.loss[(size_t)best * V];
        for (uint32_t t = 0; t < V; ++t) {
            if (lrow[t] == UINT64_MAX || visited[t]) continue;
            // PathProperties::add without volatile: -ffp-contract=off + SSE round every op
            const float x = 1.0f - sb.loss, y = 1.0f - prow[t];
            const float prod = x * y;
            const PP ns{sb.lat + lrow[t], 1.0f - prod};
            if (!seen[t] || pp_less(ns, score[t])) {
                score[t] = ns;
                seen[t] = 1;
            }
        }
    }
}

void set_err(char* buf, size_t len, const std::string& m) {
    if (buf && len) {
        std::snprintf(buf, len, "%s", m.c_str());
    }
}

// get_edge_weight (mod.rs:256-293): 0 = ok, 2 = no edge, 3 = more than one.
int edge_weight(const Graph& g, uint32_t a, uint32_t b, PP* out, char* err, size_t errlen) {
    PP first{0, 0.0f};
    uint32_t c = g.count_connecting(a, b, &first);
    if (c == 0) {
        set_err(err, errlen, "No edge connecting node " + std::to_string(g.node_id[a]) + " to " +
                                 std::to_string(g.node_id[b]));
        return 2;
    }
    if (c > 1) {
        set_err(err, errlen, "More than one edge connecting node " + std::to_string(g.node_id[a]) +
                                 " to " + std::to_string(g.node_id[b]));
        return 3;
    }
    *out = first;
    return 0;
}

int hw_threads(int n) {
    if (n > 0) return n;
    unsigned h = std::thread::hardware_concurrency();
    return h ? (int)h : 1;
}

template <class F>
void parallel_for(uint32_t count, int nthreads, F&& f) {
    nthreads = std::max(1, std::min<int>(nthreads, (int)std::max<uint32_t>(count, 1)));
    std::atomic<uint32_t> next{0};
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t)
        th.emplace_back([&, t]() {
            (void)t;
            for (;;) {
                uint32_t i = next.fetch_add(1);
                if (i >= count) break;
                f(i);
            }
        });
    for (auto& x : th) x.join();
}

inline uint64_t key2(uint32_t a, uint32_t b) { return (uint64_t)a << 32 | b; }

}  // namespace

extern "C" {

// compute_shortest_paths (mod.rs:183-228).
//   mode 0: reference-equivalent plumbing: HashMap scores, linear `nodes.contains` filter,
//           per-source HashMap, one merged HashMap (rayon collect), then dense copy-out.
//   mode 1: same Dijkstra semantics with dense scores and O(1) membership (fast checker).
//   mode 2: dense-matrix Dijkstra (dijkstra_matrix; checker for complete graphs, O(V^2)/source).
// rows/num_rows: if rows != NULL only those source POSITIONS are computed and out_* is
//           [num_rows x n]; the error checks that need all rows (n^2) are then per-row.
// Returns 0 or SRG-style codes (2 no edge, 3 multi edge, 4 unreachable, 1 arg).
int oracle_compute_shortest_paths(uint32_t V, int directed, uint64_t E, const uint32_t* src,
                                  const uint32_t* dst, const uint64_t* lat, const float* loss,
                                  const uint32_t* node_ids, const uint32_t* nodes, uint32_t n,
                                  const uint32_t* rows, uint32_t num_rows, uint64_t* out_lat,
                                  float* out_loss, int mode, int nthreads, char* err,
                                  size_t errlen) {
    for (uint64_t e = 0; e < E; ++e)
        if (src[e] >= V || dst[e] >= V) {
            set_err(err, errlen, "edge endpoint out of range");
            return 1;
        }
    for (uint32_t i = 0; i < n; ++i)
        if (nodes[i] >= V) {
            set_err(err, errlen, "node index out of range");
            return 1;
        }
    Graph g;
    g.build(V, directed, E, src, dst, lat, loss, node_ids);
    nthreads = hw_threads(nthreads);
    const bool all_rows = rows == nullptr;
    const uint32_t R = all_rows ? n : num_rows;
    std::vector<uint32_t> row_pos(R);
    for (uint32_t r = 0; r < R; ++r) row_pos[r] = all_rows ? r : rows[r];

    std::vector<int32_t> pos_of(V, -1);
    for (uint32_t i = 0; i < n; ++i) pos_of[nodes[i]] = (int32_t)i;
    std::vector<uint8_t> filled((size_t)R * n, 0);

    if (mode == 0) {
        // per-source HashMaps (flat_map body), then one sequential merge (collect)
        std::vector<std::unordered_map<uint64_t, PP>> per(R);
        parallel_for(R, nthreads, [&](uint32_t r) {
            std::unordered_map<uint32_t, PP> scores;
            std::vector<uint64_t> visited;
            const uint32_t s = nodes[row_pos[r]];
            dijkstra_hash(g, s, scores, visited);
            auto& m = per[r];
            for (auto& kv : scores) {
                bool used = false;  // nodes.contains(dst): linear scan (mod.rs:203)
                for (uint32_t i = 0; i < n; ++i)
                    if (nodes[i] == kv.first) {
                        used = true;
                        break;
                    }
                if (used) m.emplace(key2(s, kv.first), kv.second);
            }
        });
        std::unordered_map<uint64_t, PP> paths;
        for (auto& m : per)
            for (auto& kv : m) paths.insert(kv);
        per.clear();
        for (uint32_t r = 0; r < R; ++r) {
            const uint32_t s = nodes[row_pos[r]];
            for (uint32_t j = 0; j < n; ++j) {
                auto f = paths.find(key2(s, nodes[j]));
                if (f != paths.end()) {
                    out_lat[(size_t)r * n + j] = f->second.lat;
                    out_loss[(size_t)r * n + j] = f->second.loss;
                    filled[(size_t)r * n + j] = 1;
                }
            }
        }
    } else if (mode == 2) {
        DenseW w;
        w.build(g);
        parallel_for(R, nthreads, [&](uint32_t r) {
            std::vector<PP> score;
            std::vector<uint8_t> seen, visited;
            dijkstra_matrix(w, nodes[row_pos[r]], score, seen, visited);
            for (uint32_t j = 0; j < n; ++j) {
                uint32_t t = nodes[j];
                if (seen[t]) {
                    out_lat[(size_t)r * n + j] = score[t].lat;
                    out_loss[(size_t)r * n + j] = score[t].loss;
                    filled[(size_t)r * n + j] = 1;
                }
            }
        });
    } else {
        parallel_for(R, nthreads, [&](uint32_t r) {
            std::vector<PP> score;
            std::vector<uint8_t> seen, visited;
            dijkstra_dense(g, nodes[row_pos[r]], score, seen, visited);
            for (uint32_t j = 0; j < n; ++j) {
                uint32_t t = nodes[j];
                if (seen[t]) {
                    out_lat[(size_t)r * n + j] = score[t].lat;
                    out_loss[(size_t)r * n + j] = score[t].loss;
                    filled[(size_t)r * n + j] = 1;
                }
            }
        });
    }

    // diagonal: raw self-loop weight, errors in `nodes` order (mod.rs:210-217)
    for (uint32_t i = 0; i < n; ++i) {
        PP w;
        int rc = edge_weight(g, nodes[i], nodes[i], &w, err, errlen);
        if (rc) return rc;
        for (uint32_t r = 0; r < R; ++r)
            if (row_pos[r] == i) {
                out_lat[(size_t)r * n + i] = w.lat;
                out_loss[(size_t)r * n + i] = w.loss;
                filled[(size_t)r * n + i] = 1;
            }
    }
    // assert_eq!(paths.len(), nodes.len().pow(2)) (mod.rs:219)
    for (size_t k = 0; k < filled.size(); ++k)
        if (!filled[k]) {
            set_err(err, errlen,
                    "assertion `left == right` failed: paths.len() != nodes.len().pow(2) "
                    "(unreachable pair)");
            return 4;
        }
    return 0;
}

// get_direct_paths (mod.rs:230-252): src-major, dst-minor iteration; first error wins.
int oracle_get_direct_paths(uint32_t V, int directed, uint64_t E, const uint32_t* src,
                            const uint32_t* dst, const uint64_t* lat, const float* loss,
                            const uint32_t* node_ids, const uint32_t* nodes, uint32_t n,
                            uint64_t* out_lat, float* out_loss, char* err, size_t errlen) {
    for (uint64_t e = 0; e < E; ++e)
        if (src[e] >= V || dst[e] >= V) {
            set_err(err, errlen, "edge endpoint out of range");
            return 1;
        }
    Graph g;
    g.build(V, directed, E, src, dst, lat, loss, node_ids);
    for (uint32_t i = 0; i < n; ++i)
        for (uint32_t j = 0; j < n; ++j) {
            PP w;
            int rc = edge_weight(g, nodes[i], nodes[j], &w, err, errlen);
            if (rc) return rc;
            out_lat[(size_t)i * n + j] = w.lat;
            out_loss[(size_t)i * n + j] = w.loss;
        }
    return 0;
}

// PathProperties + PathProperties (mod.rs:322-331), exposed for the test_path_add KAT.
void oracle_path_add(uint64_t lat_a, float loss_a, uint64_t lat_b, float loss_b,
                     uint64_t* lat_out, float* loss_out) {
    PP r = pp_add(PP{lat_a, loss_a}, PP{lat_b, loss_b});
    *lat_out = r.lat;
    *loss_out = r.loss;
}

// CPU baseline timer: the reference-equivalent pipeline (mode 0 plumbing: HashMap scores,
// linear contains filter, per-source maps merged into one map) over a SAMPLE of source
// positions, `nthreads` worker threads (rayon's default pool = all host cores).
// Returns wall seconds; *checksum guards against dead-code elimination.
double oracle_time_sources(uint32_t V, int directed, uint64_t E, const uint32_t* src,
                           const uint32_t* dst, const uint64_t* lat, const float* loss,
                           const uint32_t* nodes, uint32_t n, const uint32_t* sample,
                           uint32_t k, int nthreads, uint64_t* checksum) {
    Graph g;
    g.build(V, directed, E, src, dst, lat, loss, nullptr);
    nthreads = hw_threads(nthreads);
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::unordered_map<uint64_t, PP>> per(k);
    parallel_for(k, nthreads, [&](uint32_t r) {
        std::unordered_map<uint32_t, PP> scores;
        std::vector<uint64_t> visited;
        const uint32_t s = nodes[sample[r]];
        dijkstra_hash(g, s, scores, visited);
        auto& m = per[r];
        for (auto& kv : scores) {
            bool used = false;
            for (uint32_t i = 0; i < n; ++i)
                if (nodes[i] == kv.first) {
                    used = true;
                    break;
                }
            if (used) m.emplace(key2(s, kv.first), kv.second);
        }
    });
    std::unordered_map<uint64_t, PP> paths;
    for (auto& m : per)
        for (auto& kv : m) paths.insert(kv);
    auto t1 = std::chrono::steady_clock::now();
    uint64_t cs = 0;
    for (auto& kv : paths) cs += kv.second.lat ^ kv.first;
    if (checksum) *checksum = cs;
    return std::chrono::duration<double>(t1 - t0).count();
}

// CPU-baseline timer with a choice of pipeline (bench.py cpu_baseline):
//   mode 0: the reference-equivalent pipeline above (oracle_time_sources)
//   mode 1: "CPU-best" for sparse graphs: the same heap Dijkstra with dense scores, O(1)
//           membership (position table instead of nodes.contains) and a dense output row
//   mode 2: "CPU-best" for dense graphs: dense-matrix Dijkstra (dijkstra_matrix), dense rows
// *setup_s = one-time preparation (graph build; mode 2 also the dense weight matrix), NOT in
// the returned seconds; the returned time covers the sample's sources (and mode 0's merge).
double oracle_time_sources_mode(uint32_t V, int directed, uint64_t E, const uint32_t* src, const uint32_t* dst,
                                const uint64_t* lat, const float* loss, const uint32_t* nodes, uint32_t n,
                                const uint32_t* sample, uint32_t k, int nthreads, int mode, double* setup_s,
                                uint64_t* checksum) {
    if (mode == 0) {
        auto s0 = std::chrono::steady_clock::now();
        Graph g0;
        g0.build(V, directed, E, src, dst, lat, loss, nullptr);
        if (setup_s) *setup_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - s0).count();
        return oracle_time_sources(V, directed, E, src, dst, lat, loss, nodes, n, sample, k, nthreads, checksum);
    }
    auto s0 = std::chrono::steady_clock::now();
    Graph g;
    g.build(V, directed, E, src, dst, lat, loss, nullptr);
    DenseW w;
    if (mode == 2) w.build(g);
    std::vector<int32_t> pos_of(V, -1);
    for (uint32_t i = 0; i < n; ++i) pos_of[nodes[i]] = (int32_t)i;
    std::vector<uint64_t> out_lat((size_t)k * n);
    std::vector<float> out_loss((size_t)k * n);
    if (setup_s) *setup_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - s0).count();
    nthreads = hw_threads(nthreads);
    auto t0 = std::chrono::steady_clock::now();
    parallel_for(k, nthreads, [&](uint32_t r) {
        std::vector<PP> score;
        std::vector<uint8_t> seen, visited;
        const uint32_t s = nodes[sample[r]];
        if (mode == 2) dijkstra_matrix(w, s, score, seen, visited);
        else dijkstra_dense(g, s, score, seen, visited);
        uint64_t* ol = &out_lat[(size_t)r * n];
        float* of = &out_loss[(size_t)r * n];
        for (uint32_t v = 0; v < V; ++v) {
            const int32_t p = pos_of[v];
            if (p >= 0 && seen[v]) {
                ol[p] = score[v].lat;
                of[p] = score[v].loss;
            }
        }
    });
    auto t1 = std::chrono::steady_clock::now();
    uint64_t cs = 0;
    for (uint64_t v : out_lat) cs += v;
    if (checksum) *checksum = cs;
    return std::chrono::duration<double>(t1 - t0).count();
}

int oracle_hw_threads(void) { return hw_threads(0); }

// ---- stretch C5: one round's cross-host packet events ----------------------
// Restates, per event i sent by src_host to dst_host at send_ns:
//   Worker::send_packet (src/main/core/worker.rs:391-424):
//     delay = RoutingInfo latency(src, dst)   -> table[src_node * tn + dst_node]
//     update_lowest_used_latency(delay)       (runahead.rs:61-116: min over used latencies)
//     deliver = current_time + delay (EmulatedTime + SimulationTime; overflow panics),
//               raised to round_end if earlier (worker.rs:411-414)
//     update_next_event_time(deliver)         (manager.rs:430-435, min at :459-464)
//     push_packet_to_host(dst_host, deliver)  (worker.rs:644-654: one EventQueue per host)
//   EventQueue pop order (event_queue.rs:38-49, BinaryHeap<Reverse<PanickingOrd<Event>>>):
//     Event::partial_cmp (event.rs:84-99): time, then EventData (Packet < Local, event.rs:103-110),
//     then PacketEventData (event.rs:131-155): src_host_id, then src_host_event_id; two events
//     equal in all of these with different packets -> None -> PanickingOrd unwrap panic.
// Output: order = per destination host (increasing HostId), that host's pop order;
// host_off[h] .. host_off[h+1] = host h's events.  Error codes: 1 = bad index, 2 = time
// overflow, 3 = two events with no relative order (the reference's panic).
int oracle_order_packet_events(uint64_t n, const uint32_t* src_node, const uint32_t* dst_node,
                               const uint32_t* src_host, const uint32_t* dst_host, const uint64_t* send_ns,
                               const uint64_t* event_id, const uint64_t* table, uint32_t tn, uint32_t num_hosts,
                               uint64_t round_end, uint64_t* deliver, uint32_t* order, uint64_t* host_off,
                               uint64_t* min_next, uint64_t* min_lat) {
    *min_next = UINT64_MAX;
    *min_lat = UINT64_MAX;
    std::vector<std::vector<uint32_t>> queues(num_hosts);
    for (uint64_t i = 0; i < n; ++i) {
        if (src_node[i] >= tn || dst_node[i] >= tn || dst_host[i] >= num_hosts) return 1;
        const uint64_t delay = table[(size_t)src_node[i] * tn + dst_node[i]];
        if (send_ns[i] > UINT64_MAX - delay) return 2;
        uint64_t t = send_ns[i] + delay;
        if (t < round_end) t = round_end;
        deliver[i] = t;
        *min_lat = std::min(*min_lat, delay);
        *min_next = std::min(*min_next, t);
        queues[dst_host[i]].push_back((uint32_t)i);
    }
    auto less = [&](uint32_t a, uint32_t b) {
        if (deliver[a] != deliver[b]) return deliver[a] < deliver[b];
        if (src_host[a] != src_host[b]) return src_host[a] < src_host[b];
        return event_id[a] < event_id[b];
    };
    uint64_t pos = 0;
    for (uint32_t h = 0; h < num_hosts; ++h) {
        host_off[h] = pos;
        auto& q = queues[h];
        std::sort(q.begin(), q.end(), less);
        for (size_t k = 0; k < q.size(); ++k) {
            if (k && !less(q[k - 1], q[k])) return 3;
            order[pos++] = q[k];
        }
    }
    host_off[num_hosts] = pos;
    return 0;
}

}  // extern "C"
