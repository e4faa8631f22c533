// routing.hip — MI355X routing-table builder: device pipeline + C ABI (include/shadow_routing.h).
//
// Replaces NetworkGraph::compute_shortest_paths (src/main/network/graph/mod.rs:183-228) and
// NetworkGraph::get_direct_paths (mod.rs:230-252) with a dense device pipeline:
//   1. k_edge_scan       validate endpoints, count self-loops per vertex, record the raw
//                        self-loop weight (diagonal, mod.rs:210-217), max edge latency
//   2. k_w_lat/k_w_loss  dense W = lexicographic min over parallel edges (mod.rs:305-313)
//   3. fw_phase1/fw_product   blocked min-plus Floyd-Warshall on latency (exact u32-sat or u64)
//   4. tight_scan        per used source, the tight predecessors of every vertex
//   5. k_loss_round      left-fold loss over the tight DAG, Jacobi rounds to a fixpoint
//                        == petgraph Dijkstra's lexicographic (latency, loss) scores
//   6. k_extract         used x used outputs, diagonal <- raw self-loop, unreachable check
// No CPU fallback: every entry point fails loudly (status code) when HIP is unavailable.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <deque>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/shadow_routing.h"
#include "internal.h"
#include "kernels.hip.h"
#include "guards.h"
#include "edge_codec.h"
#include "tight_sparse.hip.h"
#include "comm.h"
#include "sparse.hip.h"
#include "sparse_ds.hip.h"
#include "events.hip.h"
#include "xchg.hip.h"

#include <hipcub/hipcub.hpp>

using namespace srg;

namespace {

struct Failure {
    int code;
    std::string msg;
};

[[noreturn]] void fail(int code, const std::string& m) { throw Failure{code, m}; }

#define HIP_CHECK(expr)                                                                           \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess) {                                                                   \
            if (e_ == hipErrorOutOfMemory)                                                        \
                fail(SRG_ERR_OOM, std::string("device allocation failed: ") + hipGetErrorString(e_)); \
            fail(SRG_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));                  \
        }                                                                                         \
    } while (0)

void set_err(char* buf, size_t len, const std::string& m) {
    if (buf && len) std::snprintf(buf, len, "%s", m.c_str());
}

// grow-only device buffer
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    void* get(size_t need) {
        if (need <= bytes) return p;
        if (p) HIP_CHECK(hipFree(p));
        p = nullptr;
        bytes = 0;
        HIP_CHECK(hipMalloc(&p, need ? need : 16));
        bytes = need;
        return p;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
};

struct EdgeStats {
    unsigned long long max_lat;   // max latency over non-self-loop edges
    unsigned long long unit;      // gcd of the non-self-loop latencies (0: none, or all zero)
    uint32_t bad_endpoint;        // an endpoint >= V
    uint32_t lat_overflow;        // a non-self-loop latency == UINT64_MAX (ns conversion overflow)
    unsigned long long min_lat_inv;  // ~(min latency over non-self-loop edges) (0: no such edge)
};

struct Flags {
    uint32_t changed;
    uint32_t inf_in_used_row;
    uint32_t unreachable_used_pair;
    uint32_t bad_node;
    unsigned long long first_bad;  // direct paths: first (i*n+j) with edge count != 1
    uint32_t wrap;                 // k_wrap_edges: a relaxation the reference would run wraps u64
    uint32_t wrap_inf;             // k_wrap_edges: a relaxation from a vertex left at INF (unknown distance)
    uint32_t impossible;           // k_certify: a used off-diagonal key below the smallest edge key (guards.h)
};

constexpr int kThreads = 256;

inline unsigned grid_for(size_t work, size_t cap = 256 * 16) {
    size_t g = (work + kThreads - 1) / kThreads;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

// ---------------------------------------------------------------------------------------
__global__ void k_check_nodes(const uint32_t* __restrict__ nodes, uint32_t n, uint32_t V,
                              uint32_t* __restrict__ mark, Flags* flags) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t v = nodes[i];
        if (v >= V) {
            atomicOr(&flags->bad_node, 1u);
            continue;
        }
        if (atomicAdd(&mark[v], 1u) != 0) atomicOr(&flags->bad_node, 2u);
    }
}

// binary gcd (gcd(0, b) = b)
__device__ __forceinline__ unsigned long long gcd64(unsigned long long a, unsigned long long b) {
    if (a == 0) return b;
    if (b == 0) return a;
    const int sh = __builtin_ctzll(a | b);
    a >>= __builtin_ctzll(a);
    do {
        b >>= __builtin_ctzll(b);
        if (a > b) {
            const unsigned long long t = a;
            a = b;
            b = t;
        }
        b -= a;
    } while (b);
    return a << sh;
}

__global__ void k_edge_scan(uint64_t E, const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
                            const uint64_t* __restrict__ lat, const float* __restrict__ loss, uint32_t V,
                            uint32_t* __restrict__ selfcnt, uint64_t* __restrict__ self_lat,
                            float* __restrict__ self_loss, EdgeStats* st) {
    unsigned long long mx = 0, mn = 0;  // mn = ~min: a max reduction like mx (0 = no edge yet)
    uint32_t bad = 0, ovf = 0;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < E; e += (size_t)gridDim.x * blockDim.x) {
        const uint32_t s = src[e], t = dst[e];
        if (s >= V || t >= V) {
            bad = 1;
            continue;
        }
        const uint64_t l = lat[e];
        if (s == t) {
            atomicAdd(&selfcnt[s], 1u);
            self_lat[s] = l;      // meaningful only when the count ends at exactly 1
            if (loss) self_loss[s] = loss[e];  // null: the loss arrives later (k_self_loss)
        } else {
            mx = l > mx ? l : mx;
            mn = ~l > mn ? ~l : mn;
            ovf |= (l == UINT64_MAX);
        }
    }
    // wave reduction then one atomic per wave
    for (int off = 32; off > 0; off >>= 1) {
        unsigned long long o = __shfl_down(mx, off, 64);
        mx = o > mx ? o : mx;
        o = __shfl_down(mn, off, 64);
        mn = o > mn ? o : mn;
    }
    if ((threadIdx.x & 63) == 0 && mx) atomicMax(&st->max_lat, mx);
    if ((threadIdx.x & 63) == 0 && mn) atomicMax(&st->min_lat_inv, mn);
    if (bad) atomicOr(&st->bad_endpoint, 1u);
    if (ovf) atomicOr(&st->lat_overflow, 1u);
}

// The latency unit (compute_device: keys = latency / unit) = gcd of the non-self-loop latencies,
// in a pass of its own: each wave folds 256-edge chunks and publishes its gcd, and every wave stops
// once the published unit is 1 -- on nanosecond-random latencies after the first round of chunks
// (~1 M edges), on unit-granular ones after the whole list.  (Folded into k_edge_scan, the gcd
// tripled that kernel: 298 -> 884 us on C3.)
__global__ void __launch_bounds__(256) k_lat_gcd(uint64_t E, const uint32_t* __restrict__ src,
                                                 const uint32_t* __restrict__ dst, const uint64_t* __restrict__ lat,
                                                 unsigned long long* unit) {
    const uint32_t lane = threadIdx.x & 63;
    const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
    const size_t nwaves = ((size_t)gridDim.x * blockDim.x) >> 6;
    const size_t nch = (E + 255) / 256;
    for (size_t ch = wave; ch < nch; ch += nwaves) {
        if (__hip_atomic_load(unit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 1ull) return;  // whole wave
        unsigned long long un = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const size_t e = ch * 256 + (size_t)j * 64 + lane;
            if (e < E && src[e] != dst[e]) un = gcd64(un, lat[e]);
        }
        for (int off = 32; off > 0; off >>= 1) un = gcd64(un, __shfl_down(un, off, 64));
        if (lane == 0 && un) {
            // gcd has no atomic: compare-and-swap until the stored unit divides this wave's
            unsigned long long cur = __hip_atomic_load(unit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            for (;;) {
                const unsigned long long nu = gcd64(cur, un);
                if (nu == cur) break;
                const unsigned long long prev = atomicCAS(unit, cur, nu);
                if (prev == cur) break;
                cur = prev;
            }
        }
    }
}

// the self-loops' loss, when the edge losses arrive after k_edge_scan (host entry, late loss)
__global__ void k_self_loss(uint64_t E, const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
                            const float* __restrict__ loss, uint32_t V, float* __restrict__ self_loss) {
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < E; e += (size_t)gridDim.x * blockDim.x) {
        const uint32_t s = src[e];
        if (s == dst[e] && s < V) self_loss[s] = loss[e];
    }
}

template <class K>
__global__ void k_fill(K* __restrict__ p, size_t count, K v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x)
        p[i] = v;
}

// latency -> key: latency / unit, where the unit (the gcd of all non-self-loop latencies) divides
// every path sum, so keys compare and add exactly as the latencies do; outputs are key * unit
template <class K>
__device__ __forceinline__ K to_key(uint64_t l, uint64_t unit) {
    if (unit != 1) l /= unit;
    if constexpr (sizeof(K) == 4) return l >= KeyOps<K>::INF ? KeyOps<K>::INF : (uint32_t)l;
    else return (K)l;
}

template <class K>
__global__ void k_w_lat(uint64_t E, const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
                        const uint64_t* __restrict__ lat, uint64_t unit, int directed, K* __restrict__ W, size_t ld) {
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < E; e += (size_t)gridDim.x * blockDim.x) {
        const uint32_t s = src[e], t = dst[e];
        if (s == t) continue;  // self-loops never shorten a path; kept for the diagonal only
        const K l = to_key<K>(lat[e], unit);
        atomicMin(&W[(size_t)s * ld + t], l);
        if (!directed) atomicMin(&W[(size_t)t * ld + s], l);
    }
}

template <class K>
__global__ void k_w_loss(uint64_t E, const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
                         const uint64_t* __restrict__ lat, uint64_t unit, const float* __restrict__ loss, int directed,
                         const K* __restrict__ W, uint32_t* __restrict__ WL, size_t ld) {
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < E; e += (size_t)gridDim.x * blockDim.x) {
        const uint32_t s = src[e], t = dst[e];
        if (s == t) continue;
        const K l = to_key<K>(lat[e], unit);
        // -0.0 compares equal to 0.0 (partial_cmp) and folds identically: normalise it
        const uint32_t bits = __float_as_uint(loss[e] + 0.0f);
        if (W[(size_t)s * ld + t] == l) atomicMin(&WL[(size_t)s * ld + t], bits);
        if (!directed && W[(size_t)t * ld + s] == l) atomicMin(&WL[(size_t)t * ld + s], bits);
    }
}

// u32 keys: one pass over the edges with a packed lexicographic key
//   KW[s][t] = min over parallel edges of (latency << 32 | loss bits)    (mod.rs:305-313)
// (loss in [0,1] is non-negative, so its f32 bit order is its numeric order).
// (V: endpoints past it are skipped -- the FW beside the H2D builds W before the edge checks run)
__global__ void k_w_key(uint64_t E, const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
                        const uint64_t* __restrict__ lat, uint64_t unit, const float* __restrict__ loss,
                        unsigned long long* __restrict__ KW, size_t ld, uint32_t V = 0xFFFFFFFFu) {
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < E; e += (size_t)gridDim.x * blockDim.x) {
        const uint32_t s = src[e], t = dst[e];
        if (s == t || s >= V || t >= V) continue;  // self-loops never shorten a path; kept for the diagonal only
        // null loss: latency only (WL is then built by k_w_loss once the losses have arrived)
        const uint64_t l = unit != 1 ? lat[e] / unit : lat[e];  // < 2^32-1: the u32 path's precondition
        const unsigned long long k = ((unsigned long long)l << 32) | (loss ? __float_as_uint(loss[e] + 0.0f) : 0u);
        atomicMin(&KW[(size_t)s * ld + t], k);
    }
}

// 64x64 tiles: (undirected) KW = min(KW, KW^T), then split into W (latency), WL (loss bits)
// and D (= W with a zero diagonal).  grid = (nb64, nb64) over the upper triangle incl. diagonal
// blocks when undirected (each block pair handled once), all blocks when directed.
// WL_ONLY: only WL is written (late loss: W and D were split from latency-only keys before FW)
// (bi0: first 64-block row of the launch -- the FW beside the H2D splits a block-row at a time)
template <bool WL_ONLY = false>
__global__ void __launch_bounds__(256) k_w_split(const unsigned long long* __restrict__ KW, size_t ld, int directed,
                                                 uint32_t* __restrict__ W, uint32_t* __restrict__ WL,
                                                 uint32_t* __restrict__ D, uint32_t bi0 = 0) {
    __shared__ unsigned long long tb[64][65];
    const uint32_t bi = bi0 + blockIdx.y, bj = blockIdx.x;
    if (!directed && bj < bi) return;
    const uint32_t tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    if (!directed) {
        for (uint32_t r = ty; r < 64; r += 4) tb[r][tx] = KW[(size_t)(bj * 64 + r) * ld + bi * 64 + tx];  // (bj, bi)
        __syncthreads();
    }
    for (uint32_t r = ty; r < 64; r += 4) {
        const size_t i = bi * 64 + r, j = bj * 64 + tx;
        unsigned long long k = KW[i * ld + j];
        if (!directed) k = min(k, tb[tx][r]);
        const uint32_t w = min((uint32_t)(k >> 32), KeyOps<uint32_t>::INF);  // no edge / >= INF -> INF
        WL[i * ld + j] = (uint32_t)k;
        if (!WL_ONLY) {
            W[i * ld + j] = w;
            D[i * ld + j] = i == j ? 0u : w;
        }
        if (!directed && bi != bj) tb[tx][r] = k;  // the mirrored element, written below
    }
    if (!directed && bi != bj) {
        __syncthreads();
        for (uint32_t r = ty; r < 64; r += 4) {
            const size_t i = bj * 64 + r, j = bi * 64 + tx;
            const unsigned long long k = tb[r][tx];
            const uint32_t w = min((uint32_t)(k >> 32), KeyOps<uint32_t>::INF);
            WL[i * ld + j] = (uint32_t)k;
            if (!WL_ONLY) {
                W[i * ld + j] = w;
                D[i * ld + j] = w;
            }
        }
    }
}

template <class K>
__global__ void k_init_d(const K* __restrict__ W, K* __restrict__ D, size_t ld) {
    const size_t total = ld * ld;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = i / ld, c = i - r * ld;
        D[i] = (r == c) ? (K)0 : W[i];
    }
}

// INF in a used (row, column) pair (u32 certification).  Only used columns can change an
// output: a stored key <= INF plus an edge w > 0 never falsely equals a finite D[s][t], so an
// unreachable UNUSED vertex leaves the u32 result exact.
// Row kernels over (used row x used column) arrays: one workgroup per row (grid = rows), the
// threads striding over the columns -- no 64-bit division per element (the grid-stride form with
// i / ncols ran 10x below HBM rate: 0.6 ms per C3 pass).
// Also the impossible-result guard (guards.h): a used off-diagonal key below the smallest edge key
// (0 included) cannot be a path length -- a fault inside the builder, never returned as OK.
template <class K>
__global__ void __launch_bounds__(256) k_certify(const K* __restrict__ D, size_t ld, const uint32_t* __restrict__ rows,
                                                 uint32_t nrows, const uint32_t* __restrict__ cols, uint32_t ncols,
                                                 K min_key, Flags* flags) {
    const uint32_t s = rows[blockIdx.x];
    const K* Dr = D + (size_t)s * ld;
    uint32_t hit = 0, bad = 0;
    constexpr uint32_t U = 8;  // independent loads in flight per thread (the gather is latency-bound)
    for (uint32_t j0 = threadIdx.x; j0 < ncols; j0 += blockDim.x * U) {
        uint32_t cc[U];
        K d[U];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            const uint32_t j = j0 + u * blockDim.x;
            cc[u] = cols[j < ncols ? j : 0];
        }
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) d[u] = Dr[cc[u]];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            const bool in = j0 + u * blockDim.x < ncols;
            hit |= in & (d[u] == KeyOps<K>::INF);
            bad |= in & impossible_key<K>(d[u], min_key, cc[u] == s);
        }
    }
    if (__ballot(hit) && (threadIdx.x & 63) == 0) atomicOr(&flags->inf_in_used_row, 1u);
    if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(&flags->impossible, 1u);
}

template <class K>
__global__ void k_loss_round(const uint32_t* __restrict__ PRED, const K* __restrict__ D, const K* __restrict__ W,
                             const uint32_t* __restrict__ WL, const uint32_t* __restrict__ nodes, uint32_t n,
                             uint32_t V, size_t ld, const float* __restrict__ Lin, float* __restrict__ Lout,
                             Flags* flags) {
    const size_t total = (size_t)n * V;
    uint32_t changed = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = i / V, t = i - r * V;
        const uint32_t s = nodes[r];
        const uint32_t p = PRED[r * ld + t];
        const float* Lrow = Lin + r * ld;
        float v;
        if (t == s) {
            v = 0.0f;  // Dijkstra start score PathProperties::default() (mod.rs:297)
        } else if (p == PRED_NONE) {
            v = 1.0f;  // unreachable: never read by a reachable vertex
        } else if (p != PRED_MULTI) {
            const float pl = __uint_as_float(WL[(size_t)p * ld + t]);
            v = fold_loss(Lrow[p], __fsub_rn(1.0f, pl));
        } else {
            // several latency-tight predecessors: Dijkstra keeps the smallest loss
            const K dst_st = D[(size_t)s * ld + t];
            const K* Ds = D + (size_t)s * ld;
            v = 1.0f;
            for (uint32_t u = 0; u < V; ++u) {
                if (KeyOps<K>::add(Ds[u], W[(size_t)u * ld + t]) != dst_st) continue;
                const float pl = __uint_as_float(WL[(size_t)u * ld + t]);
                const float c = fold_loss(Lrow[u], __fsub_rn(1.0f, pl));
                v = c < v ? c : v;
            }
        }
        Lout[r * ld + t] = v;
        changed |= (v != Lrow[t]);
    }
    if (changed) atomicOr(&flags->changed, 1u);
}

// Wrap check (graphs whose max edge latency x V reaches 2^64 ns only).  The reference
// sums u64 latencies with wrapping arithmetic (mod.rs:327, release build): its Dijkstra from s
// relaxes every edge (u, t) of a visited u towards a not-yet-visited t, i.e. with D[s][t] >= D[s][u]
// (ties either way), and a sum D[s][u] + w >= 2^64 ns wraps and corrupts its result.  This kernel
// flags such a relaxation for the local source rows (grid = (edge blocks, rows)): D is in latency
// units (outputs are D * unit), w in ns.  A relaxation from a vertex whose key is INF can only be
// judged when INF means unreachable; `inf_known` = 0 flags it instead (the caller reruns on wider
// keys or reports the range).
template <class K>
__global__ void __launch_bounds__(256) k_wrap_edges(uint64_t E, const uint32_t* __restrict__ src,
                                                    const uint32_t* __restrict__ dst, const uint64_t* __restrict__ lat,
                                                    int directed, const K* __restrict__ D, size_t ld,
                                                    const uint32_t* __restrict__ rows, uint64_t unit, int inf_known,
                                                    Flags* flags) {
    const K* Ds = D + (size_t)rows[blockIdx.y] * ld;
    uint32_t wrap = 0, winf = 0;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < E; e += (size_t)gridDim.x * blockDim.x) {
        const uint32_t s = src[e], t = dst[e];
        if (s == t) continue;
        const uint64_t w = lat[e];
        for (int dir = 0; dir < (directed ? 1 : 2); ++dir) {
            const uint32_t u = dir ? t : s, v = dir ? s : t;
            const K du = Ds[u], dv = Ds[v];
            if (du == KeyOps<K>::INF) {
                winf |= !inf_known;  // unknown distance: the relaxation may or may not wrap
                continue;
            }
            if (dv < du) continue;  // v was visited before u: Dijkstra skips the edge
            const unsigned __int128 sum = (unsigned __int128)du * unit + w;
            wrap |= (uint32_t)(sum >> 64) != 0;
        }
    }
    if (__ballot(wrap) && (threadIdx.x & 63) == 0) atomicOr(&flags->wrap, 1u);
    if (__ballot(winf) && (threadIdx.x & 63) == 0) atomicOr(&flags->wrap_inf, 1u);
}

// (stride 2: the packed {u, 1 - loss} PRED rows of tight_v5<true>, marker in the first word)
__global__ void __launch_bounds__(256) k_count_multi(const uint32_t* __restrict__ PRED, uint32_t n, uint32_t V,
                                                     size_t ld, unsigned long long* out, uint32_t stride = 1) {
    const uint32_t* row = PRED + (size_t)blockIdx.x * ld * stride;
    unsigned long long c = 0;
    for (uint32_t t = threadIdx.x; t < V; t += blockDim.x) c += row[(size_t)t * stride] == PRED_MULTI;
    if (c) atomicAdd(out, c);
}

// Used x used outputs for the local source rows: row a (source snodes[a]) goes to output row
// rowpos[a]; columns are the full `cols` (= nodes) list.  L == nullptr: out_loss was already
// written by k_loss_rows.
template <class K>
__global__ void __launch_bounds__(256) k_extract(const K* __restrict__ D, const float* __restrict__ L, size_t ld,
                                                 const uint32_t* __restrict__ snodes, uint32_t nloc,
                                                 const uint32_t* __restrict__ cols, uint32_t ncols,
                                                 const uint32_t* __restrict__ rowpos,
                                                 const uint64_t* __restrict__ self_lat, const float* __restrict__ self_loss,
                                                 uint64_t* __restrict__ out_lat, float* __restrict__ out_loss, Flags* flags,
                                                 int mode, uint64_t unit, uint32_t* __restrict__ out_key = nullptr,
                                                 uint64_t* __restrict__ out_diag = nullptr) {
    // out_key (RoutingInfo's key table, srg_internal_compute_table): latencies as u32 keys instead of
    // ns (0xFFFFFFFF on the diagonal, whose raw self-loop latency goes to out_diag)
    // mode bit 0: latency (+ unreachable check), bit 1: loss from L; one workgroup per local row a,
    // U columns per thread in flight (the gathers are latency-bound)
    const uint32_t a = blockIdx.x;
    const uint32_t s = snodes[a], p = rowpos[a];
    const K* Ds = D + (size_t)s * ld;
    const float* La = L ? L + (size_t)a * ld : nullptr;
    uint64_t* ol = out_lat + (size_t)p * ncols;
    uint32_t* ok = out_key ? out_key + (size_t)p * ncols : nullptr;
    float* os = out_loss + (size_t)p * ncols;
    uint32_t unreach = 0;
    constexpr uint32_t U = 4;
    for (uint32_t b0 = threadIdx.x; b0 < ncols; b0 += blockDim.x * U) {
        uint32_t tt[U];
        K d[U];
        float l[U];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            const uint32_t b = b0 + u * blockDim.x;
            tt[u] = cols[b < ncols ? b : 0];
        }
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            if (mode & 1) d[u] = Ds[tt[u]];
            if (mode & 2) l[u] = La[tt[u]];
        }
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            const uint32_t b = b0 + u * blockDim.x;
            if (b >= ncols) break;
            if (p == b) {
                // raw self-loop weight, no 1-(1-p) rounding (mod.rs:211-217)
                if (mode & 1) {
                    if (ok) {
                        ok[b] = 0xFFFFFFFFu;
                        out_diag[p] = self_lat[s];
                    } else {
                        ol[b] = self_lat[s];
                    }
                }
                if (mode & 2) os[b] = self_loss[s];
            } else {
                if (mode & 1) {
                    unreach |= d[u] == KeyOps<K>::INF;
                    if (ok) ok[b] = (uint32_t)d[u];
                    else ol[b] = (uint64_t)d[u] * unit;
                }
                if (mode & 2) os[b] = l[u];
            }
        }
    }
    if (__ballot(unreach) && (threadIdx.x & 63) == 0) atomicOr(&flags->unreachable_used_pair, 1u);
}

// k_extract's latency pass when every vertex is used in vertex order (nodes[j] == j, the GML
// complete graphs): a row copy of D at 16 B per lane (the per-column index gathers of k_extract
// ran at ~1.25 TB/s), the diagonal patched in the register before the store.  ncols % 4 == 0.
template <class K>
__global__ void __launch_bounds__(256) k_extract_ident(const K* __restrict__ D, size_t ld, const uint32_t* __restrict__ snodes,
                                                       uint32_t ncols, const uint64_t* __restrict__ self_lat,
                                                       uint64_t* __restrict__ out_lat, Flags* flags, uint64_t unit,
                                                       uint32_t* __restrict__ out_key, uint64_t* __restrict__ out_diag) {
    const uint32_t s = snodes[blockIdx.x];  // (= its output row: identity)
    const K* Ds = D + (size_t)s * ld;
    uint32_t unreach = 0;
    for (uint32_t b = threadIdx.x * 4; b < ncols; b += blockDim.x * 4) {
        K d[4];
        if constexpr (sizeof(K) == 4) {
            const uint4 v = *reinterpret_cast<const uint4*>(Ds + b);
            d[0] = v.x, d[1] = v.y, d[2] = v.z, d[3] = v.w;
        } else {
            const ulonglong2 v0 = *reinterpret_cast<const ulonglong2*>(Ds + b);
            const ulonglong2 v1 = *reinterpret_cast<const ulonglong2*>(Ds + b + 2);
            d[0] = v0.x, d[1] = v0.y, d[2] = v1.x, d[3] = v1.y;
        }
        uint64_t o[4];
        uint32_t k[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const bool diag = b + u == s;
            unreach |= !diag && d[u] == KeyOps<K>::INF;
            k[u] = diag ? 0xFFFFFFFFu : (uint32_t)d[u];
            o[u] = diag ? self_lat[s] : (uint64_t)d[u] * unit;  // raw self-loop weight (mod.rs:211-217)
        }
        if (out_key) {
            *reinterpret_cast<uint4*>(out_key + (size_t)s * ncols + b) = make_uint4(k[0], k[1], k[2], k[3]);
            if (b <= s && s < b + 4) out_diag[s] = self_lat[s];
        } else {
            uint64_t* ol = out_lat + (size_t)s * ncols + b;
            *reinterpret_cast<ulonglong2*>(ol) = make_ulonglong2(o[0], o[1]);
            *reinterpret_cast<ulonglong2*>(ol + 2) = make_ulonglong2(o[2], o[3]);
        }
    }
    if (__ballot(unreach) && (threadIdx.x & 63) == 0) atomicOr(&flags->unreachable_used_pair, 1u);
}

// min over a u64 array (RoutingInfo::get_smallest_latency_ns, mod.rs:474-476: all n^2 entries,
// diagonal included)
__global__ void k_min_u64(const uint64_t* __restrict__ a, size_t count, unsigned long long* out) {
    unsigned long long m = ~0ull;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x)
        m = a[i] < m ? a[i] : m;
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_down(m, off, 64);
        m = o < m ? o : m;
    }
    if ((threadIdx.x & 63) == 0 && m != ~0ull) atomicMin(out, m);
}

// min over a key table (the diagonal's 0xFFFFFFFF excluded by being the maximum)
__global__ void k_min_u32(const uint32_t* __restrict__ a, size_t count, unsigned long long* out) {
    uint32_t m = 0xFFFFFFFFu;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x)
        m = a[i] < m ? a[i] : m;
    for (int off = 32; off > 0; off >>= 1) {
        const uint32_t o = __shfl_down(m, off, 64);
        m = o < m ? o : m;
    }
    if ((threadIdx.x & 63) == 0 && m != 0xFFFFFFFFu) atomicMin(out, (unsigned long long)m);
}

__global__ void k_positions(const uint32_t* __restrict__ nodes, uint32_t n, int32_t* __restrict__ pos) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        pos[nodes[i]] = (int32_t)i;
}

__global__ void k_direct(uint64_t E, const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
                         const uint64_t* __restrict__ lat, const float* __restrict__ loss, int directed,
                         const int32_t* __restrict__ pos, uint32_t n, uint32_t* __restrict__ cnt,
                         uint64_t* __restrict__ out_lat, float* __restrict__ out_loss) {
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < E; e += (size_t)gridDim.x * blockDim.x) {
        const int32_t ps = pos[src[e]], pt = pos[dst[e]];
        if (ps < 0 || pt < 0) continue;
        size_t k = (size_t)ps * n + pt;
        if (atomicAdd(&cnt[k], 1u) == 0) {
            out_lat[k] = lat[e];
            out_loss[k] = loss[e];
        }
        if (!directed && ps != pt) {
            k = (size_t)pt * n + ps;
            if (atomicAdd(&cnt[k], 1u) == 0) {
                out_lat[k] = lat[e];
                out_loss[k] = loss[e];
            }
        }
    }
}

__global__ void k_direct_check(const uint32_t* __restrict__ cnt, uint32_t n, Flags* flags) {
    const size_t total = (size_t)n * n;
    unsigned long long first = ~0ull;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x)
        if (cnt[i] != 1 && i < first) first = i;
    if (first != ~0ull) atomicMin(&flags->first_bad, first);
}

// ---------------------------------------------------------------------------------------
double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace

// Host-side worker pool for the host entry's H2D codec: run(f) calls f(w, nw) on nw threads
// (the caller is worker 0) and returns when all are done.
struct HostPool {
    std::vector<std::thread> th;
    std::mutex run_mu;  // one job at a time: job / pending / gen are shared (callers on several threads queue)
    std::mutex mu;
    std::condition_variable cv, done_cv;
    std::function<void(int, int)> job;
    uint64_t gen = 0;
    int pending = 0;
    bool stop = false;
    int size() const { return (int)th.size() + 1; }
    void start(int n) {
        for (int w = 1; w < n; ++w)
            th.emplace_back([this, w] {
                uint64_t seen = 0;
                for (;;) {
                    std::function<void(int, int)> f;
                    {
                        std::unique_lock<std::mutex> lk(mu);
                        cv.wait(lk, [&] { return stop || gen != seen; });
                        if (stop) return;
                        seen = gen;
                        f = job;
                    }
                    f(w, size());
                    std::lock_guard<std::mutex> lk(mu);
                    if (--pending == 0) done_cv.notify_one();
                }
            });
    }
    void run(const std::function<void(int, int)>& f) {
        std::lock_guard<std::mutex> serial(run_mu);
        {
            std::lock_guard<std::mutex> lk(mu);
            job = f;
            pending = (int)th.size();
            ++gen;
        }
        cv.notify_all();
        f(0, size());
        std::unique_lock<std::mutex> lk(mu);
        done_cv.wait(lk, [&] { return pending == 0; });
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_all();
        for (auto& t : th) t.join();
    }
};

// The HSA agents of a HIP device (matched by PCI domain / bus / device), for SDMA copies.
struct SdmaAgents {
    bool ok = false;
    hsa_agent_t gpu{}, cpu{};
    uint32_t engine = 0;  // hsa_amd_sdma_engine_id_t bit of the engine used for D2H
    void init(int device) {
        if (hsa_init() != HSA_STATUS_SUCCESS) return;
        int bus = -1, dev = -1, dom = -1;
        if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device) != hipSuccess ||
            hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, device) != hipSuccess ||
            hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, device) != hipSuccess)
            return;
        struct Q {
            int bus, dev, dom;
            hsa_agent_t gpu{}, cpu{};
            bool found = false, have_cpu = false;
        } q{bus, dev, dom};
        hsa_iterate_agents(
            [](hsa_agent_t a, void* p) -> hsa_status_t {
                Q& q = *static_cast<Q*>(p);
                hsa_device_type_t t;
                if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
                if (t == HSA_DEVICE_TYPE_CPU && !q.have_cpu) {
                    q.cpu = a;
                    q.have_cpu = true;
                } else if (t == HSA_DEVICE_TYPE_GPU && !q.found) {
                    uint32_t bdf = 0, dom = 0;
                    if (hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf) == HSA_STATUS_SUCCESS &&
                        hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom) == HSA_STATUS_SUCCESS &&
                        (int)(bdf >> 8) == q.bus && (int)((bdf >> 3) & 31) == q.dev && (int)dom == q.dom) {
                        q.gpu = a;
                        q.found = true;
                    }
                }
                return HSA_STATUS_SUCCESS;
            },
            &q);
        if (!q.found || !q.have_cpu) return;
        uint32_t mask = 0;
        if (hsa_amd_memory_copy_engine_status(q.cpu, q.gpu, &mask) != HSA_STATUS_SUCCESS || !mask) return;
        gpu = q.gpu;
        cpu = q.cpu;
        engine = mask & (~mask + 1);  // lowest available engine
        ok = true;
    }
};

// Pinned-table pool (srg_internal_table_get / _put): the host tables a RoutingInfo owns
// (routing_info.cpp) come from their context's pool and go back to it when the RoutingInfo is
// freed, still page-locked.  The first build into a table pays the prefault + hipHostRegister
// (on the host entry's helper thread, beside the H2D and FW, as for any caller's table); a later
// build into a recycled table pays neither (the 1.2 GB C3 pair: ~12 ms cold, measured r04).
// A table can outlive its context: it holds the pool by reference count, and a closed pool frees
// what comes back.
struct TablePool;
struct srg_table {
    std::shared_ptr<TablePool> pool;
    void* p = nullptr;         // 2 MB aligned (transparent huge pages)
    size_t cap = 0;            // its bytes (a multiple of 2 MB)
    void* view = nullptr;      // its device view once registered
    bool registered = false;
};
struct TablePool {
    std::mutex mu;
    std::vector<srg_table*> idle;
    size_t idle_bytes = 0;
    // idle bytes kept (SRG_OPT_TABLE_POOL_BYTES); by default no byte cap but only the most recently
    // freed pair (a RoutingInfo's latency + loss tables): page-locked memory the OS cannot reclaim
    // stays bounded by one table set per context
    size_t limit = ~(size_t)0;
    size_t max_idle = 2;  // idle tables kept (0 = no count cap once a byte cap is set)
    bool open = true;
    static void destroy(srg_table* t);
    void trim_locked(size_t keep) {  // the oldest idle tables first
        while ((idle_bytes > keep || (max_idle && idle.size() > max_idle)) && !idle.empty()) {
            srg_table* t = idle.front();
            idle.erase(idle.begin());
            idle_bytes -= t->cap;
            destroy(t);
        }
    }
    void close() {
        std::lock_guard<std::mutex> lk(mu);
        open = false;
        trim_locked(0);
    }
};
void TablePool::destroy(srg_table* t) {
    if (t->registered) (void)hipHostUnregister(t->p);
    if (t->p) munmap(t->p, t->cap);
    delete t;
}

struct srg_ctx {
    int device = 0;
    double sparse_threshold = 0.35;  // essential-edge density above which the dense scan is used
    bool profiling = false;
    bool gather_output = true;       // multi-rank: every rank ends with all n x n outputs
    int algorithm = SRG_ALGO_AUTO;   // dense FW / sparse batched Bellman-Ford
    bool sparse_locality = true;     // sparse: batch sources in BFS order
    int sparse_delta_div = 1;        // sparse: bucket width = max edge latency / this (0 = plain BF)
    bool sparse_global_bitmaps = false;  // sparse: force the vertex bitmaps into global memory
    int fw_tile = 0;                 // 0 = auto, 64 or 128
    bool fw_symmetric = true;        // undirected + one rank: FW over the tiles I <= J only (SRG_OPT_FW_SYMMETRIC)
    int d2h_mode = 1;                // host entry D2H: 1 = SDMA engine, 0 = hipMemcpyAsync (SRG_OPT_D2H_MODE)
    DevBuf b_DST2;                   // low words of the u64-key DST (the scan input)
    SdmaAgents sdma;
    int h2d_codec = 1;               // host entry: narrowed edge list over PCIe (SRG_OPT_H2D_CODEC)
    HostPool* pool = nullptr;        // its host workers
    void* h_ring = nullptr;          // its page-locked staging ring (hipHostMalloc)
    size_t h_ring_bytes = 0;
    hipEvent_t ev_ring[3] = {nullptr, nullptr, nullptr};
    DevBuf b_n16s, b_n16d, b_n32l;   // narrowed edge arrays on the device
    DevBuf b_exc;                    // sequential-pair codec: a chunk's exceptions (index, src, dst)
    std::vector<std::vector<uint32_t>> codec_ex;  // its per-worker exception lists
    std::vector<uint32_t> slice_exc;    // the slice's exceptions (global index, src, dst), all chunks
    DevBuf b_xexc;                      // edge-sharded exchange: every rank's exceptions, counts
    size_t own_row0 = 0, own_row1 = ~(size_t)0;  // the output rows this rank routed (multi-rank: [p0, p1))
    int late_loss = 1;               // host entry: edge losses shipped beside FW (SRG_OPT_LATE_LOSS)
    hipStream_t loss_stream = nullptr;  // = d2h_stream (see srg_create)
    hipEvent_t ev_ledges = nullptr, ev_lin = nullptr, ev_ldone = nullptr, ev_wlate = nullptr;
    void* h_lring = nullptr;         // pinned ring of the late loss H2D
    hipEvent_t ev_lring[3] = {nullptr, nullptr, nullptr};
    int edge_shard = -1;             // host entry, multi-rank: ship 1/N of the edges, allgatherv the rest (SRG_OPT_EDGE_SHARD)
    const uint32_t* sim_edges = nullptr;  // simulated rank: the edge list whose other slices are resident
    size_t sim_E = 0;
    int scan_groups = 0;             // host entry: v5 scan launches interleaved with the loss rows (0 = auto: 3) (SRG_OPT_SCAN_GROUPS)
    int loss_chunks = 0;             // k_loss_rows launches (0 = auto: 8 when the host entry ships rows early, else 1) (SRG_OPT_LOSS_CHUNKS)
    srg::Comm* comm = nullptr;       // null = single GPU
    // srg_multi: the caller's output arrays are page-locked once for every rank (portable); the
    // host entry then waits for that registration (returns the arrays' device views, false if it
    // failed) instead of registering them itself
    std::function<bool(void** views, double* ms)> ext_reg;
    std::vector<hipEvent_t> prof_events;
    hipStream_t stream = nullptr;
    hipStream_t aux_stream = nullptr;   // FW lookahead: phase 1/2 of the next pivot block
    hipStream_t comm_stream = nullptr;  // pivot-panel broadcasts (multi-rank)
    hipStream_t d2h_stream = nullptr;   // host entry: output rows to the caller while kernels run
    hipEvent_t ev_a = nullptr, ev_b = nullptr, ev_c = nullptr, ev_d = nullptr, ev_e = nullptr;
    std::mutex mu;
    DevBuf b_src, b_dst, b_lat, b_loss, b_ids, b_nodes, b_olat, b_oloss;  // host-entry staging
    DevBuf b_W, b_WL, b_D, b_PRED, b_PRED2, b_L0, b_L1, b_mark, b_selfcnt, b_selflat, b_selfloss;
    DevBuf b_stats, b_flags, b_multi, b_pos, b_cnt;
    // sparse tight scan
    DevBuf b_ecnt, b_eoff, b_indeg, b_cscoff, b_cscfill, b_entkey, b_entw, b_entb, b_grpu, b_grpe, b_cscent,
        b_gblk, b_DST, b_scantmp, b_ess, b_rlen, b_roff;
    // multi-rank: local sources, their output rows, exchange staging
    DevBuf b_lnodes, b_lpos, b_red, b_outoff, b_outdst;
    DevBuf b_cflags, b_tiles, b_tslot;  // symmetric FW: closure barrier words, own tiles, packed slots
    uint32_t* fw_timeout = nullptr;     // symmetric FW: raised by a closure grid barrier that timed out
    unsigned char* hbox = nullptr;      // page-locked mailbox for small device -> host readbacks (rb_async)
    uint32_t* sig[2] = {nullptr, nullptr};  // stream_hop signals (HSA signal memory), their last values
    uint32_t sig_val[2] = {0, 0};
    bool hop_values = false;            // this build's hops use the signals (stream_hop)
    unsigned long long hop_bound_ticks = 200000000ull;  // a value hop's wait bound (100 MHz ticks; SymFw::begin)
    hipEvent_t ev_fwreset = nullptr;    // SymFw::begin: the chain stream after the reset of the FW sync words
    hipEvent_t ev_dst = nullptr;        // the scan's DST columns built (on the aux stream, beside the entry fill)
    int fw_line_split = 0;              // symmetric FW: line sub-tiles per dimension (0 = auto) (SRG_OPT_FW_LINE_SPLIT)
    int fw_step = -1;                   // symmetric FW's line exchange between ranks (SRG_OPT_FW_STEP, chain_xmode)
    DevBuf b_xlb, b_xflags;             // line buffers (kept lines / the exchange's three), peers' arrival flags
    uint32_t xepoch = 0;                // device-side exchange: this build's flag value (agreed in share_ptrs)
    std::vector<hipEvent_t> ev_ov;      // FW beside the H2D: one "chunk landed" event per chunk
    uint32_t* kout_key = nullptr;       // this call's RoutingInfo key table on the device (key mode), and
    uint64_t* kout_diag = nullptr;      // its diagonal (raw self-loop latencies per position)
    DevBuf b_odiag;
    int fw_overlap = 1;                 // host entry: FW starts while the edge list arrives (SRG_OPT_FW_OVERLAP)
    int fw_xcd_order = 1;               // symmetric FW bulk: tiles dealt to the XCDs in Z-order runs (SRG_OPT_FW_XCD_ORDER)
    int test_fault = 0;                 // TEST HOOK (SRG_OPT_TEST_FAULT): 1 = zero D after FW, 2 = stale FW sync words
    std::shared_ptr<TablePool> tpool = std::make_shared<TablePool>();  // RoutingInfo's pinned tables
    double ms_create_runtime = 0, ms_create_lib = 0;  // srg_create: HIP runtime / device init vs the library's own
    // packet-event batches (events.hip.h): key / index ping-pong buffers, tile histograms
    DevBuf b_ek0, b_ek1, b_eh0, b_eh1, b_ei0, b_ei1, b_ehist, b_eoffs, b_ered;
    ~srg_ctx() {
        for (DevBuf* b : {&b_src, &b_dst, &b_lat, &b_loss, &b_ids, &b_nodes, &b_olat, &b_oloss, &b_W, &b_WL,
                          &b_D, &b_PRED, &b_PRED2, &b_L0, &b_L1, &b_mark, &b_selfcnt, &b_selflat, &b_selfloss,
                          &b_stats, &b_flags, &b_multi, &b_pos, &b_cnt, &b_ecnt, &b_eoff, &b_indeg, &b_cscoff,
                          &b_cscfill, &b_entkey, &b_entw, &b_entb, &b_grpu, &b_grpe, &b_cscent, &b_gblk, &b_DST,
                          &b_scantmp, &b_ess, &b_rlen, &b_roff, &b_lnodes, &b_lpos, &b_red, &b_cflags, &b_tiles, &b_tslot, &b_outoff, &b_outdst, &b_xlb, &b_xflags, &b_xexc, &b_odiag,
                          &b_ek0, &b_ek1, &b_eh0, &b_eh1, &b_ei0, &b_ei1, &b_ehist, &b_eoffs, &b_ered})
            b->release();
        delete comm;
        for (hipEvent_t e : prof_events) (void)hipEventDestroy(e);
        for (uint32_t* p : sig)
            if (p) (void)hipFree(p);
        for (hipEvent_t e : {ev_a, ev_b, ev_c, ev_d, ev_e, ev_ledges, ev_lin, ev_ldone, ev_wlate, ev_fwreset, ev_dst})
            if (e) (void)hipEventDestroy(e);
        for (hipEvent_t e : ev_ov) (void)hipEventDestroy(e);
        for (hipEvent_t e : ev_lring)
            if (e) (void)hipEventDestroy(e);
        if (h_lring) (void)hipHostFree(h_lring);
        if (hbox) (void)hipHostFree(hbox);
        for (hipStream_t s : {aux_stream, comm_stream, d2h_stream, stream})
            if (s) (void)hipStreamDestroy(s);
        delete pool;
        for (hipEvent_t e : ev_ring)
            if (e) (void)hipEventDestroy(e);
        if (h_ring) (void)hipHostFree(h_ring);
        for (DevBuf* b : {&b_n16s, &b_n16d, &b_n32l, &b_DST2, &b_exc})
            b->release();
        tpool->close();
    }
};

namespace {

// Host entry with SRG_OPT_LATE_LOSS: the edge losses cross PCIe on their own stream after the
// endpoints and latencies, while the W build and FW (which need no loss) run.  Every reader of
// `DevGraph::loss` first calls loss_arrive() on its stream.
struct LateLoss {
    hipStream_t ls = nullptr;   // c.loss_stream
    std::thread th;             // queues the chunked H2D of the losses (pinned ring) on c.loss_stream
    hipEvent_t ev_in = nullptr;  // recorded by `th` after the last loss chunk
    hipEvent_t ev_done = nullptr;  // the losses and the self-loop losses are on the device
    bool joined = false, applied = false;
    std::string err;
    // edge-sharded host entry: each rank shipped only its slice's losses; they are exchanged when
    // first read (loss_arrive, at the same point on every rank): allgatherv with these segments
    srg::Comm* comm = nullptr;
    std::vector<size_t> offs, lens;
    void join() {
        if (!joined) {
            if (th.joinable()) th.join();
            joined = true;
        }
        if (!err.empty()) fail(SRG_ERR_HIP, "loss H2D: " + err);
    }
    ~LateLoss() {  // no DMA into the ring or the device losses may outlive the call
        if (th.joinable()) th.join();
        if (ls) (void)hipStreamSynchronize(ls);
    }
};

struct DevGraph {
    uint32_t V;
    int directed;
    uint64_t E;
    const uint32_t* src;
    const uint32_t* dst;
    const uint64_t* lat;
    const float* loss;
    const uint32_t* ids_dev;    // may be null
    const uint32_t* ids_host;   // may be null (host entry)
    LateLoss* late = nullptr;   // non-null: `loss` is still in flight (loss_arrive before reading it)
};

// Make `s` wait until g.loss (and the self-loop losses) are on the device.
void loss_arrive(const DevGraph& g, float* self_loss, hipStream_t s) {
    LateLoss* L = g.late;
    if (!L) return;
    L->join();  // every loss chunk is queued and ev_in recorded
    if (!L->applied) {
        HIP_CHECK(hipStreamWaitEvent(s, L->ev_in, 0));
        if (L->comm) L->comm->allgatherv(const_cast<float*>(g.loss), L->offs.data(), L->lens.data(), s);
        if (g.E) k_self_loss<<<grid_for(g.E), kThreads, 0, s>>>(g.E, g.src, g.dst, g.loss, g.V, self_loss);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipEventRecord(L->ev_done, s));
        L->applied = true;
    } else {
        HIP_CHECK(hipStreamWaitEvent(s, L->ev_done, 0));
    }
}

uint32_t node_gml_id(const DevGraph& g, uint32_t v, hipStream_t st) {
    if (g.ids_host) return g.ids_host[v];
    if (!g.ids_dev) return v;
    uint32_t id = v;
    HIP_CHECK(hipMemcpyAsync(&id, g.ids_dev + v, 4, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    return id;
}

template <class F>
void set_lds(F func, size_t bytes) {
    static_assert(sizeof(F) > 0, "");
    if (bytes > 65536)
        HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(func),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
}

// Small device -> host readbacks (flags, counters) through the context's page-locked mailbox:
// one asynchronous DMA each, read after the stream's next synchronisation.  Into pageable host
// memory the runtime stages such a copy synchronously (~20 us per call on top of the sync;
// C1 paid a dozen of them per build).  64-byte slots, kMailSlots of them.
constexpr int kMailSlots = 64;
template <class T>
void rb_async(srg_ctx& c, int slot, const T* dev, hipStream_t st) {
    static_assert(sizeof(T) <= 64, "mailbox slot");
    HIP_CHECK(hipMemcpyAsync(c.hbox + 64 * slot, dev, sizeof(T), hipMemcpyDeviceToHost, st));
}
template <class T>
T rb_get(const srg_ctx& c, int slot) {
    T v;
    std::memcpy(&v, c.hbox + 64 * slot, sizeof(T));
    return v;
}
enum MailSlot { MS_EDGESTATS, MS_FLAGS, MS_TIMEOUT, MS_REDUCE, MS_TAIL0, MS_TAIL1, MS_NMULTI, MS_CHANGED, MS_MIN, MS_REDUCE2 };

// Common validation: nodes in range & unique, edge endpoints, self-loop counts, latency range.
struct Prelude {
    EdgeStats es;
    uint32_t* selfcnt;
    uint64_t* selflat;
    float* selfloss;
    Flags* flags;
    std::vector<uint32_t> nodes_h;  // host copy of `nodes` (partitioning, error text)
    bool ident = false;             // nodes == 0, 1, ..., V - 1 (k_extract_ident)
    bool range_risk = false;         // max_key * (V-1) >= 2^62: an INF used pair on the u64 keys may be a
                                     // path >= 2^62 units (SRG_ERR_LATENCY_RANGE), not an unreachable one
    bool wrap_risk = false;          // max_lat * V >= 2^64 ns: a relaxation of the reference may wrap u64
                                     // (checked after FW by k_wrap_edges; the sparse path is not taken)
    uint64_t unit = 1;               // latency unit in ns: keys = latency / unit (compute_device)
    unsigned long long max_key = 0;  // max_lat / unit
};

Prelude prelude(srg_ctx& c, const DevGraph& g, const uint32_t* nodes, uint32_t n, hipStream_t st,
                bool check_selfloops) {
    Prelude P{};
    const uint32_t V = g.V;
    uint32_t* mark = (uint32_t*)c.b_mark.get((size_t)V * 4);
    P.selfcnt = (uint32_t*)c.b_selfcnt.get((size_t)V * 4);
    P.selflat = (uint64_t*)c.b_selflat.get((size_t)V * 8);
    P.selfloss = (float*)c.b_selfloss.get((size_t)V * 4);
    EdgeStats* es = (EdgeStats*)c.b_stats.get(sizeof(EdgeStats));
    P.flags = (Flags*)c.b_flags.get(sizeof(Flags));
    HIP_CHECK(hipMemsetAsync(mark, 0, (size_t)V * 4, st));
    HIP_CHECK(hipMemsetAsync(P.selfcnt, 0, (size_t)V * 4, st));
    HIP_CHECK(hipMemsetAsync(es, 0, sizeof(EdgeStats), st));
    HIP_CHECK(hipMemsetAsync(P.flags, 0, sizeof(Flags), st));
    if (n) k_check_nodes<<<grid_for(n), kThreads, 0, st>>>(nodes, n, V, mark, P.flags);
    if (g.E) {
        k_edge_scan<<<grid_for(g.E), kThreads, 0, st>>>(g.E, g.src, g.dst, g.lat, g.late ? nullptr : g.loss, V, P.selfcnt,
                                                       P.selflat, P.selfloss, es);
        k_lat_gcd<<<grid_for(g.E / 4, 1024), kThreads, 0, st>>>(g.E, g.src, g.dst, g.lat, &es->unit);
    }
    HIP_CHECK(hipGetLastError());
    Flags fl;
    P.nodes_h.resize(n);
    rb_async(c, MS_EDGESTATS, es, st);
    rb_async(c, MS_FLAGS, P.flags, st);
    if (n) HIP_CHECK(hipMemcpyAsync(P.nodes_h.data(), nodes, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    P.es = rb_get<EdgeStats>(c, MS_EDGESTATS);
    fl = rb_get<Flags>(c, MS_FLAGS);
    P.ident = n == V;
    for (uint32_t i = 0; i < n && P.ident; ++i) P.ident = P.nodes_h[i] == i;
    if (P.es.bad_endpoint) fail(SRG_ERR_ARG, "edge endpoint out of range (>= num_vertices)");
    if (fl.bad_node & 1) fail(SRG_ERR_ARG, "node index out of range (>= num_vertices)");
    if (fl.bad_node & 2) fail(SRG_ERR_ARG, "duplicate node index in `nodes`");
    if (check_selfloops) {
        if (P.es.lat_overflow)
            fail(SRG_ERR_LATENCY_RANGE, "The resulting value is outside of the bounds [0, 18446744073709551615]");
        // there must be a single self-loop for each node (mod.rs:215-216), in `nodes` order
        std::vector<uint32_t> cnt(V);
        HIP_CHECK(hipMemcpyAsync(cnt.data(), P.selfcnt, (size_t)V * 4, hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        for (uint32_t i = 0; i < n; ++i) {
            const uint32_t v = P.nodes_h[i];
            if (cnt[v] == 1) continue;
            const uint32_t id = node_gml_id(g, v, st);
            if (cnt[v] == 0)
                fail(SRG_ERR_NO_EDGE, "No edge connecting node " + std::to_string(id) + " to " + std::to_string(id));
            fail(SRG_ERR_MULTI_EDGE,
                 "More than one edge connecting node " + std::to_string(id) + " to " + std::to_string(id));
        }
    }
    return P;
}

struct Timer {
    hipStream_t st;
    std::chrono::steady_clock::time_point t0;
    explicit Timer(hipStream_t s) : st(s) { t0 = std::chrono::steady_clock::now(); }
    double lap() {
        HIP_CHECK(hipStreamSynchronize(st));
        double m = ms_since(t0);
        t0 = std::chrono::steady_clock::now();
        return m;
    }
};

// Host entry output sink: the caller's n x n host arrays.  Finished output rows are copied
// while later kernels run (latency rows right after FW, loss rows per chunk of k_loss_rows),
// so the 1.2 GB C3 table mostly leaves during the scan and loss pass.  The caller's (pageable)
// buffers are page-locked by a helper thread that runs concurrently with the H2D copy and FW;
// until `ready()` confirms it, nothing is sent early and the host entry copies everything at
// the end instead.
// Copy engines (SRG_OPT_D2H_MODE): 1 (default) = an SDMA engine (hsa_amd_memory_async_copy_on_engine),
// issued by a helper thread once the producing kernels' event has completed -- measured to leave
// the overlapped kernels at full speed, where hipMemcpyAsync into registered memory (0) runs as a
// full-chip blit kernel that held k_ess_mask 0.26 -> 12.7 ms and each k_loss_rows chunk
// 0.48 -> 2.2 ms (profiles/r02c/).
struct HostSink {
    uint64_t* lat = nullptr;
    float* loss = nullptr;
    void* lat_view = nullptr;   // device views of the mapped host arrays (SDMA destinations)
    void* loss_view = nullptr;
    int mode = 1;
    const SdmaAgents* sdma = nullptr;
    int device = 0;
    size_t n = 0;
    hipStream_t cs = nullptr;
    hipEvent_t ev = nullptr;
    std::function<bool()> ready;
    bool checked = false, registered = false;
    bool lat_sent = false, loss_sent = false;
    uint64_t early_bytes = 0;
    // SDMA worker
    struct Job {
        hipEvent_t ev;
        void* dst;
        const void* src;
        size_t bytes;
    };
    std::thread worker;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<Job> jobs;
    bool closing = false;
    std::string err;
    std::vector<hsa_signal_t> sigs;
    std::vector<hipEvent_t> evs;
    // latency rows as the build's u32 keys (widen = true: host entry, dense u32 build, one rank):
    // half the bytes of u64 ns over PCIe; a helper thread ships them through the context's pinned
    // ring (3 slots) on the SDMA engine and the host pool widens each slot (key x unit) into the u64
    // table while the next slots cross
    bool widen = false;
    HostPool* pool = nullptr;
    unsigned char* ring = nullptr;
    size_t ring_slot = 0;
    std::thread kthread;
    std::string kerr;
    double ms_widen = 0;
    uint64_t key_unit = 1;  // the keys' latency unit (set by the build that wrote them)
    void send_keys(hipStream_t st, const uint32_t* dkey, size_t row0, size_t rows, uint64_t unit) {
        if (!rows || !n) return;
        hipEvent_t e;
        HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        evs.push_back(e);
        HIP_CHECK(hipEventRecord(e, st));
        kthread = std::thread([this, e, dkey, row0, rows, unit]() { key_worker(e, dkey, row0, rows, unit); });
        early_bytes += rows * n * 4;
    }
    void key_worker(hipEvent_t ev, const uint32_t* dkey, size_t row0, size_t rows, uint64_t unit) {
        (void)hipSetDevice(device);
        if (hipEventSynchronize(ev) != hipSuccess) {
            kerr = "hipEventSynchronize failed before the key D2H";
            return;
        }
        const auto t0 = std::chrono::steady_clock::now();
        constexpr int NS = 3;
        const size_t rpc = std::max<size_t>(1, ring_slot / (n * 4));  // rows per chunk
        const size_t nch = (rows + rpc - 1) / rpc;
        hsa_signal_t sg[NS];
        int made = 0;
        for (; made < NS; ++made)
            if (hsa_signal_create(0, 0, nullptr, &sg[made]) != HSA_STATUS_SUCCESS) break;
        if (made < NS) {
            for (int i = 0; i < made; ++i) hsa_signal_destroy(sg[i]);
            kerr = "hsa_signal_create failed";
            return;
        }
        auto issue = [&](size_t ci) {
            const size_t r = ci * rpc, cnt = std::min(rpc, rows - r);
            hsa_signal_store_relaxed(sg[ci % NS], 1);
            if (hsa_amd_memory_async_copy_on_engine(ring + (ci % NS) * ring_slot, sdma->cpu, dkey + (row0 + r) * n, sdma->gpu,
                                                    cnt * n * 4, 0, nullptr, sg[ci % NS],
                                                    (hsa_amd_sdma_engine_id_t)sdma->engine, true) != HSA_STATUS_SUCCESS) {
                kerr = "hsa_amd_memory_async_copy_on_engine failed (keys)";
                hsa_signal_store_relaxed(sg[ci % NS], 0);
                return false;
            }
            return true;
        };
        bool ok = true;
        for (size_t ci = 0; ci < std::min<size_t>(NS, nch) && ok; ++ci) ok = issue(ci);
        for (size_t ci = 0; ci < nch && ok; ++ci) {
            hsa_signal_wait_scacquire(sg[ci % NS], HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
            const size_t r = ci * rpc, cnt = std::min(rpc, rows - r);
            const uint32_t* kb = reinterpret_cast<const uint32_t*>(ring + (ci % NS) * ring_slot);
            uint64_t* ob = lat + (row0 + r) * n;
            const size_t tot = cnt * n;
            pool->run([&](int w, int nw) {  // (the diagonal's 0xFFFFFFFF is patched by the caller)
                const size_t a = tot * w / nw, z = tot * (w + 1) / nw;
                if (unit == 1)
                    for (size_t i = a; i < z; ++i) ob[i] = kb[i];
                else
                    for (size_t i = a; i < z; ++i) ob[i] = (uint64_t)kb[i] * unit;
            });
            if (ci + NS < nch) ok = issue(ci + NS);
        }
        // drain: no copy may still target the ring when the call returns
        for (int i = 0; i < NS; ++i) {
            hsa_signal_wait_scacquire(sg[i], HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
            hsa_signal_destroy(sg[i]);
        }
        ms_widen = ms_since(t0);
    }
    bool ok() {
        if (!checked) {
            registered = ready && ready();
            checked = true;
        }
        return registered;
    }
    void work() {
        (void)hipSetDevice(device);
        for (;;) {
            Job j;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return closing || !jobs.empty(); });
                if (jobs.empty()) return;
                j = jobs.front();
                jobs.pop_front();
            }
            if (!err.empty()) continue;
            if (hipEventSynchronize(j.ev) != hipSuccess) {
                err = "hipEventSynchronize failed before a D2H copy";
                continue;
            }
            hsa_signal_t sg;
            if (hsa_signal_create(1, 0, nullptr, &sg) != HSA_STATUS_SUCCESS) {
                err = "hsa_signal_create failed";
                continue;
            }
            sigs.push_back(sg);
            if (hsa_amd_memory_async_copy_on_engine(j.dst, sdma->cpu, j.src, sdma->gpu, j.bytes, 0, nullptr, sg,
                                                    (hsa_amd_sdma_engine_id_t)sdma->engine, true) != HSA_STATUS_SUCCESS)
                err = "hsa_amd_memory_async_copy_on_engine failed";
        }
    }
    // rows [row0, row0 + rows) of a row-major n-column device array, after the work queued on st
    void send_rows(hipStream_t st, const void* dev, void* host, size_t row0, size_t rows, size_t elem) {
        const size_t off = row0 * n * elem, bytes = rows * n * elem;
        if (!bytes) return;
        const unsigned char* src = (const unsigned char*)dev + off;
        void* view = host == (void*)lat ? lat_view : host == (void*)loss ? loss_view : nullptr;
        if (mode == 1 && sdma && sdma->ok) {
            hipEvent_t e;
            HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            evs.push_back(e);
            HIP_CHECK(hipEventRecord(e, st));
            {
                std::lock_guard<std::mutex> lk(mu);
                jobs.push_back(Job{e, (unsigned char*)(view ? view : host) + off, src, bytes});
            }
            if (!worker.joinable()) worker = std::thread([this] { work(); });
            cv.notify_one();
            early_bytes += bytes;
            return;
        }
        HIP_CHECK(hipEventRecord(ev, st));
        HIP_CHECK(hipStreamWaitEvent(cs, ev, 0));
        HIP_CHECK(hipMemcpyAsync((unsigned char*)host + off, src, bytes, hipMemcpyDeviceToHost, cs));
        early_bytes += bytes;
    }
    // wait for every copy; throws on a failed one
    void finish() {
        if (kthread.joinable()) kthread.join();
        if (!kerr.empty()) fail(SRG_ERR_HIP, "key D2H: " + kerr);
        if (worker.joinable()) {
            {
                std::lock_guard<std::mutex> lk(mu);
                closing = true;
            }
            cv.notify_one();
            worker.join();
        }
        for (hsa_signal_t sg : sigs) {
            hsa_signal_wait_scacquire(sg, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
            hsa_signal_destroy(sg);
        }
        sigs.clear();
        for (hipEvent_t e : evs) (void)hipEventDestroy(e);
        evs.clear();
        HIP_CHECK(hipStreamSynchronize(cs));
        if (!err.empty()) fail(SRG_ERR_HIP, "D2H copy: " + err);
    }
    ~HostSink() {  // an exception unwound past finish(): drain before the buffers go away
        if (kthread.joinable()) kthread.join();
        if (worker.joinable()) {
            {
                std::lock_guard<std::mutex> lk(mu);
                closing = true;
            }
            cv.notify_one();
            worker.join();
        }
        for (hsa_signal_t sg : sigs) {
            hsa_signal_wait_scacquire(sg, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
            hsa_signal_destroy(sg);
        }
        for (hipEvent_t e : evs) (void)hipEventDestroy(e);
    }
};

// The caller's output arrays are page-locked for the SDMA copies; a fresh array (the Rust
// binding's vec![0u64; n*n] is lazily zeroed memory) is faulted in by that registration, 4 KB at
// a time.  Advising transparent huge pages first (the boxes run THP in "madvise" mode) lets the
// not-yet-touched part of the range fault in 2 MB pages: ~600 faults for the 1.2 GB C3 table
// instead of ~300 000.  Advisory only: pages already present stay as they are.
void advise_huge(void* p, size_t bytes) {
    const uintptr_t a = ((uintptr_t)p + ((size_t)2 << 20) - 1) & ~(uintptr_t)(((size_t)2 << 20) - 1);
    const uintptr_t e = ((uintptr_t)p + bytes) & ~(uintptr_t)(((size_t)2 << 20) - 1);
    if (e > a) (void)madvise((void*)a, e - a, MADV_HUGEPAGE);
}

// Fault a fresh output range in from several threads before it is page-locked: hipHostRegister
// faults the never-touched pages in one thread (49-58 ms for the 1.2 GB C3 table even in 2 MB
// pages, exposed after FW on a fresh table); each thread writes one byte per page of its slice (the
// table is an output: its contents are overwritten anyway).
void prefault(void* p, size_t bytes, int nthreads) {
    if (!p || bytes < ((size_t)64 << 20)) return;
    const size_t pg = 4096, per = (bytes / nthreads + pg - 1) / pg * pg;
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) {
        const size_t a = (size_t)t * per, e = std::min(bytes, a + per);
        if (a >= e) break;
        th.emplace_back([=]() {
            volatile unsigned char* b = (volatile unsigned char*)p;
            for (size_t o = a; o < e; o += pg) b[o] = 0;
        });
    }
    for (auto& x : th) x.join();
}

// Contexts per device in this process (srg_create / srg_destroy): the FW's cross-stream hops
// use stream memory operations only when a context is alone on its device (stream_hop).
std::mutex g_dev_mu;
std::map<int, int> g_dev_ctx;

// `to` waits until `from` has reached this point.  hipStreamWriteValue32 + hipStreamWaitValue32 on
// HSA signal memory cost 5 us per hop against 11 us for hipEventRecord + hipStreamWaitEvent
// (tools/xq_probe.hip; 1-3 ms of FW at N = 2..8).  The wait is a polling kernel the
// runtime knows nothing about, so it is safe only while every wait is queued behind the write it
// waits for: true for one context -- ONE host thread enqueues both halves of every hop, the write
// first (fw_line_sym: the calling thread; FwOverlap: its FW thread, which issues every launch on
// the FW and chain streams, the submitting thread only the H2D stream), and streams sharing a
// hardware queue keep that order -- not for several contexts on one device (in-process rank
// groups: two waits could each block the queue holding the other's write), nor under a profiler
// that serialises dispatches (rocprofv3 --pmc hung on it): those use events (and
// SRG_STREAM_HOPS=events forces them).
// The value form is a pair of one-wave kernels of our own instead of hipStreamWriteValue32 /
// hipStreamWaitValue32 (the same mechanism: the runtime's wait is a polling blit kernel too), so
// that the wait is bounded: past its bound it raises the FW timeout word and returns, and the host
// reports SRG_ERR_HIP after FW instead of hanging on a mis-ordered enqueue.
// The wait also returns as soon as the timeout word is set (a closure barrier gave up: nothing
// after it is valid).  That word and the closure barrier words are reset per build on the FW
// stream; SymFw::begin orders the chain stream after that reset with an EVENT.  Without it (rounds
// 3-4) a chain-stream wait could run before the reset, read the previous occupant's value of the
// word (a recycled allocation: nonzero), return at once, and the reset then erased the evidence:
// the chain ran ahead of line 0 and the build returned an all-zero table with rc = 0, or a closure
// counted arrivals into words the reset then zeroed (the barrier timeouts) -- DESIGN.md §5.
__global__ void k_hop_set(uint32_t* sig, uint32_t v) {
    if (threadIdx.x == 0) __hip_atomic_store(sig, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void k_hop_wait(const uint32_t* sig, uint32_t v, uint32_t* timeout, unsigned long long bound_ticks) {
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = wall_clock64();  // 100 MHz
    while (__hip_atomic_load(sig, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - v > 0x7FFFFFFFu) {  // sig < v (mod 2^32)
        if (__hip_atomic_load(timeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;  // keep the raiser's code
        if (wall_clock64() - t0 > bound_ticks) {
            uint32_t zero = 0;  // 2 = a hop timed out, unless something else was first
            __hip_atomic_compare_exchange_strong(timeout, &zero, 2u, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

void stream_hop(srg_ctx& c, int i, hipStream_t from, hipStream_t to, hipEvent_t ev) {
    if (c.hop_values && c.sig[i] && c.fw_timeout) {
        const uint32_t v = ++c.sig_val[i];
        k_hop_set<<<1, 64, 0, from>>>(c.sig[i], v);
        k_hop_wait<<<1, 64, 0, to>>>(c.sig[i], v, c.fw_timeout, c.hop_bound_ticks);
        HIP_CHECK(hipGetLastError());
        return;
    }
    HIP_CHECK(hipEventRecord(ev, from));
    HIP_CHECK(hipStreamWaitEvent(to, ev, 0));
}

// ---- distribution plan --------------------------------------------------
// G ranks.  FW ownership: the general FW gives rank r the whole rows of the row blocks
// [blk_lo[r], blk_lo[r+1]); the symmetric FW gives it the stored tiles (I, J) with
// (I + J) mod G == r (fw_line_sym).  After FW every rank holds the whole D.  Sources: rank r
// routes the used nodes at positions [p0, p1) = [n r / G, n (r+1) / G) of `nodes`, so its output
// rows are one contiguous range whatever the node order.
struct Plan {
    int G = 1, g = 0, nb = 0, rb0 = 0, rb1 = 0;
    std::vector<int> blk_lo;               // [G+1] first row block per rank (general FW)
    uint32_t p0 = 0, p1 = 0;               // own sources = nodes[p0 .. p1)
    std::vector<uint32_t> lnodes, lpos;    // own sources (vertex) and their output rows (p0 ..)
    int owner(int b) const { return (int)(std::upper_bound(blk_lo.begin(), blk_lo.end(), b) - blk_lo.begin()) - 1; }
    bool own(int b) const { return b >= rb0 && b < rb1; }
};

inline void tri_tile_h(int nb, int idx, int& I, int& J) {  // kernels.hip.h tri_tile, on the host
    int i = 0;
    while (i + 1 < nb && (i + 1) * nb - (i + 1) * i / 2 <= idx) ++i;
    I = i;
    J = i + (idx - (i * nb - i * (i - 1) / 2));
}

Plan make_plan(int G, int g, uint32_t V, int T, const std::vector<uint32_t>& nodes_h) {
    Plan p;
    p.G = G;
    p.g = g;
    p.nb = (int)(((size_t)V + T - 1) / T);
    p.blk_lo.resize(G + 1);
    for (int r = 0; r <= G; ++r) p.blk_lo[r] = (int)((int64_t)r * p.nb / G);
    p.blk_lo[G] = p.nb;
    p.rb0 = p.blk_lo[g];
    p.rb1 = p.blk_lo[g + 1];
    const uint64_t n = nodes_h.size();
    p.p0 = (uint32_t)(n * g / G);
    p.p1 = (uint32_t)(n * (g + 1) / G);
    for (uint32_t q = p.p0; q < p.p1; ++q) {
        p.lnodes.push_back(nodes_h[q]);
        p.lpos.push_back(q);
    }
    return p;
}

// FW lookahead chain kernels raise their wave priority (s_setprio 3) beside the bulk tiles: C3 FW
// 24.1 -> 23.5 ms (profiles/r02/prio; the option that turned it off was A/B only and is gone)
constexpr int kChainPrio = 1;

#ifndef SRG_FW_KC
#define SRG_FW_KC 32
#endif
constexpr int KC = SRG_FW_KC;

// tiles of one min-plus product launch: rows [ra, rb) minus {rx...}, cols [ca, cb) minus {cx...}
struct Rect {
    TileSet ts;
    int nr, nc;
};

inline Rect make_rect(int ra, int rb, std::initializer_list<int> rx, int ca, int cb, std::initializer_list<int> cx) {
    auto norm = [](int a, int b, std::initializer_list<int> x, int& x0, int& x1) {
        std::vector<int> v;
        for (int e : x)
            if (e >= a && e < b && std::find(v.begin(), v.end(), e) == v.end()) v.push_back(e);
        std::sort(v.begin(), v.end());
        x0 = v.size() > 0 ? v[0] : -1;
        x1 = v.size() > 1 ? v[1] : -1;
        return std::max(0, b - a - (int)v.size());
    };
    Rect r;
    r.nr = norm(ra, rb, rx, r.ts.rx0, r.ts.rx1);
    r.nc = norm(ca, cb, cx, r.ts.cx0, r.ts.cx1);
    r.ts.r0 = ra;
    r.ts.c0 = ca;
    return r;
}

// split-K factor for a short launch of `tiles` workgroups (critical-path launches only)
template <int T, int KCV>
int split_for(int tiles, bool enable) {
    if (!enable) return 1;
    constexpr int maxs = T / KCV;
    int sp = 1;
    while (sp < maxs && tiles * sp * 2 <= 512) sp *= 2;
    return sp;
}

template <int PK>
constexpr int kc_for() { return PK ? pk_kc<PK>() : KC; }

template <class K, int T, int PK>
void fw_tiles(K* D, size_t ld, int kb, int ra, int rb, std::initializer_list<int> rx, int ca, int cb,
              std::initializer_list<int> cx, size_t lds, hipStream_t s, bool split = false) {
    const Rect r = make_rect(ra, rb, rx, ca, cb, cx);
    if (r.nr <= 0 || r.nc <= 0) return;
    const int sp = split_for<T, kc_for<PK>()>(r.nr * r.nc, split);
    fw_product<K, T, kc_for<PK>(), PK><<<dim3(r.nc, r.nr, sp), 256, lds, s>>>(D, ld, kb, r.ts);
}

template <class K, int T, int PK>
void fw_tiles_pair(K* D, size_t ld, int kb, const Rect& a, const Rect& b, size_t lds, hipStream_t s,
                   bool split = false) {
    const int na = std::max(0, a.nr) * std::max(0, a.nc), nb = std::max(0, b.nr) * std::max(0, b.nc);
    if (na + nb == 0) return;
    const int sp = split_for<T, kc_for<PK>()>(na + nb, split);
    fw_product_pair<K, T, kc_for<PK>(), PK><<<dim3(na + nb, 1, sp), 256, lds, s>>>(D, ld, kb, a.ts, na, std::max(1, a.nc),
                                                                        b.ts, std::max(1, b.nc));
}

// Blocked Floyd-Warshall over the rank's row blocks with a one-block lookahead:
//   pivot kb+1's owner updates row kb+1 (w.r.t. kb) first, closes pivot kb+1 and its row
//   panel on the auxiliary stream, and broadcasts the panel (T x Vp keys, in place) while
//   every rank finishes the remaining tiles of kb; then each rank updates its own column
//   panel of kb+1.  Single GPU: the same schedule with the broadcast elided.
template <class K, int T, int PK>
void fw_blocked(srg_ctx& c, const Plan& pl, K* D, size_t Vp, hipStream_t st, uint64_t& prof_relax, int& prof_n) {
    const int nb = pl.nb;
    constexpr int KCV = kc_for<PK>();
    // double-buffered LDS image: A^T + B (add + min3 tiles) or the k-pair image (packed tiles)
    const size_t lds = PK ? pk_lds_bytes<T, KCV>() : (size_t)4 * KCV * (T + 16 / (int)sizeof(K)) * sizeof(K);
    set_lds(fw_product<K, T, KCV, PK>, lds);
    set_lds(fw_product_pair<K, T, KCV, PK>, lds);
    const bool multi = c.comm && c.comm->nranks > 1;
    const bool prof = c.profiling && nb > 2;
    if (prof) {
        while (c.prof_events.size() < (size_t)2 * nb) {
            hipEvent_t e;
            HIP_CHECK(hipEventCreate(&e));
            c.prof_events.push_back(e);
        }
    }
    hipStream_t aux = c.aux_stream, cs = c.comm_stream;
    const size_t panel_bytes = (size_t)T * Vp * sizeof(K);
    auto panel = [&](int b) { return (void*)(D + (size_t)b * T * Vp); };
    const int r0 = pl.rb0, r1 = pl.rb1;
    // pivot 0
    if (pl.own(0)) {
        fw_phase1<K, T><<<1, 512, 0, st>>>(D, Vp, 0, kChainPrio);
        fw_tiles<K, T, PK>(D, Vp, 0, 0, 1, {}, 0, nb, {0}, lds, st, pl.G > 1);
    }
    if (multi) {
        HIP_CHECK(hipEventRecord(c.ev_c, st));
        HIP_CHECK(hipStreamWaitEvent(cs, c.ev_c, 0));
        c.comm->bcast(panel(0), panel_bytes, pl.owner(0), cs);
        HIP_CHECK(hipEventRecord(c.ev_c, cs));
        HIP_CHECK(hipStreamWaitEvent(st, c.ev_c, 0));
    }
    fw_tiles<K, T, PK>(D, Vp, 0, r0, r1, {0}, 0, 1, {}, lds, st);
    for (int kb = 0; kb < nb; ++kb) {
        if (kb + 1 >= nb) {
            fw_tiles<K, T, PK>(D, Vp, kb, r0, r1, {kb}, 0, nb, {kb}, lds, st);
            break;
        }
        const int k1 = kb + 1;
        // critical chain on the (high-priority) aux stream, concurrent with the bulk tiles of kb
        // on st: row k1 + own column k1 (w.r.t. kb) in one launch -> close pivot k1 -> its row +
        // column panels.  The chain's tiles are disjoint from the bulk's; both only read panel kb.
        const bool sk = pl.G > 1;  // split-K the chain's short launches when the rest is short too
        HIP_CHECK(hipEventRecord(c.ev_a, st));  // st: bulk of kb-1 (row k1 w.r.t. kb-1) done
        HIP_CHECK(hipStreamWaitEvent(aux, c.ev_a, 0));
        const Rect rowr = pl.own(k1) ? make_rect(k1, k1 + 1, {}, 0, nb, {kb}) : Rect{TileSet{0, -1, -1, 0, -1, -1}, 0, 0};
        fw_tiles_pair<K, T, PK>(D, Vp, kb, rowr, make_rect(r0, r1, {kb, k1}, k1, k1 + 1, {}), lds, aux, sk);
        const Rect colp = make_rect(r0, r1, {k1}, k1, k1 + 1, {});  // own column panel of k1
        if (pl.own(k1)) {
            fw_phase1<K, T><<<1, 512, 0, aux>>>(D, Vp, k1, kChainPrio);
            // the column panel of k1 rewrites tile (kb, k1) of panel kb: its broadcast (still the
            // last one recorded in ev_c) must have left first
            if (multi) HIP_CHECK(hipStreamWaitEvent(aux, c.ev_c, 0));
            fw_tiles_pair<K, T, PK>(D, Vp, k1, make_rect(k1, k1 + 1, {}, 0, nb, {k1}), colp, lds, aux, sk);
        }
        if (multi) {
            HIP_CHECK(hipEventRecord(c.ev_b, aux));
            HIP_CHECK(hipStreamWaitEvent(cs, c.ev_b, 0));
            c.comm->bcast(panel(k1), panel_bytes, pl.owner(k1), cs);
            HIP_CHECK(hipEventRecord(c.ev_c, cs));
            if (!pl.own(k1)) {  // the pivot tile arrives in the panel
                HIP_CHECK(hipStreamWaitEvent(aux, c.ev_c, 0));
                fw_tiles_pair<K, T, PK>(D, Vp, k1, Rect{TileSet{0, -1, -1, 0, -1, -1}, 0, 0}, colp, lds, aux, sk);
            }
        }
        HIP_CHECK(hipEventRecord(c.ev_d, aux));
        // the remaining tiles of kb (the dominant kernel), overlapped with the above
        const int nr = (r1 - r0) - (pl.own(kb) ? 1 : 0) - (pl.own(k1) ? 1 : 0);
        const bool timed = prof && nr > 0 && nb > 2;
        if (timed) HIP_CHECK(hipEventRecord(c.prof_events[2 * prof_n], st));
        fw_tiles<K, T, PK>(D, Vp, kb, r0, r1, {kb, k1}, 0, nb, {kb, k1}, lds, st);
        if (timed) {
            HIP_CHECK(hipEventRecord(c.prof_events[2 * prof_n + 1], st));
            prof_relax += (uint64_t)nr * (nb - 2) * T * T * T;
            ++prof_n;
        }
        HIP_CHECK(hipStreamWaitEvent(st, c.ev_d, 0));
        // receivers need panel k1 before their next updates; its owner only before it rewrites a
        // tile of it (the column panel of k2 on aux, which waits above), so the owner's chain of
        // k2 overlaps the broadcast of k1
        if (multi && !pl.own(k1)) HIP_CHECK(hipStreamWaitEvent(st, c.ev_c, 0));
    }
}

// low 32 bits of u64 keys (the u64 path's scan input, tight_v5 with inf_check = 0)
__global__ void k_low_words(const uint64_t* __restrict__ x, size_t n, uint32_t* __restrict__ lo) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        lo[i] = (uint32_t)x[i];
}

// Symmetric blocked FW over line buffers (undirected graph, u32 pair-packed tiles, one or
// several ranks; kernels.hip.h fw_core_lb / LineMap).  Tile (I, J) belongs to rank (I + J) mod G.
// Per pivot kb, with k1 = kb + 1:
//   chain (aux stream, raised priority), after this rank's bulk of kb - 1:
//     1. line k1 w.r.t. kb over the rank's own tiles of line k1 -> D and the line buffer LB(k1)
//     2. (ranks > 1) allgatherv of LB(k1): one contiguous segment per rank (owner-major slots)
//     3. close the pivot tile (k1, k1) inside LB(k1): eight squaring launches of 64 workgroups
//        (every rank, redundantly)
//     4. line k1 w.r.t. k1 over all of LB(k1), own tiles written back to D (every rank)
//   bulk (main stream): the rank's stored tiles off lines kb and k1 through LB(kb).
// Line 0 needs no exchange (every rank starts from the same D).  The chain of k1 overlaps the
// bulk of kb; LB(k1) is written only after the bulk of kb - 1, the last reader of its buffer.
// At the end the lower triangle is mirrored (one rank) or the ranks' tiles are all-gathered and
// unpacked with the mirror, so that every rank holds the whole D.  shadow_amd/dist.py line_fw
// restates this schedule in numpy (tests/test_dist_cpu.py runs it on gloo ranks).
template <class K, int T>
void fw_sym_finish(srg_ctx& c, const Plan& pl, K* D, size_t Vp, hipStream_t st, const std::vector<int>& own_h,
                   const std::vector<int>& slot_h, const std::vector<int>& first, double& ms_xchg);

// this rank's stored tiles (triangle indices, row-major; uploaded to c.b_tiles), and for the final
// exchange every tile's slot in the packed buffer (owner-major, each owner's tiles in triangle order)
// The bulk's launch order (SRG_OPT_FW_XCD_ORDER): workgroup b runs on XCD b % 8 (round-robin
// dispatch), and row-major order deals consecutive tiles of a block-row -- which share their row
// operand LB[I] -- to 8 different XCDs, so every XCD's L2 fetches nearly every line-buffer tile of
// the pivot.  Here the tiles are sorted along a Z-order (Morton) curve of (I, J) and cut into 8
// contiguous runs, XCD x taking run x: each XCD works on a compact block of the triangle and reads
// only that block's rows and columns of LB.  Slots past a short run hold -1 (skipped).  One list per
// pivot kb without the tiles of lines kb and kb + 1 (the chain's), so the 8 runs stay equal: with
// those tiles returning early inside one list, the XCDs whose blocks hold line kb idled (measured
// 4 % slower than triangle order).
inline uint32_t morton2(uint32_t a, uint32_t b) {
    uint32_t z = 0;
    for (int i = 0; i < 16; ++i) z |= ((a >> i) & 1u) << (2 * i + 1) | ((b >> i) & 1u) << (2 * i);
    return z;
}
inline void xcd_tile_order(const std::vector<int>& own, int nb, std::vector<int>& out, std::vector<int>& off) {
    struct Z {
        uint32_t key;
        int t, I, J;
        bool operator<(const Z& o) const { return key < o.key; }
    };
    std::vector<Z> z(own.size());
    for (size_t i = 0; i < own.size(); ++i) {
        int I, J;
        tri_tile_h(nb, own[i], I, J);
        z[i] = {morton2((uint32_t)I, (uint32_t)J), own[i], I, J};
    }
    std::sort(z.begin(), z.end());
    out.clear();
    off.assign(nb + 1, 0);
    std::vector<int> run;
    for (int kb = 0; kb < nb; ++kb) {
        const int k1 = kb + 1;
        run.clear();
        for (const Z& q : z)
            if (q.I != kb && q.J != kb && q.I != k1 && q.J != k1) run.push_back(q.t);
        const size_t per = (run.size() + 7) / 8, base = out.size();
        out.resize(base + per * 8, -1);
        for (size_t i = 0; i < run.size(); ++i) out[base + (i % per) * 8 + i / per] = run[i];
        off[kb + 1] = (int)out.size();
    }
}

inline void sym_tiles(srg_ctx& c, const Plan& pl, hipStream_t st, std::vector<int>& own_h, std::vector<int>& slot_h,
                      std::vector<int>& first, std::vector<int>& bulk_off) {
    const int nb = pl.nb, G = pl.G, g = pl.g;
    const int ntri = nb * (nb + 1) / 2;
    own_h.clear();
    slot_h.assign(ntri, 0);
    first.assign(G + 1, 0);
    for (int t = 0, I = 0; I < nb; ++I)
        for (int J = I; J < nb; ++J, ++t) {
            const int r = (I + J) % G;
            if (r == g) own_h.push_back(t);
            ++first[r + 1];
        }
    for (int r = 0; r < G; ++r) first[r + 1] += first[r];
    std::vector<int> fill(first.begin(), first.end() - 1);
    for (int t = 0, I = 0; I < nb; ++I)
        for (int J = I; J < nb; ++J, ++t) slot_h[t] = fill[(I + J) % G]++;
    // the bulk's launch order after own_h in the same buffer: one list for every pivot
    // (xcd_tile_order), or own_h itself (bulk_off empty)
    std::vector<int> bulk;
    bulk_off.clear();
    if (c.fw_xcd_order) xcd_tile_order(own_h, nb, bulk, bulk_off);
    int* tiles = (int*)c.b_tiles.get(std::max<size_t>(own_h.size() + bulk.size(), 1) * 4);
    if (!own_h.empty()) {
        HIP_CHECK(hipMemcpyAsync(tiles, own_h.data(), own_h.size() * 4, hipMemcpyHostToDevice, st));
        HIP_CHECK(hipMemcpyAsync(tiles + own_h.size(), bulk.data(), bulk.size() * 4, hipMemcpyHostToDevice, st));
        HIP_CHECK(hipStreamSynchronize(st));  // (host vectors)
    }
}

// The schedule as a stepper: begin() builds line 0, pivot(kb, maxI) enqueues the chain of kb + 1 and
// the bulk of kb (tiles of block-rows <= maxI), end() mirrors or exchanges.  fw_line_sym runs it
// straight through; the host entry's FW beside the H2D (FwOverlap) runs pivots as block-rows of the
// edge list land, with every line kept (keep_lines) for the late tiles' catch-up.
int chain_xmode(const srg_ctx& c);

template <class K, int T>
struct SymFw {
    static constexpr int KCS = 16;
    static constexpr size_t TT = (size_t)T * T;
    srg_ctx& c;
    const Plan& pl;
    K* D;
    size_t Vp;
    hipStream_t st;
    int nb, G, g, split = 1, bulk_split = 1, ntile = 0, prio = kChainPrio;
    bool multi = false, prof = false, keep_lines = false;
    LineMap lm{1, 1};
    size_t lds_bulk = 0;
    uint32_t* cflags = nullptr;
    const int* tiles = nullptr;   // own stored tiles (triangle order), then the bulk's launch order
    std::vector<int> own_h, slot_h, first;
    std::vector<int> bulk_off;    // SRG_OPT_FW_XCD_ORDER: pivot kb's launch list at tiles + ntile + bulk_off[kb]
    K* lbuf[3] = {nullptr, nullptr, nullptr};
    K* lball = nullptr;  // keep_lines: line p at lball + p * nb * TT
    int xmode = 0;       // chain_xmode: how LB(k1) is exchanged
    std::vector<void*> plb;       // xmode 2: every rank's line-buffer block, arrival words
    std::vector<uint32_t*> pfl;
    uint32_t* myflags = nullptr;
    bool sys = false;
    uint64_t* prof_relax = nullptr;
    int* prof_n = nullptr;

    SymFw(srg_ctx& c_, const Plan& pl_, K* D_, size_t Vp_, hipStream_t st_) : c(c_), pl(pl_), D(D_), Vp(Vp_), st(st_) {
        nb = pl.nb;
        G = pl.G;
        g = pl.g;
        multi = c.comm && c.comm->nranks > 1;
        lm = LineMap{nb, G};
        xmode = chain_xmode(c);
    }
    // two line buffers round-robin; three with a device-side exchange (a peer may store LB(k1) while
    // this rank's bulk of kb - 1 still reads LB(kb - 1), never earlier: the peer's chain of k1 ran
    // after its exchange of kb, which waited for this rank's line kb, i.e. this rank's bulk of kb - 2)
    K* lb(int p) const { return keep_lines ? lball + (size_t)p * nb * TT : lbuf[xmode ? p % 3 : p & 1]; }
    void line(const K* lbL, int L, K* lbK, int K1, int mode, int ntiles, hipStream_t s) const {
        if (!ntiles) return;
        if (split == 4)
            fw_line_lb<K, T, 4><<<dim3(ntiles, 16), 256, lb_lds<K, T / 4, line_kc<4>()>(), s>>>(D, Vp, lbL, L, lbK, K1, mode, lm, g, prio);
        else if (split == 2)
            fw_line_lb<K, T, 2><<<dim3(ntiles, 4), 256, lb_lds<K, T / 2, line_kc<2>()>(), s>>>(D, Vp, lbL, L, lbK, K1, mode, lm, g, prio);
        else
            fw_line_lb<K, T, 1><<<dim3(ntiles, 1), 256, lb_lds<K, T, line_kc<1>()>(), s>>>(D, Vp, lbL, L, lbK, K1, mode, lm, g, prio);
    }
    void close_pivot(K* lbk, int k, hipStream_t s) const {
        fw_close_sq<K, T><<<dim3(T / 16, T / 16), 256, 0, s>>>(lbk + (size_t)lm.slot(k, k) * TT, cflags + 16 * k, c.fw_timeout,
                                                             prio);
    }
    void begin(uint64_t& relax, int& n) {
        prof_relax = &relax;
        prof_n = &n;
        {
            const char* hv = std::getenv("SRG_STREAM_HOPS");
            std::lock_guard<std::mutex> lk(g_dev_mu);
            c.hop_values = g_dev_ctx[c.device] == 1 && !(hv && std::strcmp(hv, "events") == 0);
        }
        lds_bulk = lb_lds<K, T, KCS>();
        set_lds(fw_bulk_lb<K, T, KCS>, lds_bulk);
        // The chain's line launches.  A large bulk (C3 on one rank: ~nb^2/2 = 3 160 tiles, four rounds
        // of the chip's 768 slots) hides the chain, so the lines take whole tiles (the fewest CU slots
        // taken from the bulk).  A bulk below ~2 rounds (several ranks, or a small graph) leaves the
        // chain as the critical path: sub-tiles, S^2 x the workgroups at a fraction of the latency
        // (SRG_OPT_FW_LINE_SPLIT; FW at sim 2:0 / 4:0 / 8:0 with whole tiles, quadrants, 32 x 32:
        // 17.9 / 15.1 / 15.6, 14.9 / 12.2 / 12.1, 11.0 / 7.7 / 7.2 ms, profiles/r03c/, r03k/; one rank,
        // C2 (nb = 32) 3.6 / 2.8 / 2.6 ms, C1 (nb = 8) 0.79 / 0.48 / 0.47 ms, profiles/r03x/).  The
        // pivot closure is one launch of 64 workgroups either way (fw_close_sq; eight squaring launches
        // took 45-117 us per pivot, the one-workgroup FW closure 159 us beside the bulk: r03b/).
        const int bulk_tiles = nb * (nb + 1) / 2 / G;
        // (C2, nb = 32, 528 tiles: quadrant lines, host entry 7.16-7.27 vs 7.39-8.76 ms with 32 x 32,
        // profiles/r06/c2/)
        split = c.fw_line_split ? c.fw_line_split : bulk_tiles >= 2048 ? 1 : bulk_tiles >= 512 ? 2 : 4;
        // a bulk below one round of the slots (3 per CU) runs as quadrants (fw_bulk_lb_q): sim 8:0
        // bulk launch 59.5 -> 48.6 us, FW 6.24-6.28 -> 6.02-6.04 ms (profiles/r05/chain/)
        // (one rank too: C2, nb = 32, 528 tiles; SRG_FW_BULK_Q = 0 / 1 forces it off / on for A/B)
        const char* bq = std::getenv("SRG_FW_BULK_Q");
        if (sizeof(K) == 4 && T == 128 && !(bq && bq[0] == '0')) {
            int cus = 256;
            HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c.device));
            if (bulk_tiles < 3 * cus || (bq && bq[0] == '1')) {
                bulk_split = 2;
                set_lds(fw_bulk_lb_q<K, T, 32>, lb_lds<K, T / 2, 32>());
            }
        }
        set_lds(fw_line_lb<K, T, 1>, lb_lds<K, T, line_kc<1>()>());
        set_lds(fw_line_lb<K, T, 2>, lb_lds<K, T / 2, line_kc<2>()>());
        set_lds(fw_line_lb<K, T, 4>, lb_lds<K, T / 4, line_kc<4>()>());
        prof = c.profiling && nb > 2;
        if (prof) {
            while (c.prof_events.size() < (size_t)2 * nb) {
                hipEvent_t e;
                HIP_CHECK(hipEventCreate(&e));
                c.prof_events.push_back(e);
            }
        }
        if (keep_lines) lball = (K*)c.b_xlb.get((size_t)nb * nb * TT * sizeof(K));
        else if (xmode) {  // one block of three (the peers' stores address it by offset)
            K* x = (K*)c.b_xlb.get(3 * (size_t)nb * TT * sizeof(K));
            for (int i = 0; i < 3; ++i) lbuf[i] = x + (size_t)i * nb * TT;
        } else {
            lbuf[0] = (K*)c.b_L0.get(nb * TT * sizeof(K));
            lbuf[1] = (K*)c.b_L1.get(nb * TT * sizeof(K));
        }
        if (xmode == 2) {  // every rank's block and arrival words (a host rendezvous per build)
            const size_t fb = (size_t)nb * G * 4;
            if (c.b_xflags.bytes < fb) {
                c.b_xflags.get(fb);
                HIP_CHECK(hipMemsetAsync(c.b_xflags.p, 0, fb, st));
            }
            myflags = (uint32_t*)c.b_xflags.p;
            HIP_CHECK(hipStreamSynchronize(st));  // zeroed words before any peer may raise one
            plb.assign(G, nullptr);
            pfl.assign(G, nullptr);
            // the flag value of this build: every rank proposes its next one and all take the largest,
            // so a rank that skipped or repeated a build cannot leave the others waiting for a stale
            // value
            uint32_t ep = c.xepoch + 1 ? c.xepoch + 1 : 1;
            c.comm->share_ptrs(lbuf[0], myflags, plb.data(), pfl.data(), &sys, &ep);
            c.xepoch = ep;
        }
        // closure barrier words: 16 per pivot (arrival counter, changed flag per step), then the
        // timeout word; zeroed per build (a multiple of 16 bytes from the allocation's start)
        cflags = (uint32_t*)c.b_cflags.get(((size_t)nb * 16 + 4) * 4);
        c.fw_timeout = cflags + (size_t)nb * 16;
#ifdef SRG_TEST_HOOKS
        if (c.test_fault == 2) {
            // TEST HOOK: the state of a recycled allocation -- nonzero sync words, zero line buffers --
            // in place before this build's reset (the value-hop race of rounds 3-4, stream_hop)
            HIP_CHECK(hipMemsetAsync(cflags, 0xA5, ((size_t)nb * 16 + 4) * 4, c.aux_stream));
            if (keep_lines) HIP_CHECK(hipMemsetAsync(lball, 0, (size_t)nb * nb * TT * sizeof(K), c.aux_stream));
            HIP_CHECK(hipStreamSynchronize(c.aux_stream));
        }
#endif
        HIP_CHECK(hipMemsetAsync(cflags, 0, ((size_t)nb * 16 + 4) * 4, st));
        // the chain stream's kernels (hop waits, closures, the exchange) read and count in these
        // words: the chain stream waits for their reset by an EVENT (a value hop's wait kernel would
        // read the very word being reset; see stream_hop)
        HIP_CHECK(hipEventRecord(c.ev_fwreset, st));
        HIP_CHECK(hipStreamWaitEvent(c.aux_stream, c.ev_fwreset, 0));
        // a value hop's wait bound: 2 s, or 20 x an estimate of the longest legitimate wait (one
        // bulk launch of this rank at ~30 T relaxations/s) when that is longer
        {
            const double relax = (double)nb * (nb + 1) / 2 / G * (double)T * T * T;
            const double ticks = 20.0 * relax / 30e12 * 1e8;
            c.hop_bound_ticks = std::max<unsigned long long>(200000000ull, (unsigned long long)std::min(ticks, 1e12));
        }
        sym_tiles(c, pl, st, own_h, slot_h, first, bulk_off);
        ntile = (int)own_h.size();
        tiles = (const int*)c.b_tiles.p;
        // line 0: every rank holds the same initial D
        k_pack_line<K, T><<<nb, 256, 0, st>>>(D, Vp, lb(0), 0, lm);
        close_pivot(lb(0), 0, st);
        line(lb(0), 0, lb(0), 0, 1, nb, st);  // (with nb == 1 this only copies the closed pivot tile back to D)
        HIP_CHECK(hipGetLastError());
    }
    // the chain of k1 = kb + 1 (aux stream) and the bulk of kb over block-rows <= maxI (main stream)
    void pivot(int kb, int maxI) {
        const int k1 = kb + 1;
        hipStream_t aux = c.aux_stream;
        K* lbk = lb(kb);
        if (k1 < nb) {
            K* lbn = lb(k1);
            stream_hop(c, 0, st, aux, c.ev_a);  // st: bulk of kb - 1 done
            line(lbk, kb, lbn, k1, 0, lm.count(g, k1), aux);
            if (multi && xmode) {
                exchange(lbn, k1, aux);
            } else if (multi) {  // on the chain's own stream: no cross-queue hop around it
                std::vector<size_t> offs(G), lens(G);
                for (int r = 0; r < G; ++r) {
                    offs[r] = (size_t)lm.base(r, k1) * TT * sizeof(K);
                    lens[r] = (size_t)lm.count(r, k1) * TT * sizeof(K);
                }
                c.comm->allgatherv(lbn, offs.data(), lens.data(), aux);
            }
            close_pivot(lbn, k1, aux);
            line(lbn, k1, lbn, k1, 1, nb, aux);
            HIP_CHECK(hipGetLastError());
        }
        // the remaining tiles of kb (the dominant kernel), overlapped with the chain of k1
        const bool timed = prof && ntile > 0 && k1 < nb && maxI >= nb - 1;
        if (timed) HIP_CHECK(hipEventRecord(c.prof_events[2 * *prof_n], st));
        auto bulk = [&](int nl, const int* list) {
            if (bulk_split == 2)
                fw_bulk_lb_q<K, T, 32><<<dim3(nl, 4), 256, lb_lds<K, T / 2, 32>(), st>>>(D, Vp, lbk, kb, kb, k1 < nb ? k1 : -1,
                                                                                         lm, list, maxI);
            else
                fw_bulk_lb<K, T, KCS><<<nl, 256, lds_bulk, st>>>(D, Vp, lbk, kb, kb, k1 < nb ? k1 : -1, lm, list, maxI);
        };
        if (!bulk_off.empty() && maxI >= nb - 1) {  // (beside the H2D, with rows still missing: triangle order,
                                                    // which spreads the missing rows' idle slots over the XCDs)
            const int nl = bulk_off[kb + 1] - bulk_off[kb];
            if (nl > 0) bulk(nl, tiles + ntile + bulk_off[kb]);
        } else if (ntile > 0) {
            bulk(ntile, tiles);
        }
        HIP_CHECK(hipGetLastError());
        if (timed) {
            int64_t m = 0;  // relaxations of this launch: own tiles off lines kb and k1
            for (int t : own_h) {
                int I, J;
                tri_tile_h(nb, t, I, J);
                if (I != kb && I != k1 && J != kb && J != k1) ++m;
            }
            HIP_CHECK(hipEventRecord(c.prof_events[2 * *prof_n + 1], st));
            *prof_relax += (uint64_t)m * T * T * T;
            ++*prof_n;
        }
        if (k1 < nb) stream_hop(c, 1, aux, st, c.ev_d);  // the chain of k1 (LB(k1) final) before the bulk of k1
    }
    // device-side exchange of LB(k1) on the chain's stream (k_line_xchg)
    void exchange(K* lbn, int k1, hipStream_t s) {
        XchgArgs<K> a{};
        a.k1 = k1;
        a.G = G;
        a.g = g;
        a.sys = sys ? 1 : 0;
        a.xmode = xmode;
        a.epoch = c.xepoch;
        a.timeout = c.fw_timeout;
        a.myflags = myflags;
        a.cnt = cflags + 16 * k1 + 13;  // a free word of the pivot's group (the closure uses 0..8)
        a.off = (size_t)lm.base(g, k1) * TT;
        a.seg = lbn + a.off;
        a.n8 = (size_t)lm.count(g, k1) * TT * sizeof(K) / 8;
        int grid = 1;
        if (xmode == 1) {
            size_t mx = 0;  // the largest segment a peer sends this rank
            for (int r = 0; r < G; ++r)
                if (r != g) mx = std::max(mx, (size_t)lm.count(r, k1) * TT * sizeof(K));
            a.model_ns = (uint32_t)c.comm->model_xchg_ns(mx);
        } else {
            const size_t blk = (size_t)lbn - (size_t)lbuf[0];  // LB(k1)'s offset inside the block
            for (int r = 0; r < G && r < kMaxPeers; ++r)
                if (r != g) {
                    a.peer_lb[r] = (K*)((unsigned char*)plb[r] + blk);
                    a.peer_flags[r] = pfl[r];
                }
            grid = (int)std::max<size_t>(1, std::min<size_t>(64, (a.n8 + 255) / 256));
        }
        k_line_xchg<K><<<grid, 256, 0, s>>>(a);
        HIP_CHECK(hipGetLastError());
    }
    void end(double& ms_xchg) {
        HIP_CHECK(hipGetLastError());
        fw_sym_finish<K, T>(c, pl, D, Vp, st, own_h, slot_h, first, ms_xchg);
    }
};

template <class K, int T>
void fw_line_sym(srg_ctx& c, const Plan& pl, K* D, size_t Vp, hipStream_t st, uint64_t& prof_relax,
                 int& prof_n, double& ms_xchg) {
    SymFw<K, T> f(c, pl, D, Vp, st);
    f.begin(prof_relax, prof_n);
    for (int kb = 0; kb < f.nb; ++kb) f.pivot(kb, f.nb);
    f.end(ms_xchg);
}

// End of the symmetric FW: mirror the lower triangle (one rank), or every rank ends with the whole D:
// pack the own tiles, all-gather, unpack with the mirror.
template <class K, int T>
void fw_sym_finish(srg_ctx& c, const Plan& pl, K* D, size_t Vp, hipStream_t st, const std::vector<int>& own_h,
                   const std::vector<int>& slot_h, const std::vector<int>& first, double& ms_xchg) {
    const int nb = pl.nb, G = pl.G, g = pl.g;
    constexpr size_t TT = (size_t)T * T;
    const bool multi = c.comm && c.comm->nranks > 1;
    const int ntri = nb * (nb + 1) / 2, ntile = (int)own_h.size();
    const int* tiles = (const int*)c.b_tiles.p;
    hipStream_t cs = c.comm_stream;
    if (!multi) {
        const unsigned nb64 = (unsigned)(Vp / 64);
        k_sym_mirror<K><<<dim3(nb64, nb64), 256, 0, st>>>(D, Vp);
        return;
    }
    HIP_CHECK(hipStreamSynchronize(st));  // (FW done: the exchange is timed on its own)
    auto t0x = std::chrono::steady_clock::now();
    K* Pk = (K*)c.b_PRED.get((size_t)ntri * TT * sizeof(K));
    int* slot = (int*)c.b_tslot.get((size_t)ntri * 4);
    HIP_CHECK(hipMemcpyAsync(slot, slot_h.data(), (size_t)ntri * 4, hipMemcpyHostToDevice, st));
    if (ntile) k_pack_tiles<K, T><<<ntile, 256, 0, st>>>(D, Vp, nb, tiles, (size_t)first[g], Pk);
    std::vector<size_t> offs(G), lens(G);
    for (int r = 0; r < G; ++r) {
        offs[r] = (size_t)first[r] * TT * sizeof(K);
        lens[r] = (size_t)(first[r + 1] - first[r]) * TT * sizeof(K);
    }
    HIP_CHECK(hipEventRecord(c.ev_b, st));
    HIP_CHECK(hipStreamWaitEvent(cs, c.ev_b, 0));
    c.comm->allgatherv(Pk, offs.data(), lens.data(), cs);
    HIP_CHECK(hipEventRecord(c.ev_c, cs));
    HIP_CHECK(hipStreamWaitEvent(st, c.ev_c, 0));
    k_unpack_tiles<K, T><<<ntri, 256, 0, st>>>(Pk, slot, nb, D, Vp);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(st));
    ms_xchg += ms_since(t0x);
}

// General FW, several ranks: every rank ends with the whole D (row blocks all-gathered)
template <class K>
void gather_rows(srg_ctx& c, const Plan& pl, K* D, size_t Vp, int T, hipStream_t st, double& ms_xchg) {
    HIP_CHECK(hipStreamSynchronize(st));  // (FW done: the exchange is timed on its own)
    auto t0x = std::chrono::steady_clock::now();
    std::vector<size_t> offs(pl.G), lens(pl.G);
    for (int r = 0; r < pl.G; ++r) {
        const size_t a = std::min<size_t>(Vp, (size_t)pl.blk_lo[r] * T), b = std::min<size_t>(Vp, (size_t)pl.blk_lo[r + 1] * T);
        offs[r] = a * Vp * sizeof(K);
        lens[r] = (b - a) * Vp * sizeof(K);
    }
    HIP_CHECK(hipEventRecord(c.ev_b, st));
    HIP_CHECK(hipStreamWaitEvent(c.comm_stream, c.ev_b, 0));
    c.comm->allgatherv(D, offs.data(), lens.data(), c.comm_stream);
    HIP_CHECK(hipEventRecord(c.ev_c, c.comm_stream));
    HIP_CHECK(hipStreamWaitEvent(st, c.ev_c, 0));
    HIP_CHECK(hipStreamSynchronize(st));
    ms_xchg += ms_since(t0x);
}

// The chain's exchange of LB(k1) (xchg.hip.h): 0 = the communicator's allgather on the chain's
// stream, 1 = a simulated rank's modelled device-side exchange, 2 = stores into the peers' line
// buffers + arrival words (k_line_xchg).  Auto (SRG_OPT_FW_STEP = -1): the modelled exchange for
// simulated ranks, else the collective; 2 asks for the stores between in-process ranks.  The stores
// stay opt-in until they have run between distinct devices (only ranks sharing one GPU
// have exercised them; such ranks then need a hardware queue each for their chain streams).
int chain_xmode(const srg_ctx& c) {
    const bool multi = c.comm && c.comm->nranks > 1;
    if (!multi || c.fw_step == 0 || c.comm->nranks > kMaxPeers) return 0;
    const int dx = c.comm->device_exchange();
    if (dx == 1) return 1;
    if (dx == 2 && c.fw_step == 2) return 2;
    return 0;
}

// the symmetric FW over line buffers applies: undirected, u32 pair-packed 128-tiles or u64 64-tiles
template <class K, int T>
bool sym_fw_for(const srg_ctx& c, const DevGraph& g) {
    return ((sizeof(K) == 4 && T == 128) || (sizeof(K) == 8 && T == 64)) && c.fw_symmetric &&
           !g.directed;
}

// The host entry's FW beside the H2D (one rank, undirected graph, symmetric FW on u32
// keys counted in ns).  A GML complete graph lists its edges by source row, each (s, d) with s <= d;
// then block-row I of W (rows [128 I, 128 (I + 1))) is complete once the chunk holding the last edge
// of its rows has landed, and block-row I is all that line I and the rows' tiles need.  Per chunk:
// the chunk's latency-only keys into KW (k_w_key, on the H2D stream); per newly complete block-row:
// its tiles split from KW into W / D (k_w_split) and caught up on the pivots whose bulks already ran
// without them (fw_catchup, from the kept final lines); then every pivot whose line is complete is
// enqueued (SymFw::pivot, bulk over the complete block-rows only).  FW thus starts while the list
// is still arriving instead of after it (C3: the H2D is ~8 ms, host-bound on the codec's encoding).
// Speculative: the keys are nanoseconds (latency unit 1) -- exact whatever the unit -- and the edge
// checks run after the H2D as before (a failed check or certification discards this FW).  Any chunk
// that is not sequential-pair, or an edge (s, d) with s > d or a source row going backwards,
// abandons the overlap (ok = false): the build then runs from the landed edge list as usual.
// The FW's launches are issued by a thread of its own (enq): from the codec's submitting thread,
// ~80 pivots x ~6 launches and waits delayed the chunk submissions, H2D 8-9 -> 11-13 ms at C3
// (profiles/r04/c3_overlap_ab.txt).  The submitting thread records one event per landed chunk and
// queues (rows complete, event); the FW thread waits on the event in its stream and enqueues.
struct FwOverlap {
    static constexpr int T = 128;
    static constexpr size_t TT = (size_t)T * T;
    srg_ctx* c = nullptr;
    hipStream_t st = nullptr;   // FW (c.stream)
    hipStream_t hs = nullptr;   // H2D chunks (c.comm_stream)
    uint32_t V = 0;
    size_t Vp = 0;
    int nb = 0;
    Plan pl;
    std::unique_ptr<SymFw<uint32_t, T>> fw;
    uint32_t *W = nullptr, *WL = nullptr, *D = nullptr;
    unsigned long long* KW = nullptr;
    int A = -1, next = 0;       // block-rows complete; pivots enqueued (FW thread)
    int splitA = -1;            // block-rows split from KW on the H2D stream (submitting thread)
    std::atomic<bool> ok{false};
    bool on = false, begun = false, ended = false;
    // the FW thread and its queue of (block-rows complete, chunk event)
    std::thread enq;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::pair<int, hipEvent_t>> q;
    bool closing = false;
    std::exception_ptr err;
    size_t nev = 0;  // chunk events used this call
    static constexpr int catchup_wgs = 768;  // catch-up launch size target (128 / 256 / 1536 measured slower)
    uint32_t prev_src = 0;
    uint64_t prof_relax = 0;
    int prof_n = 0;
    double ms_xchg = 0;
    // SRG_DEBUG_OVERLAP: timing events (H2D start, each chunk's keys landed, each pivot's bulk done)
    bool dbg = false;
    hipEvent_t e0 = nullptr;
    std::vector<hipEvent_t> ce, pe;
    std::vector<int> ca;  // block-rows complete after each chunk
    hipEvent_t tev(hipStream_t s) {
        hipEvent_t e;
        HIP_CHECK(hipEventCreate(&e));
        HIP_CHECK(hipEventRecord(e, s));
        return e;
    }
    // after the FW: when each chunk landed and how far the FW had got by then (debug only: syncs)
    void report() {
        if (!dbg || !e0) return;
        HIP_CHECK(hipStreamSynchronize(st));
        auto ms = [&](hipEvent_t e) {
            float m = 0;
            HIP_CHECK(hipEventElapsedTime(&m, e0, e));
            return m;
        };
        std::vector<float> pt(pe.size());
        for (size_t i = 0; i < pe.size(); ++i) pt[i] = ms(pe[i]);
        for (size_t i = 0; i < ce.size(); ++i) {
            const float t = ms(ce[i]);
            int done = 0;
            for (float x : pt) done += x <= t;
            std::fprintf(stderr, "fw-overlap: chunk %2zu landed %6.2f ms, block-rows %3d, pivots done %3d\n", i, t, ca[i], done);
        }
        if (!pt.empty()) std::fprintf(stderr, "fw-overlap: last pivot done %.2f ms\n", pt.back());
        {  // a few entries of each buffer (debug)
            uint32_t w = 0, d = 0, l[4] = {0, 0, 0, 0};
            unsigned long long kw = 0;
            HIP_CHECK(hipMemcpy(&w, W + 1, 4, hipMemcpyDeviceToHost));
            HIP_CHECK(hipMemcpy(&d, D + 1, 4, hipMemcpyDeviceToHost));
            HIP_CHECK(hipMemcpy(&kw, KW + 1, 8, hipMemcpyDeviceToHost));
            HIP_CHECK(hipMemcpy(l, fw->lball + 1, 16, hipMemcpyDeviceToHost));
            std::fprintf(stderr, "fw-overlap: W[0][1] %u D[0][1] %u KW[0][1] %llx LB0 %u %u %u %u\n", w, d, kw, l[0], l[1],
                         l[2], l[3]);
        }
        for (hipEvent_t e : ce) HIP_CHECK(hipEventDestroy(e));
        for (hipEvent_t e : pe) HIP_CHECK(hipEventDestroy(e));
        HIP_CHECK(hipEventDestroy(e0));
        ce.clear();
        pe.clear();
        ca.clear();
        e0 = nullptr;
    }

    void init(srg_ctx& cc, uint32_t V_, const std::vector<uint32_t>& nodes_h) {
        c = &cc;
        st = cc.stream;
        hs = cc.comm_stream;
        V = V_;
        Vp = ((size_t)V + T - 1) / T * T;
        nb = (int)(Vp / T);
        pl = make_plan(1, 0, V, T, nodes_h);
        const size_t VV = Vp * Vp;
        W = (uint32_t*)cc.b_W.get(VV * 4);
        WL = (uint32_t*)cc.b_WL.get(VV * 4);
        D = (uint32_t*)cc.b_D.get(VV * 4);
        KW = (unsigned long long*)cc.b_PRED.get(VV * 8);
        HIP_CHECK(hipMemsetAsync(KW, 0xFF, VV * 8, hs));
        fw.reset(new SymFw<uint32_t, T>(cc, pl, D, Vp, st));
        fw->keep_lines = true;
        on = true;
        ok = true;
        dbg = std::getenv("SRG_DEBUG_OVERLAP") != nullptr;
        if (dbg) e0 = tev(hs);
        enq = std::thread([this]() { run(); });
    }
    void run() {  // the FW thread: wait on each landed chunk in the FW stream, enqueue what it completes
        try {
            HIP_CHECK(hipSetDevice(c->device));
            for (;;) {
                std::pair<int, hipEvent_t> it;
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&]() { return closing || !q.empty(); });
                    if (q.empty()) return;
                    it = q.front();
                    q.pop_front();
                }
                if (!ok) continue;
                HIP_CHECK(hipStreamWaitEvent(st, it.second, 0));
                advance(it.first);
            }
        } catch (...) {
            err = std::current_exception();
            ok = false;
        }
    }
    // every queued chunk enqueued (or dropped); rethrows the FW thread's error
    void finish() {
        if (!enq.joinable()) return;
        {
            std::lock_guard<std::mutex> lk(mu);
            closing = true;
        }
        cv.notify_one();
        enq.join();
        if (err) std::rethrow_exception(err);
    }
    ~FwOverlap() {
        if (enq.joinable()) {
            {
                std::lock_guard<std::mutex> lk(mu);
                closing = true;
                ok = false;
            }
            cv.notify_one();
            enq.join();
        }
    }
    // a chunk's edges [e0, e0 + ne) are on the device (in hs order); exc = its exceptions (global
    // index, src, dst) when sequential-pair, null otherwise
    void chunk(const DevGraph& dg, size_t e0, size_t ne, const uint32_t* exc, size_t nexc, bool last) {
        if (!ok) return;
        bool good = exc != nullptr;
        for (size_t k = 0; good && k < nexc; ++k) {
            const uint32_t s = exc[3 * k + 1], d = exc[3 * k + 2];
            // a self-loop whose next edge is an exception too opens no row (W ignores it): any
            // position, e.g. a block of self-loops ahead of the rows
            const bool next_exc = k + 1 < nexc ? exc[3 * (k + 1)] == exc[3 * k] + 1 : exc[3 * k] + 1 == e0 + ne;
            if (s == d && next_exc) continue;
            good = s >= prev_src && s <= d;
            prev_src = s;
        }
        if (!good) {
            ok = false;
            return;
        }
        k_w_key<<<grid_for(ne), kThreads, 0, hs>>>(ne, dg.src + e0, dg.dst + e0, dg.lat + e0, 1, nullptr, KW, Vp, V);
        HIP_CHECK(hipGetLastError());
        // rows below the chunk's last source row are complete (all of them after the last chunk):
        // their tiles are split from KW here, on the H2D stream (beside FW: k_w_split writes the
        // upper tiles of its block-row, which FW does not touch before the row is complete, and
        // lower-triangle entries FW never reads)
        const int newA = last ? nb - 1 : std::min(nb - 1, (int)(prev_src / T) - 1);
        for (int I = splitA + 1; I <= newA; ++I)
            k_w_split<false><<<dim3((unsigned)(Vp / 64), 2), 256, 0, hs>>>(KW, Vp, 0, W, WL, D, (uint32_t)(2 * I));
        splitA = std::max(splitA, newA);
        HIP_CHECK(hipGetLastError());
        // one event per chunk (the FW thread may not have waited on the previous one yet)
        if (nev == c->ev_ov.size()) {
            hipEvent_t e;
            HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            c->ev_ov.push_back(e);
        }
        hipEvent_t ev = c->ev_ov[nev++];
        HIP_CHECK(hipEventRecord(ev, hs));
        if (dbg) {
            ce.push_back(tev(hs));
            ca.push_back(newA + 1);
        }
        {
            std::lock_guard<std::mutex> lk(mu);
            q.emplace_back(newA, ev);
        }
        cv.notify_one();
    }
    void advance(int newA) {
        for (int I = A + 1; I <= newA; ++I)
            if (I > splitA)  // (only after the H2D: the submitting thread splits every landed row)
                k_w_split<false><<<dim3((unsigned)(Vp / 64), 2), 256, 0, st>>>(KW, Vp, 0, W, WL, D, (uint32_t)(2 * I));
        if (next > 0 && newA > A) {
            // the newly complete block-rows (A, newA] catch up in ONE launch over all their tiles,
            // each workgroup a K = 128 pg product over a group of the pivots run so far.  The
            // group count minimises waves x (pg + merge): a grid just past the 768 slots (3 per CU)
            // ran a second, nearly empty wave of full-length workgroups -- rounding ceil(768 /
            // tiles) groups up did that in most C3 launches (816-918 workgroups).  Host entry
            // 47.7-48.1 vs 48.1-50.1 ms in alternating runs (profiles/r05/catchup/)
            int tiles = 0;
            for (int I = A + 1; I <= newA; ++I) tiles += nb - I;
            int pg = next;
            double best = 1e300;
            for (int g = 1; g <= next; ++g) {
                const int p = (next + g - 1) / g, gg = (next + p - 1) / p;
                const double waves = std::ceil((double)tiles * gg / catchup_wgs);
                const double cost = waves * (p + 0.25);  // (0.25: C load + atomicMin merge, in pivots)
                if (cost < best - 1e-9) best = cost, pg = p;
            }
            set_lds(fw_catchup<T>, lb_lds<uint32_t, T, 16>());
            fw_catchup<T><<<dim3(tiles, (next + pg - 1) / pg), 256, lb_lds<uint32_t, T, 16>(), st>>>(
                D, Vp, fw->lball, (size_t)nb * TT, A + 1, nb, next, pg);
        }
        HIP_CHECK(hipGetLastError());
        A = std::max(A, newA);
        if (A < 0) return;
        if (!begun) {
            fw->begin(prof_relax, prof_n);
            begun = true;
        }
        while (next < nb && (next + 1 < nb ? A >= next + 1 : A >= nb - 1)) {
            fw->pivot(next, A);
            if (dbg) pe.push_back(tev(st));
            ++next;
        }
        if (next == nb && !ended) {
            fw->end(ms_xchg);
            ended = true;
        }
    }
};

// Dense path for key type K. Returns false (u32 only) when certification fails.
template <class K, int T>
bool run_dense(srg_ctx& c, const DevGraph& g, const Plan& pl, const uint32_t* nodes, uint32_t n, uint64_t* out_lat,
               float* out_loss, hipStream_t st, const Prelude& P, srg_stats* stats, HostSink* sink,
               FwOverlap* ov = nullptr) {
    // the FW already ran beside the H2D (FwOverlap): W, D and the closed D are in place
    const bool pre = ov && ov->on && ov->ok && ov->ended && sizeof(K) == 4 && T == FwOverlap::T;
    if (sizeof(K) == 8 && c.kout_key) {  // a key table needs the u32 keys
        // (the host entry's internal key shipping just falls back to the u64 latency rows)
        if (!(sink && sink->widen)) fail(SRG_INTERNAL_NEED_U64, "the build needs u64 latency keys: no u32 key table");
        sink->widen = false;
        c.kout_key = nullptr;
        c.kout_diag = nullptr;
    }
    const uint32_t V = g.V;
    const size_t Vp = ((size_t)V + T - 1) / T * T;
    const size_t VV = Vp * Vp;
    const bool multi = c.comm && c.comm->nranks > 1;
    Timer tm(st);
    c.own_row0 = pl.p0;  // this rank's output rows (the host entry ships only these without the exchange)
    c.own_row1 = pl.p1;

    K* W = (K*)c.b_W.get(VV * sizeof(K));
    uint32_t* WL = (uint32_t*)c.b_WL.get(VV * 4);
    K* D = (K*)c.b_D.get(VV * sizeof(K));
    bool wl_late = false;  // late loss: WL is built after FW, once the losses have landed
    if (pre) {
        wl_late = g.late && !g.late->applied;
    } else if constexpr (sizeof(K) == 4) {
        // packed (latency, loss) keys: one atomic pass, then a tiled symmetrize + split pass
        static_assert(T % 64 == 0, "tile");
        unsigned long long* KW = (unsigned long long*)c.b_PRED.get(VV * 8);
        HIP_CHECK(hipMemsetAsync(KW, 0xFF, VV * 8, st));
        wl_late = g.late && !g.late->applied;
        if (g.E) k_w_key<<<grid_for(g.E), kThreads, 0, st>>>(g.E, g.src, g.dst, g.lat, P.unit, wl_late ? nullptr : g.loss, KW, Vp);
        const unsigned nb64 = (unsigned)(Vp / 64);
        k_w_split<false><<<dim3(nb64, nb64), 256, 0, st>>>(KW, Vp, g.directed, (uint32_t*)W, WL, (uint32_t*)D);
    } else {
        loss_arrive(g, P.selfloss, st);
        k_fill<K><<<grid_for(VV), kThreads, 0, st>>>(W, VV, KeyOps<K>::INF);
        HIP_CHECK(hipMemsetAsync(WL, 0xFF, VV * 4, st));
        if (g.E) {
            k_w_lat<K><<<grid_for(g.E), kThreads, 0, st>>>(g.E, g.src, g.dst, g.lat, P.unit, g.directed, W, Vp);
            k_w_loss<K><<<grid_for(g.E), kThreads, 0, st>>>(g.E, g.src, g.dst, g.lat, P.unit, g.loss, g.directed, W, WL,
                                                             Vp);
        }
        k_init_d<K><<<grid_for(VV), kThreads, 0, st>>>(W, D, Vp);
    }
    // local sources and their output rows
    const uint32_t nloc = (uint32_t)pl.lnodes.size();
    uint32_t* lnodes = (uint32_t*)c.b_lnodes.get(std::max<size_t>(nloc, 1) * 4);
    uint32_t* lpos = (uint32_t*)c.b_lpos.get(std::max<size_t>(nloc, 1) * 4);
    if (nloc) {
        HIP_CHECK(hipMemcpyAsync(lnodes, pl.lnodes.data(), (size_t)nloc * 4, hipMemcpyHostToDevice, st));
        HIP_CHECK(hipMemcpyAsync(lpos, pl.lpos.data(), (size_t)nloc * 4, hipMemcpyHostToDevice, st));
    }
    HIP_CHECK(hipGetLastError());
    const double ms_build = tm.lap();

    // ---- blocked Floyd-Warshall; afterwards every rank holds the whole D ----
    uint64_t prof_relax = 0;
    int prof_n = 0;
    double ms_dx = 0;  // multi-rank: D exchange at the end of FW (inside ms_fw, also in ms_exchange)
    if (pre) {
        prof_relax = ov->prof_relax;
        prof_n = ov->prof_n;
    } else if (sym_fw_for<K, T>(c, g)) {
        if constexpr ((sizeof(K) == 4 && T == 128) || (sizeof(K) == 8 && T == 64))
            fw_line_sym<K, T>(c, pl, D, Vp, st, prof_relax, prof_n, ms_dx);
    } else {
        // u32 keys: the pair-packed tile (two relaxations per 64-bit add + v_min3); the add + min3
        // tile (PK = 0) ran the same C3 launch in 0.304 instead of 0.242 ms (profiles/r02c/fw_fold.txt)
        // and is kept for u64 keys only
        if constexpr (sizeof(K) == 4) fw_blocked<K, T, 2>(c, pl, D, Vp, st, prof_relax, prof_n);
        else fw_blocked<K, T, 0>(c, pl, D, Vp, st, prof_relax, prof_n);
        if (multi) gather_rows<K>(c, pl, D, Vp, T, st, ms_dx);
    }
    HIP_CHECK(hipGetLastError());
    if (sym_fw_for<K, T>(c, g)) rb_async(c, MS_TIMEOUT, c.fw_timeout, st);  // read after FW, on its stream
    const double ms_fw = tm.lap();
    if (sym_fw_for<K, T>(c, g) && rb_get<uint32_t>(c, MS_TIMEOUT))
        fail(SRG_ERR_HIP, fw_timeout_message(rb_get<uint32_t>(c, MS_TIMEOUT)));
#ifdef SRG_TEST_HOOKS
    if (c.test_fault == 1)  // TEST HOOK (SRG_OPT_TEST_FAULT): a lost synchronisation's result, for the guard
        HIP_CHECK(hipMemsetAsync(D, 0, VV * sizeof(K), st));
#endif
    if (wl_late) {
        // WL = min loss among the min-latency parallel edges (what k_w_split gives), from the
        // losses that crossed PCIe during FW.  Built here, after FW, rather than beside it: on a
        // narrow grid beside the FW tiles it cost the bulk launches 5 % (0.242 -> 0.255 ms,
        // FW +0.8 ms, profiles/r02g) for about the same total.
        // The packed-key pass again, now with the losses (its buffer is free until the scan
        // writes PRED), splitting out WL only: 0.8 ms where k_w_loss's random W reads took 2.3.
        // It runs on the (idle) FW lookahead stream beside the certification, extract and
        // essential-entry count, which read W and D only; st waits for it before the entry fill.
        hipStream_t ax = c.aux_stream;  // st is synchronised (tm.lap): FW is complete
        const auto tl0 = std::chrono::steady_clock::now();
        loss_arrive(g, P.selfloss, ax);
        if (std::getenv("SRG_DEBUG_OVERLAP"))
            std::fprintf(stderr, "late loss: the host waited %.2f ms for the loss thread after FW\n",
                         std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tl0).count());
        if constexpr (sizeof(K) == 4) {
            unsigned long long* KW = (unsigned long long*)c.b_PRED.get(VV * 8);
            HIP_CHECK(hipMemsetAsync(KW, 0xFF, VV * 8, ax));
            if (g.E) k_w_key<<<grid_for(g.E), kThreads, 0, ax>>>(g.E, g.src, g.dst, g.lat, P.unit, g.loss, KW, Vp);
            const unsigned nb64 = (unsigned)(Vp / 64);
            k_w_split<true><<<dim3(nb64, nb64), 256, 0, ax>>>(KW, Vp, g.directed, nullptr, WL, nullptr);
            HIP_CHECK(hipGetLastError());
        }
        HIP_CHECK(hipEventRecord(c.ev_wlate, ax));
    }
    if (prof_n && stats) {
        double sum = 0;
        for (int i = 0; i < prof_n; ++i) {
            float ms = 0;
            HIP_CHECK(hipEventElapsedTime(&ms, c.prof_events[2 * i], c.prof_events[2 * i + 1]));
            sum += ms;
        }
        stats->prof_launches += prof_n;
        stats->prof_kernel_ms += sum;
        stats->prof_relaxations += prof_relax;
    }

    // Every collective after FW runs on the comm stream, in the same order on every rank:
    // allreduce(certify) -> allreduce(unreachable) -> allgather(latency rows, overlapped with
    // the scan) -> allgather(essential bitmask) -> allgather(loss rows).
    hipStream_t cs = c.comm_stream;
    auto cs_after_st = [&]() {
        HIP_CHECK(hipEventRecord(c.ev_a, st));
        HIP_CHECK(hipStreamWaitEvent(cs, c.ev_a, 0));
    };
    auto st_after_cs = [&]() {
        HIP_CHECK(hipEventRecord(c.ev_b, cs));
        HIP_CHECK(hipStreamWaitEvent(st, c.ev_b, 0));
    };
    auto reduce_flag = [&](uint32_t* flag_dev) -> uint32_t {
        uint32_t* red = (uint32_t*)c.b_red.get(16);
        HIP_CHECK(hipMemcpyAsync(red, flag_dev, 4, hipMemcpyDeviceToDevice, st));
        if (multi) {
            cs_after_st();
            c.comm->allreduce_max_u32(red, 1, cs);
            st_after_cs();
        }
        rb_async(c, MS_REDUCE, red, st);
        HIP_CHECK(hipStreamSynchronize(st));
        return rb_get<uint32_t>(c, MS_REDUCE);
    };
    // output rows of every rank: positions [n r / G, n (r+1) / G)
    const bool exchange = multi && c.gather_output;
    auto exchange_rows = [&](void* out, size_t elem) {  // on cs, after st
        const size_t row = (size_t)n * elem;
        std::vector<size_t> offs(pl.G), lens(pl.G);
        for (int r = 0; r < pl.G; ++r) {
            const size_t a = (uint64_t)n * r / pl.G, b = (uint64_t)n * (r + 1) / pl.G;
            offs[r] = a * row;
            lens[r] = (b - a) * row;
        }
        cs_after_st();
        c.comm->allgatherv(out, offs.data(), lens.data(), cs);
    };

    // ---- essential edges (W[u][t] == D[u][t]) counted into the scan's pair-record layout ----
    // One rank: on the comm stream (idle after the H2D), beside the certification / extract and
    // their flag read-backs on st, which read D only; several ranks: on st (cs carries collectives).
    hipStream_t es = multi ? st : c.comm_stream;
    auto drain_es = [&]() {  // (before an early return: a rerun may reallocate these buffers)
        if (es != st) HIP_CHECK(hipStreamSynchronize(es));
    };
    constexpr int TS = 64;
    constexpr int VE = 16 / (int)sizeof(K);
    const size_t nmax = std::max<uint32_t>(nloc, 1);
    uint32_t* PRED = (uint32_t*)c.b_PRED.get(nmax * Vp * 4);
    unsigned long long* multi_cnt = (unsigned long long*)c.b_multi.get(8);
    int rounds = 0;
    unsigned long long nmulti = 0;
    uint64_t n_ess = 0;
    int scan_kind = SRG_SCAN_NONE;
    bool loss_written = false;  // out_loss already filled by the per-row kernel
    float* Lfin = nullptr;
    double ms_scan = 0;
    HIP_CHECK(hipMemsetAsync(multi_cnt, 0, 8, st));
    // essential bitmask (V^2/8 bytes): every rank holds the whole D and W, so each builds all of it
    const uint32_t nw64 = (V + 63) / 64;
    unsigned long long* ess = (unsigned long long*)c.b_ess.get((size_t)V * nw64 * 8);
    k_ess_mask<K><<<V, 256, 0, es>>>(W, D, Vp, V, 0u, V, nw64, ess);
    uint32_t* indeg = (uint32_t*)c.b_indeg.get(((size_t)nw64 * 64 + 1) * 4);
    uint32_t* cscoff = (uint32_t*)c.b_cscoff.get(((size_t)nw64 * 64 + 1) * 4);
    HIP_CHECK(hipMemsetAsync(indeg, 0, ((size_t)nw64 * 64 + 1) * 4, es));
    // pair-lane LDS scan (tight_v5); u64 keys run it on the keys' low words (exact together with
    // the loss pass's multi-predecessor check, tight_sparse.hip.h)
    const bool v5lo = sizeof(K) == 8;
    const uint32_t SB = V5_SB;
    const size_t npad = ((size_t)nloc + SB - 1) / SB * SB;
    const size_t dst_bytes = (size_t)nw64 * 64 * std::max<size_t>(npad, 64) * sizeof(K);
    const uint32_t NT = nw64 * 64;
    const uint32_t nK5 = (V + V5_UC - 1) / V5_UC, nbTT5 = (NT + V5_TT - 1) / V5_TT;
    const size_t NG5 = (size_t)nbTT5 * nK5 * V5_WAVES;
    uint32_t* v5_cnt = (uint32_t*)c.b_ecnt.get((size_t)nbTT5 * nK5 * V5_TT * 4);
    uint32_t* v5_goff = (uint32_t*)c.b_eoff.get((NG5 + 1) * 4);
    uint64_t E_ess = 0, E_layout = 0;
    {
        uint32_t* v5_glen = (uint32_t*)c.b_rlen.get((NG5 + 1) * 4);
        HIP_CHECK(hipMemsetAsync(v5_cnt, 0, (size_t)nbTT5 * nK5 * V5_TT * 4, es));
        HIP_CHECK(hipMemsetAsync(v5_glen, 0, (NG5 + 1) * 4, es));
        const size_t nwaves = (size_t)nw64 * nK5;
        k_v5_count<<<(unsigned)((nwaves * 64 + 255) / 256), 256, 0, es>>>(ess, V, nw64, nK5, v5_cnt, v5_glen, indeg);
        HIP_CHECK(hipGetLastError());
        size_t ta = 0, tc = 0;
        HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, ta, indeg, cscoff, (int)(NT + 1), es));
        HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tc, v5_glen, v5_goff, (int)(NG5 + 1), es));
        const size_t tbytes = std::max(ta, tc);
        void* tmp = c.b_scantmp.get(tbytes);
        HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp, ta, indeg, cscoff, (int)(NT + 1), es));
        HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp, tc, v5_glen, v5_goff, (int)(NG5 + 1), es));
        HIP_CHECK(hipGetLastError());
    }

    // u32 certification: no saturated key in any used row (every rank must agree)
    HIP_CHECK(hipMemsetAsync(&P.flags->inf_in_used_row, 0, 4, st));
    HIP_CHECK(hipMemsetAsync(&P.flags->impossible, 0, 4, st));
    if (nloc)
        k_certify<K><<<nloc, kThreads, 0, st>>>(
            D, Vp, lnodes, nloc, nodes, n,
            // (an edge of >= INF keys counts as absent: the bound is never above INF, which stays legal)
            (K)std::min<uint64_t>(min_edge_key(P.es.min_lat_inv, P.unit), (uint64_t)KeyOps<K>::INF), P.flags);
    // (a simulated rank -- SRG_OPT_SIMULATE_RANK, timing only -- never receives its peers' line
    // segments, so its table is not a result and the guard does not apply)
    const bool simulated = c.comm && std::strcmp(c.comm->kind(), "simulated") == 0;
    // both of k_certify's flags with one read-back when one rank (each read-back is a stream drain)
    uint32_t impossible = 0, inf_any = 0;
    if (multi) {
        impossible = reduce_flag(&P.flags->impossible);
        inf_any = reduce_flag(&P.flags->inf_in_used_row);
    } else {
        rb_async(c, MS_REDUCE, &P.flags->impossible, st);
        rb_async(c, MS_REDUCE2, &P.flags->inf_in_used_row, st);
        HIP_CHECK(hipStreamSynchronize(st));
        impossible = rb_get<uint32_t>(c, MS_REDUCE);
        inf_any = rb_get<uint32_t>(c, MS_REDUCE2);
    }
    if (impossible && !simulated)
        fail(SRG_ERR_INTERNAL, "FW produced an impossible table: a used pair's latency is below the smallest edge "
                               "latency (" + std::to_string(~P.es.min_lat_inv) + " ns)");
    if (sizeof(K) == 4 && inf_any) {
        // a used pair at INF: unreachable -- unless some path could reach 2^31-1 ns, in which case
        // the u64 keys decide (the u32 FW work is redone)
        const unsigned __int128 bound = (unsigned __int128)P.max_key * (V > 1 ? V - 1 : 1);
        if (bound >= KeyOps<uint32_t>::INF) {
            if (wl_late) HIP_CHECK(hipStreamWaitEvent(st, c.ev_wlate, 0));  // the u64 rerun rewrites WL
            drain_es();
            return false;
        }
        fail(SRG_ERR_UNREACHABLE,
             "assertion `left == right` failed: paths.len() != nodes.len().pow(2) (a used node is unreachable "
             "from another used node)");
    }
    if (P.wrap_risk) {
        // max edge latency x V reaches 2^64 ns: check that no relaxation the reference runs wraps
        // its u64 sum (k_wrap_edges), and that outputs D * unit fit u64 (they are below such a sum)
        const unsigned __int128 bound = (unsigned __int128)P.max_key * (V > 1 ? V - 1 : 1);
        const bool inf_known = sizeof(K) == 4 ? bound < KeyOps<uint32_t>::INF : !P.range_risk;
        HIP_CHECK(hipMemsetAsync(&P.flags->wrap, 0, 8, st));
        for (uint32_t r0 = 0; r0 < nloc && g.E; r0 += 32768) {
            const uint32_t nr = std::min<uint32_t>(32768, nloc - r0);
            k_wrap_edges<K><<<dim3(grid_for(g.E, 64), nr), 256, 0, st>>>(g.E, g.src, g.dst, g.lat, g.directed, D, Vp,
                                                                        lnodes + r0, P.unit, inf_known ? 1 : 0, P.flags);
        }
        HIP_CHECK(hipGetLastError());
        const uint32_t wrapped = reduce_flag(&P.flags->wrap);
        if (wrapped)
            fail(SRG_ERR_LATENCY_RANGE, "a shortest-path relaxation sums past 2^64 ns (max edge latency " +
                                            std::to_string(P.es.max_lat) +
                                            " ns): the reference's u64 latency sum would wrap (mod.rs:327)");
        if (reduce_flag(&P.flags->wrap_inf)) {
            if (sizeof(K) == 4) {  // a vertex past the u32 keys: decide on the u64 keys
                if (wl_late) HIP_CHECK(hipStreamWaitEvent(st, c.ev_wlate, 0));
                drain_es();
                return false;
            }
            fail(SRG_ERR_LATENCY_RANGE, "a vertex has no path below 2^62 latency units on a graph whose u64 latency "
                                        "sums can wrap (max edge latency " +
                                            std::to_string(P.es.max_lat) + " ns)");
        }
    }

    // latency outputs (+ diagonal self-loops) of the own rows, right after FW
    HIP_CHECK(hipMemsetAsync(&P.flags->unreachable_used_pair, 0, 4, st));
    // k_extract_ident moves rows by 16-B vectors: the caller's arrays (a device-entry torch view may be
    // offset) must be 16-B aligned too (row offsets are, since n % 4 == 0)
    const bool al16 = (((uintptr_t)out_lat | (uintptr_t)c.kout_key) & 15u) == 0;
    if (nloc && P.ident && n % 4 == 0 && al16)
        k_extract_ident<K><<<nloc, 256, 0, st>>>(D, Vp, lnodes, n, P.selflat, out_lat, P.flags, P.unit, c.kout_key,
                                                 c.kout_diag);
    else if (nloc)
        k_extract<K><<<nloc, kThreads, 0, st>>>(D, nullptr, Vp, lnodes, nloc, nodes, n, lpos,
                                                                      P.selflat, P.selfloss, out_lat, out_loss,
                                                                      P.flags, 1, P.unit, c.kout_key, c.kout_diag);
    HIP_CHECK(hipGetLastError());
    if (reduce_flag(&P.flags->unreachable_used_pair)) {
        if (sizeof(K) == 8 && P.range_risk)
            fail(SRG_ERR_LATENCY_RANGE, "a used pair has no path below 2^62 latency units (max edge latency " +
                                            std::to_string(P.es.max_lat) +
                                            " ns): unreachable, or a latency sum the reference's u64 would wrap");
        fail(SRG_ERR_UNREACHABLE,
             "assertion `left == right` failed: paths.len() != nodes.len().pow(2) (a used node is unreachable "
             "from another used node)");
    }
    if (exchange) exchange_rows(out_lat, 8);  // overlaps the scan and the loss pass below
    // host entry, own rows only (one rank, or several without the exchange): the latency rows are
    // final -- they leave during the scan / loss pass
    const bool sink_rows = sink && !exchange && nloc && sink->ok();
    if (sink && c.kout_key) sink->key_unit = P.unit;
    if (sink_rows) {
        if (c.kout_key && sink->widen) sink->send_keys(st, c.kout_key, pl.p0, nloc, P.unit);  // (widened on the host)
        else if (c.kout_key) sink->send_rows(st, c.kout_key, sink->lat, pl.p0, nloc, 4);  // (sink->lat: the host key table)
        else sink->send_rows(st, out_lat, sink->lat, pl.p0, nloc, 8);
        sink->lat_sent = true;
    }

    // ---- tight-predecessor scan, loss (the essential entries were counted above) ----
    {
        rb_async(c, MS_TAIL0, cscoff + NT, es);
        rb_async(c, MS_TAIL1, v5_goff + NG5, es);
        HIP_CHECK(hipStreamSynchronize(es));
        E_ess = rb_get<uint32_t>(c, MS_TAIL0);
        E_layout = 2ull * rb_get<uint32_t>(c, MS_TAIL1);
    }
    n_ess = E_ess;
    if (wl_late) HIP_CHECK(hipStreamWaitEvent(st, c.ev_wlate, 0));  // WL (late loss) before the entry fill
    const bool sparse = (double)E_ess <= c.sparse_threshold * (double)V * (double)V &&
                        E_layout + 256 < 0xF0000000ull && dst_bytes < 0xFFFFFFFFull;
    if (sparse) {
        scan_kind = SRG_SCAN_SPARSE;
        // the scan's DST (D columns of the used sources, + their low words for u64 keys) on the aux
        // stream, beside the entry fill: it reads D only (st is past FW)
        K* DST = nullptr;
        const uint32_t* DSTs = nullptr;
        uint32_t dsts_bytes = 0;
        if (nloc) {
            hipStream_t ax = c.aux_stream;
            const uint32_t nbS = (uint32_t)(npad / 64);
            DST = (K*)c.b_DST.get(dst_bytes);
            k_build_dst<K><<<dim3(nw64, nbS), 256, 0, ax>>>(D, Vp, lnodes, nloc, DST, npad);
            DSTs = (const uint32_t*)DST;
            dsts_bytes = (uint32_t)std::min<size_t>(dst_bytes, 0xFFFFFFFFull);
            if (v5lo) {
                const size_t cnt = dst_bytes / 8;
                uint32_t* lo = (uint32_t*)c.b_DST2.get(cnt * 4);
                k_low_words<<<grid_for(cnt), kThreads, 0, ax>>>(reinterpret_cast<const uint64_t*>(DST), cnt, lo);
                DSTs = lo;
                dsts_bytes = (uint32_t)(cnt * 4);
            }
            HIP_CHECK(hipGetLastError());
            HIP_CHECK(hipEventRecord(c.ev_dst, ax));
        }
        const size_t Eb = E_layout + 256;
        uint32_t* cscpos = (uint32_t*)c.b_cscfill.get((size_t)nbTT5 * nK5 * V5_TT * 4);
        K* ent_w = (K*)c.b_entw.get(Eb * sizeof(K));
        uint2* ent_ub = (uint2*)c.b_grpe.get(Eb * 8);  // {u, 1 - loss bits}: one gather in the loss pass
        uint32_t* cscent = (uint32_t*)c.b_cscent.get(std::max<uint64_t>(E_ess, 1) * 4);
        k_v5_cscpos<<<(NT + 255) / 256, 256, 0, st>>>(v5_cnt, cscoff, NT, nK5, cscpos);
        uint2* rec = (uint2*)c.b_entkey.get((Eb + V5_SLACK) * 8);
        {
            const size_t nwaves = (size_t)nw64 * nK5;
            k_v5_fill<K><<<(unsigned)((nwaves * 64 + 255) / 256), 256, 0, st>>>(ess, W, WL, Vp, V, nw64, nK5, v5_cnt,
                                                                                  v5_goff, cscpos, rec, ent_w,
                                                                                  ent_ub, cscent);
        }
        HIP_CHECK(hipGetLastError());
        // host entry, one rank, per-row LDS loss: scan groups interleaved with the loss rows
        const size_t lds_rows = loss_rows_lds(V);
        const uint32_t scan_groups = c.scan_groups ? (uint32_t)c.scan_groups : 3u;
        const bool interleave = sink_rows && lds_rows <= 150 * 1024 && scan_groups > 1;
        if (interleave) {
            set_lds(k_loss_rows<K, true>, lds_rows);
            HIP_CHECK(hipMemsetAsync(&P.flags->changed, 0, 4, st));
        }
        // the per-row LDS loss pass reads PRED packed with each single predecessor's {u, 1 - loss}
        // (k_pred_pack, after each scan group); the global-memory fold the entry indices
        uint32_t* PREDK = lds_rows <= 150 * 1024 ? (uint32_t*)c.b_PRED2.get(nmax * Vp * 8) : nullptr;
        auto pack_pred = [&](uint32_t r0, uint32_t r1) {
            const uint32_t nsb = (r1 - r0 + 127) / 128, nt8 = (nbTT5 + 7) / 8;
            k_pred_pack<<<8u * nt8 * nsb, 256, 0, st>>>(PRED, Vp, r0, r1, NT, nbTT5, nsb, ent_ub, (uint2*)PREDK,
                                                        multi_cnt);
            HIP_CHECK(hipGetLastError());
        };
        if (nloc) {
            HIP_CHECK(hipStreamWaitEvent(st, c.ev_dst, 0));  // (the scan's DST, built on the aux stream)
            const uint32_t inf_check = v5lo ? 0u : 1u;
            const uint32_t nbS5 = (uint32_t)(npad / SB);
            // host entry: the scan runs in source-block groups, each group's loss rows folded right
            // after it and shipped while later groups scan (loss rows on a second stream beside the
            // next group's scan were starved of CUs: 24.7 ms vs 20.8)
            const uint32_t ng = interleave ? std::min<uint32_t>(scan_groups, nbS5) : 1u;
            for (uint32_t gi = 0; gi < ng; ++gi) {
                // group bounds on multiples of 8 source blocks: every XCD gets the same number of
                // blocks per launch (20 blocks = 3/3/3/3/2/2/2/2 ran 33 % long)
                auto cut = [&](uint32_t q) {
                    if (q == 0) return 0u;
                    if (q == ng) return nbS5;
                    // three groups: half, then all but the last partial 8 blocks, so the loss rows
                    // left to ship after the last fold are few (C3 40 / 32 / 7 blocks: exposed D2H
                    // 1.8 -> 0.8 ms, scan + tail -0.6 ms vs thirds, profiles/r02i/scan_cuts.txt)
                    const uint32_t half = std::min(nbS5, (nbS5 / 2 + 4) / 8 * 8), last = (nbS5 - 1) / 8 * 8;
                    if (ng == 3 && half > 0 && last > half) return q == 1 ? half : last;
                    return std::min(nbS5, (nbS5 * q / ng + 4) / 8 * 8);
                };
                const uint32_t c0 = cut(gi), c1 = cut(gi + 1);
                if (c1 == c0) continue;
                const uint32_t nblk = (nbTT5 + 3) / 4 * ((c1 - c0 + 7) / 8);
                tight_v5<<<8u * 32u * ((nblk + 7) / 8), V5_WAVES * 64, 0, st>>>(
                    DSTs, npad, dsts_bytes, lnodes, nloc, V, NT, nbTT5, c1, nK5, c0, v5_goff,
                    (const uint32_t*)c.b_entkey.get(0), PRED, Vp, inf_check);
                HIP_CHECK(hipGetLastError());
                if (interleave) {
                    const uint32_t r0 = c0 * SB, r1 = std::min<uint32_t>(c1 * SB, nloc);
                    if (r1 <= r0) continue;
                    pack_pred(r0, r1);
                    k_loss_rows<K, true><<<r1 - r0, 1024, lds_rows, st>>>(PREDK, Vp, V, lnodes, nloc, ent_ub, ent_w,
                                                                   DST, npad, cscoff, cscent, P.selfloss, nodes, n,
                                                                   lpos, out_loss, &P.flags->changed, r0);
                    HIP_CHECK(hipGetLastError());
                    sink->send_rows(st, out_loss, sink->loss, pl.p0 + r0, r1 - r0, 4);
                }
            }
            if (!PREDK) k_count_multi<<<nloc, kThreads, 0, st>>>(PRED, nloc, V, Vp, multi_cnt);  // (else k_pred_pack counted)
            HIP_CHECK(hipGetLastError());
            ms_scan = tm.lap();
            if (interleave) {  // loss rows already folded and shipped, group by group
                sink->loss_sent = true;
                rb_async(c, MS_CHANGED, &P.flags->changed, st);
                HIP_CHECK(hipStreamSynchronize(st));
                rounds = (int)rb_get<uint32_t>(c, MS_CHANGED);
                loss_written = true;
            } else if (lds_rows <= 150 * 1024) {
                // per-row Gauss-Seidel in LDS, writes out_loss directly
                set_lds(k_loss_rows<K, true>, lds_rows);
                HIP_CHECK(hipMemsetAsync(&P.flags->changed, 0, 4, st));
                // host entry: row chunks, each chunk's loss rows sent as soon as it is done
                pack_pred(0, nloc);
                const uint32_t nchunk = std::max<uint32_t>(1, std::min<uint32_t>(c.loss_chunks ? c.loss_chunks : sink_rows ? 8 : 1, nloc));
                for (uint32_t q = 0; q < nchunk; ++q) {
                    const uint32_t r0 = (uint32_t)((uint64_t)nloc * q / nchunk);
                    const uint32_t r1 = (uint32_t)((uint64_t)nloc * (q + 1) / nchunk);
                    if (r1 == r0) continue;
                    k_loss_rows<K, true><<<r1 - r0, 1024, lds_rows, st>>>(PREDK, Vp, V, lnodes, nloc, ent_ub, ent_w,
                                                                   DST, npad, cscoff, cscent, P.selfloss, nodes, n,
                                                                   lpos, out_loss, &P.flags->changed, r0);
                    HIP_CHECK(hipGetLastError());
                    if (sink_rows) sink->send_rows(st, out_loss, sink->loss, pl.p0 + r0, r1 - r0, 4);
                }
                if (sink_rows) sink->loss_sent = true;
                rb_async(c, MS_CHANGED, &P.flags->changed, st);
                HIP_CHECK(hipStreamSynchronize(st));
                rounds = (int)rb_get<uint32_t>(c, MS_CHANGED);
                loss_written = true;
            } else {
                float* L0 = (float*)c.b_L0.get(nmax * Vp * 4);
                float* L1 = (float*)c.b_L1.get(nmax * Vp * 4);
                k_fill<float><<<grid_for((size_t)nloc * Vp), kThreads, 0, st>>>(L0, (size_t)nloc * Vp, 1.0f);
                float* Lin = L0;
                float* Lout = L1;
                for (;;) {
                    HIP_CHECK(hipMemsetAsync(&P.flags->changed, 0, 4, st));
                    k_loss_round_sparse<K><<<grid_for((size_t)nloc * V, 256 * 64), kThreads, 0, st>>>(
                        PRED, Vp, DST, npad, lnodes, nloc, V, ent_ub, ent_w, cscoff, cscent, Lin, Lout,
                        &P.flags->changed);
                    HIP_CHECK(hipGetLastError());
                    ++rounds;
                    rb_async(c, MS_CHANGED, &P.flags->changed, st);
                    HIP_CHECK(hipStreamSynchronize(st));
                    const uint32_t ch = rb_get<uint32_t>(c, MS_CHANGED);
                    std::swap(Lin, Lout);
                    if (!ch) break;
                    if (rounds > (int)V + 2) fail(SRG_ERR_INTERNAL, "loss rounds did not converge");
                }
                Lfin = Lin;
            }
        }
    } else {
        scan_kind = SRG_SCAN_DENSE;
        if (nloc) {
            const size_t lds3 = (size_t)2 * KC * (TS + VE) * sizeof(K);
            set_lds(tight_scan<K, TS, KC>, lds3);
            tight_scan<K, TS, KC><<<dim3((unsigned)(Vp / TS), (nloc + TS - 1) / TS), 256, lds3, st>>>(D, W, Vp, lnodes,
                                                                                                    nloc, PRED);
            k_count_multi<<<nloc, kThreads, 0, st>>>(PRED, nloc, V, Vp, multi_cnt);
            float* L0 = (float*)c.b_L0.get(nmax * Vp * 4);
            float* L1 = (float*)c.b_L1.get(nmax * Vp * 4);
            k_fill<float><<<grid_for((size_t)nloc * Vp), kThreads, 0, st>>>(L0, (size_t)nloc * Vp, 1.0f);
            HIP_CHECK(hipGetLastError());
            ms_scan = tm.lap();
            float* Lin = L0;
            float* Lout = L1;
            for (;;) {
                HIP_CHECK(hipMemsetAsync(&P.flags->changed, 0, 4, st));
                k_loss_round<K><<<grid_for((size_t)nloc * V, 256 * 64), kThreads, 0, st>>>(
                    PRED, D, W, WL, lnodes, nloc, V, Vp, Lin, Lout, P.flags);
                HIP_CHECK(hipGetLastError());
                ++rounds;
                rb_async(c, MS_CHANGED, &P.flags->changed, st);
                HIP_CHECK(hipStreamSynchronize(st));
                const uint32_t ch = rb_get<uint32_t>(c, MS_CHANGED);
                std::swap(Lin, Lout);
                if (!ch) break;
                if (rounds > (int)V + 2) fail(SRG_ERR_INTERNAL, "loss rounds did not converge");
            }
            Lfin = Lin;
        }
    }
    rb_async(c, MS_NMULTI, multi_cnt, st);
    const double ms_loss = tm.lap();
    nmulti = rb_get<unsigned long long>(c, MS_NMULTI);

    if (nloc && !loss_written)
        k_extract<K><<<nloc, kThreads, 0, st>>>(D, Lfin, Vp, lnodes, nloc, nodes, n, lpos,
                                                                      P.selflat, P.selfloss, out_lat, out_loss,
                                                                      P.flags, 2, P.unit);
    HIP_CHECK(hipGetLastError());
    const double ms_extract = tm.lap();

    // ---- output exchange: every rank ends with all n x n rows ----
    double ms_exchange = 0;
    if (exchange) {
        exchange_rows(out_loss, 4);
        st_after_cs();
        ms_exchange = tm.lap();
    }
    if (stats) {
        stats->ms_build += ms_build;
        stats->ms_fw += ms_fw;
        stats->ms_scan += ms_scan;
        stats->ms_loss += ms_loss;
        stats->ms_extract += ms_extract;
        stats->ms_exchange += ms_exchange + ms_dx;
        stats->path_kind = sizeof(K) == 4 ? SRG_PATH_DENSE_U32 : SRG_PATH_DENSE_U64;
        stats->loss_rounds = rounds;
        stats->multi_pred_pairs = nmulti;
        uint64_t own_tiles = 0;  // symmetric FW: this rank's stored tiles ((I + J) mod G == g)
        for (int I = 0; I < pl.nb; ++I)
            for (int J = I; J < pl.nb; ++J) own_tiles += (I + J) % pl.G == pl.g;
        stats->relaxations = sym_fw_for<K, T>(c, g) ? own_tiles * (uint64_t)pl.nb * T * T * T
                                                    : (uint64_t)(pl.rb1 - pl.rb0) * T * Vp * Vp;
        stats->essential_edges = n_ess;
        stats->scan_kind = scan_kind;
        stats->nranks = pl.G;
        stats->rank = pl.g;
        stats->local_sources = nloc;
    }
    return true;
}

// ---- sparse path: batched lexicographic Bellman-Ford (sparse.hip.h) ----------------------
// Rank r routes the used sources at positions [r*n/G, (r+1)*n/G) (contiguous output rows).
// Returns false when a used pair came out saturated/unreachable and the graph's latencies
// could exceed the u32 keys: the caller then reruns on the wide (u64-key) labels.
bool run_sparse(srg_ctx& c, const DevGraph& g, const uint32_t* nodes, uint32_t n, uint64_t* out_lat,
                float* out_loss, hipStream_t st, const Prelude& P, srg_stats* stats, bool wide = false) {
    if (wide && c.kout_key) fail(SRG_INTERNAL_NEED_U64, "the build needs u64 latency keys: no u32 key table");
    const uint32_t V = g.V;
    const bool multi = c.comm && c.comm->nranks > 1;
    const int G = multi ? c.comm->nranks : 1, rk = multi ? c.comm->rank : 0;
    Timer tm(st);
    uint32_t* off = (uint32_t*)c.b_indeg.get(((size_t)V + 1) * 4);
    uint32_t* cur = (uint32_t*)c.b_cscfill.get(((size_t)V + 1) * 4);
    const uint32_t* esrc = g.src;
    const uint32_t* edst = g.dst;
    const uint64_t* selflat = P.selflat;
    const float* selfloss = P.selfloss;
    const uint32_t* cols = nodes;
    // CSR of in-arcs
    HIP_CHECK(hipMemsetAsync(cur, 0, ((size_t)V + 1) * 4, st));
    if (g.E) k_csr_count<<<grid_for(g.E), kThreads, 0, st>>>(g.E, esrc, edst, g.directed, cur);
    size_t tb = 0;
    HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cur, off, (int)(V + 1), st));
    void* tmp = c.b_scantmp.get(tb);
    HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, cur, off, (int)(V + 1), st));
    uint32_t arcs = 0;
    HIP_CHECK(hipMemcpyAsync(&arcs, off + V, 4, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    uint32_t* in_src = (uint32_t*)c.b_entkey.get(std::max<size_t>(arcs, 1) * 4);
    uint32_t* in_w = (uint32_t*)c.b_entw.get(std::max<size_t>(arcs, 1) * 4);
    float* in_b = (float*)c.b_entb.get(std::max<size_t>(arcs, 1) * 4);
    uint64_t* in_w64 = wide ? (uint64_t*)c.b_cscent.get(std::max<size_t>(arcs, 1) * 8) : nullptr;
    HIP_CHECK(hipMemsetAsync(cur, 0, ((size_t)V + 1) * 4, st));
    if (g.E)
        k_csr_fill<<<grid_for(g.E), kThreads, 0, st>>>(g.E, esrc, edst, g.lat, P.unit, g.loss, g.directed, off, cur,
                                                       in_src, in_w, in_b, in_w64);
    // out-arcs for the work marks: the in-CSR itself when undirected
    const uint32_t* out_off = off;
    const uint32_t* out_dst = in_src;
    if (g.directed) {
        uint32_t* ooff = (uint32_t*)c.b_outoff.get(((size_t)V + 1) * 4);
        uint32_t* odst = (uint32_t*)c.b_outdst.get(std::max<size_t>(arcs, 1) * 4);
        HIP_CHECK(hipMemsetAsync(cur, 0, ((size_t)V + 1) * 4, st));
        k_csr_count_out<<<grid_for(g.E), kThreads, 0, st>>>(g.E, esrc, edst, cur);
        HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, cur, ooff, (int)(V + 1), st));
        HIP_CHECK(hipMemsetAsync(cur, 0, ((size_t)V + 1) * 4, st));
        k_csr_fill_out<<<grid_for(g.E), kThreads, 0, st>>>(g.E, esrc, edst, ooff, cur, odst);
        out_off = ooff;
        out_dst = odst;
    }
    // this rank's sources, in graph-locality (BFS) order, in batches of 64 lanes: sources of
    // one batch are close to each other, so their Bellman-Ford frontiers move together
    const uint32_t p0 = (uint32_t)((uint64_t)rk * n / G), p1 = (uint32_t)((uint64_t)(rk + 1) * n / G);
    c.own_row0 = p0;  // this rank's rows: positions [p0, p1) of `nodes`
    c.own_row1 = p1;
    const uint32_t nloc = p1 - p0;
    const uint32_t nbatch = (nloc + 63) / 64;
    const double ms_csr = std::getenv("SRG_DEBUG_SPARSE") ? tm.lap() : 0.0;  // (debug split of ms_build)
    const auto t_host0 = std::chrono::steady_clock::now();
    std::vector<uint32_t> h_off(V + 1), h_src(arcs);
    HIP_CHECK(hipMemcpyAsync(h_off.data(), off, ((size_t)V + 1) * 4, hipMemcpyDeviceToHost, st));
    if (arcs) HIP_CHECK(hipMemcpyAsync(h_src.data(), in_src, (size_t)arcs * 4, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    const auto t_host1 = std::chrono::steady_clock::now();
    std::vector<uint32_t> order(V, 0xFFFFFFFFu), queue;
    queue.reserve(V);
    uint32_t next = 0;
    for (uint32_t root_pass = 0; root_pass < 2 && next < V; ++root_pass) {
        for (uint32_t r = 0; r < V; ++r) {
            // first pass: start at the highest-degree vertex; then any unvisited vertex
            uint32_t start = r;
            if (root_pass == 0) {
                uint32_t best = 0;
                for (uint32_t v = 0; v < V; ++v)
                    if (h_off[v + 1] - h_off[v] > h_off[best + 1] - h_off[best]) best = v;
                start = best;
            }
            if (order[start] != 0xFFFFFFFFu) continue;
            order[start] = next++;
            queue.assign(1, start);
            for (size_t qi = 0; qi < queue.size(); ++qi) {
                const uint32_t v = queue[qi];
                for (uint32_t k = h_off[v]; k < h_off[v + 1]; ++k) {
                    const uint32_t u = h_src[k];
                    if (order[u] == 0xFFFFFFFFu) {
                        order[u] = next++;
                        queue.push_back(u);
                    }
                }
            }
            if (root_pass == 0) break;
        }
    }
    const auto t_host2 = std::chrono::steady_clock::now();
    std::vector<uint32_t> loc(nloc);
    for (uint32_t i = 0; i < nloc; ++i) loc[i] = p0 + i;
    if (c.sparse_locality) {  // stable by BFS position: a counting sort over the V positions
        std::vector<uint32_t> cnt((size_t)V + 1, 0);
        for (uint32_t i = 0; i < nloc; ++i) ++cnt[order[P.nodes_h[p0 + i]] + 1];
        for (uint32_t v = 0; v < V; ++v) cnt[v + 1] += cnt[v];
        for (uint32_t i = 0; i < nloc; ++i) loc[cnt[order[P.nodes_h[p0 + i]]]++] = p0 + i;
    }
    std::vector<uint32_t> bsrc((size_t)std::max<uint32_t>(nbatch, 1) * 64), brow(bsrc.size());
    for (uint32_t i = 0; i < (uint32_t)bsrc.size(); ++i) {
        const bool real = i < nloc;
        bsrc[i] = P.nodes_h[real ? loc[i] : (nloc ? loc[0] : 0)];
        brow[i] = real ? loc[i] : 0xFFFFFFFFu;
    }
    const auto t_host3 = std::chrono::steady_clock::now();
    uint32_t* d_bsrc = (uint32_t*)c.b_lnodes.get(bsrc.size() * 4);
    uint32_t* d_brow = (uint32_t*)c.b_lpos.get(brow.size() * 4);
    HIP_CHECK(hipMemcpyAsync(d_bsrc, bsrc.data(), bsrc.size() * 4, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(d_brow, brow.data(), brow.size() * 4, hipMemcpyHostToDevice, st));
    uint32_t* fl = (uint32_t*)c.b_red.get(128);
    HIP_CHECK(hipMemsetAsync(fl, 0, 128, st));
    HIP_CHECK(hipGetLastError());
    const double ms_build = tm.lap() + ms_csr;
    if (std::getenv("SRG_DEBUG_SPARSE"))
        std::fprintf(stderr, "sparse build: CSR %.2f ms, host order + batches %.2f ms (of %.2f): CSR to host %.2f, BFS %.2f, batches %.2f\n", ms_csr,
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_host0).count(), ms_build,
                     std::chrono::duration<double, std::milli>(t_host1 - t_host0).count(),
                     std::chrono::duration<double, std::milli>(t_host2 - t_host1).count(),
                     std::chrono::duration<double, std::milli>(t_host3 - t_host2).count());

    int dev_cus = 256;
    HIP_CHECK(hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, c.device));
    // wide labels take the 128-VGPR budget: one workgroup per CU
    const int wpc = wide ? 1 : 2;
    uint32_t grid = std::max<uint32_t>(1, std::min<uint32_t>(nbatch, (uint32_t)dev_cus * (uint32_t)wpc));

    // u32 latency keys take the two-phase kernel (latency-only delta-stepping, then the loss fold
    // over the tight arcs, sparse_ds.hip.h); wide labels keep the lexicographic sweeps.
    // SRG_SPARSE_KERNEL=bf selects the lexicographic sweeps for u32 keys too (A/B)
    const char* sk = std::getenv("SRG_SPARSE_KERNEL");
    const bool two_phase = !wide && !(sk && std::strcmp(sk, "bf") == 0);
    // per resident batch: labels V x 64 x 8 B (16 B wide); two-phase: u32 latency + f32 loss
    // labels, a u64 tight mask per arc and a u64 final-lane mask per vertex
    size_t free_b = 0, total_b = 0;
    HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
    const size_t slot_bytes = (size_t)V * 64 * (wide ? 16 : two_phase ? 4 : 8);
    const size_t ds_extra = two_phase ? (size_t)V * 64 * 4 + (size_t)std::max<uint32_t>(arcs, 1) * 16 + (size_t)V * 16 : 0;
    // two launches (phase 1, then phases 2 + output) when every batch's latency labels fit beside the
    // rest (C4: 782 x 12.8 MB = 10 GB): each launch gets its own register allocation
    // (SRG_SPARSE_SPLIT=0: one fused launch, A/B)
    const char* sp_env = std::getenv("SRG_SPARSE_SPLIT");
    const size_t d_all = (size_t)nbatch * V * 64 * 4;
    const bool split = two_phase && nbatch && !(sp_env && sp_env[0] == '0') && d_all <= free_b / 3;
    grid = (uint32_t)std::max<size_t>(
        1, std::min<size_t>(grid, (free_b / 2 - (split ? d_all : 0)) / std::max<size_t>((split ? 0 : slot_bytes) + ds_extra, 1)));
    const uint32_t nwv = (V + 63) / 64;
    const size_t bitmap_bytes = two_phase ? ds_state_bytes(V) : (size_t)nwv * 5 * 8;
    const size_t scr_bytes = two_phase ? ds_scratch_bytes() : sp_scratch_bytes();
    // bitmaps in LDS while a CU still fits the requested workgroups, else in global memory
    const bool gbits = c.sparse_global_bitmaps || bitmap_bytes + scr_bytes > (size_t)160 * 1024 / wpc;
    const size_t lds = (gbits ? 0 : bitmap_bytes) + scr_bytes;
    if (nbatch) {
        unsigned long long* slots = (unsigned long long*)c.b_D.get(split ? d_all : (size_t)grid * slot_bytes);
        unsigned long long* gb = gbits ? (unsigned long long*)c.b_W.get((size_t)grid * bitmap_bytes) : nullptr;
        // 16 rows in flight was measured 2.5x slower (the row array no longer unrolls into
        // registers); 4 ties with 8 at 2 workgroups per CU
        // 8 rows in flight at two workgroups per CU: 4 rows tied, 16 rows / one workgroup per CU
        // (128 VGPRs, no spills) ran 2.5x / 1.2x slower
        auto kern = gbits ? k_sparse_bf<SP_G, true> : k_sparse_bf<SP_G, false>;
        if (wide) kern = gbits ? k_sparse_bf<SP_G, true, 4, LabelU64> : k_sparse_bf<SP_G, false, 4, LabelU64>;
        if (two_phase) {
            // 8 rows in flight per wave: 16 and 32 spill at the 64-VGPR budget and measured 375 / 712 ms
            // against 293 on C4 (profiles/r06/sparse_ds/c4_g*.json)
            kern = gbits ? k_sparse_ds<true, 8, 8> : k_sparse_ds<false, 8, 8>;
        }
        set_lds(kern, lds);
        SparseArgs a{off, in_src, in_w, in_b, out_off, out_dst, V, d_bsrc, d_brow, nbatch, slots, fl + 4, cols, n,
                     selflat, selfloss, out_lat, out_loss, fl, P.unit, ~0ull, gb, c.kout_key, c.kout_diag,
                     in_w64, min_edge_key(P.es.min_lat_inv, P.unit), nullptr, nullptr, nullptr, arcs};
        if (two_phase) {
            a.lo_slots = (float*)c.b_WL.get((size_t)grid * V * 64 * 4);
            // tight records (16 B per in-arc slot), final-lane masks + tight-record counts (16 B per vertex)
            a.tmask = (unsigned long long*)c.b_PRED.get((size_t)grid * std::max<uint32_t>(arcs, 1) * 16);
            a.fmask = (unsigned long long*)c.b_L0.get((size_t)grid * V * 16);
        }
        // bucket width: the largest edge latency / sparse_delta_div (0 = one bucket, plain BF)
        if (c.sparse_delta_div > 0)
            a.delta = std::max<unsigned long long>(1ull, P.max_key / (unsigned long long)c.sparse_delta_div);
        const char* dbg_env = std::getenv("SRG_DEBUG_SPARSE");
        const bool dbg_batches = two_phase && dbg_env && dbg_env[0] == '2';
        if (dbg_batches) {
            a.dbg = (uint32_t*)c.b_L1.get((size_t)nbatch * 6 * 4);
            HIP_CHECK(hipMemsetAsync(a.dbg, 0, (size_t)nbatch * 6 * 4, st));
        }
        if (c.profiling) {
            while (c.prof_events.size() < 2) {
                hipEvent_t e;
                HIP_CHECK(hipEventCreate(&e));
                c.prof_events.push_back(e);
            }
            HIP_CHECK(hipEventRecord(c.prof_events[0], st));
        }
        if (split) {
            auto k1 = gbits ? k_sparse_ds<true, 8, 8, 1> : k_sparse_ds<false, 8, 8, 1>;
            auto k2 = gbits ? k_sparse_ds<true, 8, 8, 2> : k_sparse_ds<false, 8, 8, 2>;
            // (phase 1 in 8-wave workgroups at 128 VGPRs with 32 rows in flight per wave, no spills, was
            // measured slower: 151 vs 115 ms per workgroup, profiles/r06/sparse_p1w/)
            set_lds(k1, lds);
            set_lds(k2, lds);
            k1<<<grid, SP_THREADS, lds, st>>>(a);
            SparseArgs a2 = a;
            a2.queue = fl + 9;  // (zeroed with the flags)
            k2<<<grid, SP_THREADS, lds, st>>>(a2);
        } else {
            kern<<<grid, SP_THREADS, lds, st>>>(a);
        }
        HIP_CHECK(hipGetLastError());
        if (c.profiling) HIP_CHECK(hipEventRecord(c.prof_events[1], st));
        if (dbg_batches) {  // per-batch durations (100-MHz ticks): what sets the launches' makespan
            std::vector<uint32_t> h((size_t)nbatch * 6);
            HIP_CHECK(hipMemcpyAsync(h.data(), a.dbg, h.size() * 4, hipMemcpyDeviceToHost, st));
            HIP_CHECK(hipStreamSynchronize(st));
            for (int ph = 0; ph < 2; ++ph) {
                std::vector<double> d(nbatch);
                for (uint32_t b = 0; b < nbatch; ++b) {
                    d[b] = h[b * 6 + 1 + 4 * ph] / 1e5;
                }
                std::vector<double> srt = d;
                std::sort(srt.begin(), srt.end());
                std::fprintf(stderr, "sparse batches phase %d (ms): min %.1f p10 %.1f median %.1f p90 %.1f max %.1f; by batch decile:",
                             ph + 1, srt[0], srt[nbatch / 10], srt[nbatch / 2], srt[nbatch * 9 / 10], srt[nbatch - 1]);
                for (int q = 0; q < 10; ++q) {
                    double m = 0;
                    uint32_t cnt = 0;
                    for (uint32_t b = q * nbatch / 10; b < (q + 1) * nbatch / 10; ++b) m += d[b], ++cnt;
                    std::fprintf(stderr, " %.1f", cnt ? m / cnt : 0.0);
                }
                std::fprintf(stderr, "\n");
            }
            std::fprintf(stderr, "sparse batches phase-1 sweeps:");
            for (uint32_t b = 0; b < nbatch; b += std::max<uint32_t>(1, nbatch / 20)) std::fprintf(stderr, " %u", h[b * 6 + 3]);
            std::fprintf(stderr, "\n");
        }
    }
    // every rank agrees on the outcome before any exchange
    if (multi) {
        c.comm->allreduce_max_u32(fl, 2, st);
        c.comm->allreduce_max_u32(fl + 5, 3, st);  // saturated, impossible, fold incomplete
    }
    uint32_t hfl[26] = {};
    HIP_CHECK(hipMemcpyAsync(hfl, fl, 104, hipMemcpyDeviceToHost, st));
    const double ms_sssp = tm.lap();
    if (hfl[7])
        fail(SRG_ERR_INTERNAL, "the sparse build's loss fold left a used pair without a final loss");
    if (hfl[6])
        fail(SRG_ERR_INTERNAL, "the sparse build produced an impossible table: a used pair's latency is below the "
                               "smallest edge latency (" + std::to_string(~P.es.min_lat_inv) + " ns)");
    if (std::getenv("SRG_DEBUG_SPARSE")) {
        const unsigned long long ev = (unsigned long long)hfl[2] | (unsigned long long)hfl[3] << 32;
        const unsigned long long p2 = (unsigned long long)hfl[10] | (unsigned long long)hfl[11] << 32;
        std::fprintf(stderr,
                     "sparse: %s, %u batches, grid %u, max sweeps %u, lane evaluations %llu, fold sweeps %u, "
                     "fold row pulls %llu, arcs %u\n",
                     two_phase ? "two-phase" : "lexicographic", nbatch, grid, hfl[1], ev, hfl[8], p2, arcs);
        if (two_phase) {  // per-phase wall clock summed over workgroups (100 MHz), as ms per workgroup
            double t[4];
            for (int p = 0; p < 4; ++p)
                t[p] = (double)((unsigned long long)hfl[12 + 2 * p] | (unsigned long long)hfl[13 + 2 * p] << 32) / 1e5 / grid;
            std::fprintf(stderr, "sparse phases (ms per workgroup): latency %.1f, tight masks %.1f, fold %.1f, output %.1f\n",
                         t[0], t[1], t[2], t[3]);
            double b[3];  // wave utilisation: ticks inside window visits / (16 waves x the phase's ticks)
            for (int p = 0; p < 3; ++p)
                b[p] = (double)((unsigned long long)hfl[20 + 2 * p] | (unsigned long long)hfl[21 + 2 * p] << 32) / 1e5 / grid /
                       (16.0 * std::max(t[p], 1e-9));
            std::fprintf(stderr, "sparse wave utilisation: latency %.2f, tight masks %.2f, fold %.2f\n", b[0], b[1], b[2]);
        }
    }
    if (hfl[0]) {
        // a used pair came out INF: only a relaxation that saturated the u32 key can have hidden a
        // finite (>= 2^32-1 ns) path; otherwise the pair is unreachable -- the reference's panic
        if (hfl[5] && !wide) return false;  // rerun on the wide labels
        fail(SRG_ERR_UNREACHABLE,
             "assertion `left == right` failed: paths.len() != nodes.len().pow(2) (a used node is unreachable "
             "from another used node)");
    }
    double ms_exchange = 0;
    if (multi && c.gather_output) {
        std::vector<size_t> offs(G), lens(G);
        for (int elem : {8, 4}) {
            for (int r = 0; r < G; ++r) {
                const size_t a0 = (uint64_t)r * n / G, a1 = (uint64_t)(r + 1) * n / G;
                offs[r] = a0 * n * elem;
                lens[r] = (a1 - a0) * n * elem;
            }
            c.comm->allgatherv(elem == 8 ? (void*)out_lat : (void*)out_loss, offs.data(), lens.data(), st);
        }
        ms_exchange = tm.lap();
    }
    if (stats && c.profiling && nbatch) {
        float ms = 0;
        HIP_CHECK(hipEventElapsedTime(&ms, c.prof_events[0], c.prof_events[1]));
        stats->prof_launches += 1;
        stats->prof_kernel_ms += ms;
        stats->prof_relaxations += nloc;  // sparse: sources routed by the profiled launch
    }
    if (stats) {
        stats->ms_build += ms_build;
        stats->ms_fw += ms_sssp;
        stats->ms_exchange += ms_exchange;
        stats->path_kind = wide ? SRG_PATH_SPARSE_U64 : SRG_PATH_SPARSE_U32;
        stats->loss_rounds = (int)hfl[1];
        stats->relaxations = (((uint64_t)hfl[3] << 32) | hfl[2]) * 64;
        stats->nranks = G;
        stats->rank = rk;
        stats->local_sources = nloc;
    }
    return true;
}

bool choose_sparse(const srg_ctx& c, const DevGraph& g) {
    if (c.algorithm == SRG_ALGO_DENSE) return false;
    if (c.algorithm == SRG_ALGO_SPARSE) return true;
    const double arcs = (double)g.E * (g.directed ? 1.0 : 2.0);
    return g.V >= 2048 && arcs * 32.0 < (double)g.V * g.V;
}

void compute_device(srg_ctx& c, const DevGraph& g, const uint32_t* nodes, uint32_t n, uint64_t* out_lat,
                    float* out_loss, hipStream_t st, srg_stats* stats, HostSink* sink = nullptr,
                    FwOverlap* ov = nullptr) {
    HIP_CHECK(hipStreamSynchronize(c.aux_stream));  // nothing of an aborted call still writes WL / PRED
    HIP_CHECK(hipStreamSynchronize(c.comm_stream));  // ... or the essential-entry counts
    if (g.V == 0) {
        if (n) fail(SRG_ERR_ARG, "nodes given for an empty graph");
        return;
    }
    // with the FW already queued beside the H2D the edge checks go on the (idle) H2D stream: on st
    // they would wait behind the whole FW before the host could read them
    const bool ov_fw = ov && ov->on && ov->ok && ov->begun;
    Prelude P = prelude(c, g, nodes, n, ov_fw ? c.comm_stream : st, true);
    if (n == 0) return;
    // u64 keys hold path sums below INF = 2^62 (a sum of two keys never wraps); a graph whose
    // worst-case path could reach 2^62 still runs, and only a used pair left at INF is an error:
    // SRG_ERR_LATENCY_RANGE then, since it may be a path the reference would wrap (mod.rs:327)
    // latency unit: every non-self-loop latency is a multiple of their gcd, hence so is every path
    // sum; keys count units (a ms-granular graph fits u32 keys up to 2^31-1 ms of path), outputs
    // are key * unit -- exact.  SRG_LATENCY_UNIT=1 keeps nanosecond keys (tests, A/B).
    const char* lu = std::getenv("SRG_LATENCY_UNIT");
    const uint64_t unit = (P.es.unit > 1 && !(lu && std::strcmp(lu, "1") == 0)) ? P.es.unit : 1;
    P.unit = unit;
    // the FW that ran beside the H2D counted nanoseconds (exact for any unit; its certification
    // decides as usual, a failure reruns on the u64 keys)
    const bool pre = ov && ov->on && ov->ok && ov->ended && P.es.max_lat < 0xFFFFFFFFull;
    if (pre) P.unit = 1;
    P.max_key = P.es.max_lat / P.unit;
    if (stats) stats->latency_unit_ns = P.unit;
    const unsigned __int128 bound = (unsigned __int128)P.max_key * (g.V > 1 ? g.V - 1 : 1);
    P.range_risk = bound >= ((unsigned __int128)1 << 62);
    // every shortest path is at most max_lat * (V - 1) ns and every relaxation the reference runs
    // at most max_lat * V: below 2^64 nothing wraps, and outputs D * unit fit u64
    P.wrap_risk = (unsigned __int128)P.es.max_lat * g.V >= ((unsigned __int128)1 << 64);
    const int G = c.comm ? c.comm->nranks : 1, rk = c.comm ? c.comm->rank : 0;
    if (choose_sparse(c, g) && !P.wrap_risk) {
        // u32 latency keys first; a graph whose arcs or used paths pass 2^32-1 units takes the
        // wide (u64-key) labels: exact, since max_lat * V < 2^64 (no wrap risk) bounds every sum
        loss_arrive(g, P.selfloss, st);
        if (P.max_key < 0xFFFFFFFFull && run_sparse(c, g, nodes, n, out_lat, out_loss, st, P, stats)) return;
        run_sparse(c, g, nodes, n, out_lat, out_loss, st, P, stats, true);
        return;
    }
    if (pre) {
        if (run_dense<uint32_t, FwOverlap::T>(c, g, ov->pl, nodes, n, out_lat, out_loss, st, P, stats, sink, ov)) {
            if (stats) stats->fw_overlap_kept = 1;
            return;
        }
        // the overlapped FW counted nanoseconds and failed its certification: the latencies' gcd unit
        // may still fit u32 keys -- the normal u32 build before the u64 one
        P.unit = unit;
        P.max_key = P.es.max_lat / P.unit;
        if (stats) stats->latency_unit_ns = P.unit;
        P.range_risk = (unsigned __int128)P.max_key * (g.V > 1 ? g.V - 1 : 1) >= ((unsigned __int128)1 << 62);
    }
    if ((!pre || P.unit > 1) && P.max_key < 0xFFFFFFFFull) {
        // FW tile: 128 (more work per launch) on one GPU; the multi-rank schedule is bound by
        // the per-pivot chain (close pivot -> panels), whose latency scales with T^3
        const int tile = c.fw_tile ? c.fw_tile : 128;
        if (tile == 64) {
            Plan pl = make_plan(G, rk, g.V, 64, P.nodes_h);
            if (run_dense<uint32_t, 64>(c, g, pl, nodes, n, out_lat, out_loss, st, P, stats, sink)) return;
        } else {
            Plan pl = make_plan(G, rk, g.V, 128, P.nodes_h);
            if (run_dense<uint32_t, 128>(c, g, pl, nodes, n, out_lat, out_loss, st, P, stats, sink)) return;
        }
    }
    Plan pl = make_plan(G, rk, g.V, 64, P.nodes_h);
    run_dense<uint64_t, 64>(c, g, pl, nodes, n, out_lat, out_loss, st, P, stats, sink);
}

void direct_device(srg_ctx& c, const DevGraph& g, const uint32_t* nodes, uint32_t n, uint64_t* out_lat,
                   float* out_loss, hipStream_t st) {
    Prelude P = prelude(c, g, nodes, n, st, false);
    loss_arrive(g, P.selfloss, st);
    if (n == 0) return;
    int32_t* pos = (int32_t*)c.b_pos.get((size_t)g.V * 4);
    uint32_t* cnt = (uint32_t*)c.b_cnt.get((size_t)n * n * 4);
    HIP_CHECK(hipMemsetAsync(pos, 0xFF, (size_t)g.V * 4, st));
    HIP_CHECK(hipMemsetAsync(cnt, 0, (size_t)n * n * 4, st));
    HIP_CHECK(hipMemsetAsync(&P.flags->first_bad, 0xFF, 8, st));
    k_positions<<<grid_for(n), kThreads, 0, st>>>(nodes, n, pos);
    if (g.E)
        k_direct<<<grid_for(g.E), kThreads, 0, st>>>(g.E, g.src, g.dst, g.lat, g.loss, g.directed, pos, n, cnt,
                                                     out_lat, out_loss);
    k_direct_check<<<grid_for((size_t)n * n), kThreads, 0, st>>>(cnt, n, P.flags);
    HIP_CHECK(hipGetLastError());
    Flags fl;
    HIP_CHECK(hipMemcpyAsync(&fl, P.flags, sizeof(Flags), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    if (fl.first_bad != ~0ull) {
        const size_t k = fl.first_bad;
        uint32_t cv = 0, a = 0, b = 0;
        HIP_CHECK(hipMemcpy(&cv, cnt + k, 4, hipMemcpyDeviceToHost));
        HIP_CHECK(hipMemcpy(&a, nodes + k / n, 4, hipMemcpyDeviceToHost));
        HIP_CHECK(hipMemcpy(&b, nodes + k % n, 4, hipMemcpyDeviceToHost));
        const std::string ia = std::to_string(node_gml_id(g, a, st)), ib = std::to_string(node_gml_id(g, b, st));
        if (cv == 0) fail(SRG_ERR_NO_EDGE, "No edge connecting node " + ia + " to " + ib);
        fail(SRG_ERR_MULTI_EDGE, "More than one edge connecting node " + ia + " to " + ib);
    }
    // get_direct_paths converts every used edge to ns with unwrap (mod.rs:240, 336)
    if (P.es.lat_overflow || P.es.max_lat == UINT64_MAX) {
        // only an error when an overflowing edge is among the outputs
        std::vector<uint64_t> lat((size_t)n * n);
        HIP_CHECK(hipMemcpy(lat.data(), out_lat, lat.size() * 8, hipMemcpyDeviceToHost));
        for (uint64_t v : lat)
            if (v == UINT64_MAX)
                fail(SRG_ERR_LATENCY_RANGE, "The resulting value is outside of the bounds [0, 18446744073709551615]");
    }
}

// ---- stretch C5: packet-event batch (events.hip.h) ---------------------------------------
inline uint32_t bit_width64(uint64_t v) { return v ? 64u - (uint32_t)__builtin_clzll(v) : 0u; }

template <bool WIDE>
void events_sort(srg_ctx& c, const EvIn& in, const uint64_t* deliver, const EvKeyFmt& f, uint32_t bits,
                 uint32_t* out_order, uint64_t* host_off, hipStream_t st, uint32_t& passes) {
    const uint64_t n = in.n;
    unsigned long long* k0 = (unsigned long long*)c.b_ek0.get(n * 8);
    unsigned long long* k1 = (unsigned long long*)c.b_ek1.get(n * 8);
    unsigned long long* h0 = WIDE ? (unsigned long long*)c.b_eh0.get(n * 8) : nullptr;
    unsigned long long* h1 = WIDE ? (unsigned long long*)c.b_eh1.get(n * 8) : nullptr;
    uint32_t* i0 = (uint32_t*)c.b_ei0.get(n * 4);
    uint32_t* i1 = (uint32_t*)c.b_ei1.get(n * 4);
    k_ev_keys<WIDE><<<grid_for(n, 256 * 64), kThreads, 0, st>>>(in, deliver, f, k0, h0, i0);
    const uint32_t ntiles = (uint32_t)((n + RS_TILE - 1) / RS_TILE);
    const int nh = (int)(256 * (size_t)ntiles);
    uint32_t* hist = (uint32_t*)c.b_ehist.get((size_t)nh * 4);
    uint32_t* offs = (uint32_t*)c.b_eoffs.get((size_t)nh * 4);
    size_t tb = 0;
    HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, hist, offs, nh, st));
    void* tmp = c.b_scantmp.get(tb);
    passes = 0;
    for (uint32_t p = 0; p < bits; p += 8) {
        k_rs_hist<WIDE><<<ntiles, RS_THREADS, 0, st>>>(k0, h0, n, p, ntiles, hist);
        HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, hist, offs, nh, st));
        k_rs_scatter<WIDE><<<ntiles, RS_THREADS, 0, st>>>(k0, h0, i0, k1, h1, i1, n, p, ntiles, hist, offs);
        std::swap(k0, k1);
        std::swap(h0, h1);
        std::swap(i0, i1);
        ++passes;
    }
    HIP_CHECK(hipGetLastError());
    uint32_t* flag = (uint32_t*)c.b_red.get(64);
    HIP_CHECK(hipMemsetAsync(flag, 0, 4, st));
    k_ev_finish<WIDE><<<grid_for(n, 256 * 64), kThreads, 0, st>>>(k0, h0, n, f.sh_dst, in.num_hosts, host_off, flag);
    HIP_CHECK(hipMemcpyAsync(out_order, i0, n * 4, hipMemcpyDeviceToDevice, st));
    uint32_t hflag = 0;
    HIP_CHECK(hipMemcpyAsync(&hflag, flag, 4, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    if (hflag)
        fail(SRG_ERR_EVENT_ORDER,
             "called `Option::unwrap()` on a `None` value: two packet events with equal (time, src_host_id, "
             "src_host_event_id) have no relative order");
}

void order_events_device(srg_ctx& c, const EvIn& in, uint64_t* deliver, uint32_t* out_order, uint64_t* host_off,
                         hipStream_t st, srg_event_result* res) {
    if (res) {
        res->min_next_event_ns = UINT64_MAX;
        res->min_used_latency_ns = UINT64_MAX;
        res->key_bits = 0;
        res->radix_passes = 0;
    }
    HIP_CHECK(hipMemsetAsync(host_off, 0, ((size_t)in.num_hosts + 1) * 8, st));
    if (in.n == 0) {
        HIP_CHECK(hipStreamSynchronize(st));
        return;
    }
    if (in.n >= 0xFFFFFFFFull) fail(SRG_ERR_ARG, "event batch too large (>= 2^32 events)");
    EvReduce* red = (EvReduce*)c.b_ered.get(sizeof(EvReduce));
    EvReduce init{~0ull, 0ull, ~0ull, 0ull, ~0ull, 0u, 0u, 0u, 0u};
    HIP_CHECK(hipMemcpyAsync(red, &init, sizeof(EvReduce), hipMemcpyHostToDevice, st));
    k_ev_prep<<<grid_for(in.n, 2048), kThreads, 0, st>>>(in, deliver, red);
    HIP_CHECK(hipGetLastError());
    EvReduce r;
    HIP_CHECK(hipMemcpyAsync(&r, red, sizeof(EvReduce), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    if (r.bad & 2) fail(SRG_ERR_ARG, "event node position out of range (>= table_n)");
    if (r.bad & 1) fail(SRG_ERR_ARG, "event dst_host out of range (>= num_hosts)");
    if (r.bad & 4) fail(SRG_ERR_LATENCY_RANGE, "deliver time overflows EmulatedTime (send + latency)");
    EvKeyFmt f{};
    const uint32_t b_id = bit_width64(r.id_max - r.id_min), b_src = bit_width64(r.src_max),
                   b_t = bit_width64(r.t_max - r.t_min), b_dst = bit_width64(r.dst_max);
    f.t_min = r.t_min;
    f.id_min = r.id_min;
    f.sh_src = b_id;
    f.sh_t = b_id + b_src;
    f.sh_dst = b_id + b_src + b_t;
    const uint32_t bits = f.sh_dst + b_dst;
    if (bits > 128) fail(SRG_ERR_ARG, "event batch key wider than 128 bits");
    uint32_t passes = 0;
    // an all-equal key (bits == 0) needs no pass; a 1-event batch is trivially ordered
    if (bits <= 64) events_sort<false>(c, in, deliver, f, bits, out_order, host_off, st, passes);
    else events_sort<true>(c, in, deliver, f, bits, out_order, host_off, st, passes);
    if (res) {
        res->min_next_event_ns = r.t_min;
        res->min_used_latency_ns = r.lat_min;
        res->key_bits = bits;
        res->radix_passes = passes;
    }
}

__global__ void k_widen_edges(size_t n, const uint16_t* __restrict__ s16, const uint16_t* __restrict__ d16,
                              const uint32_t* __restrict__ l32, uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                              uint64_t* __restrict__ lat) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        src[i] = s16[i];
        dst[i] = d16[i];
        lat[i] = l32[i];
    }
}

// H2D codec of the host entry (SRG_OPT_H2D_CODEC): the edge list crosses PCIe narrowed -- u16
// endpoints (V <= 65536) and u32 latencies -- 12 B instead of 20 B per edge, then is widened on
// the device.  Host threads narrow chunk i+1 into a page-locked ring while chunk i is in flight.
// Returns false (nothing usable staged) when an endpoint >= 65536 or a latency >= 2^32 is seen:
// the caller then ships the plain arrays, whose checks report such edges as the reference does.
// on_chunk(e0, ne, exc, nexc, last): edges [e0, e0 + ne) are decoded on the device (in st order); exc =
// their exceptions (global index, src, dst) when the chunk went sequential-pair, else null
using ChunkFn = std::function<void(size_t, size_t, const uint32_t*, size_t, bool)>;
bool codec_in(srg_ctx& c, const srg_edge_list* g, DevGraph& dg, hipStream_t st, size_t a0, size_t a1, bool with_loss,
              bool& all_narrow, bool& all_seq, const ChunkFn& on_chunk = nullptr);

// Sequential-pair codec, device side: edge i of a chunk is (src, dst) = (es[j], ed[j] + i - ei[j])
// for the last exception j with ei[j] <= i (ei[0] = 0: a chunk starts with one), latency = l32[i].
// Consecutive lanes search the same few exceptions (wave-broadcast loads).
__global__ void k_decode_seq(size_t ne, const uint32_t* __restrict__ l32, const uint32_t* __restrict__ exc, uint32_t nexc,
                             uint32_t* __restrict__ src, uint32_t* __restrict__ dst, uint64_t* __restrict__ lat) {
    const uint32_t* ei = exc;
    const uint32_t* es = exc + nexc;
    const uint32_t* ed = exc + 2 * (size_t)nexc;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < ne; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t lo = 0, hi = nexc - 1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (ei[mid] <= (uint32_t)i) lo = mid;
            else hi = mid - 1;
        }
        src[i] = es[lo];
        dst[i] = ed[lo] + ((uint32_t)i - ei[lo]);
        lat[i] = l32[i];
    }
}

// The edge-sharded exchange's sequential-pair form: edges [e0, e1) of the whole list from every
// slice's exceptions ex = (global index, src, dst) x nexc in index order (each slice starts with
// one, so index 0 is covered) and the u32 latencies.
__global__ void k_decode_seq_global(size_t e0, size_t e1, const uint32_t* __restrict__ l32,
                                    const uint32_t* __restrict__ ex, uint32_t nexc, uint32_t* __restrict__ src,
                                    uint32_t* __restrict__ dst, uint64_t* __restrict__ lat) {
    for (size_t i = e0 + blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < e1; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t lo = 0, hi = nexc - 1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (ex[3 * (size_t)mid] <= (uint32_t)i) lo = mid;
            else hi = mid - 1;
        }
        src[i] = ex[3 * (size_t)lo + 1];
        dst[i] = ex[3 * (size_t)lo + 2] + ((uint32_t)i - ex[3 * (size_t)lo]);
        lat[i] = l32[i];
    }
}

template <class T>
T* stage_in(DevBuf& b, const T* host, size_t count, hipStream_t st) {
    T* d = (T*)b.get(std::max<size_t>(count, 1) * sizeof(T));
    if (count) HIP_CHECK(hipMemcpyAsync(d, host, count * sizeof(T), hipMemcpyHostToDevice, st));
    return d;
}

// Ships edges [a0, a1) into the full-length device arrays (the rank's slice when the edge list
// is sharded, else all of it).
// Sequential-pair mode (whole lists only; SRG_CODEC_SEQ=0 turns it off): an edge list in
// row order -- a GML complete graph lists (i, i), (i, i+1), ... (i, V-1), then row i+1 -- needs
// no endpoints over PCIe: an edge (s, d) following (s, d - 1) is implied, and only the others
// (row starts, ~V of them) cross as exceptions, so a chunk is its u32 latencies (4 B per edge
// instead of 8) plus ~12 B per row.  A chunk with more than 1/8 exceptions is re-narrowed to
// u16 endpoints and the rest of the list stays in that mode.
// all_narrow: every edge of the slice also stays narrowed on the device (b_n16s / b_n16d / b_n32l),
// false when the host-slow switch shipped the rest of the slice plain.
// all_seq: every chunk of the slice went sequential-pair: its u32 latencies are in b_n32l and its
// exceptions (GLOBAL edge index, src, dst) in c.slice_exc -- the edge-sharded exchange then ships
// that form (4 B per edge) instead of the u16 narrowing (8 B).
// the host entry's codec worker pool and its page-locked rings (first use, or srg_create's warm-up)
constexpr size_t kCodecChunk = (size_t)2 << 20;  // edges per chunk: 32 MB narrowed (+ loss)
constexpr int kRingSlots = 3;
void ensure_pool(srg_ctx& c) {
    if (c.pool) return;
    c.pool = new HostPool();
    const unsigned hw = std::thread::hardware_concurrency();
    int nt = (int)std::max(1u, std::min(8u, hw ? hw : 1u));
    if (const char* e = std::getenv("SRG_CODEC_THREADS")) nt = std::max(1, std::atoi(e));  // experiments
    c.pool->start(nt);
}
void ensure_rings(srg_ctx& c) {
    const size_t slot = kCodecChunk * 16;
    if (c.h_ring_bytes < slot * kRingSlots) {
        if (c.h_ring) HIP_CHECK(hipHostFree(c.h_ring));
        c.h_ring = nullptr;
        c.h_ring_bytes = 0;
        HIP_CHECK(hipHostMalloc(&c.h_ring, slot * kRingSlots, hipHostMallocDefault));
        c.h_ring_bytes = slot * kRingSlots;
    }
    for (hipEvent_t& e : c.ev_ring)
        if (!e) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    if (!c.h_lring) HIP_CHECK(hipHostMalloc(&c.h_lring, kCodecChunk * 4 * kRingSlots, hipHostMallocDefault));
    for (hipEvent_t* e : {&c.ev_lring[0], &c.ev_lring[1], &c.ev_lring[2], &c.ev_lin, &c.ev_ldone})
        if (!*e) HIP_CHECK(hipEventCreateWithFlags(e, hipEventDisableTiming));
}

bool codec_in(srg_ctx& c, const srg_edge_list* g, DevGraph& dg, hipStream_t st, size_t a0, size_t a1, bool with_loss,
              bool& all_narrow, bool& all_seq, const ChunkFn& on_chunk) {
    all_narrow = true;
    all_seq = false;
    c.slice_exc.clear();
    const auto t_setup = std::chrono::steady_clock::now();
    const size_t E = g->num_edges, A = a1 - a0;
    constexpr size_t CE = kCodecChunk;  // edges per chunk: 32 MB narrowed (+ loss)
    constexpr int NB = kRingSlots;      // ring slots
    const size_t slot = CE * 16;
    ensure_pool(c);
    ensure_rings(c);
    uint16_t* s16 = (uint16_t*)c.b_n16s.get(E * 2);
    uint16_t* d16 = (uint16_t*)c.b_n16d.get(E * 2);
    uint32_t* l32 = (uint32_t*)c.b_n32l.get(E * 4);
    dg.src = (uint32_t*)c.b_src.get(E * 4);
    dg.dst = (uint32_t*)c.b_dst.get(E * 4);
    dg.lat = (uint64_t*)c.b_lat.get(E * 8);
    dg.loss = (float*)c.b_loss.get(E * 4);
    const double ms_setup = ms_since(t_setup);  // (first call: worker threads, pinned ring, device arrays)
    std::atomic<bool> bad{false};     // a latency >= 2^32: the codec cannot carry the list
    std::atomic<bool> bad_ep{false};  // an endpoint >= 65536: only the sequential-pair chunks can
    const bool dbg = std::getenv("SRG_DEBUG_CODEC") != nullptr;
    double t_conv = 0, t_wait = 0;
    const size_t nch = (A + CE - 1) / CE;
    const char* sq = std::getenv("SRG_CODEC_SEQ");
    bool seq = !(sq && std::strcmp(sq, "0") == 0);  // (a slice of a row-ordered list is row-ordered too)
    uint32_t* dexc = seq ? (uint32_t*)c.b_exc.get(CE * 4) : nullptr;
    const int nwk = c.pool->size();
    if ((int)c.codec_ex.size() < nwk) c.codec_ex.resize(nwk);
    size_t seq_chunks = 0;
    for (size_t ch = 0; ch < nch; ++ch) {
        const int b = (int)(ch % NB);
        auto tw = std::chrono::steady_clock::now();
        if (ch >= (size_t)NB) HIP_CHECK(hipEventSynchronize(c.ev_ring[b]));  // the slot's previous DMA is done
        const size_t e0 = a0 + ch * CE, ne = std::min(CE, a1 - e0);
        unsigned char* base = (unsigned char*)c.h_ring + (size_t)b * slot;
        uint16_t* hs = (uint16_t*)base;
        uint16_t* hd = hs + CE;
        uint32_t* hl = (uint32_t*)(hd + CE);
        float* hb = (float*)(hl + CE);
        auto tc = std::chrono::steady_clock::now();
        t_wait += std::chrono::duration<double, std::milli>(tc - tw).count();
        std::atomic<bool> dense{false};
        const bool seq_ch = seq;
        c.pool->run([&](int w, int nw) {
            const size_t a = ne * w / nw, z = ne * (w + 1) / nw;
            const uint32_t* src = g->src + e0;
            const uint32_t* dst = g->dst + e0;
            const uint64_t* lat = g->latency_ns + e0;
            uint32_t orx = 0;
            uint64_t orl = 0;
            if (seq_ch) {
                std::vector<uint32_t>& ex = c.codec_ex[w];
                ex.clear();
                if (!seq_encode_slice(src, dst, lat, hl, a, z, ex, 3 * ((z - a) / 8 + 1), orx, orl))
                    dense.store(true, std::memory_order_relaxed);  // (redone below with u16 endpoints)
            } else {
                for (size_t i = a; i < z; ++i) {
                    const uint32_t x = src[i], y = dst[i];
                    const uint64_t l = lat[i];
                    orx |= x | y;
                    orl |= l;
                    hs[i] = (uint16_t)x;
                    hd[i] = (uint16_t)y;
                    hl[i] = (uint32_t)l;
                }
            }
            if (with_loss) std::memcpy(hb + a, g->packet_loss + e0 + a, (z - a) * 4);  // f32 as is
            if (orl >> 32) bad.store(true, std::memory_order_relaxed);
            if (orx >> 16) bad_ep.store(true, std::memory_order_relaxed);
        });
        // sequential-pair chunks never carry u16 endpoints (exceptions are u32): only the u16
        // narrowing needs every endpoint below 65536
        if (seq_ch && dense.load() && bad_ep.load()) bad.store(true);
        if (seq_ch && dense.load() && !bad.load()) {
            // not a row-ordered list: this chunk's endpoints narrowed after all, u16 from here on
            seq = false;
            c.pool->run([&](int w, int nw) {
                const size_t a = ne * w / nw, z = ne * (w + 1) / nw;
                for (size_t i = a; i < z; ++i) {
                    hs[i] = (uint16_t)g->src[e0 + i];
                    hd[i] = (uint16_t)g->dst[e0 + i];
                }
            });
        }
        const bool chunk_seq = seq_ch && !dense.load();
        if (!chunk_seq && bad_ep.load()) bad.store(true);
        const double dt = ms_since(tc);
        t_conv += dt;
        if (bad.load()) {
            HIP_CHECK(hipStreamSynchronize(st));  // no DMA may still read the ring
            return false;
        }
        // the host is busy (narrowing takes longer than shipping the chunks plain would at ~55 GB/s):
        // the remaining edges go plain, straight from the caller's arrays.  Judged on the average over
        // the chunks so far, past the first, with a 1.5x margin: shipping plain also gives up the FW
        // beside the H2D (~5 ms at C3), and a single chunk slowed by the caller's fresh table being
        // faulted in beside it (0.79 ms against 0.76) switched a C3 first call over (round 6)
        const double plain_ms = (double)ne * 20.0 / 55e9 * 1e3;
        bool slow = ch + 1 < nch && ch >= 1 && t_conv / (double)(ch + 1) > 1.5 * plain_ms;
        if (const char* f = std::getenv("SRG_CODEC_SLOW_AFTER")) slow = ch + 1 < nch && ch >= (size_t)std::atoll(f);  // tests
        if (chunk_seq) {
            // the workers' exception lists, in order, as SoA (index | src | dst) where the u16
            // endpoints would have gone
            size_t nexc = 0;
            for (int w = 0; w < nwk; ++w) nexc += c.codec_ex[w].size() / 3;
            uint32_t* hx = (uint32_t*)hs;
            size_t q = 0;
            const size_t x0 = c.slice_exc.size();
            for (int w = 0; w < nwk; ++w) {
                const std::vector<uint32_t>& ex = c.codec_ex[w];
                for (size_t k = 0; k + 2 < ex.size(); k += 3, ++q) {
                    hx[q] = ex[k];
                    hx[nexc + q] = ex[k + 1];
                    hx[2 * nexc + q] = ex[k + 2];
                    c.slice_exc.push_back((uint32_t)(e0 + ex[k]));  // global index, src, dst
                    c.slice_exc.push_back(ex[k + 1]);
                    c.slice_exc.push_back(ex[k + 2]);
                }
            }
            HIP_CHECK(hipMemcpyAsync(l32 + e0, hl, ne * 4, hipMemcpyHostToDevice, st));
            HIP_CHECK(hipMemcpyAsync(dexc, hx, nexc * 12, hipMemcpyHostToDevice, st));
            if (with_loss) HIP_CHECK(hipMemcpyAsync((float*)dg.loss + e0, hb, ne * 4, hipMemcpyHostToDevice, st));
            HIP_CHECK(hipEventRecord(c.ev_ring[b], st));
            k_decode_seq<<<grid_for(ne), kThreads, 0, st>>>(ne, l32 + e0, dexc, (uint32_t)nexc, (uint32_t*)dg.src + e0,
                                                             (uint32_t*)dg.dst + e0, (uint64_t*)dg.lat + e0);
            ++seq_chunks;
            if (on_chunk) on_chunk(e0, ne, c.slice_exc.data() + x0, nexc, ch + 1 == nch && !slow);
        } else {
            HIP_CHECK(hipMemcpyAsync(s16 + e0, hs, ne * 2, hipMemcpyHostToDevice, st));
            HIP_CHECK(hipMemcpyAsync(d16 + e0, hd, ne * 2, hipMemcpyHostToDevice, st));
            HIP_CHECK(hipMemcpyAsync(l32 + e0, hl, ne * 4, hipMemcpyHostToDevice, st));
            if (with_loss) HIP_CHECK(hipMemcpyAsync((float*)dg.loss + e0, hb, ne * 4, hipMemcpyHostToDevice, st));
            HIP_CHECK(hipEventRecord(c.ev_ring[b], st));
            k_widen_edges<<<grid_for(ne), kThreads, 0, st>>>(ne, s16 + e0, d16 + e0, l32 + e0, (uint32_t*)dg.src + e0,
                                                              (uint32_t*)dg.dst + e0, (uint64_t*)dg.lat + e0);
            if (on_chunk) on_chunk(e0, ne, nullptr, 0, ch + 1 == nch && !slow);
        }
        HIP_CHECK(hipGetLastError());
        if (slow) {
            const size_t r0 = e0 + ne, rn = a1 - r0;
            HIP_CHECK(hipMemcpyAsync((uint32_t*)dg.src + r0, g->src + r0, rn * 4, hipMemcpyHostToDevice, st));
            HIP_CHECK(hipMemcpyAsync((uint32_t*)dg.dst + r0, g->dst + r0, rn * 4, hipMemcpyHostToDevice, st));
            HIP_CHECK(hipMemcpyAsync((uint64_t*)dg.lat + r0, g->latency_ns + r0, rn * 8, hipMemcpyHostToDevice, st));
            if (with_loss)
                HIP_CHECK(hipMemcpyAsync((float*)dg.loss + r0, g->packet_loss + r0, rn * 4, hipMemcpyHostToDevice, st));
            if (dbg) std::fprintf(stderr, "codec: host slow after chunk %zu (%.2f ms), rest plain\n", ch, dt);
            if (on_chunk) on_chunk(r0, rn, nullptr, 0, true);
            all_narrow = false;
            break;
        }
    }
    if (seq_chunks) all_narrow = false;  // (the endpoints are not on the device narrowed)
    all_seq = seq_chunks == nch && nch > 0;
    if (dbg) std::fprintf(stderr, "codec: %zu chunks (%zu sequential-pair), %d threads, setup %.2f ms, convert %.2f ms, slot waits %.2f ms\n",
                          nch, seq_chunks, c.pool->size(), ms_setup, t_conv, t_wait);
    return true;
}

// Late loss H2D: a helper thread copies the losses chunk by chunk into a pinned ring and queues
// each chunk's DMA on c.loss_stream behind the last endpoint/latency chunk (so the two never
// share the PCIe link); loss_arrive() later joins it and orders the readers after the last DMA.
void start_late_loss(srg_ctx& c, const srg_edge_list* g, DevGraph& dg, hipStream_t st, LateLoss& L, size_t a0 = 0,
                     size_t a1 = ~(size_t)0) {
    constexpr size_t CE = kCodecChunk;
    constexpr int NB = kRingSlots;
    ensure_rings(c);
    L.ev_in = c.ev_lin;
    L.ev_done = c.ev_ldone;
    HIP_CHECK(hipEventRecord(c.ev_ledges, st));
    HIP_CHECK(hipStreamWaitEvent(c.loss_stream, c.ev_ledges, 0));
    dg.late = &L;
    const int device = c.device;
    L.th = std::thread([&c, g, &dg, &L, device, a0, a1]() {
        constexpr size_t CE = (size_t)2 << 20;  // losses per chunk (8 MB)
        constexpr int NB = 3;
        try {
            HIP_CHECK(hipSetDevice(device));
            const bool dbg = std::getenv("SRG_DEBUG_OVERLAP") != nullptr;
            const auto t0 = std::chrono::steady_clock::now();
            double t_copy = 0, t_wait = 0;
            const size_t E = std::min<size_t>(g->num_edges, a1);  // this rank's slice [a0, E)
            float* dloss = const_cast<float*>(dg.loss);
            for (size_t ch = 0, e0 = a0; e0 < E; ++ch, e0 += CE) {
                const int b = (int)(ch % NB);
                auto ta = std::chrono::steady_clock::now();
                if (ch >= (size_t)NB) HIP_CHECK(hipEventSynchronize(c.ev_lring[b]));
                auto tb = std::chrono::steady_clock::now();
                const size_t ne = std::min(CE, E - e0);
                float* slot = (float*)c.h_lring + (size_t)b * CE;
                c.pool->run([&](int w, int nw) {
                    const size_t a = ne * w / nw, z = ne * (w + 1) / nw;
                    std::memcpy(slot + a, g->packet_loss + e0 + a, (z - a) * 4);
                });
                t_wait += std::chrono::duration<double, std::milli>(tb - ta).count();
                t_copy += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tb).count();
                HIP_CHECK(hipMemcpyAsync(dloss + e0, slot, ne * 4, hipMemcpyHostToDevice, c.loss_stream));
                HIP_CHECK(hipEventRecord(c.ev_lring[b], c.loss_stream));
            }
            HIP_CHECK(hipEventRecord(L.ev_in, c.loss_stream));
            if (dbg) {
                HIP_CHECK(hipEventSynchronize(L.ev_in));
                std::fprintf(stderr, "late loss thread: %.2f ms to the last DMA, host copies %.2f ms, ring waits %.2f ms\n",
                             std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(),
                             t_copy, t_wait);
            }
        } catch (const Failure& f) {
            L.err = f.msg;
        } catch (const std::exception& e) {
            L.err = e.what();
        }
    });
}

int guard(char* errbuf, size_t errlen, const std::function<void()>& body) {
    try {
        body();
        if (errbuf && errlen) errbuf[0] = 0;
        return SRG_OK;
    } catch (const Failure& f) {
        set_err(errbuf, errlen, f.msg);
        return f.code;
    } catch (const srg::CommError& e) {
        set_err(errbuf, errlen, std::string("collective: ") + e.what());
        return SRG_ERR_RCCL;
    } catch (const std::bad_alloc&) {
        set_err(errbuf, errlen, "out of host memory");
        return SRG_ERR_OOM;
    } catch (const std::exception& e) {
        set_err(errbuf, errlen, std::string("internal error: ") + e.what());
        return SRG_ERR_INTERNAL;
    } catch (...) {
        set_err(errbuf, errlen, "internal error");
        return SRG_ERR_INTERNAL;
    }
}

// out_key / out_diag (srg_internal_compute_table, RoutingInfo's key table): non-null = the latencies
// leave as the build's u32 keys plus the diagonal's raw self-loop latencies; out_lat is unused then
int host_entry(srg_ctx* c, const srg_edge_list* g, const uint32_t* nodes, uint32_t num_nodes, uint64_t* out_lat,
               float* out_loss, srg_stats* stats, char* errbuf, size_t errlen, bool direct,
               uint32_t* out_key = nullptr, uint64_t* out_diag = nullptr, srg_table* const* tabs = nullptr) {
    const bool keys = out_key != nullptr;
    if (keys && (direct || (c && c->comm && c->comm->nranks > 1) || (num_nodes && !out_diag))) {
        set_err(errbuf, errlen, "key table: one rank, shortest paths only");
        return SRG_ERR_ARG;
    }
    if (!c || !g || (num_nodes && (!nodes || !(out_lat || keys) || !out_loss)) ||
        (g->num_edges && (!g->src || !g->dst || !g->latency_ns || !g->packet_loss))) {
        set_err(errbuf, errlen, "null argument");
        return SRG_ERR_ARG;
    }
    std::lock_guard<std::mutex> lk(c->mu);
    // Page-lock the caller's output arrays on a helper thread, concurrently with the H2D copy
    // and FW (≈10 ms for the 1.2 GB C3 table, measured), so finished rows can be DMA'd out
    // asynchronously while later kernels run.  Small tables are copied at the end.
    const size_t nn = (size_t)num_nodes * num_nodes;
    struct Registration {
        int device = 0;
        std::thread th;
        bool ok = false;
        double ms = 0;
        void* p[2] = {nullptr, nullptr};
        void* view[2] = {nullptr, nullptr};  // device pointers of the mapped registrations
        size_t b[2] = {0, 0};
        hipStream_t wait = nullptr;
        bool fault = true;
        srg_table* tab[2] = {nullptr, nullptr};  // pooled tables (RoutingInfo): stay registered after the call
        bool join() {
            if (th.joinable()) th.join();
            return ok;
        }
        void run() {
            const auto t0 = std::chrono::steady_clock::now();
            if (!b[0] || hipSetDevice(device) != hipSuccess) return;
            for (int i = 0; i < 2; ++i) {
                if (tab[i] && tab[i]->registered) {  // a recycled pooled table: nothing to do
                    view[i] = tab[i]->view;
                    continue;
                }
                advise_huge(p[i], b[i]);
                if (fault) prefault(p[i], b[i], 8);
                if (hipHostRegister(p[i], b[i], hipHostRegisterMapped) != hipSuccess) {
                    if (i == 1 && !tab[0]) (void)hipHostUnregister(p[0]);
                    return;
                }
                if (hipHostGetDevicePointer(&view[i], p[i], 0) != hipSuccess) view[i] = nullptr;
                if (tab[i]) tab[i]->registered = true, tab[i]->view = view[i];
            }
            ms = ms_since(t0);
            ok = true;
        }
        ~Registration() {
            if (th.joinable()) th.join();
            if (ok) {
                (void)hipStreamSynchronize(wait);  // no copy into the buffers may be in flight
                for (int i = 0; i < 2; ++i)
                    if (!tab[i]) (void)hipHostUnregister(p[i]);
            }
        }
    } reg;
    reg.device = c->device;
    reg.wait = c->d2h_stream;
    if (const char* e = std::getenv("SRG_PREFAULT")) reg.fault = std::strcmp(e, "0") != 0;  // A/B
    const bool early = !direct && nn * 12 >= ((size_t)64 << 20);
    const bool ext = (bool)c->ext_reg;
    // a rank of a group that fills only its own rows [n r / N, n (r+1) / N) of a table the ranks
    // share (SRG_OPT_GATHER_OUTPUT 0, one process per GPU) page-locks only those rows: N processes
    // pinning the whole shared table each cost N times the pinning, and a shared-memory table is
    // typically 4-KB pages (~50 ms per 1.2 GB)
    const bool rows_part = !direct && c->comm && c->comm->nranks > 1 && !c->gather_output;
    const size_t reg_r0 = rows_part ? (size_t)num_nodes * c->comm->rank / c->comm->nranks : 0;
    const size_t reg_r1 = rows_part ? (size_t)num_nodes * (c->comm->rank + 1) / c->comm->nranks : num_nodes;
    const size_t lat_elem = keys ? 4 : 8;
    unsigned char* out_lat_b = keys ? (unsigned char*)out_key : (unsigned char*)out_lat;  // the latency table
    // pooled tables (srg_internal_compute_table): the whole mapping is registered once and kept
    const bool pooled = early && !ext && !rows_part && tabs && tabs[0] && tabs[1] && tabs[0]->p == out_lat_b &&
                        tabs[1]->p == (void*)out_loss && tabs[0]->cap >= nn * lat_elem && tabs[1]->cap >= nn * 4;
    if (early && !ext) {
        reg.p[0] = out_lat_b + reg_r0 * num_nodes * lat_elem;
        reg.b[0] = (reg_r1 - reg_r0) * num_nodes * lat_elem;
        reg.p[1] = out_loss + reg_r0 * num_nodes;
        reg.b[1] = (reg_r1 - reg_r0) * num_nodes * 4;
        if (pooled)
            for (int i = 0; i < 2; ++i) reg.tab[i] = tabs[i], reg.b[i] = tabs[i]->cap;
        reg.th = std::thread([&reg]() { reg.run(); });
    }
    return guard(errbuf, errlen, [&]() {
        auto t0 = std::chrono::steady_clock::now();
        if (stats) std::memset(stats, 0, sizeof(*stats));
        HIP_CHECK(hipSetDevice(c->device));
        hipStream_t st = c->stream;
        const size_t E = g->num_edges, n = num_nodes;
        DevGraph dg{g->num_vertices, (int)g->directed, g->num_edges, nullptr, nullptr, nullptr, nullptr,
                    nullptr, g->node_ids};
        // Multi-rank: every rank needs the whole edge list (W's rows feed the essential-entry
        // records of every source), but each GPU has its own PCIe link and the GPUs a mesh of
        // their own: rank r ships edges [E r/N, E (r+1)/N) and the slices are exchanged device to
        // device.  The slice ranges are a function of (E, N) only, so every rank agrees on them.
        const int nr = c->comm ? c->comm->nranks : 1, rk = c->comm ? c->comm->rank : 0;
        const bool shard = nr > 1 && (c->edge_shard == 1 || (c->edge_shard < 0 && nr >= 4));
        const size_t a0 = shard ? E * rk / nr : 0, a1 = shard ? E * (rk + 1) / nr : E;
        // narrowed edge list over PCIe when it fits (falls back to the plain arrays otherwise)
        // late loss: the losses follow the endpoints and latencies on their own stream, beside
        // the W build and FW (dense u32 path: WL is built from them on c->loss_stream)
        // (edge-sharded ranks ship their slices' losses late too; the slices are exchanged when
        // the losses are first read, after FW -- loss_arrive)
        const bool want_late = c->late_loss && !direct;
        bool all_narrow = false, all_seq = false;
        // FW beside the H2D (FwOverlap): one rank, undirected, the dense symmetric two-stream FW on
        // 128-tiles, the codec with late losses; the chunks then cross on the comm stream (idle on
        // one rank) while FW runs on the main stream
        FwOverlap ov;
        {
            DevGraph probe{g->num_vertices, (int)g->directed, E};
            const bool ov_want = c->fw_overlap && !direct && nr == 1 && want_late && c->h2d_codec && E >= ((size_t)1 << 20) &&
                                 !g->directed && c->fw_symmetric && (c->fw_tile == 0 || c->fw_tile == 128) &&
                                 g->num_vertices >= 256 && n > 0 && !choose_sparse(*c, probe);
            if (ov_want) {
                HIP_CHECK(hipStreamSynchronize(c->aux_stream));  // nothing of an aborted call still runs
                ov.init(*c, g->num_vertices, std::vector<uint32_t>(nodes, nodes + n));
            }
        }
        const hipStream_t hst = ov.on ? c->comm_stream : st;
        ChunkFn on_chunk = nullptr;
        if (ov.on) on_chunk = [&](size_t e0, size_t ne, const uint32_t* exc, size_t nexc, bool last) {
            ov.chunk(dg, e0, ne, exc, nexc, last);
        };
        // (V > 65536: only a row-ordered list, through the sequential-pair chunks, can be narrowed;
        // codec_in gives up on the first chunk that is neither)
        const bool coded = c->h2d_codec && a1 - a0 >= ((size_t)1 << 20) &&
                           codec_in(*c, g, dg, hst, a0, a1, !want_late, all_narrow, all_seq, on_chunk);
        if (ov.on) ov.finish();  // the FW thread has enqueued every landed chunk's work
        if (ov.on && !coded) ov.ok = false;
        const int ov_early = ov.next;  // pivots enqueued while chunks were still crossing
        if (stats && ov.on && ov.ok) stats->fw_overlap_pivots = ov_early;
        if (ov.on && ov.ok && !ov.ended) ov.advance(ov.nb - 1);
        if (ov.on && std::getenv("SRG_DEBUG_OVERLAP")) {
            std::fprintf(stderr, "fw-overlap: ok=%d pivots_during_h2d=%d of %d\n", ov.ok ? 1 : 0, ov_early, ov.nb);
            if (ov.ok) ov.report();
        }
        // (started here, after the remaining pivots are enqueued -- an enqueue that holds this thread
        // until FW nears its end -- the losses land ~3 ms after FW, but that wait overlaps GPU work:
        // starting the thread before it measured 46.9-47.4 vs 46.5-46.6 ms, profiles/r06/late_loss/)
        LateLoss late;
        late.ls = c->loss_stream;
        if (coded && want_late) start_late_loss(*c, g, dg, hst, late, a0, a1);
        if (!coded) {
            const size_t cnt = std::max<size_t>(E, 1);
            dg.src = (uint32_t*)c->b_src.get(cnt * 4);
            dg.dst = (uint32_t*)c->b_dst.get(cnt * 4);
            dg.lat = (uint64_t*)c->b_lat.get(cnt * 8);
            dg.loss = (float*)c->b_loss.get(cnt * 4);
            if (a1 > a0) {
                HIP_CHECK(hipMemcpyAsync((uint32_t*)dg.src + a0, g->src + a0, (a1 - a0) * 4, hipMemcpyHostToDevice, st));
                HIP_CHECK(hipMemcpyAsync((uint32_t*)dg.dst + a0, g->dst + a0, (a1 - a0) * 4, hipMemcpyHostToDevice, st));
                HIP_CHECK(hipMemcpyAsync((uint64_t*)dg.lat + a0, g->latency_ns + a0, (a1 - a0) * 8,
                                         hipMemcpyHostToDevice, st));
                HIP_CHECK(hipMemcpyAsync((float*)dg.loss + a0, g->packet_loss + a0, (a1 - a0) * 4,
                                         hipMemcpyHostToDevice, st));
            }
        }
        const bool sim = shard && std::strcmp(c->comm->kind(), "simulated") == 0;
        if (sim && (c->sim_edges != g->src || c->sim_E != E)) {
            // SRG_OPT_SIMULATE_RANK elides the exchange: the other slices are shipped once per
            // edge list (a warm-up call), so later calls time this rank's slice and stay valid
            auto put = [&](size_t e0, size_t e1) {
                if (e1 <= e0) return;
                HIP_CHECK(hipMemcpyAsync((uint32_t*)dg.src + e0, g->src + e0, (e1 - e0) * 4, hipMemcpyHostToDevice, st));
                HIP_CHECK(hipMemcpyAsync((uint32_t*)dg.dst + e0, g->dst + e0, (e1 - e0) * 4, hipMemcpyHostToDevice, st));
                HIP_CHECK(hipMemcpyAsync((uint64_t*)dg.lat + e0, g->latency_ns + e0, (e1 - e0) * 8,
                                         hipMemcpyHostToDevice, st));
                HIP_CHECK(hipMemcpyAsync((float*)dg.loss + e0, g->packet_loss + e0, (e1 - e0) * 4,
                                         hipMemcpyHostToDevice, st));
            };
            put(0, a0);
            put(a1, E);
            c->sim_edges = g->src;
            c->sim_E = E;
        }
        if (shard) {
            std::vector<size_t> offs(nr), lens(nr);
            auto gather = [&](const void* p, size_t elem) {
                for (int q = 0; q < nr; ++q) {
                    const size_t q0 = E * q / nr, q1 = E * (q + 1) / nr;
                    offs[q] = q0 * elem;
                    lens[q] = (q1 - q0) * elem;
                }
                c->comm->allgatherv(const_cast<void*>(p), offs.data(), lens.data(), st);
            };
            // the narrowest form every rank has: 0 = sequential-pair (each slice's u32 latencies +
            // exceptions: 4 B per edge with the loss 8), 1 = u16 narrowing (8 B, 12 with the loss),
            // 2 = plain (a rank shipped its slice plain: 20 B)
            // forms 0 / 1: every rank is coded, so every rank ships its losses late -- exchanged when
            // first read (loss_arrive); else now
            auto late_or_gather_loss = [&]() {
                if (dg.late) {
                    dg.late->comm = c->comm;
                    dg.late->offs.resize(nr);
                    dg.late->lens.resize(nr);
                    for (int q = 0; q < nr; ++q) {
                        dg.late->offs[q] = E * q / nr * 4;
                        dg.late->lens[q] = (E * (q + 1) / nr - E * q / nr) * 4;
                    }
                } else {
                    gather(dg.loss, 4);
                }
            };
            uint32_t* plain = (uint32_t*)c->b_red.get(16);
            const uint32_t mine = !coded ? 2u : all_seq ? 0u : all_narrow ? 1u : 2u;
            HIP_CHECK(hipMemcpyAsync(plain, &mine, 4, hipMemcpyHostToDevice, st));
            c->comm->allreduce_max_u32(plain, 1, st);
            uint32_t form = 2;
            HIP_CHECK(hipMemcpyAsync(&form, plain, 4, hipMemcpyDeviceToHost, st));
            HIP_CHECK(hipStreamSynchronize(st));
            if (form == 0) {
                // every slice's exception count, then every slice's exceptions (global index, src,
                // dst), the u32 latencies and the losses; the other slices are decoded here
                const size_t xbase = ((size_t)nr * 4 + 255) / 256 * 256;
                uint32_t* xc = (uint32_t*)c->b_xexc.get(xbase);
                const uint32_t my_n = (uint32_t)(c->slice_exc.size() / 3);
                HIP_CHECK(hipMemcpyAsync(xc + rk, &my_n, 4, hipMemcpyHostToDevice, st));
                for (int q = 0; q < nr; ++q) {
                    offs[q] = (size_t)q * 4;
                    lens[q] = 4;
                }
                c->comm->allgatherv(xc, offs.data(), lens.data(), st);
                std::vector<uint32_t> cnt(nr);
                HIP_CHECK(hipMemcpyAsync(cnt.data(), xc, (size_t)nr * 4, hipMemcpyDeviceToHost, st));
                HIP_CHECK(hipStreamSynchronize(st));
                if (sim)
                    for (int q = 0; q < nr; ++q) cnt[q] = my_n;  // (a simulated rank hears nothing: its own size)
                size_t tot = 0, mine_at = 0;
                for (int q = 0; q < nr; ++q) {
                    if (q == rk) mine_at = tot;
                    offs[q] = xbase + tot * 12;
                    lens[q] = (size_t)cnt[q] * 12;
                    tot += cnt[q];
                }
                unsigned char* xb = (unsigned char*)c->b_xexc.get(xbase + std::max<size_t>(tot, 1) * 12);
                if (my_n)
                    HIP_CHECK(hipMemcpyAsync(xb + xbase + mine_at * 12, c->slice_exc.data(), (size_t)my_n * 12,
                                             hipMemcpyHostToDevice, st));
                c->comm->allgatherv(xb, offs.data(), lens.data(), st);
                uint32_t* l32 = (uint32_t*)c->b_n32l.p;
                gather(l32, 4);
                late_or_gather_loss();
                for (auto [e0, e1] : {std::pair<size_t, size_t>{0, a0}, std::pair<size_t, size_t>{a1, E}})
                    if (e1 > e0 && !sim)
                        k_decode_seq_global<<<grid_for(e1 - e0), kThreads, 0, st>>>(
                            e0, e1, l32, (const uint32_t*)(xb + xbase), (uint32_t)tot, (uint32_t*)dg.src,
                            (uint32_t*)dg.dst, (uint64_t*)dg.lat);
                HIP_CHECK(hipGetLastError());
            } else if (form == 1) {
                uint16_t* s16 = (uint16_t*)c->b_n16s.p;
                uint16_t* d16 = (uint16_t*)c->b_n16d.p;
                uint32_t* l32 = (uint32_t*)c->b_n32l.p;
                gather(s16, 2);
                gather(d16, 2);
                gather(l32, 4);
                late_or_gather_loss();
                // (a simulated rank received nothing: its other slices are the wide ones put once)
                for (auto [e0, e1] : {std::pair<size_t, size_t>{0, a0}, std::pair<size_t, size_t>{a1, E}})
                    if (e1 > e0 && !sim)
                        k_widen_edges<<<grid_for(e1 - e0), kThreads, 0, st>>>(e1 - e0, s16 + e0, d16 + e0, l32 + e0,
                                                                               (uint32_t*)dg.src + e0, (uint32_t*)dg.dst + e0,
                                                                               (uint64_t*)dg.lat + e0);
                HIP_CHECK(hipGetLastError());
            } else {
                gather(dg.src, 4);
                gather(dg.dst, 4);
                gather(dg.lat, 8);
                if (dg.late) {  // (some rank shipped plain: no late exchange; this rank's losses first)
                    dg.late->join();
                    HIP_CHECK(hipStreamWaitEvent(st, dg.late->ev_in, 0));
                }
                gather(dg.loss, 4);
            }
        }
        const uint32_t* dn = stage_in(c->b_nodes, nodes, n, hst);
        if (hst != st) {  // the main stream's later work reads the landed edges and nodes
            HIP_CHECK(hipEventRecord(c->ev_c, hst));
            HIP_CHECK(hipStreamWaitEvent(st, c->ev_c, 0));
        }
        // multi-rank without the output exchange: the device holds only this rank's rows [p0, p1)
        // (the plan's split, make_plan / run_sparse); dol / dos then point p0 rows before that
        // allocation, so the kernels' absolute row indices land in it (C4 at 8 ranks: 3.75 GB per
        // GPU instead of 30 GB)
        const bool own_rows_only = !direct && c->comm && c->comm->nranks > 1 && !c->gather_output;
        const size_t q0 = own_rows_only ? (uint64_t)n * c->comm->rank / c->comm->nranks : 0;
        const size_t q1 = own_rows_only ? (uint64_t)n * (c->comm->rank + 1) / c->comm->nranks : n;
        const size_t dev_nn = (q1 - q0) * n;
        uint64_t* dol = reinterpret_cast<uint64_t*>(reinterpret_cast<uintptr_t>(c->b_olat.get(std::max<size_t>(dev_nn, 1) * 8)) -
                                                    q0 * n * 8);
        float* dos = reinterpret_cast<float*>(reinterpret_cast<uintptr_t>(c->b_oloss.get(std::max<size_t>(dev_nn, 1) * 4)) -
                                              q0 * n * 4);
        HIP_CHECK(hipStreamSynchronize(hst));  // (beside FW when it started early: st still runs it)
        const double ms_h2d = ms_since(t0);
        // u64 output of a dense u32 build on one rank: the latency rows cross PCIe as the build's u32
        // keys and are widened on the host (HostSink::send_keys; 0.6 GB less D2H at C3); a build that
        // turns out to need u64 keys ships the u64 rows instead (run_dense clears sink.widen)
        bool ikeys = !keys && !direct && early && nr == 1 && c->sdma.ok && c->d2h_mode == 1 && c->h_ring &&
                     c->pool && (size_t)n * 4 <= c->h_ring_bytes / 3 && !std::getenv("SRG_NO_KEY_D2H");
        {
            DevGraph probe{g->num_vertices, (int)g->directed, E};
            ikeys = ikeys && !choose_sparse(*c, probe);
        }
        bool kmode = keys || ikeys;
        // key mode: the device key table in the latency buffer's room, the diagonal beside it; the
        // kernels see them through the context for this call
        uint32_t* dkey = kmode ? reinterpret_cast<uint32_t*>(dol) : nullptr;
        uint64_t* ddiag = kmode ? (uint64_t*)c->b_odiag.get(std::max<size_t>(n, 1) * 8) : nullptr;
        struct KeyScope {
            srg_ctx* c;
            ~KeyScope() { c->kout_key = nullptr, c->kout_diag = nullptr; }
        } key_scope{c};
        c->kout_key = dkey;
        c->kout_diag = ddiag;
        HostSink sink;
        sink.lat = keys ? reinterpret_cast<uint64_t*>(out_key) : out_lat;  // (a host table pointer either way)
        sink.widen = ikeys;
        sink.pool = c->pool;
        sink.ring = (unsigned char*)c->h_ring;
        sink.ring_slot = c->h_ring_bytes / 3;
        sink.loss = out_loss;
        sink.n = n;
        sink.cs = c->d2h_stream;
        sink.ev = c->ev_e;
        if (early) {
            sink.mode = c->d2h_mode;
            sink.sdma = &c->sdma;
            sink.device = c->device;
            if (ext) {
                sink.ready = [c, &reg, &sink]() {
                    void* v[2] = {nullptr, nullptr};
                    if (!c->ext_reg(v, &reg.ms)) return false;
                    sink.lat_view = v[0];
                    sink.loss_view = v[1];
                    return true;
                };
            } else {
                sink.ready = [&reg, &sink, reg_r0, num_nodes]() {
                    if (!reg.join()) return false;
                    // views of rows [reg_r0, ...): based so that row r lands at view + r * n
                    sink.lat_view = (unsigned char*)reg.view[0] - reg_r0 * num_nodes * 8;
                    sink.loss_view = (unsigned char*)reg.view[1] - reg_r0 * num_nodes * 4;
                    return true;
                };
            }
        }
        c->own_row0 = 0;
        c->own_row1 = ~(size_t)0;
        if (direct) {
            direct_device(*c, dg, dn, num_nodes, dol, dos, st);
        } else {
            compute_device(*c, dg, dn, num_nodes, dol, dos, st, stats, early ? &sink : nullptr, ov.on ? &ov : nullptr);
            if (ikeys && !sink.widen) {  // the build took u64 keys (run_dense dropped the key table)
                ikeys = false;
                kmode = keys;
                dkey = nullptr;
                ddiag = nullptr;
            }
        }
        if (dg.late) {  // a path that never read the losses (error-free early return): drain
            dg.late->join();
            HIP_CHECK(hipStreamSynchronize(c->loss_stream));
        }
        // multi-rank without the output exchange: only this rank's rows [own_row0, own_row1) leave
        // the device (possibly none), and min_latency_ns is over those rows only
        const bool rows_only = c->comm && c->comm->nranks > 1 && !c->gather_output && !direct;
        const size_t r0 = rows_only ? std::min<size_t>(c->own_row0, n) : 0;
        const size_t r1 = rows_only ? std::min<size_t>(c->own_row1, n) : n;
        const size_t rows_off = r0 * n, rows_nn = r1 > r0 ? (r1 - r0) * n : 0;
        auto t1 = std::chrono::steady_clock::now();
        unsigned long long hmin = ~0ull;
        if (rows_nn && stats) {  // smallest latency over the table (feeds the runahead, manager.rs:238-243)
            unsigned long long* dmin = (unsigned long long*)c->b_multi.get(16);
            HIP_CHECK(hipMemsetAsync(dmin, 0xFF, 16, st));
            if (kmode) {  // smallest key (x unit below) and smallest diagonal latency
                k_min_u32<<<grid_for(rows_nn, 1024), kThreads, 0, st>>>(dkey + rows_off, rows_nn, dmin);
                k_min_u64<<<grid_for(n, 1024), kThreads, 0, st>>>(ddiag, n, dmin + 1);
            } else {
                k_min_u64<<<grid_for(rows_nn, 1024), kThreads, 0, st>>>(dol + rows_off, rows_nn, dmin);
            }
            HIP_CHECK(hipMemcpyAsync(c->hbox + 64 * MS_MIN, dmin, 16, hipMemcpyDeviceToHost, st));
        }
        if (rows_nn && !sink.lat_sent) {
            if (keys)
                HIP_CHECK(hipMemcpyAsync(out_key + rows_off, dkey + rows_off, rows_nn * 4, hipMemcpyDeviceToHost, st));
            else if (!ikeys)
                HIP_CHECK(hipMemcpyAsync(out_lat + rows_off, dol + rows_off, rows_nn * 8, hipMemcpyDeviceToHost, st));
        }
        if (keys && n) HIP_CHECK(hipMemcpyAsync(out_diag, ddiag, n * 8, hipMemcpyDeviceToHost, st));
        std::vector<uint64_t> hdiag(ikeys ? n : 0);  // the diagonal the widened rows are patched with
        if (ikeys && n) HIP_CHECK(hipMemcpyAsync(hdiag.data(), ddiag, n * 8, hipMemcpyDeviceToHost, st));
        if (rows_nn && !sink.loss_sent)
            HIP_CHECK(hipMemcpyAsync(out_loss + rows_off, dos + rows_off, rows_nn * 4, hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        if (rows_nn && stats) {
            hmin = rb_get<unsigned long long>(*c, MS_MIN);
            if (kmode) {
                const unsigned long long dmin = *reinterpret_cast<const unsigned long long*>(c->hbox + 64 * MS_MIN + 8);
                const uint64_t unit = stats->latency_unit_ns ? stats->latency_unit_ns : 1;
                hmin = std::min<unsigned long long>(hmin == ~0ull ? ~0ull : hmin * unit, dmin);
            }
        }
        if (ikeys && rows_nn && !sink.lat_sent) {
            // the rows were not shipped early (the caller's tables could not be page-locked): keys now
            sink.send_keys(st, dkey, r0, r1 - r0, sink.key_unit);
            sink.lat_sent = true;
        }
        sink.finish();
        if (ikeys)
            for (size_t r = r0; r < r1; ++r) out_lat[r * n + r] = hdiag[r];  // raw self-loop weights (mod.rs:211-217)
        if (stats) {
            stats->ms_h2d = ms_h2d;
            stats->ms_d2h = ms_since(t1);  // the D2H not hidden behind kernels
            stats->ms_total = ms_since(t0);
            stats->ms_host_register = ext ? (sink.registered ? reg.ms : -1.0) : reg.join() ? reg.ms : -1.0;
            stats->d2h_overlapped_bytes = sink.early_bytes;
            stats->d2h_key_rows = ikeys ? 1 : 0;
            stats->ms_key_widen = sink.ms_widen;
            stats->min_latency_ns = hmin;
            if (direct) stats->path_kind = SRG_PATH_DIRECT;
        }
    });
}
}  // namespace

extern "C" {

__global__ void k_warm(uint32_t* p) {
    if (threadIdx.x == 0 && blockIdx.x == 0) p[0] = 0;
}

// srg_create's warm-up (SRG_CREATE_WARM=0 skips it, for A/B): what the first host-entry call would
// otherwise pay on the routing path -- the code object's load on the device (the first launch), each
// stream's first dispatch, the codec worker pool, the page-locked H2D rings (96 + 24 MB), the first
// copy of each kind (H2D and D2H by the runtime, D2H on the SDMA engine).  Shadow creates its context
// before parsing the GML, so this runs off the routing path.
void warm_context(srg_ctx& c) {
    ensure_pool(c);
    ensure_rings(c);
    uint32_t* d = (uint32_t*)c.b_red.get(128);
    const hipStream_t ss[4] = {c.stream, c.aux_stream, c.comm_stream, c.d2h_stream};
    for (hipStream_t s : ss) k_warm<<<1, 64, 0, s>>>(d);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipMemcpyAsync(d, c.h_ring, 64, hipMemcpyHostToDevice, c.comm_stream));
    HIP_CHECK(hipMemcpyAsync(c.h_lring, d + 16, 64, hipMemcpyDeviceToHost, c.d2h_stream));
    for (hipStream_t s : ss) HIP_CHECK(hipStreamSynchronize(s));
    if (c.sdma.ok) {
        hsa_signal_t sg;
        if (hsa_signal_create(1, 0, nullptr, &sg) == HSA_STATUS_SUCCESS) {
            if (hsa_amd_memory_async_copy_on_engine(c.h_ring, c.sdma.cpu, d, c.sdma.gpu, 64, 0, nullptr, sg,
                                                    (hsa_amd_sdma_engine_id_t)c.sdma.engine, true) == HSA_STATUS_SUCCESS)
                hsa_signal_wait_scacquire(sg, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
            hsa_signal_destroy(sg);
        }
    }
}

int srg_create(srg_ctx** out, int device, char* errbuf, size_t errlen) {
    if (!out) {
        set_err(errbuf, errlen, "null argument");
        return SRG_ERR_ARG;
    }
    *out = nullptr;
    srg_ctx* c = nullptr;
    int rc = guard(errbuf, errlen, [&]() {
        // SRG_DEBUG_CREATE: where srg_create's time goes (the cold call Shadow pays once)
        const bool dbg = std::getenv("SRG_DEBUG_CREATE") != nullptr;
        auto tc = std::chrono::steady_clock::now();
        auto lap = [&](const char* what) {
            if (dbg) std::fprintf(stderr, "srg_create: %-28s %7.2f ms\n", what, ms_since(tc));
            tc = std::chrono::steady_clock::now();
        };
        const auto tcreate = std::chrono::steady_clock::now();
        int count = 0;
        hipError_t e = hipGetDeviceCount(&count);
        lap("hipGetDeviceCount");
        if (e != hipSuccess || count == 0)
            fail(SRG_ERR_HIP, std::string("no HIP device available (") + hipGetErrorString(e) +
                                  "); the routing builder has no CPU fallback");
        if (device < 0 || device >= count) fail(SRG_ERR_ARG, "device index out of range");
        c = new srg_ctx();
        c->device = device;
        HIP_CHECK(hipSetDevice(device));
        HIP_CHECK(hipFree(nullptr));  // (the device's runtime context, if this process has none yet)
        lap("hipSetDevice");
        // the first stream is where the runtime initialises the device for this process (80-145 ms
        // on the boxes, the next streams ~5 ms each; creating the four from four threads at once took
        // as long, profiles/r05/create/): counted as the runtime's part
        HIP_CHECK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        lap("stream main");
        c->ms_create_runtime = ms_since(tcreate);
        const auto tlib = std::chrono::steady_clock::now();
        // the FW lookahead chain (pivot close, row/col panels) is latency-critical: its workgroups
        // should be dispatched ahead of the bulk phase-3 tiles
        int prio_lo = 0, prio_hi = 0;
        HIP_CHECK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
        HIP_CHECK(hipStreamCreateWithPriority(&c->aux_stream, hipStreamNonBlocking, prio_hi));
        HIP_CHECK(hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking));
        HIP_CHECK(hipStreamCreateWithFlags(&c->d2h_stream, hipStreamNonBlocking));
        lap("streams aux, comm, d2h");
        HIP_CHECK(hipHostMalloc((void**)&c->hbox, 64 * kMailSlots, hipHostMallocDefault));
        lap("mailbox");
        c->sdma.init(device);  // SDMA engine for the host entry's early D2H (else hipMemcpyAsync)
        lap("sdma agents");
        // the late-loss H2D and WL build share the D2H stream (idle until FW ends): a fifth
        // stream would share a hardware queue (GPU_MAX_HW_QUEUES = 4) with the main stream and
        // serialise the W build and FW behind the loss DMAs (measured: build 1.0 -> 3.6 ms)
        c->loss_stream = c->d2h_stream;
        for (hipEvent_t* e : {&c->ev_a, &c->ev_b, &c->ev_c, &c->ev_d, &c->ev_e, &c->ev_ledges, &c->ev_wlate, &c->ev_fwreset,
                              &c->ev_dst})
            HIP_CHECK(hipEventCreateWithFlags(e, hipEventDisableTiming));
        int wv = 0;
        if (hipDeviceGetAttribute(&wv, hipDeviceAttributeCanUseStreamWaitValue, device) == hipSuccess && wv) {
            for (uint32_t*& p : c->sig) HIP_CHECK(hipExtMallocWithFlags((void**)&p, 8, hipMallocSignalMemory));
            HIP_CHECK(hipStreamWriteValue32(c->stream, c->sig[0], 0, 0));
            HIP_CHECK(hipStreamWriteValue32(c->stream, c->sig[1], 0, 0));
            HIP_CHECK(hipStreamSynchronize(c->stream));
        }
        lap("events, signals");
        const char* wv_env = std::getenv("SRG_CREATE_WARM");
        if (!(wv_env && wv_env[0] == '0')) {
            warm_context(*c);
            lap("warm-up (module, rings, copies)");
        }
        c->ms_create_lib = ms_since(tlib);
        std::lock_guard<std::mutex> lk(g_dev_mu);
        ++g_dev_ctx[device];
    });
    if (rc != SRG_OK) {
        delete c;
        return rc;
    }
    *out = c;
    return SRG_OK;
}

int srg_set_option(srg_ctx* ctx, int option, double value) {
    if (!ctx) return SRG_ERR_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    switch (option) {
        case SRG_OPT_PROFILING:
            ctx->profiling = value != 0.0;
            return SRG_OK;
        case SRG_OPT_SPARSE_THRESHOLD:
            if (!(value >= 0.0)) return SRG_ERR_ARG;
            ctx->sparse_threshold = value;
            return SRG_OK;
        case SRG_OPT_GATHER_OUTPUT:
            ctx->gather_output = value != 0.0;
            return SRG_OK;
        case SRG_OPT_SIMULATE_RANK: {
            // value = nranks * 1000 + rank; 0 detaches
            const int v = (int)value;
            delete ctx->comm;
            ctx->comm = nullptr;
            ctx->sim_edges = nullptr;
            if (v > 0) {
                const int nr = v / 1000, rk = v % 1000;
                if (nr < 1 || rk >= nr) return SRG_ERR_ARG;
                ctx->comm = srg::null_create(nr, rk);
            }
            return SRG_OK;
        }
        case SRG_OPT_FW_TILE:
            if (value != 0 && value != 64 && value != 128) return SRG_ERR_ARG;
            ctx->fw_tile = (int)value;
            return SRG_OK;
        case SRG_OPT_SPARSE_LOCALITY:
            ctx->sparse_locality = value != 0.0;
            return SRG_OK;
        case SRG_OPT_SPARSE_DELTA_DIV:
            if (!(value >= 0.0 && value <= 1e6)) return SRG_ERR_ARG;
            ctx->sparse_delta_div = (int)value;
            return SRG_OK;
        case SRG_OPT_SPARSE_GLOBAL_BITMAPS:
            ctx->sparse_global_bitmaps = value != 0.0;
            return SRG_OK;
        case SRG_OPT_FW_SYMMETRIC:
            ctx->fw_symmetric = value != 0.0;
            return SRG_OK;
        case SRG_OPT_LATE_LOSS:
            if (value != 0 && value != 1) return SRG_ERR_ARG;
            ctx->late_loss = (int)value;
            return SRG_OK;
        case SRG_OPT_EDGE_SHARD:
            if (value != 0 && value != 1 && value != -1) return SRG_ERR_ARG;
            ctx->edge_shard = (int)value;
            return SRG_OK;
        case SRG_OPT_H2D_CODEC:
            if (value != 0 && value != 1) return SRG_ERR_ARG;
            ctx->h2d_codec = (int)value;
            return SRG_OK;
        case SRG_OPT_SCAN_GROUPS:
            if (value < 0 || value > 1024) return SRG_ERR_ARG;
            ctx->scan_groups = (int)value;
            return SRG_OK;
        case SRG_OPT_LOSS_CHUNKS:
            if (value < 0 || value > 1024) return SRG_ERR_ARG;
            ctx->loss_chunks = (int)value;
            return SRG_OK;
        case SRG_OPT_D2H_MODE:
            if (value != 0 && value != 1) return SRG_ERR_ARG;
            ctx->d2h_mode = (int)value;
            return SRG_OK;
        case SRG_OPT_FW_LINE_SPLIT:
            if (value != 0 && value != 1 && value != 2 && value != 4) return SRG_ERR_ARG;
            ctx->fw_line_split = (int)value;
            return SRG_OK;
        case SRG_OPT_FW_STEP:
            // (1, the fused one-launch-per-pivot FW, was removed in round 5: DESIGN.md §7)
            if (value != 0 && value != 2 && value != -1) return SRG_ERR_ARG;
            ctx->fw_step = (int)value;
            return SRG_OK;
        case SRG_OPT_FW_OVERLAP:
            if (value != 0 && value != 1) return SRG_ERR_ARG;
            ctx->fw_overlap = (int)value;
            return SRG_OK;
        case SRG_OPT_TEST_FAULT:
            // test hooks exist only in the test build (libshadow_routing_testhooks.so, -DSRG_TEST_HOOKS);
            // the product library accepts 0 (off) and refuses the rest
            if (value != 0 && value != 1 && value != 2) return SRG_ERR_ARG;
#ifndef SRG_TEST_HOOKS
            if (value != 0) return SRG_ERR_ARG;
#endif
            ctx->test_fault = (int)value;
            return SRG_OK;
        case SRG_OPT_FW_XCD_ORDER:
            if (value != 0 && value != 1) return SRG_ERR_ARG;
            ctx->fw_xcd_order = (int)value;
            return SRG_OK;
        case SRG_OPT_TABLE_POOL_BYTES: {
            if (!(value >= 0.0 && value <= 1e15)) return SRG_ERR_ARG;
            std::lock_guard<std::mutex> pl(ctx->tpool->mu);
            ctx->tpool->limit = (size_t)value;
            ctx->tpool->max_idle = 0;  // an explicit byte cap replaces the one-pair default
            ctx->tpool->trim_locked(ctx->tpool->limit);
            return SRG_OK;
        }
        case SRG_OPT_ALGORITHM:
            if (value != SRG_ALGO_AUTO && value != SRG_ALGO_DENSE && value != SRG_ALGO_SPARSE) return SRG_ERR_ARG;
            ctx->algorithm = (int)value;
            return SRG_OK;
        default:
            return SRG_ERR_ARG;
    }
}

int srg_get_option(srg_ctx* ctx, int option, double* value) {
    if (!ctx || !value) return SRG_ERR_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    switch (option) {
        case SRG_OPT_PROFILING: *value = ctx->profiling; break;
        case SRG_OPT_SPARSE_THRESHOLD: *value = ctx->sparse_threshold; break;
        case SRG_OPT_GATHER_OUTPUT: *value = ctx->gather_output; break;
        case SRG_OPT_ALGORITHM: *value = ctx->algorithm; break;
        case SRG_OPT_SPARSE_LOCALITY: *value = ctx->sparse_locality; break;
        case SRG_OPT_FW_TILE: *value = ctx->fw_tile; break;
        case SRG_OPT_SPARSE_DELTA_DIV: *value = ctx->sparse_delta_div; break;
        case SRG_OPT_SPARSE_GLOBAL_BITMAPS: *value = ctx->sparse_global_bitmaps; break;
        case SRG_OPT_FW_SYMMETRIC: *value = ctx->fw_symmetric; break;
        case SRG_OPT_D2H_MODE: *value = ctx->d2h_mode; break;
        case SRG_OPT_LOSS_CHUNKS: *value = ctx->loss_chunks; break;
        case SRG_OPT_SCAN_GROUPS: *value = ctx->scan_groups; break;
        case SRG_OPT_H2D_CODEC: *value = ctx->h2d_codec; break;
        case SRG_OPT_EDGE_SHARD: *value = ctx->edge_shard; break;
        case SRG_OPT_LATE_LOSS: *value = ctx->late_loss; break;
        case SRG_OPT_FW_LINE_SPLIT: *value = ctx->fw_line_split; break;
        case SRG_OPT_FW_STEP: *value = ctx->fw_step; break;
        case SRG_OPT_FW_OVERLAP: *value = ctx->fw_overlap; break;
        case SRG_OPT_TEST_FAULT: *value = ctx->test_fault; break;
        case SRG_OPT_TABLE_POOL_BYTES: {
            std::lock_guard<std::mutex> pl(ctx->tpool->mu);
            *value = (double)ctx->tpool->limit;
            break;
        }
        case SRG_OPT_TABLE_POOL_IDLE_BYTES: {
            std::lock_guard<std::mutex> pl(ctx->tpool->mu);
            *value = (double)ctx->tpool->idle_bytes;
            break;
        }
        case SRG_OPT_CREATE_MS_RUNTIME: *value = ctx->ms_create_runtime; break;
        case SRG_OPT_FW_XCD_ORDER: *value = ctx->fw_xcd_order; break;
        case SRG_OPT_CREATE_MS_LIBRARY: *value = ctx->ms_create_lib; break;
        default: return SRG_ERR_ARG;
    }
    return SRG_OK;
}

void srg_destroy(srg_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    {
        std::lock_guard<std::mutex> lk(g_dev_mu);
        --g_dev_ctx[ctx->device];
    }
    delete ctx;
}

int srg_internal_compute_table(srg_ctx* ctx, const srg_edge_list* graph, const uint32_t* nodes, uint32_t num_nodes,
                               int shortest, uint64_t* out_lat, uint32_t* out_key, uint64_t* out_diag, float* out_loss,
                               uint64_t* unit_ns, srg_table* tab_lat, srg_table* tab_loss, srg_stats* stats,
                               char* errbuf, size_t errlen) {
    srg_stats local{};
    srg_stats* st = stats ? stats : &local;
    srg_table* tabs[2] = {tab_lat, tab_loss};
    const int rc = host_entry(ctx, graph, nodes, num_nodes, out_key ? nullptr : out_lat, out_loss, st, errbuf, errlen,
                              !shortest, out_key, out_diag, tabs);
    if (unit_ns) *unit_ns = out_key && st->latency_unit_ns ? st->latency_unit_ns : 1;
    return rc;
}

srg_table* srg_internal_table_get(srg_ctx* ctx, size_t bytes, void** host) {
    if (!ctx || !host) return nullptr;
    *host = nullptr;
    constexpr size_t HP = (size_t)2 << 20;
    const size_t cap = (std::max<size_t>(bytes, 1) + HP - 1) / HP * HP;
    TablePool& P = *ctx->tpool;
    {
        std::lock_guard<std::mutex> lk(P.mu);
        size_t best = SIZE_MAX;
        for (size_t i = 0; i < P.idle.size(); ++i)  // the smallest idle table that holds it (and < 2x)
            if (P.idle[i]->cap >= cap && P.idle[i]->cap <= 2 * cap && (best == SIZE_MAX || P.idle[i]->cap < P.idle[best]->cap))
                best = i;
        if (best != SIZE_MAX) {
            srg_table* t = P.idle[best];
            P.idle.erase(P.idle.begin() + best);
            P.idle_bytes -= t->cap;
            *host = t->p;
            return t;
        }
    }
    // a fresh mapping, 2 MB aligned; its pages are faulted in and locked by the first build into
    // it (host_entry's registration thread, beside the H2D and FW)
    void* m = mmap(nullptr, cap + HP, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    if (m == MAP_FAILED) return nullptr;
    const uintptr_t a = ((uintptr_t)m + HP - 1) / HP * HP;
    if (a > (uintptr_t)m) munmap(m, a - (uintptr_t)m);
    if ((uintptr_t)m + cap + HP > a + cap) munmap((void*)(a + cap), (uintptr_t)m + cap + HP - (a + cap));
    srg_table* t = new (std::nothrow) srg_table();
    if (!t) {
        munmap((void*)a, cap);
        return nullptr;
    }
    t->pool = ctx->tpool;
    t->p = (void*)a;
    t->cap = cap;
    *host = t->p;
    return t;
}

void srg_internal_table_put(srg_table* t) {
    if (!t) return;
    std::shared_ptr<TablePool> P = t->pool;  // (keeps the pool alive past this table)
    std::lock_guard<std::mutex> lk(P->mu);
    if (P->open && t->cap <= P->limit) {
        P->idle.push_back(t);
        P->idle_bytes += t->cap;
        P->trim_locked(P->limit);
    } else {
        TablePool::destroy(t);
    }
}

int srg_compute_shortest_paths(srg_ctx* ctx, const srg_edge_list* graph, const uint32_t* nodes, uint32_t num_nodes,
                               uint64_t* out_latency_ns, float* out_packet_loss, srg_stats* stats, char* errbuf,
                               size_t errlen) {
    return host_entry(ctx, graph, nodes, num_nodes, out_latency_ns, out_packet_loss, stats, errbuf, errlen, false);
}

int srg_get_direct_paths(srg_ctx* ctx, const srg_edge_list* graph, const uint32_t* nodes, uint32_t num_nodes,
                         uint64_t* out_latency_ns, float* out_packet_loss, srg_stats* stats, char* errbuf,
                         size_t errlen) {
    return host_entry(ctx, graph, nodes, num_nodes, out_latency_ns, out_packet_loss, stats, errbuf, errlen, true);
}

int srg_compute_shortest_paths_device(srg_ctx* ctx, const srg_edge_list* g, const uint32_t* nodes_dev,
                                      uint32_t num_nodes, uint64_t* out_lat_dev, float* out_loss_dev,
                                      void* hip_stream, srg_stats* stats, char* errbuf, size_t errlen) {
    if (!ctx || !g || (num_nodes && (!nodes_dev || !out_lat_dev || !out_loss_dev))) {
        set_err(errbuf, errlen, "null argument");
        return SRG_ERR_ARG;
    }
    std::lock_guard<std::mutex> lk(ctx->mu);
    return guard(errbuf, errlen, [&]() {
        auto t0 = std::chrono::steady_clock::now();
        if (stats) std::memset(stats, 0, sizeof(*stats));
        HIP_CHECK(hipSetDevice(ctx->device));
        hipStream_t st = hip_stream ? (hipStream_t)hip_stream : ctx->stream;
        DevGraph dg{g->num_vertices, (int)g->directed, g->num_edges, g->src, g->dst, g->latency_ns,
                    g->packet_loss, g->node_ids, nullptr};
        compute_device(*ctx, dg, nodes_dev, num_nodes, out_lat_dev, out_loss_dev, st, stats);
        HIP_CHECK(hipStreamSynchronize(st));
        if (stats) stats->ms_total = ms_since(t0);
    });
}

int srg_comm_unique_id(unsigned char id[SRG_UNIQUE_ID_BYTES], char* errbuf, size_t errlen) {
    if (!id) {
        set_err(errbuf, errlen, "null argument");
        return SRG_ERR_ARG;
    }
    return guard(errbuf, errlen, [&]() {
        const std::string e = srg::rccl_unique_id(id);
        if (!e.empty()) fail(SRG_ERR_RCCL, e);
    });
}

int srg_comm_init(srg_ctx* ctx, int nranks, int rank, const unsigned char id[SRG_UNIQUE_ID_BYTES], char* errbuf,
                  size_t errlen) {
    if (!ctx || !id || nranks < 1 || rank < 0 || rank >= nranks) {
        set_err(errbuf, errlen, "bad argument");
        return SRG_ERR_ARG;
    }
    std::lock_guard<std::mutex> lk(ctx->mu);
    return guard(errbuf, errlen, [&]() {
        srg::Comm* cm = nullptr;
        const std::string e = srg::rccl_create(nranks, rank, id, ctx->device, &cm);
        if (!e.empty()) fail(SRG_ERR_RCCL, e);
        delete ctx->comm;
        ctx->comm = cm;
    });
}

int srg_local_group_create(int nranks, srg_local_group** out) {
    if (!out || nranks < 1) return SRG_ERR_ARG;
    *out = reinterpret_cast<srg_local_group*>(srg::local_group_create(nranks));
    return SRG_OK;
}

void srg_local_group_release(srg_local_group* g) { srg::local_group_release(reinterpret_cast<srg::LocalGroup*>(g)); }

int srg_comm_init_local(srg_ctx* ctx, srg_local_group* g, int rank, char* errbuf, size_t errlen) {
    if (!ctx || !g) {
        set_err(errbuf, errlen, "null argument");
        return SRG_ERR_ARG;
    }
    std::lock_guard<std::mutex> lk(ctx->mu);
    return guard(errbuf, errlen, [&]() {
        srg::Comm* cm = nullptr;
        const std::string e = srg::local_create(reinterpret_cast<srg::LocalGroup*>(g), rank, ctx->device, &cm);
        if (!e.empty()) fail(SRG_ERR_ARG, e);
        delete ctx->comm;
        ctx->comm = cm;
    });
}

int srg_comm_size(srg_ctx* ctx, int* nranks, int* rank) {
    if (!ctx || !nranks || !rank) return SRG_ERR_ARG;
    *nranks = ctx->comm ? ctx->comm->nranks : 1;
    *rank = ctx->comm ? ctx->comm->rank : 0;
    return SRG_OK;
}

// ---- one call site, several GPUs of this process (srg_multi) ----------------------------------
// Shadow builds its RoutingInfo once, in one process (sim_config.rs:137-141 -> manager.rs:301-324).
// srg_multi drives N GPUs from that one call: one context per device attached to an in-process
// group (collectives = pull kernels over xGMI), one worker thread per rank, and the caller's two
// host arrays page-locked once (portable) while the ranks ship their edges and run FW.  Every rank
// runs the SPMD build with the output exchange off and ships its own sources' rows over its own
// PCIe link straight into the caller's arrays, so the call returns with the whole table there.
struct srg_multi {
    std::vector<srg_ctx*> ranks;
    std::vector<int> devices;
    srg::LocalGroup* group = nullptr;
    std::mutex mu;
    ~srg_multi() {
        for (srg_ctx* c : ranks) srg_destroy(c);
        if (group) srg::local_group_release(group);
    }
};

int srg_multi_create(srg_multi** out, const int* devices, int num_devices, char* errbuf, size_t errlen) {
    if (!out || !devices || num_devices < 1) {
        set_err(errbuf, errlen, "bad argument");
        return SRG_ERR_ARG;
    }
    *out = nullptr;
    auto* m = new srg_multi();
    m->devices.assign(devices, devices + num_devices);
    m->group = srg::local_group_create(num_devices);
    for (int r = 0; r < num_devices; ++r) {
        srg_ctx* c = nullptr;
        int rc = srg_create(&c, devices[r], errbuf, errlen);
        if (rc == SRG_OK) {
            m->ranks.push_back(c);
            if (num_devices > 1) rc = srg_comm_init_local(c, reinterpret_cast<srg_local_group*>(m->group), r, errbuf, errlen);
        }
        if (rc != SRG_OK) {
            delete m;
            return rc;
        }
    }
    *out = m;
    return SRG_OK;
}

void srg_multi_destroy(srg_multi* m) { delete m; }

int srg_multi_size(const srg_multi* m) { return m ? (int)m->ranks.size() : 0; }

int srg_multi_set_option(srg_multi* m, int option, double value) {
    if (!m) return SRG_ERR_ARG;
    if (option == SRG_OPT_GATHER_OUTPUT || option == SRG_OPT_SIMULATE_RANK) return SRG_ERR_ARG;  // fixed by srg_multi
    // all or nothing: the ranks must keep one option set (a split FW tile or line split would run
    // mismatched multi-rank schedules), so a rank that rejects the value rolls the others back
    std::vector<double> old(m->ranks.size(), 0.0);
    for (size_t r = 0; r < m->ranks.size(); ++r)
        if (srg_get_option(m->ranks[r], option, &old[r]) != SRG_OK) return SRG_ERR_ARG;
    for (size_t r = 0; r < m->ranks.size(); ++r) {
        const int rc = srg_set_option(m->ranks[r], option, value);
        if (rc != SRG_OK) {
            for (size_t q = 0; q < r; ++q) (void)srg_set_option(m->ranks[q], option, old[q]);
            return rc;
        }
    }
    return SRG_OK;
}

int srg_multi_compute_shortest_paths(srg_multi* m, const srg_edge_list* graph, const uint32_t* nodes,
                                     uint32_t num_nodes, uint64_t* out_latency_ns, float* out_packet_loss,
                                     srg_stats* stats, char* errbuf, size_t errlen) {
    if (!m || !graph || (num_nodes && (!nodes || !out_latency_ns || !out_packet_loss))) {
        set_err(errbuf, errlen, "null argument");
        return SRG_ERR_ARG;
    }
    std::lock_guard<std::mutex> lk(m->mu);
    const int G = (int)m->ranks.size();
    if (G == 1) return srg_compute_shortest_paths(m->ranks[0], graph, nodes, num_nodes, out_latency_ns, out_packet_loss,
                                                  stats, errbuf, errlen);
    const auto t0 = std::chrono::steady_clock::now();
    const size_t nn = (size_t)num_nodes * num_nodes;
    // one registration of the caller's arrays for every rank, beside the ranks' H2D and FW
    struct Reg {
        std::mutex mu;
        std::thread th;
        bool done = false, ok = false;
        double ms = 0;
        void* p[2] = {nullptr, nullptr};
        size_t b[2] = {0, 0};
        bool wait() {
            std::lock_guard<std::mutex> l(mu);
            if (!done) {
                if (th.joinable()) th.join();
                done = true;
            }
            return ok;
        }
    } reg;
    reg.p[0] = out_latency_ns;
    reg.b[0] = nn * 8;
    reg.p[1] = out_packet_loss;
    reg.b[1] = nn * 4;
    const bool big = nn * 12 >= ((size_t)64 << 20);
    if (big) {
        const int dev0 = m->devices[0];
        reg.th = std::thread([&reg, dev0]() {
            const auto ts = std::chrono::steady_clock::now();
            if (hipSetDevice(dev0) != hipSuccess) return;
            const unsigned fl = hipHostRegisterPortable | hipHostRegisterMapped;
            advise_huge(reg.p[0], reg.b[0]);
            advise_huge(reg.p[1], reg.b[1]);
            if (hipHostRegister(reg.p[0], reg.b[0], fl) != hipSuccess) return;
            if (hipHostRegister(reg.p[1], reg.b[1], fl) != hipSuccess) {
                (void)hipHostUnregister(reg.p[0]);
                return;
            }
            reg.ms = ms_since(ts);
            reg.ok = true;
        });
    }
    std::vector<int> rc(G, SRG_OK);
    std::vector<std::string> msg(G);
    std::vector<srg_stats> st(G);
    std::vector<std::thread> th;
    for (int r = 0; r < G; ++r) {
        srg_ctx* c = m->ranks[r];
        c->gather_output = false;
        if (big)
            c->ext_reg = [&reg](void** views, double* ms) {
                if (!reg.wait()) return false;
                for (int i = 0; i < 2; ++i)
                    if (hipHostGetDevicePointer(&views[i], reg.p[i], 0) != hipSuccess) views[i] = nullptr;
                *ms = reg.ms;
                return true;
            };
        th.emplace_back([&, r, c]() {
            char eb[1024];
            rc[r] = srg_compute_shortest_paths(c, graph, nodes, num_nodes, out_latency_ns, out_packet_loss, &st[r], eb,
                                               sizeof(eb));
            msg[r] = eb;
            if (rc[r] != SRG_OK) srg::local_group_abort(m->group);  // release peers waiting in a collective
        });
    }
    for (auto& t : th) t.join();
    for (srg_ctx* c : m->ranks) c->ext_reg = nullptr;
    srg::local_group_reset(m->group);
    if (big && reg.wait()) {  // every rank's copies into the arrays are complete (their sinks finished)
        (void)hipHostUnregister(reg.p[0]);
        (void)hipHostUnregister(reg.p[1]);
    }
    // the first rank that failed for its own reason (the others report the abort)
    int first = -1;
    for (int r = 0; r < G && first < 0; ++r)
        if (rc[r] != SRG_OK && rc[r] != SRG_ERR_RCCL) first = r;
    for (int r = 0; r < G && first < 0; ++r)
        if (rc[r] != SRG_OK) first = r;
    if (first >= 0) {
        set_err(errbuf, errlen, msg[first]);
        return rc[first];
    }
    if (stats) {
        // wall times: the slowest rank; counts: summed; minimum latency: over every rank's rows
        *stats = st[0];
        stats->local_sources = 0;
        stats->d2h_overlapped_bytes = 0;
        stats->prof_launches = 0;
        stats->prof_kernel_ms = 0;
        stats->prof_relaxations = 0;
        stats->relaxations = 0;
        stats->multi_pred_pairs = 0;
        for (const srg_stats& x : st) {
            for (double srg_stats::*f : {&srg_stats::ms_h2d, &srg_stats::ms_build, &srg_stats::ms_fw, &srg_stats::ms_scan,
                                          &srg_stats::ms_loss, &srg_stats::ms_extract, &srg_stats::ms_d2h,
                                          &srg_stats::ms_exchange, &srg_stats::ms_host_register})
                stats->*f = std::max(stats->*f, x.*f);
            stats->loss_rounds = std::max(stats->loss_rounds, x.loss_rounds);
            stats->local_sources += x.local_sources;
            stats->d2h_overlapped_bytes += x.d2h_overlapped_bytes;
            stats->prof_launches += x.prof_launches;
            stats->prof_kernel_ms += x.prof_kernel_ms;
            stats->prof_relaxations += x.prof_relaxations;
            stats->relaxations += x.relaxations;
            stats->multi_pred_pairs += x.multi_pred_pairs;
            stats->min_latency_ns = std::min(stats->min_latency_ns, x.min_latency_ns);
        }
        stats->rank = 0;
        stats->nranks = G;
        stats->ms_total = ms_since(t0);
    }
    if (errbuf && errlen) errbuf[0] = 0;
    return SRG_OK;
}

int srg_multi_get_direct_paths(srg_multi* m, const srg_edge_list* graph, const uint32_t* nodes, uint32_t num_nodes,
                               uint64_t* out_latency_ns, float* out_packet_loss, srg_stats* stats, char* errbuf,
                               size_t errlen) {
    if (!m) {
        set_err(errbuf, errlen, "null argument");
        return SRG_ERR_ARG;
    }
    std::lock_guard<std::mutex> lk(m->mu);
    // rank 0 alone: its context must not wait for peers in a collective
    srg_ctx* c = m->ranks[0];
    srg::Comm* cm = nullptr;
    {
        std::lock_guard<std::mutex> l2(c->mu);
        std::swap(cm, c->comm);
    }
    const int rc = srg_get_direct_paths(c, graph, nodes, num_nodes, out_latency_ns, out_packet_loss, stats, errbuf, errlen);
    {
        std::lock_guard<std::mutex> l2(c->mu);
        std::swap(cm, c->comm);
    }
    return rc;
}

int srg_order_packet_events_device(srg_ctx* ctx, const srg_event_batch* b, const uint64_t* table, uint32_t table_n,
                                   uint64_t* out_deliver, uint32_t* out_order, uint64_t* out_host_off,
                                   void* hip_stream, srg_event_result* res, char* errbuf, size_t errlen) {
    if (!ctx || !b || !out_host_off ||
        (b->num_events && (!table || !out_deliver || !out_order || !b->src_node || !b->dst_node || !b->src_host ||
                           !b->dst_host || !b->send_time_ns || !b->src_event_id))) {
        set_err(errbuf, errlen, "null argument");
        return SRG_ERR_ARG;
    }
    std::lock_guard<std::mutex> lk(ctx->mu);
    return guard(errbuf, errlen, [&]() {
        auto t0 = std::chrono::steady_clock::now();
        HIP_CHECK(hipSetDevice(ctx->device));
        hipStream_t st = hip_stream ? (hipStream_t)hip_stream : ctx->stream;
        EvIn in{b->num_events, b->src_node, b->dst_node, b->src_host, b->dst_host, b->send_time_ns,
                b->src_event_id, table, table_n, b->num_hosts, b->round_end_ns};
        order_events_device(*ctx, in, out_deliver, out_order, out_host_off, st, res);
        HIP_CHECK(hipStreamSynchronize(st));
        if (res) res->ms_total = ms_since(t0);
    });
}

const char* srg_version(void) { return "shadow_amd routing 0.3 (gfx950, dense FW u32/u64 + tight-DAG loss, RCCL row-block FW, sparse BF, event batches)"; }

}  // extern "C"
