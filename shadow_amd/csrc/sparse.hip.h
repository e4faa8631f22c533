// sparse.hip.h — batched lexicographic Bellman-Ford over CSR for sparse graphs (gfx950).
//
// Per used source the reference runs petgraph's Dijkstra with PathProperties scores
// (mod.rs:190-208, 305-331).  Its result is the unique solution of
//     label(s) = (0, 0.0),   label(t) = lexmin over in-arcs (u,t) of label(u) (+) arc
// where (+) is PathProperties::add (u64 latency sum, left-fold f32 loss) and lexmin compares
// latency then loss (positive latencies make the tight graph a DAG, so the fixpoint is unique
// and equals Dijkstra's scores bit for bit).  Any relaxation order that reaches the fixpoint
// therefore reproduces the reference; this file reaches it with pull-style Bellman-Ford sweeps.
//
// Batching: one 64-lane wave relaxes ONE vertex for 64 sources at once (lane = source), so
// every label access is one coalesced 512-byte row.  A label is the lexicographic key
//     (latency_u32 << 32) | float_bits(loss)        (loss >= +0: bit order == numeric order)
// so lexmin is a single u64 min.  Latency keys saturate at 2^32-1 (= "unreachable or too
// long"); the host re-runs such graphs on the wide labels (LabelU64: u64 latency + u32 loss).
//
// Layout (HBM):
//   in_off [V+1], in_src/in_w/in_b [arcs]  CSR of IN-arcs (self-loops dropped; undirected
//                                          edges give both arcs; parallel arcs kept)
//   slot labels [V][64] u64 per resident workgroup (one batch of 64 sources at a time)
// One workgroup owns one batch for all of its sweeps (no inter-workgroup synchronisation):
// per sweep every wave pulls the vertices it owns, skipping arcs whose source vertex did not
// change in the previous sweep (bit flags in LDS), and the batch ends when a sweep changes
// nothing.  Workgroups take batches from an atomic queue until none are left.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.hip.h"
#include "guards.h"

namespace srg {

constexpr unsigned long long LBL_INF = ~0ull;
constexpr int SP_WAVES = 16;           // waves per workgroup (1024 threads)
constexpr int SP_THREADS = SP_WAVES * 64;
constexpr int SP_CAP = 128;            // active-arc list entries per wave
constexpr int SP_G = 8;                // label rows in flight per wave
constexpr size_t sp_scratch_bytes() {
    return (size_t)SP_WAVES * (128 + 3 * SP_CAP) * 4 > 64 * 65 * 8 ? (size_t)SP_WAVES * (128 + 3 * SP_CAP) * 4
                                                                   : (size_t)64 * 65 * 8;
}
static_assert(sp_scratch_bytes() >= (size_t)SP_WAVES * (128 + 3 * SP_CAP) * 4, "per-wave scratch");
constexpr uint32_t SP_OWN = 0xFFFFFFFFu;  // w_b tag of a list entry that is a vertex's own row (b is never NaN)

__device__ __forceinline__ unsigned long long lbl_relax(unsigned long long lu, uint32_t w, float b) {
    const uint32_t lat = (uint32_t)(lu >> 32);
    const uint32_t nl = __builtin_elementwise_add_sat(lat, w);
    const float loss = fold_loss(__uint_as_float((uint32_t)lu), b);
    const unsigned long long c = ((unsigned long long)nl << 32) | __float_as_uint(loss);
    return nl == 0xFFFFFFFFu ? LBL_INF : c;
}

// Label policies.  Narrow (u32 latency keys): one u64 per lane, (key << 32) | loss bits, lexmin =
// u64 min.  Wide (u64 latency keys, for graphs whose used paths pass 2^32-1 units): one 16-byte
// slot per lane {latency u64, loss bits}, read and written by single 16-B vector accesses so that
// a wave pulling a row another wave is lowering sees either label whole (two separate arrays let a
// reader pair a new latency with an old, smaller loss, and that candidate could stick: a 1050-vertex
// case differed in loss); lexmin compares both words.  The host only takes it when
// max_lat * V < 2^64, so sums never wrap (saturation is a guard).
struct LabelU32 {
    using T = unsigned long long;
    static constexpr bool wide = false;
    static constexpr uint64_t LAT_MAX = 0xFFFFFFFFull;
    unsigned long long* L;
    __device__ static T inf() { return LBL_INF; }
    __device__ static T zero() { return 0ull; }
    __device__ static bool lt(T a, T b) { return a < b; }
    __device__ static bool is_inf(T a) { return a == LBL_INF; }
    __device__ static uint64_t lat(T a) { return a >> 32; }
    __device__ static uint32_t loss_bits(T a) { return (uint32_t)a; }
    // plain loads: C4 274-276 ms against 281-304 with the nontemporal hint (profiles/r06/sparse_cache/)
    __device__ T ld(size_t i) const { return L[i]; }
    __device__ void st(size_t i, T v) const { L[i] = v; }
    // arc weight: the list holds the u32 key itself
    __device__ static T relax(T u, uint32_t wtag, float b, const uint64_t*) { return lbl_relax(u, wtag, b); }
    __device__ static uint32_t wtag(uint32_t k, const uint32_t* in_w) { return in_w[k]; }
};

struct LabelU64 {
    struct T {
        uint64_t l;
        uint32_t s;
    };
    static constexpr bool wide = true;
    static constexpr uint64_t LAT_MAX = ~0ull;
    typedef unsigned long long v2u64 __attribute__((ext_vector_type(2)));
    v2u64* L;  // [V][64] slots: x = latency key, y = loss bits
    __device__ static T inf() { return T{~0ull, 0xFFFFFFFFu}; }
    __device__ static T zero() { return T{0ull, 0u}; }
    __device__ static bool lt(T a, T b) { return a.l < b.l || (a.l == b.l && a.s < b.s); }
    __device__ static bool is_inf(T a) { return a.l == ~0ull; }
    __device__ static uint64_t lat(T a) { return a.l; }
    __device__ static uint32_t loss_bits(T a) { return a.s; }
    __device__ T ld(size_t i) const {
        const v2u64 v = L[i];
        return T{v.x, (uint32_t)v.y};
    }
    __device__ void st(size_t i, T v) const {
        v2u64 w;
        w.x = v.l;
        w.y = v.s;
        L[i] = w;
    }
    // arc weight: the list holds the arc index, the u64 key is read per relaxation (wave-uniform)
    __device__ static T relax(T u, uint32_t wtag, float b, const uint64_t* in_w64) {
        const uint64_t w = in_w64[wtag];
        const uint64_t nl = u.l + w;
        if (nl < u.l || nl == ~0ull) return inf();
        return T{nl, __float_as_uint(fold_loss(__uint_as_float(u.s), b))};
    }
    __device__ static uint32_t wtag(uint32_t k, const uint32_t*) { return k; }
};

// ---- CSR of in-arcs -------------------------------------------------------------------
__device__ __forceinline__ uint32_t lat_key32(uint64_t l) { return l >= 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)l; }

__global__ void k_csr_count(uint64_t E, const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
                            int directed, uint32_t* __restrict__ indeg) {
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < E; e += (size_t)gridDim.x * blockDim.x) {
        const uint32_t s = src[e], t = dst[e];
        if (s == t) continue;
        atomicAdd(&indeg[t], 1u);
        if (!directed) atomicAdd(&indeg[s], 1u);
    }
}

// out-arcs (directed graphs only): targets per source vertex
__global__ void k_csr_count_out(uint64_t E, const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
                                uint32_t* __restrict__ outdeg) {
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < E; e += (size_t)gridDim.x * blockDim.x)
        if (src[e] != dst[e]) atomicAdd(&outdeg[src[e]], 1u);
}

__global__ void k_csr_fill_out(uint64_t E, const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
                               const uint32_t* __restrict__ off, uint32_t* __restrict__ cur,
                               uint32_t* __restrict__ out_dst) {
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < E; e += (size_t)gridDim.x * blockDim.x) {
        const uint32_t s = src[e], t = dst[e];
        if (s != t) out_dst[off[s] + atomicAdd(&cur[s], 1u)] = t;
    }
}

__global__ void k_csr_fill(uint64_t E, const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
                           const uint64_t* __restrict__ lat, uint64_t unit, const float* __restrict__ loss, int directed,
                           const uint32_t* __restrict__ off, uint32_t* __restrict__ cur, uint32_t* __restrict__ in_src,
                           uint32_t* __restrict__ in_w, float* __restrict__ in_b, uint64_t* __restrict__ in_w64) {
    // in_w64 (wide labels): the u64 key per arc beside the saturated u32 one
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < E; e += (size_t)gridDim.x * blockDim.x) {
        const uint32_t s = src[e], t = dst[e];
        if (s == t) continue;
        const uint64_t w64 = unit != 1 ? lat[e] / unit : lat[e];  // latency units (compute_device)
        const uint32_t w = lat_key32(w64);
        const float b = __fsub_rn(1.0f, loss[e] + 0.0f);
        uint32_t k = off[t] + atomicAdd(&cur[t], 1u);
        in_src[k] = s;
        in_w[k] = w;
        in_b[k] = b;
        if (in_w64) in_w64[k] = w64;
        if (!directed) {
            k = off[s] + atomicAdd(&cur[s], 1u);
            in_src[k] = t;
            in_w[k] = w;
            in_b[k] = b;
            if (in_w64) in_w64[k] = w64;
        }
    }
}

// ---- the batched sweep kernel ------------------------------------------------------------
struct SparseArgs {
    const uint32_t* in_off;
    const uint32_t* in_src;
    const uint32_t* in_w;
    const float* in_b;
    const uint32_t* out_off;     // CSR of OUT-arcs (== the in-CSR for undirected graphs)
    const uint32_t* out_dst;
    uint32_t V;
    const uint32_t* batch_src;   // [nbatch*64] source vertex per lane
    const uint32_t* batch_row;   // [nbatch*64] output row per lane (0xFFFFFFFF = padding lane)
    uint32_t nbatch;
    unsigned long long* slots;   // [gridDim.x][V][64]
    uint32_t* queue;             // next batch
    const uint32_t* cols;        // [ncols] used target vertices (output columns)
    uint32_t ncols;
    const uint64_t* self_lat;    // raw self-loop weight (diagonal, mod.rs:211-217)
    const float* self_loss;
    uint64_t* out_lat;           // [rows][ncols]
    float* out_loss;
    uint32_t* flags;             // [0] unreachable/saturated used pair, [1] max sweeps, [2..3] total evaluations,
                                 // [5] some relaxation saturated the u32 latency key (a path >= 2^32-1 ns)
    uint64_t unit;               // latency unit in ns (outputs = key * unit)
    uint64_t delta;              // bucket width in latency units (~0 = one bucket: plain Bellman-Ford)
    unsigned long long* gbits;   // [gridDim.x][5][nw] vertex bitmaps when they do not fit in LDS (GB = true)
    uint32_t* out_key;           // RoutingInfo key table (null: ns latencies into out_lat), diagonal 0xFFFFFFFF
    uint64_t* out_diag;          // with out_key: the raw self-loop latency per output row
    const uint64_t* in_w64;      // wide labels: u64 arc keys (`slots` then holds 16-byte labels)
    uint64_t min_key;            // smallest arc key: a used off-diagonal latency below it is impossible
                                 // (guards.h) -> flags[6]
    // two-phase kernel (k_sparse_ds, sparse_ds.hip.h): `slots` then holds u32 latency labels
    float* lo_slots;             // [gridDim.x][V][64] loss labels
    unsigned long long* tmask;   // [gridDim.x][arcs] tight-lane masks per in-arc
    unsigned long long* fmask;   // [gridDim.x][V] final-lane masks of the loss fold
    uint32_t arcs;
    uint32_t* dbg;  // per-batch {start, phase-1 ticks, workgroup, sweeps, phase-2 start, phase-2 ticks} (SRG_DEBUG_SPARSE=2)
};

// a vertex whose label dropped in some lanes is pushed now if some dropped lane's new latency is
// below the bucket bound (requiring every dropped lane below it was measured slower)
__device__ __forceinline__ bool bucket_ready(bool dropped, bool below) { return __ballot(dropped && below) != 0; }

// Vertex bitmaps (one bit per vertex): fprev = changed in the previous sweep (the arcs worth
// pulling), fcur = changed in this sweep, mark/mnext = vertices to evaluate in this / the next
// sweep (the out-neighbours of changed vertices, pushed when a vertex changes).  A sweep
// only visits marked vertices, 64 per wave step (one bitmap word pair).  The five bitmaps take
// 5 V / 8 bytes: in LDS up to V ~ 190k (GB = false), beyond that in a per-workgroup global
// slice (GB = true; the same accesses, separated by the same barriers, L2-resident).
// WPE = waves per SIMD the register budget is sized for: 8 for the u32 labels (two 1024-thread
// workgroups per CU, <= 64 VGPRs: the kernel spills ~48 B per lane to scratch; one workgroup per CU
// without spills measured 1.2x slower), 4 for the wide labels (one workgroup per CU).
// LB = label policy (LabelU32 / LabelU64 above).
template <int G, bool GB, int WPE = 8, class LB = LabelU32>
__global__ void __launch_bounds__(SP_THREADS, WPE) k_sparse_bf(SparseArgs a) {
    using Lbl = typename LB::T;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const uint32_t V = a.V;
    const uint32_t nw = (V + 63) / 64;  // 64-vertex windows
    unsigned long long* fprev =
        GB ? a.gbits + (size_t)blockIdx.x * 5 * nw : reinterpret_cast<unsigned long long*>(smem_raw);
    unsigned long long* fcur = fprev + nw;
    unsigned long long* mark = fcur + nw;
    unsigned long long* mnext = mark + nw;
    unsigned long long* pend = mnext + nw;  // changed, but above the bucket bound: not pushed yet
    __shared__ uint32_t s_batch, s_changed, s_pend;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // per-wave scratch: vertex prefix/offsets (64 + 64) and the active-arc list (3 x SP_CAP);
    // the output transpose tile [64][65] u64 reuses the same region after convergence
    uint32_t* scratch = GB ? reinterpret_cast<uint32_t*>(smem_raw) : reinterpret_cast<uint32_t*>(pend + nw);
    uint32_t* w_st = scratch + wave * (128 + 3 * SP_CAP);  // stride = sp_scratch_bytes() / SP_WAVES
    uint32_t* w_lo = w_st + 64;
    uint32_t* w_u = w_lo + 64;
    uint32_t* w_w = w_u + SP_CAP;   // arc weight, or the window index of an own-row entry
    uint32_t* w_b = w_w + SP_CAP;   // 1 - arc loss, or SP_OWN
    unsigned long long* tile = reinterpret_cast<unsigned long long*>(scratch);
    LB lab;
    if constexpr (LB::wide)
        lab.L = reinterpret_cast<typename LabelU64::v2u64*>(a.slots) + (size_t)blockIdx.x * V * 64;
    else
        lab.L = a.slots + (size_t)blockIdx.x * V * 64;
    uint32_t max_sweeps = 0;
    unsigned long long evals = 0;
    uint32_t saturated = 0;  // a finite label + arc reached 2^32-1: INF may then mean "too long", not unreachable

    auto push_out = [&](uint32_t v) {  // mark the out-neighbours of v for the next sweep
        const uint32_t o0 = a.out_off[v], o1 = a.out_off[v + 1];
        for (uint32_t k = o0 + lane; k < o1; k += 64) {
            const uint32_t t = a.out_dst[k];
            atomicOr(&mnext[t >> 6], 1ull << (t & 63));
        }
    };

    for (;;) {
        if (threadIdx.x == 0) s_batch = atomicAdd(a.queue, 1u);
        __syncthreads();
        const uint32_t bt = s_batch;
        __syncthreads();
        if (bt >= a.nbatch) break;
        const uint32_t my_src = a.batch_src[bt * 64 + lane];
        // init: labels INF except the sources; changed = the sources; marks = their out-neighbours
        for (uint32_t v = wave; v < V; v += SP_WAVES)
            lab.st((size_t)v * 64 + lane, (v == my_src) ? LB::zero() : LB::inf());
        for (uint32_t w = threadIdx.x; w < nw; w += SP_THREADS) {
            fprev[w] = 0;
            fcur[w] = 0;
            mark[w] = 0;
            mnext[w] = 0;
            pend[w] = 0;
        }
        if (threadIdx.x == 0) s_pend = 0;
        // bucket bound (delta-stepping): a changed vertex is pushed to its out-neighbours only
        // once some lane's new latency is below the bound; the others wait in `pend` until the
        // bucket is exhausted and the bound moves on.  Any push order reaches the same unique
        // lexicographic fixpoint; the order only changes the work.
        uint64_t bound = a.delta >= LB::LAT_MAX ? LB::LAT_MAX : a.delta;
        __syncthreads();
        if (wave == 0) atomicOr(&fprev[my_src >> 6], 1ull << (my_src & 63));
        for (uint32_t q = wave; q < 64; q += SP_WAVES) {
            const uint32_t sv = (uint32_t)__builtin_amdgcn_readlane((int)my_src, q);
            push_out(sv);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();
        for (uint32_t w = threadIdx.x; w < nw; w += SP_THREADS) {
            mark[w] = mnext[w];
            mnext[w] = 0;
        }
        __syncthreads();
        uint32_t sweeps = 0;
        for (;;) {
            if (threadIdx.x == 0) s_changed = 0;
            __syncthreads();
            uint32_t chg = 0;
            for (uint32_t w = wave; w < nw; w += SP_WAVES) {
                const unsigned long long mk = mark[w];
                if (!mk) continue;
                // (1) offsets of the window's 64 vertices: one load for all of them
                const uint32_t vl = w * 64 + lane;
                const bool marked = (mk >> lane) & 1ull;
                const uint32_t lo = vl < V ? a.in_off[vl] : 0u;
                const uint32_t hi = vl < V ? a.in_off[vl + 1] : 0u;
                // flattened slots per marked vertex: slot 0 = its own row (the old label), then
                // one slot per in-arc
                const uint32_t deg = marked ? hi - lo + 1 : 0u;
                uint32_t incl = deg;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t t = __shfl_up(incl, o, 64);
                    if ((int)lane >= o) incl += t;
                }
                const uint32_t total = (uint32_t)__shfl(incl, 63, 64);
                w_st[lane] = incl - deg;
                w_lo[lane] = lo;
                __builtin_amdgcn_wave_barrier();
                // (2) flattened scan of the marked vertices' in-arcs -> LDS list of the active
                //     ones (source vertex changed last sweep), grouped by target vertex, each
                //     group led by the vertex's own row (w_vi high bit set)
                uint32_t n = 0;
                unsigned long long changed = 0;  // window vertices whose label dropped (pushed now)
                unsigned long long deferred = 0; // ... whose new label is above the bound
                auto process = [&](uint32_t cnt) {
                    // (3) consume the list in groups of G rows, all loads of a group in flight
                    int cur = -1;
                    Lbl best = LB::zero(), old = LB::zero();
                    for (uint32_t j0 = 0; j0 < cnt; j0 += G) {
                        Lbl row[G];
#pragma unroll
                        for (int q = 0; q < G; ++q)
                            if (j0 + q < cnt) row[q] = lab.ld((size_t)w_u[j0 + q] * 64 + lane);
#pragma unroll
                        for (int q = 0; q < G; ++q) {
                            const uint32_t e = j0 + q;
                            if (e >= cnt) break;
                            const uint32_t tagb = w_b[e];
                            if (tagb == SP_OWN) {  // a new vertex: its current label
                                if (cur >= 0) {
                                    const bool dr = LB::lt(best, old);
                                    if (__ballot(dr)) {
                                        if (dr) lab.st((size_t)(w * 64 + cur) * 64 + lane, best);
                                        if (bucket_ready(dr, LB::lat(best) < bound))
                                            changed |= 1ull << cur;
                                        else
                                            deferred |= 1ull << cur;
                                    }
                                }
                                cur = (int)(w_w[e] & 63u);
                                old = best = row[q];
                            } else {
                                const bool rinf = LB::is_inf(row[q]);
                                const Lbl c = rinf ? LB::inf() : LB::relax(row[q], w_w[e], __uint_as_float(tagb), a.in_w64);
                                saturated |= LB::is_inf(c) & !rinf;
                                best = LB::lt(c, best) ? c : best;
                                ++evals;
                            }
                        }
                    }
                    if (cur >= 0) {
                        const bool dr = LB::lt(best, old);
                        if (__ballot(dr)) {
                            if (dr) lab.st((size_t)(w * 64 + cur) * 64 + lane, best);
                            if (bucket_ready(dr, LB::lat(best) < bound))
                                changed |= 1ull << cur;
                            else
                                deferred |= 1ull << cur;
                        }
                    }
                };
                for (uint32_t f0 = 0; f0 < total; f0 += 64) {
                    const uint32_t f = f0 + lane;
                    bool act = false;
                    uint32_t u = 0, k = 0, vi = 0;
                    if (f < total) {
                        uint32_t i = 0;
#pragma unroll
                        for (uint32_t step = 32; step; step >>= 1)
                            if (i + step < 64 && w_st[i + step] <= f) i += step;
                        const uint32_t slot = f - w_st[i];
                        if (slot == 0) {
                            u = w * 64 + i;
                            vi = 0x80000000u | i;
                            act = true;
                            k = i;
                        } else {
                            k = w_lo[i] + slot - 1;
                            u = a.in_src[k];
                            vi = i;
                            act = (fprev[u >> 6] >> (u & 63)) & 1ull;
                        }
                    }
                    const unsigned long long m = __ballot(act);
                    if (act) {
                        const uint32_t pos = n + (uint32_t)__builtin_amdgcn_mbcnt_hi(
                                                     (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                        w_u[pos] = u;
                        if (!(vi & 0x80000000u)) {
                            w_w[pos] = LB::wtag(k, a.in_w);
                            w_b[pos] = __float_as_uint(a.in_b[k]);
                        } else {
                            w_w[pos] = k;  // window index of the vertex
                            w_b[pos] = SP_OWN;
                        }
                    }
                    __builtin_amdgcn_wave_barrier();
                    n += (uint32_t)__popcll(m);
                    if (n > SP_CAP - 64) {
                        process(n);
                        n = 0;
                        // a vertex whose arcs continue past this chunk restarts its group with
                        // its (possibly just lowered) label: our stores must land first
                        const uint32_t fn = f0 + 64;
                        if (fn < total) {
                            uint32_t i = 0;
                            for (uint32_t step = 32; step; step >>= 1)
                                if (i + step < 64 && w_st[i + step] <= fn) i += step;
                            if (fn != w_st[i]) {
                                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                                if (lane == 0) {
                                    w_u[0] = w * 64 + i;
                                    w_w[0] = i;
                                    w_b[0] = SP_OWN;
                                }
                                __builtin_amdgcn_wave_barrier();
                                n = 1;
                            }
                        }
                    }
                }
                if (n) process(n);
                if ((deferred | changed) && lane == 0) {
                    // this wave owns window w for the sweep: a vertex pushed now leaves `pend`
                    const unsigned long long p = (pend[w] | deferred) & ~changed;
                    pend[w] = p;
                    if (p) s_pend = 1;
                }
                // (4) mark the out-neighbours of the changed vertices for the next sweep
                if (changed) {
                    if (lane == 0) atomicOr(&fcur[w], changed);
                    chg = 1;
                    const bool ch = (changed >> lane) & 1ull;
                    uint32_t olo = lo, ohi = hi;
                    if (a.out_off != a.in_off) {
                        olo = ch ? a.out_off[vl] : 0u;
                        ohi = ch ? a.out_off[vl + 1] : 0u;
                    }
                    const uint32_t odeg = ch ? ohi - olo : 0u;
                    uint32_t oin = odeg;
#pragma unroll
                    for (int o = 1; o < 64; o <<= 1) {
                        const uint32_t t = __shfl_up(oin, o, 64);
                        if ((int)lane >= o) oin += t;
                    }
                    const uint32_t ototal = (uint32_t)__shfl(oin, 63, 64);
                    __builtin_amdgcn_wave_barrier();
                    w_st[lane] = oin - odeg;
                    w_lo[lane] = olo;
                    __builtin_amdgcn_wave_barrier();
                    for (uint32_t f0 = 0; f0 < ototal; f0 += 64) {
                        const uint32_t f = f0 + lane;
                        if (f < ototal) {
                            uint32_t i = 0;
#pragma unroll
                            for (uint32_t step = 32; step; step >>= 1)
                                if (w_st[i + step < 64 ? i + step : 63] <= f && i + step < 64) i += step;
                            const uint32_t t = a.out_dst[w_lo[i] + (f - w_st[i])];
                            atomicOr(&mnext[t >> 6], 1ull << (t & 63));
                        }
                    }
                }
                __builtin_amdgcn_wave_barrier();
            }
            if (chg && lane == 0) s_changed = 1;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // label stores reached L2
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __syncthreads();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            ++sweeps;
            const bool more = s_changed != 0;
            for (uint32_t w = threadIdx.x; w < nw; w += SP_THREADS) {
                fprev[w] = fcur[w];
                fcur[w] = 0;
                mark[w] = mnext[w];
                mnext[w] = 0;
            }
            __syncthreads();
            if (!more) {
                if (!s_pend) break;
                // bucket exhausted: release every deferred vertex (pushed as if it had just
                // changed) and move the bound on.  Releasing only those below the new bound was
                // measured slower on C4 (more, emptier sweeps).
                __syncthreads();  // every thread has read s_pend
                bound = (a.delta >= LB::LAT_MAX || bound > LB::LAT_MAX - a.delta) ? LB::LAT_MAX : bound + a.delta;
                for (uint32_t w = threadIdx.x; w < nw; w += SP_THREADS) {
                    fprev[w] = pend[w];
                    pend[w] = 0;
                }
                __syncthreads();
                if (threadIdx.x == 0) s_pend = 0;
                for (uint32_t w = wave; w < nw; w += SP_WAVES) {
                    unsigned long long mk = fprev[w];
                    while (mk) {
                        const uint32_t b = (uint32_t)__builtin_ctzll(mk);
                        mk &= mk - 1;
                        push_out(w * 64 + b);
                    }
                }
                __syncthreads();
                for (uint32_t w = threadIdx.x; w < nw; w += SP_THREADS) {
                    mark[w] = mnext[w];
                    mnext[w] = 0;
                }
                __syncthreads();
            }
        }
        max_sweeps = sweeps > max_sweeps ? sweeps : max_sweeps;
        // ---- output rows: 64 targets x 64 sources tiles transposed through LDS ----
        // narrow labels: one pass (the tile holds the packed label); wide: pass 0 the latencies,
        // pass 1 the loss bits
        uint32_t bad = 0, imp = 0;
        for (uint32_t j0 = 0; j0 < a.ncols; j0 += 64) {
            for (int pass = 0; pass < (LB::wide ? 2 : 1); ++pass) {
                for (uint32_t i = wave; i < 64; i += SP_WAVES) {
                    const uint32_t j = j0 + i;
                    unsigned long long v = 0;
                    if (j < a.ncols) {
                        const size_t idx = (size_t)a.cols[j] * 64 + lane;
                        if constexpr (LB::wide) {
                            const auto w = lab.ld(idx);
                            v = pass ? (unsigned long long)w.s : w.l;
                        } else
                            v = lab.ld(idx);
                    }
                    tile[i * 65 + lane] = v;
                }
                __syncthreads();
                for (uint32_t sl = wave; sl < 64; sl += SP_WAVES) {
                    const uint32_t row = a.batch_row[bt * 64 + sl];
                    const uint32_t j = j0 + lane;
                    if (row == 0xFFFFFFFFu || j >= a.ncols) continue;
                    const unsigned long long l = tile[lane * 65 + sl];
                    const size_t o = (size_t)row * a.ncols + j;
                    const uint32_t s = a.batch_src[bt * 64 + sl];
                    if (!LB::wide || pass == 0) {  // latency
                        uint64_t ol;
                        if (j == row) {  // diagonal: the raw self-loop weight
                            ol = a.self_lat[s];
                        } else {
                            const uint64_t lat = LB::wide ? l : l >> 32;
                            bad |= lat == LB::LAT_MAX;
                            imp |= impossible_key<uint64_t>(lat, a.min_key, false);
                            ol = lat * a.unit;
                        }
                        if (a.out_key) {  // narrow only (the host never asks wide labels for keys)
                            a.out_key[o] = j == row ? 0xFFFFFFFFu : (uint32_t)(l >> 32);
                            if (j == row) a.out_diag[row] = ol;
                        } else {
                            a.out_lat[o] = ol;
                        }
                    }
                    if (!LB::wide || pass == 1)  // loss
                        a.out_loss[o] = j == row ? a.self_loss[s] : __uint_as_float((uint32_t)l);
                }
                __syncthreads();
            }
        }
        if (bad) atomicOr(&a.flags[0], 1u);
        if (imp) atomicOr(&a.flags[6], 1u);
    }
    if (threadIdx.x == 0) atomicMax(&a.flags[1], max_sweeps);
    if (__ballot(saturated) && lane == 0) atomicOr(&a.flags[5], 1u);
    if (lane == 0 && evals) atomicAdd(reinterpret_cast<unsigned long long*>(&a.flags[2]), evals);
}

}  // namespace srg
