// sparse_ds.hip.h — two-phase batched SSSP for sparse graphs with u32 latency keys (gfx950).
//
// What it computes is the same as k_sparse_bf (sparse.hip.h): per used source the reference's
// petgraph Dijkstra with PathProperties scores (mod.rs:190-208, 305-331), i.e. per target the
// exact u64 latency D[s][t] and the lexicographic-minimum left-fold loss over the latency-tight
// paths.  It splits them, because the loss never decides a latency and the latency alone
// converges with half the label bytes:
//
//   phase 1  latency-only delta-stepping, 64 sources per workgroup (lane = source), labels
//            D[V][64] u32 = 256-B rows.  Pull sweeps over the in-CSR: a marked vertex folds the
//            rows of its in-neighbours that changed in the previous sweep; a vertex whose label
//            dropped below the bucket bound is pushed (its out-neighbours marked for the next
//            sweep), one above it waits in the pending bucket until the bucket is exhausted.
//            The marks are wavefront-aggregated: a 64-vertex window that receives its first mark
//            is appended to the next sweep's window list with one ballot and one LDS atomic per
//            wave, and a sweep walks only that list.
//   phase 2a tight records: per in-arc k = (u, t) the 64-bit lane mask of D[u] + w_k == D[t]
//            (one pull of D[u] per arc); the arcs tight in some lane are kept as records
//            {u, 1 - loss, mask} at the head of t's own in-arc range (31 % of C4's arcs), so the fold
//            walks only them.  Only these arcs can carry a lexicographic minimum (SURVEY §8a
//            "Derived semantics"); every reachable non-source (t, lane) has one.
//   phase 2b loss fold over the tight arcs: lane l of t is computed once every tight
//            predecessor of t in lane l is final there, as min over them of
//            fold(L[u][l], 1 - p_k) (the left fold of mod.rs:322-331, separately rounded).
//            Per lane this is Kahn's order on the tight DAG (latencies > 0 make it acyclic), so
//            each (t, lane) is folded exactly once from final inputs; a row of L[u] is pulled
//            only for the arcs that are tight in a lane being completed.  Final-lane masks F[V]
//            (u64) publish completion: L stores, release fence, F store; readers load F, acquire
//            fence, then L — so a final lane's value is visible to every wave that sees its bit.
//
// CPU model of the schedule (tools/sparse2_sim.cpp, C4, 64-source BFS-local batches): phase 1
// 5.6 row pulls per arc (the lexicographic kernel: 6.4 pulls of 512-B rows), phase 2a 1 pull per
// arc, phase 2b 1.12 pulls per arc; result equal to a per-lane lexicographic Dijkstra.
//
// Layout (HBM, per resident workgroup): D [V][64] u32, L [V][64] f32, TR [arcs] 16-B tight records,
// F [V] u64 final-lane masks + TC [V] u32 tight-record counts; vertex bitmaps + window lists in LDS
// (GB = false) or a global slice.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sparse.hip.h"

namespace srg {

constexpr uint32_t DS_INF = 0xFFFFFFFFu;
constexpr uint32_t DS_CAP = SP_CAP;  // list entries per wave
constexpr uint32_t DS_WS = 128 + 3 * DS_CAP + DS_CAP / 4;  // per-wave scratch (u32): starts, offsets, list, vertex idx
constexpr size_t ds_scratch_bytes() {
    return (size_t)SP_WAVES * DS_WS * 4 > 64 * 65 * 8 ? (size_t)SP_WAVES * DS_WS * 4 : (size_t)64 * 65 * 8;
}
// bitmaps (5 x nw u64) + two window lists (2 x nw u32) per workgroup
__host__ __device__ inline size_t ds_state_bytes(uint32_t V) {
    const size_t nw = (V + 63) / 64;
    return nw * 5 * 8 + ((nw * 2 * 4 + 15) & ~(size_t)15);
}

// label rows are plain loads: the streaming hint kept them out of the caches, and a hub's row is
// pulled by every neighbour (C4 253 -> 239 ms against the nontemporal loads)
__device__ __forceinline__ uint32_t ds_row_load(const uint32_t* p) { return *p; }
// the output rows (30 GB at C4) stream past the caches the labels live in: 14.2 -> 13.6 ms of output
// per workgroup
template <class T>
__device__ __forceinline__ void ds_out_store(T* p, T v) { __builtin_nontemporal_store(v, p); }
__device__ __forceinline__ uint32_t ds_mbcnt(unsigned long long m) {
    return (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ unsigned long long ds_shfl64(unsigned long long v, uint32_t src) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, (int)src, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), (int)src, 64);
    return ((unsigned long long)hi << 32) | lo;
}
// exclusive prefix of deg over the wave; total in *tot
__device__ __forceinline__ uint32_t ds_prefix(uint32_t deg, uint32_t lane, uint32_t* tot) {
    uint32_t incl = deg;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(incl, o, 64);
        if ((int)lane >= o) incl += t;
    }
    *tot = (uint32_t)__shfl(incl, 63, 64);
    return incl - deg;
}
// the window vertex whose flattened slot range holds f (largest i with st[i] <= f)
__device__ __forceinline__ uint32_t ds_find(const uint32_t* st, uint32_t f) {
    uint32_t i = 0;
#pragma unroll
    for (uint32_t step = 32; step; step >>= 1)
        if (i + step < 64 && st[i + step] <= f) i += step;
    return i;
}

// G1: label rows in flight per wave in phases 1 and 2a (u32 rows), G2: in the fold (f32 rows + masks)
// MODE 0: one kernel runs every phase of a batch (labels per resident workgroup); MODE 1: phase 1
// only and MODE 2: phases 2 + the output only, as two launches with the latency labels kept per BATCH
// in between -- each launch then gets its own register allocation (the fused kernel spills 28 VGPRs
// at the 64-VGPR budget, phase 1 alone none: 105.9 vs 117.6 ms per workgroup, profiles/r06/sparse_split/)
template <bool GB, int G1, int G2, int MODE = 0, int NW = 16>
__global__ void __launch_bounds__(NW * 64, NW == 16 ? 8 : 4) k_sparse_ds(SparseArgs a) {
    // (NW = 8 with 128 VGPRs and 32 rows in flight per wave ran phase 1 slower: 151 vs 115 ms per
    // workgroup -- the 16-wave form keeps twice the waves' worth of rows in flight per CU)
    static_assert(NW == 16 || MODE == 1, "the output phase is laid out for 16 waves");
    constexpr int WV = NW, TH = NW * 64;  // waves / threads per workgroup
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const uint32_t V = a.V;
    const uint32_t nw = (V + 63) / 64;
    unsigned char* state = GB ? reinterpret_cast<unsigned char*>(a.gbits) + (size_t)blockIdx.x * ds_state_bytes(V) : smem_raw;
    unsigned long long* fprev = reinterpret_cast<unsigned long long*>(state);
    unsigned long long* fcur = fprev + nw;
    unsigned long long* mark = fcur + nw;
    unsigned long long* mnext = mark + nw;
    unsigned long long* pend = mnext + nw;
    uint32_t* wl_a = reinterpret_cast<uint32_t*>(pend + nw);
    uint32_t* wl_b = wl_a + nw;
    __shared__ uint32_t s_batch, s_changed, s_pend, s_ncur, s_nnext, s_take, s_take2;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t* scratch = reinterpret_cast<uint32_t*>(GB ? smem_raw : smem_raw + ds_state_bytes(V));
    uint32_t* w_st = scratch + wave * DS_WS;
    uint32_t* w_lo = w_st + 64;
    uint32_t* w_u = w_lo + 64;
    uint32_t* w_w = w_u + DS_CAP;
    uint32_t* w_b = w_w + DS_CAP;
    unsigned char* w_i = reinterpret_cast<unsigned char*>(w_b + DS_CAP);
    unsigned long long* blk = reinterpret_cast<unsigned long long*>(w_u);  // phase 2b pass A: 64 x u64
    unsigned long long* tile = reinterpret_cast<unsigned long long*>(scratch);
    uint32_t* const Dbase = reinterpret_cast<uint32_t*>(a.slots);
    uint32_t* D = Dbase + (size_t)blockIdx.x * V * 64;
    float* LO = a.lo_slots + (size_t)blockIdx.x * V * 64;
    // tight records: vertex t's tight in-arcs at TR[in_off[t] .. in_off[t] + TC[t]) as {u, bits of
    // 1 - loss, lane mask lo, hi} -- inside t's own arc range, so no global offsets are needed
    uint4* TR = reinterpret_cast<uint4*>(a.tmask) + (size_t)blockIdx.x * a.arcs;
    unsigned long long* FM = a.fmask + (size_t)blockIdx.x * V * 2;
    uint32_t* TC = reinterpret_cast<uint32_t*>(FM + V);
    uint32_t max_sweeps = 0, max_sweeps2 = 0;
    uint32_t evals = 0, pulls2 = 0;  // (per wave, flushed per batch)
    uint32_t saturated = 0;
    uint32_t* wl_cur = wl_a;
    uint32_t* wl_next = wl_b;
    // windows are taken dynamically, one LDS atomic per wave: a window holding a high-degree vertex
    // takes several times the average, and a static stride left the other waves idle at the sweep's
    // barrier
    auto take = [&](uint32_t* ctr) {
        uint32_t i = 0;
        if (lane == 0) i = atomicAdd(ctr, 1u);
        return (uint32_t)__shfl((int)i, 0, 64);
    };
    // wall-clock ticks per phase (1, 2a, 2b, output) summed over the workgroup's batches (thread 0)
    __shared__ unsigned long long s_ph[5];
    __shared__ unsigned long long s_busy[3];  // wave-ticks inside window visits (phases 1, 2a, 2b)
    if (threadIdx.x < 5) s_ph[threadIdx.x] = 0;
    if (threadIdx.x < 3) s_busy[threadIdx.x] = 0;
    unsigned long long tv0 = 0;
    auto vis_begin = [&]() { tv0 = wall_clock64(); };
    auto vis_end = [&](int p) {
        if (lane == 0) atomicAdd(&s_busy[p], wall_clock64() - tv0);
    };
    auto stamp = [&](int p) {
        if (threadIdx.x == 0) {
            const unsigned long long t = wall_clock64();
            if (p >= 0) s_ph[p] += t - s_ph[4];
            s_ph[4] = t;
        }
    };

    // mark vertex t (lanes with on) for the next sweep; a window's first mark appends it to the
    // next window list: one ballot + one LDS atomic per wave (called by the whole wave)
    auto mark_next = [&](uint32_t t, bool on) {
        bool first = false;
        if (on) first = atomicOr(&mnext[t >> 6], 1ull << (t & 63)) == 0ull;
        const unsigned long long m = __ballot(first);
        if (m) {
            const uint32_t ld = (uint32_t)__builtin_ctzll(m);
            uint32_t base = 0;
            if (lane == ld) base = atomicAdd(&s_nnext, (uint32_t)__popcll(m));
            base = (uint32_t)__shfl((int)base, (int)ld, 64);
            if (first) wl_next[base + ds_mbcnt(m)] = t >> 6;
        }
    };
    // mark the out-neighbours of the window vertices in `which` (bit i = vertex w*64+i)
    auto push_window = [&](uint32_t w, unsigned long long which) {
        const uint32_t vl = w * 64 + lane;
        const bool ch = (which >> lane) & 1ull;
        const uint32_t olo = ch ? a.out_off[vl] : 0u, ohi = ch ? a.out_off[vl + 1] : 0u;
        uint32_t ototal;
        const uint32_t ost = ds_prefix(ch ? ohi - olo : 0u, lane, &ototal);
        __builtin_amdgcn_wave_barrier();
        w_st[lane] = ost;
        w_lo[lane] = olo;
        __builtin_amdgcn_wave_barrier();
        for (uint32_t f0 = 0; f0 < ototal; f0 += 64) {
            const uint32_t f = f0 + lane;
            const bool on = f < ototal;
            uint32_t t = 0;
            if (on) {
                const uint32_t i = ds_find(w_st, f);
                t = a.out_dst[w_lo[i] + (f - w_st[i])];
            }
            mark_next(t, on);
        }
        __builtin_amdgcn_wave_barrier();
    };
    // sweep boundary: mnext -> mark, window lists swapped (caller synchronises before and after)
    auto rotate_marks = [&]() {
        for (uint32_t w = threadIdx.x; w < nw; w += TH) {
            mark[w] = mnext[w];
            mnext[w] = 0;
        }
        uint32_t* t = wl_cur;
        wl_cur = wl_next;
        wl_next = t;
    };
    auto sync_lists = [&]() {  // (all threads) s_ncur <- s_nnext, s_nnext <- 0
        __syncthreads();
        const uint32_t nn = s_nnext;
        __syncthreads();
        if (threadIdx.x == 0) {
            s_ncur = nn;
            s_nnext = 0;
        }
        __syncthreads();
    };

    for (;;) {
        if (threadIdx.x == 0) {
            s_batch = atomicAdd(a.queue, 1u);
            s_take2 = 0;
        }
        __syncthreads();
        const uint32_t bt = s_batch;
        __syncthreads();
        if (bt >= a.nbatch) break;
        if constexpr (MODE != 0) D = Dbase + (size_t)bt * V * 64;  // this batch's labels
        const uint32_t my_src = a.batch_src[bt * 64 + lane];
        stamp(-1);
        const unsigned long long tb0 = wall_clock64();
        if constexpr (MODE != 2) {

        // ================= phase 1: latency-only delta-stepping =================
        for (uint32_t v = wave; v < V; v += WV) D[(size_t)v * 64 + lane] = (v == my_src) ? 0u : DS_INF;
        for (uint32_t w = threadIdx.x; w < nw; w += TH) {
            fprev[w] = 0;
            fcur[w] = 0;
            mark[w] = 0;
            mnext[w] = 0;
            pend[w] = 0;
        }
        if (threadIdx.x == 0) {
            s_pend = 0;
            s_nnext = 0;
            s_ncur = 0;
        }
        uint64_t bound = a.delta >= 0xFFFFFFFFull ? 0xFFFFFFFFull : a.delta;
        __syncthreads();
        if (wave == 0) atomicOr(&fprev[my_src >> 6], 1ull << (my_src & 63));
        // the sources' out-neighbours: one lane set per wave, each wave a few sources
        for (uint32_t q = wave; q < 64; q += WV) {
            const uint32_t sv = (uint32_t)__builtin_amdgcn_readlane((int)my_src, q);
            const uint32_t o0 = a.out_off[sv], o1 = a.out_off[sv + 1];
            for (uint32_t k0 = o0; k0 < o1; k0 += 64) {
                const bool on = k0 + lane < o1;
                mark_next(on ? a.out_dst[k0 + lane] : 0u, on);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();
        rotate_marks();
        sync_lists();
        uint32_t sweeps = 0;
        for (;;) {
            if (threadIdx.x == 0) {
                s_changed = 0;
                s_take = 0;
            }
            __syncthreads();
            uint32_t chg = 0;
            const uint32_t ncur = s_ncur;
            for (uint32_t idx = take(&s_take); idx < ncur; idx = take(&s_take)) {
                vis_begin();
                const uint32_t w = wl_cur[idx];
                const unsigned long long mk = mark[w];
                const uint32_t vl = w * 64 + lane;
                const bool marked = (mk >> lane) & 1ull;
                const uint32_t lo = marked ? a.in_off[vl] : 0u;
                const uint32_t hi = marked ? a.in_off[vl + 1] : 0u;
                uint32_t total;
                const uint32_t st = ds_prefix(marked ? hi - lo + 1 : 0u, lane, &total);
                w_st[lane] = st;
                w_lo[lane] = lo;
                __builtin_amdgcn_wave_barrier();
                uint32_t n = 0;
                unsigned long long changed = 0, deferred = 0;
                auto finish = [&](int cur, uint32_t best, uint32_t old) {
                    if (cur < 0) return;
                    const bool dr = best < old;
                    if (__ballot(dr)) {
                        if (dr) D[(size_t)(w * 64 + cur) * 64 + lane] = best;
                        if (__ballot(dr && best < bound))
                            changed |= 1ull << cur;
                        else
                            deferred |= 1ull << cur;
                    }
                };
                auto process = [&](uint32_t cnt) {
                    int cur = -1;
                    uint32_t best = 0, old = 0;
                    for (uint32_t j0 = 0; j0 < cnt; j0 += G1) {
                        uint32_t row[G1];
#pragma unroll
                        for (int q = 0; q < G1; ++q)
                            if (j0 + q < cnt) row[q] = ds_row_load(&D[(size_t)w_u[j0 + q] * 64 + lane]);
#pragma unroll
                        for (int q = 0; q < G1; ++q) {
                            const uint32_t e = j0 + q;
                            if (e >= cnt) break;
                            if (w_b[e] == SP_OWN) {
                                finish(cur, best, old);
                                cur = (int)(w_w[e] & 63u);
                                old = best = row[q];
                            } else {
                                const uint32_t r = row[q];
                                const uint32_t c = __builtin_elementwise_add_sat(r, w_w[e]);
                                saturated |= (c == DS_INF) & (r != DS_INF);
                                best = c < best ? c : best;
                                ++evals;
                            }
                        }
                    }
                    finish(cur, best, old);
                };
                for (uint32_t f0 = 0; f0 < total; f0 += 64) {
                    const uint32_t f = f0 + lane;
                    bool act = false, own = false;
                    uint32_t u = 0, k = 0, i = 0;
                    if (f < total) {
                        i = ds_find(w_st, f);
                        const uint32_t slot = f - w_st[i];
                        if (slot == 0) {
                            u = w * 64 + i;
                            own = act = true;
                        } else {
                            k = w_lo[i] + slot - 1;
                            u = a.in_src[k];
                            act = (fprev[u >> 6] >> (u & 63)) & 1ull;
                        }
                    }
                    const unsigned long long m = __ballot(act);
                    if (act) {
                        const uint32_t pos = n + ds_mbcnt(m);
                        w_u[pos] = u;
                        w_w[pos] = own ? i : a.in_w[k];
                        w_b[pos] = own ? SP_OWN : 0u;
                    }
                    __builtin_amdgcn_wave_barrier();
                    n += (uint32_t)__popcll(m);
                    if (n > SP_CAP - 64) {
                        process(n);
                        n = 0;
                        // a vertex whose arcs continue past this chunk restarts its group with its
                        // (possibly just lowered) label: our stores must land first
                        const uint32_t fn = f0 + 64;
                        if (fn < total) {
                            const uint32_t i2 = ds_find(w_st, fn);
                            if (fn != w_st[i2]) {
                                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                                if (lane == 0) {
                                    w_u[0] = w * 64 + i2;
                                    w_w[0] = i2;
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
                    const unsigned long long p = (pend[w] | deferred) & ~changed;
                    pend[w] = p;
                    if (p) s_pend = 1;
                }
                if (changed) {
                    if (lane == 0) atomicOr(&fcur[w], changed);
                    chg = 1;
                    push_window(w, changed);
                }
                __builtin_amdgcn_wave_barrier();
                vis_end(0);
            }
            if (chg && lane == 0) s_changed = 1;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // label stores reached L2
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __syncthreads();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            ++sweeps;
            const bool more = s_changed != 0;
            for (uint32_t w = threadIdx.x; w < nw; w += TH) {
                fprev[w] = fcur[w];
                fcur[w] = 0;
            }
            rotate_marks();
            sync_lists();
            if (!more) {
                if (!s_pend) break;
                // bucket exhausted: every pending vertex is pushed as if it had just changed, and
                // the bound moves on by one bucket
                __syncthreads();  // every thread has read s_pend
                bound = (a.delta >= 0xFFFFFFFFull || bound > 0xFFFFFFFFull - a.delta) ? 0xFFFFFFFFull : bound + a.delta;
                for (uint32_t w = threadIdx.x; w < nw; w += TH) {
                    fprev[w] = pend[w];
                    pend[w] = 0;
                }
                __syncthreads();
                if (threadIdx.x == 0) s_pend = 0;
                for (uint32_t w = wave; w < nw; w += WV) {
                    const unsigned long long pw = fprev[w];
                    if (pw) push_window(w, pw);
                }
                __syncthreads();
                rotate_marks();
                sync_lists();
            }
        }
        max_sweeps = sweeps > max_sweeps ? sweeps : max_sweeps;
        stamp(0);
        if (a.dbg && threadIdx.x == 0) {
            a.dbg[bt * 6 + 0] = (uint32_t)tb0;
            a.dbg[bt * 6 + 1] = (uint32_t)(wall_clock64() - tb0);
            a.dbg[bt * 6 + 2] = blockIdx.x;
            a.dbg[bt * 6 + 3] = sweeps;
        }
        }  // (MODE != 2)
        if constexpr (MODE == 1) {  // (the lane evaluations are flushed here, the rest after the output)
            if (lane == 0 && evals) atomicAdd(reinterpret_cast<unsigned long long*>(&a.flags[2]), (unsigned long long)evals);
            evals = 0;
            continue;
        }

        // ================= phase 2a: tight records, final-lane init =================
        for (uint32_t w = take(&s_take2); w < nw; w = take(&s_take2)) {
            vis_begin();
            const uint32_t vl = w * 64 + lane;
            const bool valid = vl < V;
            const uint32_t lo = valid ? a.in_off[vl] : 0u;
            const uint32_t hi = valid ? a.in_off[vl + 1] : 0u;
            uint32_t total;
            const uint32_t st = ds_prefix(valid ? hi - lo + 1 : 0u, lane, &total);
            w_st[lane] = st;
            w_lo[lane] = lo;
            __builtin_amdgcn_wave_barrier();
            uint32_t dt = 0, tcnt = 0;  // tcnt: lane i counts vertex i's tight arcs
            int cur = 0;
            auto process = [&](uint32_t cnt) {
                for (uint32_t j0 = 0; j0 < cnt; j0 += G1) {
                    uint32_t row[G1];
#pragma unroll
                    for (int q = 0; q < G1; ++q)
                        if (j0 + q < cnt) row[q] = ds_row_load(&D[(size_t)w_u[j0 + q] * 64 + lane]);
#pragma unroll
                    for (int q = 0; q < G1; ++q) {
                        const uint32_t e = j0 + q;
                        if (e >= cnt) break;
                        if (w_b[e] == SP_OWN) {
                            cur = (int)(w_w[e] & 63u);
                            const uint32_t t = w * 64 + cur;
                            dt = row[q];
                            const unsigned long long fin = __ballot(dt == DS_INF) | __ballot(my_src == t);
                            if (lane == 0) FM[t] = fin;
                            if (my_src == t) LO[(size_t)t * 64 + lane] = 0.0f;
                        } else {
                            const uint32_t r = row[q];
                            const bool tight =
                                r != DS_INF && dt != DS_INF && __builtin_elementwise_add_sat(r, w_w[e]) == dt;
                            const unsigned long long m = __ballot(tight);
                            if (m) {
                                const uint32_t pos = (uint32_t)__builtin_amdgcn_readlane((int)tcnt, cur);
                                if (lane == 0)
                                    TR[w_lo[cur] + pos] = make_uint4(w_u[e], w_b[e], (uint32_t)m, (uint32_t)(m >> 32));
                                tcnt += lane == (uint32_t)cur;
                            }
                        }
                    }
                }
            };
            uint32_t n = 0;
            for (uint32_t f0 = 0; f0 < total; f0 += 64) {
                const uint32_t f = f0 + lane;
                const bool act = f < total;
                const unsigned long long m = __ballot(act);
                if (act) {
                    const uint32_t i = ds_find(w_st, f);
                    const uint32_t slot = f - w_st[i];
                    const uint32_t pos = n + ds_mbcnt(m);
                    if (slot == 0) {
                        w_u[pos] = w * 64 + i;
                        w_w[pos] = i;
                        w_b[pos] = SP_OWN;
                    } else {
                        const uint32_t k = w_lo[i] + slot - 1;
                        w_u[pos] = a.in_src[k];
                        w_w[pos] = a.in_w[k];
                        w_b[pos] = __float_as_uint(a.in_b[k]);  // (b in [0, 1]: never SP_OWN's bits)
                    }
                }
                __builtin_amdgcn_wave_barrier();
                n += (uint32_t)__popcll(m);
                if (n > DS_CAP - 64) {
                    process(n);
                    __builtin_amdgcn_wave_barrier();
                    n = 0;
                    const uint32_t fn = f0 + 64;  // a vertex continuing past the chunk: its own row first
                    if (fn < total) {
                        const uint32_t i2 = ds_find(w_st, fn);
                        if (fn != w_st[i2]) {
                            if (lane == 0) {
                                w_u[0] = w * 64 + i2;
                                w_w[0] = i2;
                                w_b[0] = SP_OWN;
                            }
                            __builtin_amdgcn_wave_barrier();
                            n = 1;
                        }
                    }
                }
            }
            if (n) process(n);
            __builtin_amdgcn_wave_barrier();
            if (valid) TC[vl] = tcnt;
            vis_end(1);
        }
        // ================= phase 2b: loss fold in per-lane Kahn order =================
        __syncthreads();
        stamp(1);
        for (uint32_t w = threadIdx.x; w < nw; w += TH) {
            mark[w] = 0;
            mnext[w] = 0;
        }
        if (threadIdx.x == 0) s_nnext = 0;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        for (uint32_t q = wave; q < 64; q += WV) {
            const uint32_t sv = (uint32_t)__builtin_amdgcn_readlane((int)my_src, q);
            const uint32_t o0 = a.out_off[sv], o1 = a.out_off[sv + 1];
            for (uint32_t k0 = o0; k0 < o1; k0 += 64) {
                const bool on = k0 + lane < o1;
                mark_next(on ? a.out_dst[k0 + lane] : 0u, on);
            }
        }
        __syncthreads();
        rotate_marks();
        sync_lists();
        uint32_t sweeps2 = 0;
        for (;;) {
            if (threadIdx.x == 0) {
                s_changed = 0;
                s_take = 0;
            }
            __syncthreads();
            uint32_t chg = 0;
            const uint32_t ncur = s_ncur;
            for (uint32_t idx = take(&s_take); idx < ncur; idx = take(&s_take)) {
                vis_begin();
                const uint32_t w = wl_cur[idx];
                const unsigned long long mk = mark[w];
                const uint32_t vl = w * 64 + lane;
                const bool marked = (mk >> lane) & 1ull;
                unsigned long long fold_now = 0, nf = 0;
                if (marked) {
                    fold_now = __hip_atomic_load(&FM[vl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    nf = ~fold_now;  // reachable lanes not final yet (unreachable ones start final)
                }
                const uint32_t lo = nf ? a.in_off[vl] : 0u;
                const uint32_t tc = nf ? TC[vl] : 0u;
                // pass A: lanes blocked by a tight predecessor that is not final there
                uint32_t total;
                uint32_t st = ds_prefix(tc, lane, &total);
                w_st[lane] = st;
                w_lo[lane] = lo;
                blk[lane] = 0;
                __builtin_amdgcn_wave_barrier();
                for (uint32_t f0 = 0; f0 < total; f0 += 64) {
                    const uint32_t f = f0 + lane;
                    const bool on = f < total;
                    uint32_t i = 0, k = 0;
                    if (on) {
                        i = ds_find(w_st, f);
                        k = w_lo[i] + (f - w_st[i]);
                    }
                    const unsigned long long nfi = ds_shfl64(nf, i);
                    if (on) {
                        const uint4 rc = TR[k];
                        const unsigned long long m = (((unsigned long long)rc.w << 32) | rc.z) & nfi;
                        if (m) {
                            const unsigned long long fu =
                                __hip_atomic_load(&FM[rc.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            const unsigned long long b = m & ~fu;
                            if (b) atomicOr(&blk[i], b);
                        }
                    }
                }
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                const unsigned long long comp = nf & ~blk[lane];
                __builtin_amdgcn_wave_barrier();
                if (!__ballot(comp != 0)) {
                    vis_end(2);
                    continue;
                }
                // pass B: fold the tight arcs of the completed lanes
                st = ds_prefix(comp ? tc : 0u, lane, &total);
                w_st[lane] = st;
                __builtin_amdgcn_wave_barrier();
                int cur = -1;
                unsigned long long ccur = 0;
                float acc = __builtin_inff();
                auto flush = [&]() {
                    if (cur >= 0 && ((ccur >> lane) & 1ull)) LO[(size_t)(w * 64 + cur) * 64 + lane] = acc;
                };
                const unsigned long long* TRm = reinterpret_cast<const unsigned long long*>(TR);
                auto process = [&](uint32_t cnt) {
                    for (uint32_t j0 = 0; j0 < cnt; j0 += G2) {
                        float row[G2];
                        unsigned long long tq[G2];
#pragma unroll
                        for (int q = 0; q < G2; ++q)
                            if (j0 + q < cnt) {
                                row[q] = LO[(size_t)w_u[j0 + q] * 64 + lane];
                                tq[q] = TRm[2 * (size_t)w_b[j0 + q] + 1];  // the record's lane mask
                            }
#pragma unroll
                        for (int q = 0; q < G2; ++q) {
                            const uint32_t e = j0 + q;
                            if (e >= cnt) break;
                            const int ie = (int)w_i[e];
                            if (ie != cur) {
                                flush();
                                cur = ie;
                                ccur = ds_shfl64(comp, (uint32_t)ie);
                                acc = __builtin_inff();
                            }
                            if (((tq[q] & ccur) >> lane) & 1ull) {
                                const float c = fold_loss(row[q], __uint_as_float(w_w[e]));
                                acc = c < acc ? c : acc;
                            }
                        }
                    }
                    pulls2 += cnt;
                };
                uint32_t n = 0;
                for (uint32_t f0 = 0; f0 < total; f0 += 64) {
                    const uint32_t f = f0 + lane;
                    const bool on = f < total;
                    uint32_t i = 0, k = 0;
                    if (on) {
                        i = ds_find(w_st, f);
                        k = w_lo[i] + (f - w_st[i]);
                    }
                    const unsigned long long ci = ds_shfl64(comp, i);
                    uint4 rc = make_uint4(0u, 0u, 0u, 0u);
                    if (on) rc = TR[k];
                    const bool act = on && ((((unsigned long long)rc.w << 32) | rc.z) & ci) != 0ull;
                    const unsigned long long m = __ballot(act);
                    if (act) {
                        const uint32_t pos = n + ds_mbcnt(m);
                        w_u[pos] = rc.x;
                        w_w[pos] = rc.y;
                        w_b[pos] = k;
                        w_i[pos] = (unsigned char)i;
                    }
                    __builtin_amdgcn_wave_barrier();
                    n += (uint32_t)__popcll(m);
                    if (n > DS_CAP - 64) {
                        process(n);
                        n = 0;
                        __builtin_amdgcn_wave_barrier();
                    }
                }
                if (n) process(n);
                flush();
                // publish: the L stores of the completed lanes before their final bits
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (comp)
                    __hip_atomic_store(&FM[vl], fold_now | comp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                const unsigned long long done = __ballot(comp != 0);
                chg = 1;
                push_window(w, done);
                __builtin_amdgcn_wave_barrier();
                vis_end(2);
            }
            if (chg && lane == 0) s_changed = 1;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __syncthreads();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            ++sweeps2;
            const bool more = s_changed != 0;
            rotate_marks();
            sync_lists();
            if (!more) break;
        }
        max_sweeps2 = sweeps2 > max_sweeps2 ? sweeps2 : max_sweeps2;
        stamp(2);

        // ================= output rows: 64 targets x 64 sources tiles through LDS =================
        // D and L of a block of 64 used columns staged together ([64][65] u32 each), then every
        // wave writes its sources' row segments (latency u64 + loss f32)
        uint32_t bad = 0, imp = 0, incomplete = 0;
        uint32_t* tD = reinterpret_cast<uint32_t*>(tile);
        uint32_t* tL = tD + 64 * 65;
        for (uint32_t j0 = 0; j0 < a.ncols; j0 += 64) {
            uint32_t dv[4], lv[4];
            unsigned long long fm[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t j = j0 + wave + WV * q;
                dv[q] = 0;
                lv[q] = 0;
                fm[q] = ~0ull;
                if (j < a.ncols) {
                    const uint32_t t = a.cols[j];
                    dv[q] = D[(size_t)t * 64 + lane];
                    lv[q] = __float_as_uint(LO[(size_t)t * 64 + lane]);
                    fm[q] = FM[t];
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t i = wave + WV * q;
                tD[i * 65 + lane] = dv[q];
                tL[i * 65 + lane] = lv[q];
                // every reachable lane of a used column final, with a loss a tight arc gave it
                // (unreachable lanes hold no loss: the unreachable check reports them)
                incomplete |= (uint32_t)(dv[q] != DS_INF) & ((uint32_t)((~fm[q] >> lane) & 1ull) | (uint32_t)(lv[q] > 0x3F800000u));
            }
            __syncthreads();
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t sl = wave + WV * q;
                const uint32_t row = a.batch_row[bt * 64 + sl];
                const uint32_t j = j0 + lane;
                if (row == 0xFFFFFFFFu || j >= a.ncols) continue;
                const uint32_t l = tD[lane * 65 + sl];
                const size_t o = (size_t)row * a.ncols + j;
                const uint32_t s = a.batch_src[bt * 64 + sl];
                uint64_t ol;
                if (j == row) {  // diagonal: the raw self-loop weight (mod.rs:211-217)
                    ol = a.self_lat[s];
                } else {
                    bad |= l == DS_INF;
                    imp |= impossible_key<uint64_t>(l, a.min_key, false);
                    ol = (uint64_t)l * a.unit;
                }
                if (a.out_key) {
                    ds_out_store(&a.out_key[o], j == row ? 0xFFFFFFFFu : l);
                    if (j == row) a.out_diag[row] = ol;
                } else {
                    ds_out_store(&a.out_lat[o], ol);
                }
                ds_out_store(&a.out_loss[o], j == row ? a.self_loss[s] : __uint_as_float(tL[lane * 65 + sl]));
            }
            __syncthreads();
        }
        if (bad) atomicOr(&a.flags[0], 1u);
        if (imp) atomicOr(&a.flags[6], 1u);
        if (__ballot(incomplete) && lane == 0) atomicOr(&a.flags[7], 1u);
        if (lane == 0 && evals) atomicAdd(reinterpret_cast<unsigned long long*>(&a.flags[2]), (unsigned long long)evals);
        if (lane == 0 && pulls2) atomicAdd(reinterpret_cast<unsigned long long*>(&a.flags[10]), (unsigned long long)pulls2);
        evals = pulls2 = 0;
        stamp(3);
        if (a.dbg && threadIdx.x == 0) {
            a.dbg[bt * 6 + 4] = (uint32_t)tb0;
            a.dbg[bt * 6 + 5] = (uint32_t)(wall_clock64() - tb0);
        }
    }
    if (threadIdx.x < 4) atomicAdd(reinterpret_cast<unsigned long long*>(&a.flags[12 + 2 * threadIdx.x]), s_ph[threadIdx.x]);
    if (threadIdx.x < 3) atomicAdd(reinterpret_cast<unsigned long long*>(&a.flags[20 + 2 * threadIdx.x]), s_busy[threadIdx.x]);
    if (threadIdx.x == 0) {
        atomicMax(&a.flags[1], max_sweeps);
        atomicMax(&a.flags[8], max_sweeps2);
    }
    if (__ballot(saturated) && lane == 0) atomicOr(&a.flags[5], 1u);
}

}  // namespace srg
