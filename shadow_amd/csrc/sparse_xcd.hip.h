// sparse_xcd.hip.h — XCD-cooperative batched Bellman-Ford for sparse graphs (gfx950, round 5).
//
// Per used source the reference runs petgraph's Dijkstra with PathProperties scores
// (mod.rs:190-208, 305-331).  As in sparse.hip.h, the result is the unique lexicographic fixpoint
// label(t) = lexmin over in-arcs (u, t) of label(u) (+) arc with labels (latency << 32) | loss bits
// (u32 latency keys, one u64 min), reached here by pull-style Bellman-Ford sweeps with
// delta-stepping buckets; any order that reaches the fixpoint reproduces the reference bit for bit.
//
// What is different from k_sparse_bf (one 64-source batch per workgroup, 25.6 MB of labels per
// batch, 512 batches resident = every label row an HBM read: 1.25 TB of traffic per C4 launch):
//   * a batch is B = 8 sources and its labels [V][B] (V x 64 B: 3.2 MB at C4) live in ONE XCD's
//     4 MB L2; all workgroups on that XCD relax that batch together, so every label pull is an L2
//     hit and HBM sees only the CSR (from the Infinity Cache) and the output rows;
//   * the workgroups of an XCD find each other at run time: each reads its XCC id (hwreg
//     HW_REG_XCC_ID), registers with that XCD's group, and the group's first arrival closes the
//     registration after a short window -- late workgroups leave, so nothing ever waits for a
//     workgroup that is not running (no co-residency assumption, no cooperative launch).  Groups
//     claim batches from one queue, so an XCD with few (or no) workgroups just does fewer batches;
//   * one sweep = every participant's statically owned 64-vertex windows, then a group barrier
//     (one counter per group, arrivals by memory-side atomic add, polled with L1-bypassing loads).
//     Only the window's owner writes its vertices' labels and bitmap words (plain stores: the L2 is
//     the coherence point of the XCD); every cross-workgroup read is an sc1 (L1-bypassing) load;
//   * "changed" pushes are aggregated per workgroup in an LDS bitmap (ds_or) and published once
//     per sweep as that workgroup's slice; a window's mark word is the OR of the participants'
//     slices (one sc1 gather per window) -- the wavefront-aggregated bucket push: no global atomic
//     per pushed arc (1e10 of them at C4);
//   * within a window a wave relaxes 64 / B arcs per instruction (B lanes per label row), each
//     candidate folded into an LDS best[64][B] with ds_min_u64, then compared with the owner's old
//     label (kept in registers).
// Outputs (B rows x ncols per batch) are written write-through (sc1 stores drop the line from L2,
// so the 4.8 MB of rows per batch do not evict the label slice).  The wide (u64-key) labels and
// graphs whose bitmap does not fit LDS keep k_sparse_bf.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "guards.h"
#include "kernels.hip.h"
#include "sparse.hip.h"

namespace srg {

constexpr int SX_B = 8;                // sources per batch = lanes per label row (64-B rows)
constexpr int SX_WAVES = 16;           // waves per workgroup (one 1024-thread workgroup per CU)
constexpr int SX_THREADS = SX_WAVES * 64;
constexpr int SX_CAP = 128;            // active-arc list entries per wave
constexpr int SX_MAXG = 16;            // group slots (XCC ids 0..15)
constexpr int SX_MAXP = 64;            // participants per group
constexpr uint32_t SX_CLOSED = 0x80000000u;
constexpr unsigned long long SX_TMO = 400000000ull;  // 4 s of 100 MHz ticks: a bounded wait gives up

struct SxGroup {      // one per XCC id, zeroed before the launch
    uint32_t reg;     // registration: count | SX_CLOSED once the leader closed it
    uint32_t P;       // participants (the first P registrants), published by the leader
    uint32_t go;      // 1: P is published
    uint32_t bar;     // barrier arrivals (monotonic)
    uint32_t batch;   // the group's current batch (claimed by the leader before a barrier)
    uint32_t chg_seq;   // step + 1 of the last step in which a vertex changed and was pushed
    uint32_t pend_seq;  // step + 1 of the last step that left a deferred vertex
    uint32_t pad[57];
};
static_assert(sizeof(SxGroup) == 256, "group block");

struct SxArgs {
    const uint32_t* in_off;
    const uint32_t* in_src;
    const uint32_t* in_w;
    const float* in_b;
    const uint32_t* out_off;     // out-arcs (== the in-CSR for undirected graphs)
    const uint32_t* out_dst;
    uint32_t V;
    const uint32_t* batch_src;   // [nbatch * B] source vertex per lane slot
    const uint32_t* batch_row;   // [nbatch * B] output row (0xFFFFFFFF = padding)
    uint32_t nbatch;
    SxGroup* groups;             // [SX_MAXG]
    unsigned long long* labels;  // [SX_MAXG][V][B]
    unsigned long long* bits;    // [SX_MAXG][sx_bits_words(nw)]
    uint32_t* queue;             // next batch
    uint32_t* abort;             // raised by a wait that gave up: every participant leaves
    const uint32_t* cols;
    uint32_t ncols;
    const uint64_t* self_lat;
    const float* self_loss;
    uint64_t* out_lat;
    float* out_loss;
    uint32_t* flags;             // as SparseArgs: [0] unreachable pair, [1] max sweeps, [2..3] evaluations,
                                 // [5] saturated key, [6] impossible latency, [7] groups that ran
    uint64_t unit;
    uint64_t delta;
    uint32_t* out_key;
    uint64_t* out_diag;
    uint64_t min_key;
    uint32_t reg_ticks;          // registration window (100 MHz ticks)
};

// per-group bitmap words: chg[2][nw], pend[nw], pub[2][SX_MAXP][nw]
__host__ __device__ constexpr size_t sx_bits_words(uint32_t nw) { return (size_t)(3 + 2 * SX_MAXP) * nw; }

// LDS: the workgroup's push bitmap, then per wave: window prefix / offsets, the active-arc list,
// best[64][B]
template <int B>
__host__ __device__ constexpr size_t sx_wave_bytes() {
    return (size_t)2 * 64 * 4 + (size_t)4 * SX_CAP * 4 + (size_t)64 * B * 8;
}
template <int B>
__host__ __device__ constexpr size_t sx_lds_bytes(uint32_t nw) {
    return ((size_t)nw * 8 + 15) / 16 * 16 + (size_t)SX_WAVES * sx_wave_bytes<B>();
}

__device__ __forceinline__ unsigned long long sx_ld64(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1: bypasses L1
}
__device__ __forceinline__ uint32_t sx_ld32(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long wave_or64(unsigned long long x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x |= __shfl_xor(x, o, 64);
    return x;
}

template <int B>
__global__ void __launch_bounds__(SX_THREADS, 1) k_sparse_xcd(SxArgs a) {
    static_assert(B == 8 || B == 16, "label row = 8 or 16 sources");
    constexpr int NG = 64 / B;         // label rows per wave instruction (lane groups)
    constexpr int IT = 64 / NG;        // instructions per 64-vertex window
    constexpr uint64_t LAT_MAX = 0xFFFFFFFFull;
    using Lbl = unsigned long long;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    __shared__ uint32_t s_ok, s_rank, s_P, s_batch, s_chg_seq, s_pend_seq, s_chg, s_pend;
    const uint32_t V = a.V, nw = (V + 63) / 64;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t grp = lane / B, q = lane % B;
    unsigned long long* lmark = reinterpret_cast<unsigned long long*>(smem_raw);
    unsigned char* wb = smem_raw + ((size_t)nw * 8 + 15) / 16 * 16 + (size_t)wave * sx_wave_bytes<B>();
    uint32_t* w_st = reinterpret_cast<uint32_t*>(wb);
    uint32_t* w_lo = w_st + 64;
    uint32_t* w_u = w_lo + 64;
    uint32_t* w_w = w_u + SX_CAP;
    uint32_t* w_b = w_w + SX_CAP;
    uint32_t* w_t = w_b + SX_CAP;
    Lbl* best = reinterpret_cast<Lbl*>(w_t + SX_CAP);

    // ---- registration with this XCD's group ----
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (xcc >= (uint32_t)SX_MAXG) return;
    SxGroup* G = a.groups + xcc;
    if (threadIdx.x == 0) {
        const uint32_t old = __hip_atomic_fetch_add(&G->reg, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t ok = !(old & SX_CLOSED);
        const uint32_t rank = old & 0xFFFFu;
        uint32_t P = 0;
        if (ok && rank == 0) {  // the leader: a short window for the others, then close
            const unsigned long long t0 = wall_clock64();
            while (wall_clock64() - t0 < a.reg_ticks) __builtin_amdgcn_s_sleep(2);
            const uint32_t cnt = __hip_atomic_fetch_or(&G->reg, SX_CLOSED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            P = min(cnt & 0xFFFFu, (uint32_t)SX_MAXP);
            __hip_atomic_store(&G->P, P, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // the first batch, claimed before the first barrier (every participant reads it there)
            const uint32_t b = atomicAdd(a.queue, 1u);
            __hip_atomic_store(&G->batch, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(&G->go, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            atomicAdd(&a.flags[7], 1u);
        } else if (ok) {
            const unsigned long long t0 = wall_clock64();
            while (!sx_ld32(&G->go)) {
                if (wall_clock64() - t0 > SX_TMO || sx_ld32(a.abort)) {
                    __hip_atomic_store(a.abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            if (ok) P = sx_ld32(&G->P);
        }
        s_ok = ok && rank < P;
        s_rank = rank;
        s_P = P;
    }
    __syncthreads();
    if (!s_ok) return;
    const uint32_t rank = s_rank, P = s_P;
    const uint32_t gw = rank * SX_WAVES + wave, NWT = P * SX_WAVES;  // this wave, all participant waves
    Lbl* L = a.labels + (size_t)xcc * V * B;
    unsigned long long* bits = a.bits + (size_t)xcc * sx_bits_words(nw);
    unsigned long long* chgb[2] = {bits, bits + nw};
    unsigned long long* pend = bits + 2 * (size_t)nw;
    unsigned long long* pub = bits + 3 * (size_t)nw;  // [2][SX_MAXP][nw]
    auto pubp = [&](int p, uint32_t r) { return pub + ((size_t)p * SX_MAXP + r) * nw; };

    uint32_t nbar = 0;
    unsigned long long t_wait = 0, t_work0 = wall_clock64();  // SRG_DEBUG_SPARSE: barrier wait vs all
    // group barrier: every storing wave's stores have reached the L2 before the arrival; returns
    // false when the wait gave up (abort)
    auto bar = [&]() -> bool {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        ++nbar;
        if (threadIdx.x == 0) {
            __hip_atomic_fetch_add(&G->bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t target = nbar * P;
            uint32_t ok = 1;
            const unsigned long long t0 = wall_clock64();
            while ((int)(sx_ld32(&G->bar) - target) < 0) {
                if (wall_clock64() - t0 > SX_TMO || sx_ld32(a.abort)) {
                    __hip_atomic_store(a.abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            t_wait += wall_clock64() - t0;
            s_ok = ok;
            s_batch = sx_ld32(&G->batch);
            s_chg_seq = sx_ld32(&G->chg_seq);
            s_pend_seq = sx_ld32(&G->pend_seq);
        }
        __syncthreads();
        return s_ok != 0;
    };
    // publish this workgroup's push bitmap as its slice of pub[p] (and clear it)
    auto publish = [&](int p) {
        __syncthreads();
        unsigned long long* dst = pubp(p, rank);
        for (uint32_t i = threadIdx.x; i < nw; i += SX_THREADS) {
            dst[i] = lmark[i];
            lmark[i] = 0;
        }
    };
    // mark the out-neighbours of the vertices in `vm` (window w) in the LDS push bitmap (one wave)
    auto push_window = [&](uint32_t w, unsigned long long vm) {
        const uint32_t vl = w * 64 + lane;
        const bool ch = (vm >> lane) & 1ull;
        const uint32_t olo = ch ? a.out_off[vl] : 0u, ohi = ch ? a.out_off[vl + 1] : 0u;
        const uint32_t odeg = ohi - olo;
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
                    if (i + step < 64 && w_st[i + step] <= f) i += step;
                const uint32_t t = a.out_dst[w_lo[i] + (f - w_st[i])];
                __hip_atomic_fetch_or(&lmark[t >> 6], 1ull << (t & 63), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        __builtin_amdgcn_wave_barrier();
    };

    uint32_t max_sweeps = 0, saturated = 0, bad = 0, imp = 0;
    unsigned long long evals = 0;
    for (uint32_t i = threadIdx.x; i < nw; i += SX_THREADS) lmark[i] = 0;
    if (!bar()) return;
    uint32_t gs = 0;  // group step counter (every participant counts the same steps)
    for (;;) {
        const uint32_t bt = s_batch;
        if (bt >= a.nbatch) break;
        const uint32_t src_q = a.batch_src[bt * B + q];  // this lane's source
        // ---- init: labels, change bits and pending bits of the owned windows ----
        for (uint32_t w = gw; w < nw; w += NWT) {
#pragma unroll
            for (int it = 0; it < IT; ++it) {
                const uint32_t v = w * 64 + it * NG + grp;
                if (v < V) L[(size_t)v * B + q] = v == src_q ? 0ull : LBL_INF;
            }
            // the batch's sources in this window: "changed in the step before the first"
            const bool in = lane < (uint32_t)B && (src_q >> 6) == w;
            unsigned long long m = __ballot(in), sb = 0;
            while (m) {
                const int l = __builtin_ctzll(m);
                m &= m - 1;
                sb |= 1ull << (__builtin_amdgcn_readlane((int)src_q, l) & 63);
            }
            if (lane == 0) {
                chgb[(gs + 1) & 1][w] = sb;
                chgb[gs & 1][w] = 0;
                pend[w] = 0;
            }
        }
        // the sources' out-neighbours: the marks of the first step
        for (uint32_t qq = rank; qq < (uint32_t)B; qq += P) {
            const uint32_t s = a.batch_src[bt * B + qq];
            const uint32_t o0 = a.out_off[s], o1 = a.out_off[s + 1];
            for (uint32_t k = o0 + threadIdx.x; k < o1; k += SX_THREADS) {
                const uint32_t t = a.out_dst[k];
                __hip_atomic_fetch_or(&lmark[t >> 6], 1ull << (t & 63), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        publish(gs & 1);
        if (!bar()) return;
        uint64_t bound = a.delta >= LAT_MAX ? LAT_MAX : a.delta;
        uint32_t last_rel = gs, sweeps = 0;  // pending exists iff pend_seq > last_rel
        for (;;) {
            const int p = gs & 1;
            const unsigned long long* chg_prev = chgb[p ^ 1];
            if (threadIdx.x == 0) s_chg = s_pend = 0;
            __syncthreads();
            for (uint32_t w = gw; w < nw; w += NWT) {
                // marks: the OR of the participants' slices
                unsigned long long mk = lane < P ? sx_ld64(pubp(p, lane) + w) : 0ull;
                mk = wave_or64(mk);
                if (w == nw - 1 && (V & 63)) mk &= (1ull << (V & 63)) - 1;
                if (!mk) {
                    if (lane == 0) chgb[p][w] = 0;
                    continue;
                }
                // (1) offsets of the marked vertices, prefix over the window
                const uint32_t vl = w * 64 + lane;
                const bool marked = (mk >> lane) & 1ull;
                const uint32_t lo = marked ? a.in_off[vl] : 0u, hi = marked ? a.in_off[vl + 1] : 0u;
                const uint32_t deg = hi - lo;
                uint32_t incl = deg;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t t = __shfl_up(incl, o, 64);
                    if ((int)lane >= o) incl += t;
                }
                const uint32_t total = (uint32_t)__shfl(incl, 63, 64);
                w_st[lane] = incl - deg;
                w_lo[lane] = lo;
                // (2) the owner's labels: old (registers), best (LDS)
                Lbl old[IT];
#pragma unroll
                for (int it = 0; it < IT; ++it) {
                    const uint32_t v = it * NG + grp;
                    old[it] = LBL_INF;
                    if ((mk >> v) & 1ull) {
                        old[it] = sx_ld64(L + (size_t)(w * 64 + v) * B + q);
                        best[v * B + q] = old[it];
                    }
                }
                __builtin_amdgcn_wave_barrier();
                // (3) the marked vertices' in-arcs whose source changed in the previous step ->
                //     list; (4) relax the list, B lanes per label row, into best with ds_min
                auto process = [&](uint32_t cnt) {
                    constexpr int U = 4;
                    for (uint32_t e0 = 0; e0 < cnt; e0 += NG * U) {
                        Lbl row[U];
                        uint32_t tt[U], ww[U], bb[U];
#pragma unroll
                        for (int uu = 0; uu < U; ++uu) {
                            const uint32_t e = e0 + uu * NG + grp;
                            row[uu] = LBL_INF;
                            tt[uu] = 0xFFFFFFFFu;
                            if (e < cnt) {
                                const uint32_t u = w_u[e];
                                ww[uu] = w_w[e];
                                bb[uu] = w_b[e];
                                tt[uu] = w_t[e];
                                row[uu] = sx_ld64(L + (size_t)u * B + q);
                            }
                        }
#pragma unroll
                        for (int uu = 0; uu < U; ++uu) {
                            if (tt[uu] == 0xFFFFFFFFu) continue;
                            const bool rinf = row[uu] == LBL_INF;
                            const Lbl c = rinf ? LBL_INF : lbl_relax(row[uu], ww[uu], __uint_as_float(bb[uu]));
                            saturated |= (c == LBL_INF) & !rinf;
                            __hip_atomic_fetch_min(&best[tt[uu] * B + q], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            ++evals;
                        }
                    }
                    __builtin_amdgcn_wave_barrier();
                };
                uint32_t n = 0;
                for (uint32_t f0 = 0; f0 < total; f0 += 64) {
                    const uint32_t f = f0 + lane;
                    bool act = false;
                    uint32_t u = 0, k = 0, i = 0;
                    if (f < total) {
#pragma unroll
                        for (uint32_t step = 32; step; step >>= 1)
                            if (i + step < 64 && w_st[i + step] <= f) i += step;
                        k = w_lo[i] + (f - w_st[i]);
                        u = a.in_src[k];
                        act = (sx_ld64(chg_prev + (u >> 6)) >> (u & 63)) & 1ull;
                    }
                    const unsigned long long m = __ballot(act);
                    if (act) {
                        const uint32_t pos = n + (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                        w_u[pos] = u;
                        w_w[pos] = a.in_w[k];
                        w_b[pos] = __float_as_uint(a.in_b[k]);
                        w_t[pos] = i;
                    }
                    __builtin_amdgcn_wave_barrier();
                    n += (uint32_t)__popcll(m);
                    if (n > SX_CAP - 64) {
                        process(n);
                        n = 0;
                    }
                }
                if (n) process(n);
                __builtin_amdgcn_wave_barrier();
                // (5) compare with the old labels: store the dropped ones; a vertex is pushed now if
                //     some dropped lane's new latency is below the bucket bound, else deferred
                unsigned long long changed = 0, deferred = 0;
#pragma unroll
                for (int it = 0; it < IT; ++it) {
                    const uint32_t v = it * NG + grp;
                    const bool vm = (mk >> v) & 1ull;
                    const Lbl nb = vm ? best[v * B + q] : LBL_INF;
                    const bool dr = vm && nb < old[it];
                    if (dr) L[(size_t)(w * 64 + v) * B + q] = nb;
                    const unsigned long long mdr = __ballot(dr), mbd = __ballot(dr && (nb >> 32) < bound);
                    constexpr unsigned long long gmask = B == 64 ? ~0ull : ((1ull << B) - 1);
#pragma unroll
                    for (int g = 0; g < NG; ++g) {
                        if ((mdr >> (g * B)) & gmask) {
                            const unsigned long long vb = 1ull << (it * NG + g);
                            if ((mbd >> (g * B)) & gmask) changed |= vb;
                            else deferred |= vb;
                        }
                    }
                }
                if (lane == 0) {
                    chgb[p][w] = changed;
                    if (changed | deferred) {
                        const unsigned long long pn = (pend[w] | deferred) & ~changed;
                        pend[w] = pn;
                        if (pn) s_pend = 1;
                    }
                    if (changed) s_chg = 1;
                }
                if (changed) push_window(w, changed);
            }
            publish(p ^ 1);
            if (threadIdx.x == 0) {
                if (s_chg) __hip_atomic_fetch_max(&G->chg_seq, gs + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (s_pend) __hip_atomic_fetch_max(&G->pend_seq, gs + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (!bar()) return;
            ++gs;
            ++sweeps;
            if (s_chg_seq >= gs) continue;  // a vertex changed in the step just done
            if (s_pend_seq <= last_rel) break;  // converged: nothing changed, nothing deferred
            // bucket exhausted: release every deferred vertex as if it had just changed (a step of
            // its own: pend -> the step's change bits, their out-neighbours -> the next marks)
            bound = (a.delta >= LAT_MAX || bound > LAT_MAX - a.delta) ? LAT_MAX : bound + a.delta;
            const int pr = gs & 1;
            for (uint32_t w = gw; w < nw; w += NWT) {
                const unsigned long long pb = lane == 0 ? pend[w] : 0ull;
                const unsigned long long bits_w = __shfl(pb, 0, 64);
                if (lane == 0) {
                    chgb[pr][w] = bits_w;
                    pend[w] = 0;
                }
                if (bits_w) push_window(w, bits_w);
            }
            publish(pr ^ 1);
            if (!bar()) return;
            ++gs;
            last_rel = gs;
        }
        max_sweeps = sweeps > max_sweeps ? sweeps : max_sweeps;
        // ---- output rows: B rows x ncols, write-through (the label slice stays in L2) ----
        for (uint32_t c0 = gw * 64; c0 < a.ncols; c0 += NWT * 64) {
            const uint32_t j = c0 + lane;
            const bool in = j < a.ncols;
            const uint32_t v = in ? a.cols[j] : 0u;
            Lbl lab[B];
#pragma unroll
            for (int qq = 0; qq < B; ++qq) lab[qq] = in ? sx_ld64(L + (size_t)v * B + qq) : 0ull;
#pragma unroll
            for (int qq = 0; qq < B; ++qq) {
                const uint32_t row = a.batch_row[bt * B + qq];
                if (row == 0xFFFFFFFFu || !in) continue;
                const size_t o = (size_t)row * a.ncols + j;
                const uint32_t s = a.batch_src[bt * B + qq];
                uint64_t ol;
                float ls;
                if (j == row) {  // diagonal: the raw self-loop weight (mod.rs:211-217)
                    ol = a.self_lat[s];
                    ls = a.self_loss[s];
                } else {
                    const uint64_t lat = lab[qq] >> 32;
                    bad |= lat == LAT_MAX;
                    imp |= impossible_key<uint64_t>(lat, a.min_key, false);
                    ol = lat * a.unit;
                    ls = __uint_as_float((uint32_t)lab[qq]);
                }
                if (a.out_key) {
                    __hip_atomic_store(a.out_key + o, j == row ? 0xFFFFFFFFu : (uint32_t)(lab[qq] >> 32), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                    if (j == row) a.out_diag[row] = ol;
                } else {
                    __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.out_lat) + o, (unsigned long long)ol,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                __hip_atomic_store(reinterpret_cast<uint32_t*>(a.out_loss) + o, __float_as_uint(ls), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        // the next batch (claimed by the leader before the barrier that ends this one)
        if (rank == 0 && threadIdx.x == 0)
            __hip_atomic_store(&G->batch, atomicAdd(a.queue, 1u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!bar()) return;
    }
    if (threadIdx.x == 0) {
        atomicMax(&a.flags[1], max_sweeps);
        atomicAdd(reinterpret_cast<unsigned long long*>(&a.flags[8]), t_wait);
        atomicAdd(reinterpret_cast<unsigned long long*>(&a.flags[10]), wall_clock64() - t_work0);
        atomicAdd(&a.flags[12], nbar);
    }
    if (__ballot(saturated) && lane == 0) atomicOr(&a.flags[5], 1u);
    if (__ballot(bad) && lane == 0) atomicOr(&a.flags[0], 1u);
    if (__ballot(imp) && lane == 0) atomicOr(&a.flags[6], 1u);
    unsigned long long ev = evals;
    for (int o = 32; o > 0; o >>= 1) ev += __shfl_xor(ev, o, 64);
    if (lane == 0 && ev) atomicAdd(reinterpret_cast<unsigned long long*>(&a.flags[2]), ev);
}

}  // namespace srg
