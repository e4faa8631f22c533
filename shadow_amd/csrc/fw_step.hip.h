// fw_step.hip.h — the symmetric line-buffer FW as ONE launch per pivot (gfx950).
//
// routing.hip fw_line_sym runs pivot kb's bulk on the main stream and the next pivot's chain (line
// k1 = kb + 1 w.r.t. kb, exchange, closure of the pivot tile, line k1 w.r.t. k1) as four launches
// on a second stream, with two cross-stream hops per pivot.  At 8 ranks that chain is the FW's
// critical path: 79 x ~90 us of dependent launches, modelled collectives and hops against a
// ~56-us bulk (profiles/r03c/chain_trace_sim8_0.txt).  Here both are one launch on one stream:
//   * workgroups [0, CH) run the chain of k1 as phases inside the launch,
//       A  this rank's tiles of line k1 w.r.t. kb (sub-tiles) -> D, LB(k1), and every peer's LB(k1)
//       X  exchange: arrival counter; workgroup 0 waits for the peers' segments (device flags
//          raised by their phase A, or the modelled link time of a simulated rank) and says "go"
//       C  the closure of the pivot tile inside LB(k1) (repeated squaring, grid barriers among the
//          first (T/16)^2 chain workgroups), then "closure done"
//       D  line k1 w.r.t. its closed pivot, every tile (sub-tiles), own tiles back to D
//   * workgroups [CH, CH + bulk items) run pivot kb's bulk (whole tiles or quadrants).
// The chain of k1 needs LB(kb) final and the bulk of kb - 1 done (line k1's tiles current through
// kb - 1): both are the previous launch, so stream order is the only dependency left -- no hops.
// Chain workgroups are dispatched first (lowest block ids) and are few, so they are co-resident;
// bulk workgroups wait on nothing, so every spin inside the launch ends.
//
// Hand-offs inside the launch follow MI355X_MICROARCH.md's write-through form: line-buffer bytes
// produced in phase A / C are stored sc1 (16-B or 8-B vector stores) and drained
// (s_waitcnt vmcnt(0)) before the arrival counter / flag; readers poll, then acquire (agent scope,
// system scope when peers are on other devices) before plain loads.  Line buffers are used
// round-robin over three (peers may run one pivot ahead of a slow rank, never two: their phase X
// waits for this rank's segment of the pivot before).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.hip.h"

namespace srg {

constexpr int kMaxPeers = 16;

// sync words of one pivot (16 u32, zeroed per build): closure barrier + changed flags, arrivals,
// go, closure done
enum StepSync { SS_CLOSE = 0, SS_ARRIVE = 9, SS_GO = 10, SS_CDONE = 11, SS_DNEXT = 12 };

template <class K>
struct StepArgs {
    K* D;
    size_t ld;
    const K* lbk;       // LB(kb): final (previous launch)
    K* lbn;             // LB(k1): built by this launch's chain
    int kb, k1;         // k1 < 0: the last pivot, bulk only
    LineMap lm;
    int g;              // this rank
    const int* tiles;   // this rank's stored tiles (triangle indices)
    int ntile;
    int CH;             // chain workgroups
    uint32_t* sync;     // this pivot's 16 sync words
    uint32_t* timeout;  // raised by any bounded wait that gave up (host: SRG_ERR_HIP)
    int xmode;          // 0 = no exchange (one rank), 1 = modelled link time, 2 = device flags
    uint32_t model_ns;  // xmode 1: the modelled exchange time
    int sys;            // xmode 2: peers on other devices (system-scope fences and stores)
    uint32_t epoch;     // xmode 2: this build's flag value
    uint32_t* myflags;  // xmode 2: [pivot * G + from] arrival words that peers raise here
    unsigned long long* trace;  // SRG_FW_TRACE: 8 wall-clock stamps of this launch (null = off), see TraceAt
    K* peer_lbn[kMaxPeers];          // xmode 2: each peer's LB(k1) (null for this rank)
    uint32_t* peer_flags[kMaxPeers]; // xmode 2: each peer's arrival words
};

// trace stamps (wall_clock64, 100 MHz) of one launch: first workgroup start, all phase-A arrivals
// seen, go, closure done, last chain workgroup done, last bulk workgroup done
enum TraceAt { TR_START = 0, TR_ARRIVED = 1, TR_GO = 2, TR_CDONE = 3, TR_CHAIN_END = 4, TR_BULK_END = 5 };
__device__ __forceinline__ void trace_min(unsigned long long* t, int at) {
    if (t && threadIdx.x == 0) atomicMin(t + at, wall_clock64());
}
__device__ __forceinline__ void trace_max(unsigned long long* t, int at) {
    if (t && threadIdx.x == 0) atomicMax(t + at, wall_clock64());
}

// bounded poll of *p until pred(value) (one lane); false after ~2 s (raises *timeout)
template <class Pred>
__device__ __forceinline__ bool poll_until(const uint32_t* p, int sys, uint32_t* timeout, Pred pred) {
    const unsigned long long t0 = wall_clock64();
    for (;;) {
        const uint32_t v = sys ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                               : __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (pred(v)) return true;
        if (wall_clock64() - t0 > 200000000ull || __hip_atomic_load(timeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            __hip_atomic_store(timeout, 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

__device__ __forceinline__ void acquire_for(int sys) {
    if (sys) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// 8 bytes at p, write-through: agent scope (sc1) or system scope (sc0 sc1)
__device__ __forceinline__ void st8_wt(void* p, uint64_t v, int sys) {
    if (sys) __hip_atomic_store(reinterpret_cast<uint64_t*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else __hip_atomic_store(reinterpret_cast<uint64_t*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One (T/S) x (T/S) sub-tile q of line tile j: mode 0 = line K1 w.r.t. L (C read from the D tile, the
// result to LB(K1) and the peers' LB(K1) only, write-through), mode 1 = line K1 w.r.t. its closed
// pivot (C = LB(K1) tile in place, own tiles back to D).  fw_line_lb's work item (kernels.hip.h),
// except that mode 0 does not write D: phase D writes the same D sub-tile later in the SAME launch,
// from another workgroup, maybe on another XCD, and two plain stores of one line dirty in two XCD
// L2s are written back in no particular order at the launch's end -- the stale phase-A value won
// (measured: in-process ranks at line split 2 lost up to 5 % of their latencies).  Mode 1 is the
// only D writer of a line tile.
template <class K, int T, int S>
__device__ __forceinline__ void line_item(const StepArgs<K>& a, int mode, int j, int q) {
    static_assert(S >= 2, "quadrant or smaller line items (a whole-tile line core beside the bulk's spills)");
    constexpr bool PEERS = true;
    constexpr int TM = T / S;
    constexpr int KCL = line_kc<S>();
    constexpr size_t TT = (size_t)T * T;
    const int L = a.kb, K1 = a.k1;
    const LineMap& lm = a.lm;
    const int qi = q / S, qj = q % S;
    const int I = min(j, K1), J = max(j, K1);
    const bool own = lm.owner(j, K1) == a.g;
    const size_t slot = (size_t)lm.slot(j, K1) * TT;
    K* Dt = a.D + (size_t)I * T * a.ld + (size_t)J * T + (size_t)qi * TM * a.ld + qj * TM;
    K* Lt = a.lbn + slot + (size_t)qi * TM * T + qj * TM;
    const int npeer = PEERS && a.xmode == 2 ? a.lm.G : 0;
    // mode 0 results go to LB(k1) here and at every peer, write-through (read in this launch)
    auto out_lb = [&](int r, int c, uint64_t bits) {
        const size_t off = ((size_t)r * T + c) * sizeof(K);
        st8_wt(reinterpret_cast<unsigned char*>(Lt) + off, bits, 0);
        if constexpr (PEERS)
            for (int p = 0; p < npeer; ++p)
            if (a.peer_lbn[p])
                st8_wt(reinterpret_cast<unsigned char*>(a.peer_lbn[p] + slot + (size_t)qi * TM * T + qj * TM) + off,
                       bits, a.sys);
    };
    if (mode == 1 && j == K1) {  // the closed pivot tile: back to D on its owner
        if (own) {
            constexpr int VE = 16 / (int)sizeof(K);
            for (int e = threadIdx.x; e < TM * TM / VE; e += 256) {
                const int r = e / (TM / VE), cv = e % (TM / VE);
                st16(Dt + (size_t)r * a.ld + cv * VE, ld16(Lt + (size_t)r * T + cv * VE));
            }
        }
        return;
    }
    if (mode == 0 && j == L) {  // the final tile (L, K1) of line L: copied into LB(K1)
        const K* src = a.lbk + (size_t)lm.slot(K1, L) * TT + (size_t)qi * TM * T + qj * TM;
        for (int e = threadIdx.x; e < TM * TM / 2 * (int)sizeof(K) / 4; e += 256) {
            // 8-byte pieces
            const int per_row = TM * (int)sizeof(K) / 8;
            const int r = e / per_row, cb = e % per_row;
            const uint64_t v = *reinterpret_cast<const uint64_t*>(reinterpret_cast<const unsigned char*>(src + (size_t)r * T) + cb * 8);
            out_lb(r, cb * 8 / (int)sizeof(K), v);
        }
        return;
    }
    const K* lb = mode == 0 ? a.lbk : a.lbn;
    const int P = mode == 0 ? L : K1;
    const bool acol = I > P, bcol = J >= P;
    const K* Ab = lb + lm.slot(I, P) * TT + (acol ? (size_t)qi * TM : (size_t)qi * TM * T);
    const K* Bb = lb + lm.slot(J, P) * TT + (bcol ? (size_t)qj * TM : (size_t)qj * TM * T);
    if (mode == 0) {
        fw_core_e<K, TM, T, KCL, false>(Dt, a.ld, Ab, acol, Bb, bcol, T, out_lb);
    } else {
        K* Dd = own ? Dt : nullptr;
        fw_core_e<K, TM, T, KCL>(Lt, T, Ab, acol, Bb, bcol, T, [&](int r, int c, uint64_t bits) {
            if (Dd) *reinterpret_cast<uint64_t*>(Dd + (size_t)r * a.ld + c) = bits;
        });
    }
}

// arrival after a phase: every wave drains its stores, then one lane adds to the counter
__device__ __forceinline__ void arrive(uint32_t* cnt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// all threads of the workgroup wait until lane 0 saw *p satisfy pred, then acquire
template <class Pred>
__device__ __forceinline__ void wg_wait(const uint32_t* p, int sys, uint32_t* timeout, Pred pred) {
    if (threadIdx.x == 0) (void)poll_until(p, 0, timeout, pred);
    __syncthreads();
    acquire_for(sys);
    __syncthreads();
}

template <class K, int T, int SL>
__device__ __forceinline__ void help_d(const StepArgs<K>& a);

template <class K, int T, int SL>
__device__ __forceinline__ void chain(const StepArgs<K>& a, int w) {
    const LineMap& lm = a.lm;
    const int CH = a.CH, G = lm.G;
    uint32_t* sy = a.sync;
    constexpr int SS = SL * SL;
    // ---- A: own tiles of line k1 w.r.t. kb -------------------------------------------------
    const int nA = lm.count(a.g, a.k1) * SS;
    const int j0 = lm.j0(a.g, a.k1);
    for (int i = w; i < nA; i += CH) {
        line_item<K, T, SL>(a, 0, j0 + G * (i / SS), i % SS);
        __syncthreads();  // the LDS image is reused by the next item
    }
    arrive(&sy[SS_ARRIVE]);
    // ---- X: exchange (workgroup 0), then "go" -------------------------------------------------
    if (w == 0) {
        if (threadIdx.x == 0) {
            const uint32_t ch = (uint32_t)CH;
            if (poll_until(&sy[SS_ARRIVE], 0, a.timeout, [ch](uint32_t v) { return v >= ch; })) {
                if (a.trace) a.trace[TR_ARRIVED] = wall_clock64();
                if (a.xmode == 1) {
                    const unsigned long long t0 = wall_clock64(), ticks = a.model_ns / 10;  // 100 MHz
                    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
                } else if (a.xmode == 2) {
                    // every storing wave of this rank drained its peer stores before arriving; make
                    // them visible beyond this XCD / device, then raise this rank's flag at every peer
                    if (a.sys) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                    else __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    for (int p = 0; p < G; ++p)
                        if (a.peer_flags[p]) {
                            uint32_t* f = a.peer_flags[p] + (size_t)a.k1 * G + a.g;
                            if (a.sys) __hip_atomic_store(f, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                            else __hip_atomic_store(f, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        }
                    const uint32_t ep = a.epoch;
                    for (int p = 0; p < G; ++p)
                        if (p != a.g && !poll_until(a.myflags + (size_t)a.k1 * G + p, a.sys, a.timeout,
                                                    [ep](uint32_t v) { return v == ep; }))
                            break;
                    acquire_for(a.sys);
                }
            }
            if (a.trace) a.trace[TR_GO] = wall_clock64();
            __hip_atomic_store(&sy[SS_GO], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
    }
    // ---- C: closure of the pivot tile (first (T/16)^2 chain workgroups) ------------------------
    constexpr int NB16 = T / 16;
    constexpr int NC = NB16 * NB16;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    if (w < NC) {
        wg_wait(&sy[SS_GO], a.sys, a.timeout, [](uint32_t v) { return v != 0; });
        K(*A)[T + 1] = reinterpret_cast<K(*)[T + 1]>(smem_raw);
        K(*B)[17] = reinterpret_cast<K(*)[17]>(smem_raw + sizeof(K) * 16 * (T + 1));
        uint32_t* sh = reinterpret_cast<uint32_t*>(smem_raw + sizeof(K) * (16 * (T + 1) + T * 17));
        close_body<K, T>(a.lbn + (size_t)lm.slot(a.k1, a.k1) * T * T, sy + SS_CLOSE, a.timeout, w / NB16, w % NB16,
                         (uint32_t)NC, A, B, sh);
        __syncthreads();
        if (w == 0 && threadIdx.x == 0) {
            if (a.trace) a.trace[TR_CDONE] = wall_clock64();
            __hip_atomic_store(&sy[SS_CDONE], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        acquire_for(0);
        __syncthreads();
    } else {
        wg_wait(&sy[SS_CDONE], 0, a.timeout, [](uint32_t v) { return v != 0; });
    }
    // ---- D: the whole line w.r.t. its closed pivot (shared with bulk workgroups that are free) ----
    help_d<K, T, SL>(a);
    trace_max(a.trace, TR_CHAIN_END);
}

// Phase D's items are dealt from a counter: the chain workgroups take them once the pivot is closed,
// and so does every bulk workgroup that finds the closure done when its own tile is finished -- the
// line w.r.t. its closed pivot is the launch's critical path, the bulk is not.
template <class K, int T, int SL>
__device__ __forceinline__ void help_d(const StepArgs<K>& a) {
    constexpr int SS = SL * SL;
    __shared__ int s_item;
    const int nD = a.lm.nb * SS;
    for (;;) {
        if (threadIdx.x == 0) s_item = (int)__hip_atomic_fetch_add(&a.sync[SS_DNEXT], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        const int i = s_item;
        __syncthreads();
        if (i >= nD) break;
        line_item<K, T, SL>(a, 1, i / SS, i % SS);
        __syncthreads();  // the LDS image is reused by the next item
    }
}

// bulk item: this rank's stored tile (sub-tile q of SB x SB) off lines kb and k1, operands LB(kb)
template <class K, int T, int SB>
__device__ __forceinline__ void bulk_item(const StepArgs<K>& a, int b) {
    constexpr int TM = T / SB;
    constexpr int KCB = SB == 1 ? 16 : 32;
    constexpr size_t TT = (size_t)T * T;
    const int t = b / (SB * SB), q = b % (SB * SB), qi = q / SB, qj = q % SB;
    int I, J;
    tri_tile(a.lm.nb, a.tiles[t], I, J);
    if (I == a.kb || J == a.kb || I == a.k1 || J == a.k1) return;
    const int L = a.kb;
    const bool acol = I > L, bcol = J >= L;
    const K* Ab = a.lbk + a.lm.slot(I, L) * TT + (acol ? (size_t)qi * TM : (size_t)qi * TM * T);
    const K* Bb = a.lbk + a.lm.slot(J, L) * TT + (bcol ? (size_t)qj * TM : (size_t)qj * TM * T);
    K* C = a.D + (size_t)I * T * a.ld + (size_t)J * T + (size_t)qi * TM * a.ld + qj * TM;
    fw_core_e<K, TM, T, KCB>(C, a.ld, Ab, acol, Bb, bcol, T, [](int, int, uint64_t) {});
}

template <class K, int T, int SB, int SL>
constexpr size_t step_lds() {
    constexpr size_t bulk = lb_lds<K, T / SB, SB == 1 ? 16 : 32>();
    constexpr size_t line = lb_lds<K, T / SL, line_kc<SL>()>();
    constexpr size_t close = sizeof(K) * (16 * (T + 1) + T * 17) + 16;
    constexpr size_t m = bulk > line ? bulk : line;
    return m > close ? m : close;
}

template <class K, int T, int SB, int SL>
__global__ void __launch_bounds__(256, SB == 1 ? 3 : 4) fw_step(StepArgs<K> a) {
    const int w = (int)blockIdx.x;
    trace_min(a.trace, TR_START);
    if (w >= a.CH) {
        bulk_item<K, T, SB>(a, w - a.CH);
        trace_max(a.trace, TR_BULK_END);
        // free now: help with the chain's last phase if the pivot is already closed
        if (a.k1 >= 0) {
            __shared__ uint32_t s_cd;
            if (threadIdx.x == 0) s_cd = __hip_atomic_load(&a.sync[SS_CDONE], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __syncthreads();
            if (s_cd) {
                acquire_for(a.sys);
                __syncthreads();
                help_d<K, T, SL>(a);
            }
        }
        return;
    }
    __builtin_amdgcn_s_setprio(3);  // the chain is the launch's critical path
    chain<K, T, SL>(a, w);
}

// ---- the two-stream chain's device-side exchange (routing.hip SymFw, xmode 1 / 2) ----------------
// In place of the allgather of LB(k1) on the chain's stream: xmode 2 -- the workgroups copy this
// rank's segment of LB(k1) (just written by the line launch before it) into every peer's LB(k1) with
// write-through stores, drain, and the last one to arrive raises this rank's word at every peer, then
// waits for every peer's word (their segments are in this rank's LB(k1) by then); xmode 1 -- a
// simulated rank: one workgroup waits the modelled link time.  The next launch on the stream (the
// pivot closure) starts after this one ends, so its loads see the peers' bytes.
template <class K>
struct XchgArgs {
    const K* seg;                     // this rank's segment of LB(k1)
    size_t off;                       // its element offset inside LB(k1)
    size_t n8;                        // its size in 8-byte words
    K* peer_lb[kMaxPeers];            // each peer's LB(k1) (null for this rank)
    uint32_t* peer_flags[kMaxPeers];  // each peer's arrival words [pivot * G + from]
    uint32_t* myflags;
    uint32_t* cnt;                    // a zeroed word of this pivot: workgroups done copying
    uint32_t* timeout;
    int k1, G, g, sys, xmode;
    uint32_t epoch;
    uint32_t model_ns;
};

template <class K>
__global__ void __launch_bounds__(256) k_line_xchg(XchgArgs<K> a) {
    __builtin_amdgcn_s_setprio(3);
    if (a.xmode == 1) {
        if (threadIdx.x == 0) {
            const unsigned long long t0 = wall_clock64(), ticks = a.model_ns / 10;  // 100 MHz
            while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
        }
        return;
    }
    const uint64_t* src = reinterpret_cast<const uint64_t*>(a.seg);
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < a.n8; i += (size_t)gridDim.x * blockDim.x) {
        const uint64_t v = src[i];
        for (int p = 0; p < a.G; ++p)
            if (a.peer_lb[p]) st8_wt(reinterpret_cast<uint64_t*>(a.peer_lb[p] + a.off) + i, v, a.sys);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __shared__ uint32_t last;
    if (threadIdx.x == 0) last = __hip_atomic_fetch_add(a.cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    __syncthreads();
    if (!last || threadIdx.x != 0) return;
    // every workgroup's stores have drained: publish, then wait for the peers
    if (a.sys) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    else __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int p = 0; p < a.G; ++p)
        if (a.peer_flags[p]) {
            uint32_t* f = a.peer_flags[p] + (size_t)a.k1 * a.G + a.g;
            if (a.sys) __hip_atomic_store(f, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            else __hip_atomic_store(f, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    const uint32_t ep = a.epoch;
    for (int p = 0; p < a.G; ++p)
        if (p != a.g && !poll_until(a.myflags + (size_t)a.k1 * a.G + p, a.sys, a.timeout, [ep](uint32_t v) { return v == ep; }))
            break;
    acquire_for(a.sys);
}

}  // namespace srg
