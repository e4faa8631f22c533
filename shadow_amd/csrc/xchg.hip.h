// xchg.hip.h — device-side exchange of the FW line buffers between ranks (gfx950).
//
// The symmetric line-buffer FW (routing.hip SymFw) builds, per pivot k1, the line buffer LB(k1) from
// every rank's tiles of line k1; ranks exchange their segments of it once per pivot.  The default is
// the communicator's allgather on the chain's stream (RCCL between processes, pull kernels in an
// in-process group).  This file is the alternative that needs no host rendezvous per pivot:
//   xmode 2 (in-process ranks, SRG_OPT_FW_STEP = 2): k_line_xchg stores this rank's segment straight
//           into every peer's LB(k1) (write-through, system scope when a peer is on another device)
//           and raises an arrival word at every peer, then waits for every peer's word;
//   xmode 1 (a simulated rank, SRG_OPT_SIMULATE_RANK): one workgroup waits the modelled link time.
// (Round 4 also carried a fused one-launch-per-pivot FW built on the same hand-offs; it measured
// slower at every rank count and was removed in round 5 -- DESIGN.md §7 keeps the A/B.)
// Hand-offs follow MI355X_MICROARCH.md: segment bytes stored write-through and drained before the
// arrival word; the reader polls relaxed, then one acquire before plain loads.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.hip.h"

namespace srg {

constexpr int kMaxPeers = 16;

// bounded poll of *p until pred(value) (one lane); false after ~2 s (raises *timeout)
template <class Pred>
__device__ __forceinline__ bool poll_until(const uint32_t* p, int sys, uint32_t* timeout, Pred pred) {
    const unsigned long long t0 = wall_clock64();
    for (;;) {
        const uint32_t v = sys ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                               : __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (pred(v)) return true;
        if (__hip_atomic_load(timeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return false;  // keep the raiser's code
        if (wall_clock64() - t0 > 200000000ull) {
            uint32_t zero = 0;  // 3 = an exchange wait timed out, unless something else was first
            __hip_atomic_compare_exchange_strong(timeout, &zero, 3u, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
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
