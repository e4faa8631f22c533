// guards.h — impossible-result guards, shared by the device kernels (k_certify, the sparse
// kernels' output phase) and a CPU unit test (tests/cpp/guard_check.cpp, built with g++).
//
// The reference cannot return a used off-diagonal pair whose latency is below the smallest edge
// latency: every edge latency is positive (ShadowEdge, mod.rs:62-111 rejects 0) and a shortest
// path between two distinct nodes has at least one edge, so its latency -- a sum of edge latencies
// (PathProperties::add, mod.rs:322-331) -- is at least the smallest one.  In latency keys (latency
// / unit, exact) the same bound holds with the smallest edge KEY.  A smaller value (0 included:
// an all-zero table) is a fault inside the builder -- a lost synchronisation, a buffer read
// before it was written -- and the build fails with SRG_ERR_INTERNAL instead of returning it.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define SRG_GUARD_HD __host__ __device__
#else
#define SRG_GUARD_HD
#endif

namespace srg {

// d: a used pair's latency key; min_key: the smallest non-self-loop edge key, clamped by the caller
// to the key type's INF (an edge of >= INF keys counts as absent, so INF itself stays legal: it is
// the unreachable / out-of-range marker the other checks decide on); diagonal: the pair
// is (s, s) (its output is the raw self-loop weight, mod.rs:211-217, not a path)
template <class K>
SRG_GUARD_HD inline bool impossible_key(K d, K min_key, bool diagonal) {
    return !diagonal && d < min_key;
}

// the smallest edge key from the edge scan's ~min (0 = no non-self-loop edge: nothing to guard)
SRG_GUARD_HD inline uint64_t min_edge_key(unsigned long long min_lat_inv, uint64_t unit) {
    if (!min_lat_inv) return 0;
    const uint64_t mn = ~(uint64_t)min_lat_inv;
    return unit > 1 ? mn / unit : mn;
}

// The symmetric FW's timeout word (zeroed per build; the first raiser's code stays, later raisers
// compare-and-swap from 0): 1 = a pivot-closure grid barrier, 2 = a cross-stream value hop,
// 3 = a line-exchange wait for a peer's arrival word (xchg.hip.h poll_until).  The host reports the
// kernel that gave up, so a hang is looked for where it happened.
inline const char* fw_timeout_message(uint32_t code) {
    switch (code) {
        case 2: return "FW chain: a cross-stream hop waited past its bound (mis-ordered enqueue)";
        case 3: return "FW line exchange: a peer's arrival word did not come within the bound (peer stalled or gone)";
        default: return "FW pivot closure: a grid barrier timed out (workgroups not co-resident)";
    }
}

}  // namespace srg
