// CPU check of the impossible-result guard (shadow_amd/csrc/guards.h) as k_certify applies it: a
// row-major key matrix D over used rows x used columns is flagged when any off-diagonal key is
// below the smallest edge key.  Feeds it (1) a zeroed D -- the all-zero table of the round-4 value-hop
// race -- which must be flagged, (2) a valid closure of a small graph, which must pass, (3) a valid
// table with one entry lowered below the smallest edge, flagged, (4) a diagonal of zeros and INF
// (unreachable) entries, which the guard leaves to the other checks.  Prints "ok" or exits 1.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "../../shadow_amd/csrc/guards.h"

template <class K>
static bool certify(const std::vector<K>& D, uint32_t V, const std::vector<uint32_t>& rows,
                    const std::vector<uint32_t>& cols, K min_key) {
    bool bad = false;
    for (uint32_t s : rows)
        for (uint32_t t : cols) bad |= srg::impossible_key<K>(D[(size_t)s * V + t], min_key, s == t);
    return bad;
}

int main() {
    const uint32_t V = 6;
    const uint32_t INF = 0x7FFFFFFFu;
    // a 6-cycle with chords; latencies in ns, unit 1000 ns
    struct E { uint32_t a, b; uint64_t ns; } es[] = {{0, 1, 5000}, {1, 2, 3000}, {2, 3, 7000}, {3, 4, 2000},
                                                      {4, 5, 9000}, {5, 0, 4000}, {0, 3, 11000}, {1, 4, 6000}};
    const uint64_t unit = 1000;
    unsigned long long min_inv = 0;
    for (auto& e : es) min_inv = ~e.ns > min_inv ? ~e.ns : min_inv;  // k_edge_scan's reduction
    const uint32_t min_key = (uint32_t)srg::min_edge_key(min_inv, unit);
    if (min_key != 2) return std::fprintf(stderr, "min key %u\n", min_key), 1;
    std::vector<uint32_t> D((size_t)V * V, INF);
    for (uint32_t i = 0; i < V; ++i) D[(size_t)i * V + i] = 0;
    for (auto& e : es) {
        const uint32_t k = (uint32_t)(e.ns / unit);
        D[(size_t)e.a * V + e.b] = std::min(D[(size_t)e.a * V + e.b], k);
        D[(size_t)e.b * V + e.a] = std::min(D[(size_t)e.b * V + e.a], k);
    }
    for (uint32_t k = 0; k < V; ++k)
        for (uint32_t i = 0; i < V; ++i)
            for (uint32_t j = 0; j < V; ++j)
                D[(size_t)i * V + j] = std::min(D[(size_t)i * V + j], D[(size_t)i * V + k] + D[(size_t)k * V + j]);
    std::vector<uint32_t> all = {0, 1, 2, 3, 4, 5}, sub = {4, 1, 3};
    if (certify(D, V, all, all, min_key)) return std::fprintf(stderr, "valid closure flagged\n"), 1;
    if (certify(D, V, sub, sub, min_key)) return std::fprintf(stderr, "valid subset flagged\n"), 1;
    std::vector<uint32_t> Z((size_t)V * V, 0);
    if (!certify(Z, V, all, all, min_key)) return std::fprintf(stderr, "zeroed table passed\n"), 1;
    if (!certify(Z, V, sub, sub, min_key)) return std::fprintf(stderr, "zeroed subset passed\n"), 1;
    auto L = D;
    L[(size_t)2 * V + 5] = 1;  // below the smallest edge key
    if (!certify(L, V, all, all, min_key)) return std::fprintf(stderr, "lowered entry passed\n"), 1;
    auto U = D;
    U[(size_t)2 * V + 5] = INF;  // unreachable: the certification's business, not the guard's
    if (certify(U, V, all, all, min_key)) return std::fprintf(stderr, "INF flagged\n"), 1;
    std::vector<uint64_t> D64(D.begin(), D.end()), Z64((size_t)V * V, 0);
    if (certify<uint64_t>(D64, V, all, all, min_key) || !certify<uint64_t>(Z64, V, all, all, min_key))
        return std::fprintf(stderr, "u64 keys\n"), 1;
    if (srg::min_edge_key(0, unit) != 0) return std::fprintf(stderr, "no edges\n"), 1;
    // the FW timeout word names the kernel that gave up (code 3 is the line exchange)
    const std::string m1 = srg::fw_timeout_message(1), m2 = srg::fw_timeout_message(2), m3 = srg::fw_timeout_message(3);
    if (m1.find("pivot closure") == std::string::npos || m2.find("cross-stream hop") == std::string::npos ||
        m3.find("line exchange") == std::string::npos || m3.find("arrival word") == std::string::npos)
        return std::fprintf(stderr, "timeout messages\n"), 1;
    std::printf("ok\n");
    return 0;
}
