// CPU check of the sequential-pair encoder (shadow_amd/csrc/edge_codec.h): split a chunk into
// worker slices as codec_in does, encode, concatenate the exceptions in slice order, decode with
// the device formula (k_decode_seq) and compare.  Prints "ok <chunks> <exceptions>" or exits 1.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../../shadow_amd/csrc/edge_codec.h"

static int check(const std::vector<uint32_t>& src, const std::vector<uint32_t>& dst, const std::vector<uint64_t>& lat,
                 int nw, bool expect_dense, size_t& nexc_out) {
    const size_t ne = src.size();
    std::vector<uint32_t> hl(ne);
    std::vector<std::vector<uint32_t>> ex(nw);
    bool dense = false;
    uint32_t orx = 0;
    uint64_t orl = 0;
    for (int w = 0; w < nw; ++w) {
        const size_t a = ne * w / nw, z = ne * (w + 1) / nw;
        if (!srg::seq_encode_slice(src.data(), dst.data(), lat.data(), hl.data(), a, z, ex[w], 3 * ((z - a) / 8 + 1),
                                   orx, orl))
            dense = true;
    }
    for (size_t i = 0; i < ne; ++i)
        if (hl[i] != (uint32_t)lat[i]) return std::fprintf(stderr, "latency %zu\n", i), 1;
    if (dense != expect_dense) return std::fprintf(stderr, "dense %d expected %d\n", dense, expect_dense), 1;
    if (dense) return 0;
    std::vector<uint32_t> ei, es, ed;
    for (int w = 0; w < nw; ++w)
        for (size_t k = 0; k + 2 < ex[w].size(); k += 3) {
            ei.push_back(ex[w][k]);
            es.push_back(ex[w][k + 1]);
            ed.push_back(ex[w][k + 2]);
        }
    nexc_out += ei.size();
    if (ei.empty() || ei[0] != 0) return std::fprintf(stderr, "first edge is not an exception\n"), 1;
    for (size_t j = 1; j < ei.size(); ++j)
        if (ei[j] <= ei[j - 1]) return std::fprintf(stderr, "exceptions out of order\n"), 1;
    for (size_t i = 0; i < ne; ++i) {
        size_t lo = 0, hi = ei.size() - 1;  // last exception <= i (k_decode_seq)
        while (lo < hi) {
            const size_t mid = (lo + hi + 1) >> 1;
            if (ei[mid] <= i) lo = mid;
            else hi = mid - 1;
        }
        const uint32_t s = es[lo], d = ed[lo] + (uint32_t)(i - ei[lo]);
        if (s != src[i] || d != dst[i])
            return std::fprintf(stderr, "edge %zu: (%u,%u) decoded as (%u,%u)\n", i, src[i], dst[i], s, d), 1;
    }
    return 0;
}

int main() {
    std::mt19937_64 rng(7);
    size_t chunks = 0, nexc = 0;
    for (int V : {1, 2, 3, 64, 777, 1500}) {
        // GML complete-graph order with self-loops inline, the synthetic generator's order (self-loops
        // first), and rows with gaps
        for (int variant = 0; variant < 3; ++variant) {
            std::vector<uint32_t> src, dst;
            if (variant == 1)
                for (int i = 0; i < V; ++i) src.push_back(i), dst.push_back(i);
            for (int i = 0; i < V; ++i)
                for (int j = variant == 1 ? i + 1 : i; j < V; ++j) {
                    if (variant == 2 && rng() % 20 == 0) continue;
                    src.push_back(i);
                    dst.push_back(j);
                }
            if (src.empty()) continue;
            std::vector<uint64_t> lat(src.size());
            for (auto& l : lat) l = rng() % 4000000000ull;
            // whole list, and chunk boundaries at arbitrary offsets (every chunk restarts the encoding)
            for (size_t ce : {src.size(), (size_t)1000, (size_t)4096}) {
                for (size_t e0 = 0; e0 < src.size(); e0 += ce) {
                    const size_t e1 = std::min(src.size(), e0 + ce);
                    std::vector<uint32_t> s(src.begin() + e0, src.begin() + e1), d(dst.begin() + e0, dst.begin() + e1);
                    std::vector<uint64_t> l(lat.begin() + e0, lat.begin() + e1);
                    // dense only when a slice of some worker has > 1/8 exceptions: tiny rows can be
                    for (int nw : {1, 3, 8}) {
                        size_t ex = 0;
                        // decide the expectation by counting per slice like the encoder
                        bool exp_dense = false;
                        for (int w = 0; w < nw; ++w) {
                            const size_t a = s.size() * w / nw, z = s.size() * (w + 1) / nw;
                            size_t cnt = 0;
                            for (size_t i = a; i < z; ++i)
                                if (i == 0 || !(i > 0 && s[i] == s[i - 1] && d[i] == d[i - 1] + 1)) ++cnt;
                            if (3 * cnt > 3 * ((z - a) / 8 + 1)) exp_dense = true;
                        }
                        if (check(s, d, l, nw, exp_dense, ex)) return 1;
                        nexc += ex;
                        ++chunks;
                    }
                }
            }
        }
    }
    // a shuffled list is dense
    std::vector<uint32_t> s(100000), d(100000);
    std::vector<uint64_t> l(100000, 5);
    for (size_t i = 0; i < s.size(); ++i) s[i] = rng() % 1000, d[i] = rng() % 1000;
    size_t ex = 0;
    if (check(s, d, l, 8, true, ex)) return 1;
    std::printf("ok %zu %zu\n", chunks, nexc);
    return 0;
}
