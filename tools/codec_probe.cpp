// codec_probe.cpp -- host-side throughput of the H2D codec's encoder (edge_codec.h seq_encode_slice)
// on a C3-shaped edge list (V = 10000 upper triangle, 50 M edges), chunk by chunk as codec_in runs
// it, with T worker threads per chunk; plus a plain read of the same bytes.  Built three ways by
// tools/gpu_r05n.sh (baseline x86-64, -mavx2, -mavx512f) to see what the ISA and the thread count
// buy on the GPU box's host.  Not product code.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../shadow_amd/csrc/edge_codec.h"

static double ms_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main(int argc, char** argv) {
    const uint32_t V = argc > 1 ? atoi(argv[1]) : 10000;
    size_t E = (size_t)V * (V + 1) / 2;
    std::vector<uint32_t> src(E), dst(E);
    std::vector<uint64_t> lat(E);
    size_t e = 0;
    uint64_t x = 88172645463325252ull;
    for (uint32_t i = 0; i < V; ++i)
        for (uint32_t j = i; j < V; ++j, ++e) {
            src[e] = i, dst[e] = j;
            x ^= x << 13, x ^= x >> 7, x ^= x << 17;
            lat[e] = 1000 + (x % 200000000ull);
        }
    constexpr size_t CE = (size_t)2 << 20;
    uint32_t* hl = (uint32_t*)aligned_alloc(64, CE * 4 * 3);
    std::memset(hl, 0, CE * 4 * 3);
    for (int T : {4, 8, 12, 16}) {
        for (int rep = 0; rep < 3; ++rep) {
            std::vector<std::vector<uint32_t>> ex(T);
            uint64_t orl = 0;
            // (1) chunked as codec_in: persistent workers, a spin barrier per 2 M-edge chunk
            std::atomic<size_t> go{0}, done{0};
            std::vector<uint64_t> ol(T, 0);
            auto work = [&](int w, size_t ch) {
                const size_t e0 = ch * CE, ne = std::min(CE, E - e0);
                const size_t a = ne * w / T, z = ne * (w + 1) / T;
                uint32_t orx = 0;
                ex[w].clear();
                srg::seq_encode_slice(src.data() + e0, dst.data() + e0, lat.data() + e0, hl + (ch % 3) * CE, a, z, ex[w],
                                      3 * ((z - a) / 8 + 1), orx, ol[w]);
            };
            const size_t nch = (E + CE - 1) / CE;
            std::vector<std::thread> pool;
            for (int w = 1; w < T; ++w)
                pool.emplace_back([&, w]() {
                    for (size_t ch = 0; ch < nch; ++ch) {
                        while (go.load(std::memory_order_acquire) <= ch) {}
                        work(w, ch);
                        done.fetch_add(1, std::memory_order_acq_rel);
                    }
                });
            const auto t0 = std::chrono::steady_clock::now();
            for (size_t ch = 0; ch < nch; ++ch) {
                go.store(ch + 1, std::memory_order_release);
                work(0, ch);
                while (done.load(std::memory_order_acquire) < (ch + 1) * (T - 1)) {}
            }
            const double enc = ms_since(t0);
            for (auto& t : pool) t.join();
            for (uint64_t v : ol) orl |= v;
            // (2) one slice per thread over the whole list (no chunk barriers)
            const auto t2 = std::chrono::steady_clock::now();
            {
                std::vector<std::thread> th;
                std::vector<uint32_t> big;
                for (int w = 0; w < T; ++w)
                    th.emplace_back([&, w]() {
                        const size_t a = E * w / T, z = E * (w + 1) / T;
                        uint32_t orx = 0;
                        std::vector<uint32_t> ex2;
                        for (size_t c0 = a; c0 < z; c0 += CE) {  // into a private 3-slot window
                            const size_t c1 = std::min(z, c0 + CE);
                            srg::seq_encode_slice(src.data() + c0, dst.data() + c0, lat.data() + c0,
                                                  hl + (size_t)((c0 / CE) % 3) * CE - 0, 0, c1 - c0, ex2, 1u << 30, orx, ol[w]);
                        }
                    });
                for (auto& t : th) t.join();
            }
            const double flat = ms_since(t2);
            // plain read of the same 16 B per edge
            const auto t1 = std::chrono::steady_clock::now();
            std::vector<uint64_t> acc(T, 0);
            std::vector<std::thread> th;
            for (int w = 0; w < T; ++w)
                th.emplace_back([&, w]() {
                    const size_t a = E * w / T, z = E * (w + 1) / T;
                    uint64_t s = 0;
                    for (size_t i = a; i < z; ++i) s += lat[i] ^ src[i] ^ dst[i];
                    acc[w] = s;
                });
            for (auto& t : th) t.join();
            const double rd = ms_since(t1);
            uint64_t chk = orl;
            for (uint64_t v : acc) chk ^= v;
            std::printf("{\"threads\": %d, \"rep\": %d, \"encode_ms\": %.2f, \"flat_ms\": %.2f, \"read_ms\": %.2f, \"chk\": %llu}\n", T, rep,
                        enc, flat, rd, (unsigned long long)(chk & 0xFF));
            std::fflush(stdout);
        }
    }
    return 0;
}
