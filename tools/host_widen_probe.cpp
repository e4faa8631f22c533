// Host widening rate probe (round 4): u32 keys -> u64 into a pre-faulted table, T threads, NT stores or plain
// build: g++ -O3 -mavx2 -pthread tools/host_widen_probe.cpp -o tools/host_widen_probe; usage: host_widen_probe T [nt]
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>
#include <immintrin.h>
int main(int argc, char** argv) {
    int T = atoi(argv[1]); size_t n = 100000000; int nt = argc > 2 ? atoi(argv[2]) : 1;
    uint32_t* k = (uint32_t*)aligned_alloc(4096, n * 4);
    uint64_t* o = (uint64_t*)aligned_alloc(4096, n * 8);
    memset(k, 1, n * 4); memset(o, 0, n * 8);
    for (int rep = 0; rep < 4; ++rep) {
        auto t0 = std::chrono::steady_clock::now();
        std::vector<std::thread> th;
        for (int w = 0; w < T; ++w) th.emplace_back([=]() {
            size_t a = n * w / T, z = n * (w + 1) / T;
            a &= ~(size_t)7; if (w == T - 1) z = n; else z &= ~(size_t)7;
            if (nt) {
                for (size_t i = a; i < z; i += 8) {
                    __m256i kk = _mm256_loadu_si256((const __m256i*)(k + i));
                    __m256i lo = _mm256_cvtepu32_epi64(_mm256_castsi256_si128(kk));
                    __m256i hi = _mm256_cvtepu32_epi64(_mm256_extracti128_si256(kk, 1));
                    _mm256_stream_si256((__m256i*)(o + i), lo);
                    _mm256_stream_si256((__m256i*)(o + i + 4), hi);
                }
            } else for (size_t i = a; i < z; ++i) o[i] = (uint64_t)k[i] * 1000;
        });
        for (auto& x : th) x.join();
        double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        printf("T=%d nt=%d %.1f ms  %.1f GB/s out\n", T, nt, ms, n * 8 / ms / 1e6);
    }
}
