// Integer atomicMin throughput on device memory (round 4; VERDICT r03 item 2 asks for it before
// any atomic-based sparse redesign).  u32 atomicMin with and without a used return value, against
// plain loads and stores of the same pattern, over footprints from L2-sized to HBM-sized.
// Patterns: "row" = each wave hits one 256-B row (lane = consecutive dword, the label-row shape of
// k_sparse_bf), the rows random; "scatter" = every lane a random dword.
// build: hipcc --offload-arch=gfx950 -O3 tools/atomic_probe.hip -o tools/atomic_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

// op: 0 = atomicMin no return, 1 = atomicMin with return (summed), 2 = load (summed), 3 = store
template <int OP, bool ROW>
__global__ void __launch_bounds__(256) k_probe(uint32_t* __restrict__ buf, uint32_t mask_words, int iters,
                                               uint32_t seed, uint32_t* __restrict__ sink) {
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x, lane = threadIdx.x & 63;
    const uint32_t wv = gid >> 6;
    uint32_t acc = 0;
    for (int i = 0; i < iters; ++i) {
        uint32_t idx;
        if (ROW) idx = ((hash32(wv * 1315423911u + i * 2654435761u + seed) << 6) | lane) & mask_words;
        else idx = hash32(gid * 1315423911u + i * 2654435761u + seed) & mask_words;
        const uint32_t v = hash32(idx ^ seed ^ i);
        if constexpr (OP == 0) atomicMin(&buf[idx], v);
        else if constexpr (OP == 1) acc += atomicMin(&buf[idx], v);
        else if constexpr (OP == 2) acc += buf[idx];
        else buf[idx] = v;
    }
    if (OP == 1 || OP == 2)
        if (acc == 0x9e3779b9u) sink[0] = acc;  // keep the returned values live
}

template <int OP, bool ROW>
static float run(uint32_t* buf, uint32_t words, int iters, uint32_t* sink, hipEvent_t a, hipEvent_t b, int blocks) {
    k_probe<OP, ROW><<<blocks, 256>>>(buf, words - 1, iters, 1u, sink);  // warm
    CK(hipEventRecord(a));
    for (int r = 0; r < 5; ++r) k_probe<OP, ROW><<<blocks, 256>>>(buf, words - 1, iters, 7u + r, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / 5;
}

int main() {
    const int blocks = 256 * 8, iters = 64;
    const double ops = (double)blocks * 256 * iters;
    const size_t maxw = (size_t)1 << 30;  // 4 GiB of u32
    uint32_t *buf, *sink;
    CK(hipMalloc(&buf, maxw * 4));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(buf, 0xFF, maxw * 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const char* names[4] = {"atomicMin no-ret", "atomicMin ret", "load", "store"};
    std::printf("%-18s %-8s %10s %12s %12s\n", "op", "pattern", "footprint", "Gop/s", "GB/s (4 B/op)");
    for (size_t fp : {(size_t)4 << 20, (size_t)64 << 20, (size_t)1 << 30, (size_t)4 << 30}) {
        const uint32_t words = (uint32_t)(fp / 4);
        for (int row = 1; row >= 0; --row) {
            float t[4];
            if (row) {
                t[0] = run<0, true>(buf, words, iters, sink, a, b, blocks);
                t[1] = run<1, true>(buf, words, iters, sink, a, b, blocks);
                t[2] = run<2, true>(buf, words, iters, sink, a, b, blocks);
                t[3] = run<3, true>(buf, words, iters, sink, a, b, blocks);
            } else {
                t[0] = run<0, false>(buf, words, iters, sink, a, b, blocks);
                t[1] = run<1, false>(buf, words, iters, sink, a, b, blocks);
                t[2] = run<2, false>(buf, words, iters, sink, a, b, blocks);
                t[3] = run<3, false>(buf, words, iters, sink, a, b, blocks);
            }
            for (int o = 0; o < 4; ++o)
                std::printf("%-18s %-8s %8zu MB %12.2f %12.1f\n", names[o], row ? "row" : "scatter", fp >> 20,
                            ops / (t[o] * 1e-3) / 1e9, ops * 4 / (t[o] * 1e-3) / 1e9);
        }
    }
    return 0;
}
