// Cross-stream hand-off latency probe (gfx950): a ping-pong of tiny kernels between two streams,
// joined by (a) hipEventRecord + hipStreamWaitEvent, (b) hipStreamWriteValue32 +
// hipStreamWaitValue32 on signal memory, against (c) the same kernels on one stream.
// Build: hipcc -O2 --offload-arch=gfx950 tools/xq_probe.hip -o tools/xq_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                \
        }                                                                                \
    } while (0)

__global__ void k_tiny(unsigned* p, int spin_ticks) {
    // wall_clock64 ticks at 100 MHz: spin so that the GPU, not the host enqueue, paces the loop
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < (unsigned long long)spin_ticks) __builtin_amdgcn_s_sleep(1);
    if (threadIdx.x == 0) p[blockIdx.x] += 1;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 400;
    const int wgs = argc > 2 ? std::atoi(argv[2]) : 64;
    const int spin = argc > 3 ? std::atoi(argv[3]) * 100 : 0;  // us -> ticks
    int can = 0;
    CK(hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, 0));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    unsigned* buf;
    CK(hipMalloc(&buf, 4096));
    CK(hipMemset(buf, 0, 4096));
    hipEvent_t ea, eb;
    CK(hipEventCreateWithFlags(&ea, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&eb, hipEventDisableTiming));
    unsigned *sig = nullptr, *sig2 = nullptr;  // one HSA signal (8 B) each
    if (can) {
        CK(hipExtMallocWithFlags((void**)&sig, 8, hipMallocSignalMemory));
        CK(hipExtMallocWithFlags((void**)&sig2, 8, hipMallocSignalMemory));
    }
    CK(hipDeviceSynchronize());
    auto run = [&](int mode) {
        // warm
        for (int i = 0; i < 20; ++i) k_tiny<<<wgs, 64, 0, s1>>>(buf, spin);
        CK(hipDeviceSynchronize());
        if (sig) {
            CK(hipStreamWriteValue32(s1, sig, 0, 0));
            CK(hipStreamWriteValue32(s1, sig2, 0, 0));
        }
        CK(hipDeviceSynchronize());
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < iters; ++i) {
            if (mode == 0) {  // one stream
                k_tiny<<<wgs, 64, 0, s1>>>(buf, spin);
                k_tiny<<<wgs, 64, 0, s1>>>(buf, spin);
            } else if (mode == 1) {  // events
                k_tiny<<<wgs, 64, 0, s1>>>(buf, spin);
                CK(hipEventRecord(ea, s1));
                CK(hipStreamWaitEvent(s2, ea, 0));
                k_tiny<<<wgs, 64, 0, s2>>>(buf, spin);
                CK(hipEventRecord(eb, s2));
                CK(hipStreamWaitEvent(s1, eb, 0));
            } else {  // stream memory ops on signal memory
                k_tiny<<<wgs, 64, 0, s1>>>(buf, spin);
                CK(hipStreamWriteValue32(s1, sig, 2 * i + 1, 0));
                CK(hipStreamWaitValue32(s2, sig, 2 * i + 1, hipStreamWaitValueGte, 0xFFFFFFFFu));
                k_tiny<<<wgs, 64, 0, s2>>>(buf, spin);
                CK(hipStreamWriteValue32(s2, sig2, 2 * i + 2, 0));
                CK(hipStreamWaitValue32(s1, sig2, 2 * i + 2, hipStreamWaitValueGte, 0xFFFFFFFFu));
            }
        }
        auto t1 = std::chrono::steady_clock::now();
        CK(hipDeviceSynchronize());
        auto t2 = std::chrono::steady_clock::now();
        const double enq = std::chrono::duration<double, std::micro>(t1 - t0).count() / iters;
        const double tot = std::chrono::duration<double, std::micro>(t2 - t0).count() / iters;
        std::printf("{\"mode\": \"%s\", \"us_per_iter\": %.2f, \"host_enqueue_us_per_iter\": %.2f, \"kernels_per_iter\": 2, \"kernel_spin_us\": %d}\n",
                    mode == 0 ? "one stream" : mode == 1 ? "events" : "wait/write value32", tot, enq, spin / 100);
    };
    run(0);
    run(1);
    if (can) run(2);
    else std::printf("{\"mode\": \"wait/write value32\", \"unsupported\": true}\n");
    run(0);
    run(1);
    if (can) run(2);
    return 0;
}
