// Where a process's first HIP costs go (round 4 cold-call study): runtime init, stream creation,
// the first dispatch on each new stream (hardware queue creation), device / pinned allocations.
// build: hipcc --offload-arch=gfx950 -O2 tools/init_probe.hip -o tools/init_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

__global__ void k_nop(int* p) { if (p && threadIdx.x == 0 && blockIdx.x == 0) p[0] = 1; }

static double ms(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// usage: init_probe [par]   (par: the first four streams created by four threads at once)
int main(int argc, char** argv) {
    const bool par = argc > 1 && std::strcmp(argv[1], "par") == 0;
    auto T = std::chrono::steady_clock::now();
    auto t = T;
    int n = 0;
    CK(hipGetDeviceCount(&n));
    std::printf("hipGetDeviceCount (%d devices)      %8.2f ms\n", n, ms(t));
    t = std::chrono::steady_clock::now();
    CK(hipSetDevice(0));
    std::printf("hipSetDevice                        %8.2f ms\n", ms(t));
    hipStream_t s[6];
    if (par) {
        t = std::chrono::steady_clock::now();
        std::vector<std::thread> th;
        for (int i = 0; i < 4; ++i)
            th.emplace_back([&s, i]() {
                CK(hipSetDevice(0));
                CK(hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking));
            });
        for (auto& x : th) x.join();
        std::printf("4 x hipStreamCreate in 4 threads    %8.2f ms\n", ms(t));
    }
    for (int i = par ? 4 : 0; i < 6; ++i) {
        t = std::chrono::steady_clock::now();
        CK(hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking));
        std::printf("hipStreamCreate #%d                  %8.2f ms\n", i, ms(t));
    }
    for (int i = 0; i < 6; ++i) {
        t = std::chrono::steady_clock::now();
        k_nop<<<1, 64, 0, s[i]>>>(nullptr);
        CK(hipStreamSynchronize(s[i]));
        std::printf("first launch+sync on stream #%d      %8.2f ms\n", i, ms(t));
    }
    t = std::chrono::steady_clock::now();
    k_nop<<<1, 64, 0, s[0]>>>(nullptr);
    CK(hipStreamSynchronize(s[0]));
    std::printf("second launch+sync on stream #0     %8.2f ms\n", ms(t));
    void* d = nullptr;
    t = std::chrono::steady_clock::now();
    CK(hipMalloc(&d, (size_t)400 << 20));
    std::printf("hipMalloc 400 MB                    %8.2f ms\n", ms(t));
    t = std::chrono::steady_clock::now();
    CK(hipMemsetAsync(d, 0, (size_t)400 << 20, s[0]));
    CK(hipStreamSynchronize(s[0]));
    std::printf("first memset 400 MB                 %8.2f ms\n", ms(t));
    void* h = nullptr;
    t = std::chrono::steady_clock::now();
    CK(hipHostMalloc(&h, (size_t)64 << 20, hipHostMallocDefault));
    std::printf("hipHostMalloc 64 MB                 %8.2f ms\n", ms(t));
    t = std::chrono::steady_clock::now();
    CK(hipMemcpyAsync(d, h, (size_t)64 << 20, hipMemcpyHostToDevice, s[1]));
    CK(hipStreamSynchronize(s[1]));
    std::printf("first H2D 64 MB                     %8.2f ms\n", ms(t));
    hipEvent_t e;
    t = std::chrono::steady_clock::now();
    CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    CK(hipEventRecord(e, s[2]));
    CK(hipStreamWaitEvent(s[3], e, 0));
    CK(hipStreamSynchronize(s[3]));
    std::printf("event record + cross-stream wait    %8.2f ms\n", ms(t));
    std::printf("total                               %8.2f ms\n", ms(T));
    return 0;
}
