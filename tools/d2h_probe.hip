// d2h_probe.hip — how much does a concurrent device->host copy slow the kernels it overlaps?
// Measures a streaming kernel (reads 800 MB, like k_ess_mask) and an LDS/VALU-bound kernel
// alone and beside an 800 MB D2H done four ways: hipMemcpyAsync into registered (mapped) user
// memory (ROCclr blit kernel), hipMemcpyAsync into hipHostMalloc memory, a narrow copy kernel,
// and hsa_amd_memory_async_copy_on_engine (an SDMA engine).  Exploration tool, not product code.
//   build: hipcc --offload-arch=gfx950 -O3 -o tools/d2h_probe tools/d2h_probe.hip -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

__global__ void __launch_bounds__(256) k_stream(const uint4* __restrict__ a, size_t n, unsigned* out) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        acc ^= a[i].x + a[i].y + a[i].z + a[i].w;
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void __launch_bounds__(256) k_valu(unsigned* out, int iters) {
    __shared__ unsigned s[256];
    unsigned x = threadIdx.x * 2654435761u;
    s[threadIdx.x] = x;
    __syncthreads();
    for (int i = 0; i < iters; ++i) {
        x = x * 1664525u + s[(threadIdx.x + i) & 255];
        x ^= x >> 7;
    }
    if (x == 0x12345678u) out[1] = x;
}

__global__ void __launch_bounds__(256) k_copy(const uint4* __restrict__ s, uint4* __restrict__ d, size_t n) {
    const size_t nt = (size_t)gridDim.x * 256;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += nt) d[i] = s[i];
}

static hsa_agent_t g_gpu, g_cpu;
static hsa_status_t find_agents(hsa_agent_t a, void*) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU && g_gpu.handle == 0) g_gpu = a;
    if (t == HSA_DEVICE_TYPE_CPU && g_cpu.handle == 0) g_cpu = a;
    return HSA_STATUS_SUCCESS;
}

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    const size_t B = 800ull << 20;
    CK(hipSetDevice(0));
    void *src, *big;
    unsigned* out;
    CK(hipMalloc(&src, B));
    CK(hipMalloc(&big, B));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(src, 1, B));
    CK(hipMemset(big, 2, B));
    void* user = aligned_alloc(4096, B);
    memset(user, 0, B);
    CK(hipHostRegister(user, B, hipHostRegisterMapped));
    void* view = nullptr;
    CK(hipHostGetDevicePointer(&view, user, 0));
    void* pinned = nullptr;
    CK(hipHostMalloc(&pinned, B, 0));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hsa_iterate_agents(find_agents, nullptr);
    hsa_signal_t sig;
    hsa_signal_create(1, 0, nullptr, &sig);
    uint32_t engines = 0;
    hsa_amd_memory_copy_engine_status(g_cpu, g_gpu, &engines);
    printf("view==user %d, sdma engine mask (gpu->cpu) 0x%x\n", view == user, engines);

    auto time_kernel = [&](int which) {  // ms of one launch on s1
        CK(hipEventRecord(e0, s1));
        if (which == 0) k_stream<<<8192, 256, 0, s1>>>((const uint4*)big, B / 16, out);
        else k_valu<<<4096, 256, 0, s1>>>(out, 20000);
        CK(hipEventRecord(e1, s1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        return ms;
    };
    const char* kname[2] = {"stream800MB", "valu"};
    for (int k = 0; k < 2; ++k) {
        time_kernel(k);
        float alone = 0;
        for (int r = 0; r < 3; ++r) alone += time_kernel(k) / 3;
        printf("%-12s alone %.3f ms\n", kname[k], alone);
        for (int mode = 0; mode < 5; ++mode) {
            // start the copy, then run the kernel 3x back to back while it is in flight
            double t0 = now_ms();
            bool hsa_ok = true;
            if (mode == 0) CK(hipMemcpyAsync(user, src, B, hipMemcpyDeviceToHost, s2));
            else if (mode == 1) CK(hipMemcpyAsync(pinned, src, B, hipMemcpyDeviceToHost, s2));
            else if (mode == 2) k_copy<<<32, 256, 0, s2>>>((const uint4*)src, (uint4*)view, B / 16);
            else if (mode == 3) k_copy<<<8, 256, 0, s2>>>((const uint4*)src, (uint4*)view, B / 16);
            else {
                hsa_signal_store_relaxed(sig, 1);
                int eng = 0;
                while (eng < 16 && !(engines & (1u << eng))) ++eng;
                hsa_status_t st = hsa_amd_memory_async_copy_on_engine(view, g_cpu, src, g_gpu, B, 0, nullptr, sig,
                                                                       (hsa_amd_sdma_engine_id_t)(1u << eng), true);
                if (st != HSA_STATUS_SUCCESS) {
                    st = hsa_amd_memory_async_copy(view, g_cpu, src, g_gpu, B, 0, nullptr, sig);
                    printf("  (on_engine failed, plain async copy: %d)\n", (int)st);
                }
                hsa_ok = st == HSA_STATUS_SUCCESS;
            }
            const double t_issue = now_ms() - t0;
            // kernels back to back until the copy has finished: the average launch while it runs
            float beside = 0;
            int runs = 0;
            for (;;) {
                bool done;
                if (mode == 4) done = !hsa_ok || hsa_signal_load_scacquire(sig) < 1;
                else done = hipStreamQuery(s2) == hipSuccess;
                if (done && runs >= 1) break;
                beside += time_kernel(k);
                ++runs;
                if (runs > 2000) break;
            }
            beside /= runs;
            if (mode == 4) {
                if (hsa_ok) hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
            } else {
                CK(hipStreamSynchronize(s2));
            }
            double tc = now_ms() - t0;
            printf("  [issue returned after %.2f ms, %d kernel runs during the copy]\n", t_issue, runs);
            const char* mname[5] = {"memcpy->registered", "memcpy->hostmalloc", "copykernel32", "copykernel8", "hsa_sdma"};
            printf("  beside %-20s %.3f ms (x%.2f)   copy wall %.2f ms (%.1f GB/s)\n", mname[mode], beside,
                   beside / alone, tc, B / tc / 1e6);
        }
    }
    // correctness of the SDMA path: user must equal src bytes (1s)
    size_t bad = 0;
    for (size_t i = 0; i < B; i += 4097) bad += ((unsigned char*)user)[i] != 1;
    printf("user bytes wrong (sampled): %zu\n", bad);
    return 0;
}
