// xcc_probe.hip -- which XCD a workgroup runs on: HW_REG_XCC_ID per workgroup vs blockIdx % 8.
// Exploration tool (not product code).  hipcc --offload-arch=gfx950 -O2 xcc_probe.hip -o xcc_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void probe(unsigned* out) {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    if (threadIdx.x == 0) out[blockIdx.x] = x;
}

int main() {
    const int n = 1024;
    unsigned* d = nullptr;
    if (hipMalloc(&d, n * 4) != hipSuccess) return 1;
    probe<<<n, 512>>>(d);
    std::vector<unsigned> h(n);
    if (hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    int match = 0;
    unsigned ormask = 0;
    for (int i = 0; i < n; ++i) {
        match += (h[i] & 7) == (unsigned)(i % 8);
        ormask |= h[i];
    }
    std::printf("blocks %d, (xcc & 7) == blockIdx %% 8 for %d, raw values OR 0x%x, first 16:", n, match, ormask);
    for (int i = 0; i < 16; ++i) std::printf(" %x", h[i]);
    std::printf("\n");
    return 0;
}
