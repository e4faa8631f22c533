// Hardware-queue sharing probe (gfx950): which of a routing context's four streams (srg_create's
// main stream, the high-priority chain stream, comm, d2h) can run kernels concurrently, after 0..3
// earlier contexts' streams were created and destroyed in the process.  Two streams that share a
// hardware queue serialise their kernels; the value-hop race of rounds 3-4 needs the
// main and chain streams on different queues.  For each pair (main, x): a 200-us spin kernel on
// main, then a tiny kernel on x that stamps wall_clock64; x ran concurrently iff its stamp is before
// the spin's end.  Prints one JSON line per configuration.
// Build: hipcc -O2 --offload-arch=gfx950 tools/queue_probe.hip -o tools/queue_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                       \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) {                                                                     \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                           \
        }                                                                                           \
    } while (0)

__global__ void k_spin(unsigned long long* stamp, int us) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < (unsigned long long)us * 100) __builtin_amdgcn_s_sleep(2);
    if (threadIdx.x == 0) stamp[0] = wall_clock64();
}
__global__ void k_stamp(unsigned long long* stamp) {
    if (threadIdx.x == 0) stamp[0] = wall_clock64();
}

struct Ctx {
    hipStream_t s[4];
    void create() {
        int lo = 0, hi = 0;
        CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        CK(hipStreamCreateWithFlags(&s[0], hipStreamNonBlocking));
        CK(hipStreamCreateWithPriority(&s[1], hipStreamNonBlocking, hi));
        CK(hipStreamCreateWithFlags(&s[2], hipStreamNonBlocking));
        CK(hipStreamCreateWithFlags(&s[3], hipStreamNonBlocking));
    }
    void destroy() {
        for (auto x : s) CK(hipStreamDestroy(x));
    }
};

int main(int argc, char** argv) {
    const int maxprior = argc > 1 ? std::atoi(argv[1]) : 3;
    unsigned long long* st;
    CK(hipMalloc(&st, 64));
    for (int prior = 0; prior <= maxprior; ++prior) {
        std::vector<Ctx> old(prior);
        for (auto& c : old) c.create();
        for (auto& c : old) c.destroy();
        Ctx c;
        c.create();
        int conc[4] = {0, 0, 0, 0};
        for (int x = 1; x < 4; ++x) {
            int hits = 0;
            for (int rep = 0; rep < 5; ++rep) {
                CK(hipDeviceSynchronize());
                k_spin<<<1, 64, 0, c.s[0]>>>(st, 200);
                k_stamp<<<1, 64, 0, c.s[x]>>>(st + 1);
                CK(hipDeviceSynchronize());
                unsigned long long h[2];
                CK(hipMemcpy(h, st, 16, hipMemcpyDeviceToHost));
                hits += h[1] < h[0];
            }
            conc[x] = hits;
        }
        std::printf("{\"prior_contexts\": %d, \"concurrent_with_main_of_5\": {\"chain\": %d, \"comm\": %d, \"d2h\": %d}}\n", prior,
                    conc[1], conc[2], conc[3]);
        std::fflush(stdout);
        c.destroy();
    }
    return 0;
}
