// Value-hop ordering probe (gfx950).  Reproduces the FW chain's cross-stream hand-off in
// isolation: a producer kernel on stream A writes a 64 MB buffer from every XCD, a one-wave
// "set" kernel behind it on A raises a signal word, a one-wave "wait" kernel on stream B polls
// it, and a consumer kernel behind the wait on B checks every word of the buffer.  Meanwhile B
// runs an unrelated long kernel (the bulk) before the wait, as the FW's main stream does.
//
// Per iteration it records
//   early : the set kernel ran before every producer workgroup had finished (read from a
//           completion counter the producer's workgroups bump at their very end) -- i.e. the
//           runtime let the set packet start while the previous packet on its stream still ran;
//   stale : consumer words != this iteration's value although the hop said go.
// Modes: 0 value hops (the product's k_hop_set / k_hop_wait), 1 events, 2 value hops with an
// agent-scope release in every producer workgroup and an agent-scope acquire in every consumer
// workgroup.  `extra` pre-creates that many streams (more streams than GPU_MAX_HW_QUEUES make
// HIP streams share hardware queues, as after earlier contexts in one process).
// Build: hipcc -O2 --offload-arch=gfx950 tools/hop_probe.hip -o tools/hop_probe
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

constexpr int kWG = 1024;
constexpr size_t kWords = (size_t)16 << 20;  // 64 MB

__global__ void __launch_bounds__(256) k_prod(unsigned* B, unsigned v, unsigned* done, int fence) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < kWords; i += (size_t)gridDim.x * blockDim.x)
        B[i] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        if (fence) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ void k_set(unsigned* sig, unsigned v, const unsigned* done, unsigned want, unsigned* early) {
    if (threadIdx.x != 0) return;
    const unsigned d = __hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (d != want) atomicAdd(early, 1u);
    __hip_atomic_store(sig, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_wait(const unsigned* sig, unsigned v, unsigned* timeout) {
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = wall_clock64();
    while (__hip_atomic_load(sig, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - v > 0x7FFFFFFFu) {
        if (wall_clock64() - t0 > 200000000ull) {
            atomicAdd(timeout, 1u);
            return;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

__global__ void __launch_bounds__(256) k_cons(const unsigned* B, unsigned v, unsigned* stale, int fence) {
    if (fence) {
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
    }
    unsigned bad = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < kWords; i += (size_t)gridDim.x * blockDim.x)
        bad += B[i] != v;
    if (bad) atomicAdd(stale, bad);
}

// the unrelated long kernel on the consumer's stream ahead of its wait (the FW bulk's role)
__global__ void __launch_bounds__(256) k_busy(unsigned* X, int ticks) {
    const unsigned long long t0 = wall_clock64();
    unsigned a = threadIdx.x;
    while (wall_clock64() - t0 < (unsigned long long)ticks) a = a * 1664525u + 1013904223u;
    if (a == 0x12345678u) X[blockIdx.x] = a;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 300;
    const int extra = argc > 2 ? std::atoi(argv[2]) : 0;
    const int busy_us = argc > 3 ? std::atoi(argv[3]) : 50;
    std::vector<hipStream_t> pre(extra);
    for (auto& s : pre) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipStream_t A, Bs;
    CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&Bs, hipStreamNonBlocking));
    unsigned *buf, *cnt, *X;
    CK(hipMalloc(&buf, kWords * 4));
    CK(hipMalloc(&cnt, 4096));
    CK(hipMalloc(&X, 4096));
    unsigned *sig0, *sig1;
    CK(hipExtMallocWithFlags((void**)&sig0, 8, hipMallocSignalMemory));
    CK(hipExtMallocWithFlags((void**)&sig1, 8, hipMallocSignalMemory));
    hipEvent_t ea, eb;
    CK(hipEventCreateWithFlags(&ea, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&eb, hipEventDisableTiming));
    for (int mode = 0; mode < 3; ++mode) {
        CK(hipMemset(buf, 0xFF, kWords * 4));
        CK(hipMemset(cnt, 0, 4096));
        CK(hipStreamWriteValue32(A, sig0, 0, 0));
        CK(hipStreamWriteValue32(A, sig1, 0, 0));
        CK(hipDeviceSynchronize());
        // cnt: [0] early, [1] stale words, [2] stale iterations (unused), [3] timeouts, [16 + i%2] done counters
        unsigned* early = cnt;
        unsigned* stale = cnt + 1;
        unsigned* tmo = cnt + 3;
        for (int i = 0; i < iters; ++i) {
            const unsigned v = (unsigned)i + 1;
            unsigned* done = cnt + 16 + (i & 1);
            // done counter of this iteration reset on A (in order before the producer)
            CK(hipMemsetAsync(done, 0, 4, A));
            // B -> A: the previous consumer is finished before the producer overwrites the buffer
            if (mode == 1) {
                CK(hipEventRecord(eb, Bs));
                CK(hipStreamWaitEvent(A, eb, 0));
            } else {
                k_set<<<1, 64, 0, Bs>>>(sig0, v, cnt + 15, 0, cnt + 14);  // (no completion check here)
                k_wait<<<1, 64, 0, A>>>(sig0, v, tmo);
            }
            k_prod<<<kWG, 256, 0, A>>>(buf, v, done, mode == 2);
            k_busy<<<512, 256, 0, Bs>>>(X, busy_us * 100);
            if (mode == 1) {
                CK(hipEventRecord(ea, A));
                CK(hipStreamWaitEvent(Bs, ea, 0));
            } else {
                k_set<<<1, 64, 0, A>>>(sig1, v, done, kWG, early);
                k_wait<<<1, 64, 0, Bs>>>(sig1, v, tmo);
            }
            k_cons<<<kWG, 256, 0, Bs>>>(buf, v, stale, mode == 2);
        }
        CK(hipDeviceSynchronize());
        unsigned h[4];
        CK(hipMemcpy(h, cnt, 16, hipMemcpyDeviceToHost));
        std::printf("{\"mode\": \"%s\", \"extra_streams\": %d, \"iters\": %d, \"early_sets\": %u, \"stale_words\": %u, "
                    "\"timeouts\": %u}\n",
                    mode == 0 ? "value hops" : mode == 1 ? "events" : "value hops + agent release/acquire in kernels", extra,
                    iters, h[0], h[1], h[3]);
        std::fflush(stdout);
    }
    return 0;
}
