// Microbenchmark: issue rate of the u32 min-plus building blocks on gfx950.
// Each kernel runs independent chains (8 per lane) of one instruction mix; reports
// wave-instructions per SIMD-cycle relative to the 1-per-2-cycles wave64 peak.
// build: hipcc -O3 --offload-arch=gfx950 tools/valu_rate.hip -o /tmp/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

#define N_ITER 4096

template <int MODE>
__global__ void __launch_bounds__(256) k(unsigned* out, unsigned seed) {
    unsigned a[8], b[8], c[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        a[i] = seed * (threadIdx.x + i);
        b[i] = seed ^ (threadIdx.x * 7 + i);
        c[i] = 0xFFFFFFFFu - i;
    }
    for (int it = 0; it < N_ITER; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            unsigned x, y, r;
            if constexpr (MODE == 0) {  // add clamp x2 + min3
                asm volatile("v_add_u32_e64 %0, %1, %2 clamp" : "=v"(x) : "v"(a[i]), "v"(b[i]));
                asm volatile("v_add_u32_e64 %0, %1, %2 clamp" : "=v"(y) : "v"(b[i]), "v"(a[i]));
                asm volatile("v_min3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(c[i]), "v"(x), "v"(y));
            } else if constexpr (MODE == 1) {  // add (VOP2) x2 + min3
                asm volatile("v_add_u32_e32 %0, %1, %2" : "=v"(x) : "v"(a[i]), "v"(b[i]));
                asm volatile("v_add_u32_e32 %0, %1, %2" : "=v"(y) : "v"(b[i]), "v"(a[i]));
                asm volatile("v_min3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(c[i]), "v"(x), "v"(y));
            } else if constexpr (MODE == 2) {  // add (VOP2) x2 + min (VOP2) x2
                asm volatile("v_add_u32_e32 %0, %1, %2" : "=v"(x) : "v"(a[i]), "v"(b[i]));
                asm volatile("v_add_u32_e32 %0, %1, %2" : "=v"(y) : "v"(b[i]), "v"(a[i]));
                asm volatile("v_min_u32_e32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(c[i]));
                asm volatile("v_min_u32_e32 %0, %1, %2" : "=v"(r) : "v"(y), "v"(r));
            } else if constexpr (MODE == 3) {  // add clamp only x3
                asm volatile("v_add_u32_e64 %0, %1, %2 clamp" : "=v"(x) : "v"(a[i]), "v"(b[i]));
                asm volatile("v_add_u32_e64 %0, %1, %2 clamp" : "=v"(y) : "v"(b[i]), "v"(a[i]));
                asm volatile("v_add_u32_e64 %0, %1, %2 clamp" : "=v"(r) : "v"(c[i]), "v"(x));
            } else if constexpr (MODE == 4) {  // min3 only x3
                asm volatile("v_min3_u32 %0, %1, %2, %3" : "=v"(x) : "v"(a[i]), "v"(b[i]), "v"(c[i]));
                asm volatile("v_min3_u32 %0, %1, %2, %3" : "=v"(y) : "v"(b[i]), "v"(a[i]), "v"(c[i]));
                asm volatile("v_min3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(c[i]), "v"(x), "v"(y));
            } else if constexpr (MODE == 6) {  // add x2 + min3_f32 on the u32 bit patterns
                asm volatile("v_add_u32_e32 %0, %1, %2" : "=v"(x) : "v"(a[i]), "v"(b[i]));
                asm volatile("v_add_u32_e32 %0, %1, %2" : "=v"(y) : "v"(b[i]), "v"(a[i]));
                asm volatile("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(c[i]), "v"(x), "v"(y));
            } else if constexpr (MODE == 7) {  // min3_f32 only x3
                asm volatile("v_min3_f32 %0, %1, %2, %3" : "=v"(x) : "v"(a[i]), "v"(b[i]), "v"(c[i]));
                asm volatile("v_min3_f32 %0, %1, %2, %3" : "=v"(y) : "v"(b[i]), "v"(a[i]), "v"(c[i]));
                asm volatile("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(c[i]), "v"(x), "v"(y));
            } else if constexpr (MODE == 8) {  // min_f32 (VOP2) only x3
                asm volatile("v_min_f32_e32 %0, %1, %2" : "=v"(x) : "v"(a[i]), "v"(b[i]));
                asm volatile("v_min_f32_e32 %0, %1, %2" : "=v"(y) : "v"(b[i]), "v"(a[i]));
                asm volatile("v_min_f32_e32 %0, %1, %2" : "=v"(r) : "v"(c[i]), "v"(x));
            } else if constexpr (MODE == 9) {  // min_u32 (VOP2) only x3
                asm volatile("v_min_u32_e32 %0, %1, %2" : "=v"(x) : "v"(a[i]), "v"(b[i]));
                asm volatile("v_min_u32_e32 %0, %1, %2" : "=v"(y) : "v"(b[i]), "v"(a[i]));
                asm volatile("v_min_u32_e32 %0, %1, %2" : "=v"(r) : "v"(c[i]), "v"(x));
            } else if constexpr (MODE == 10) {  // min_i32 (VOP2) only x3
                asm volatile("v_min_i32_e32 %0, %1, %2" : "=v"(x) : "v"(a[i]), "v"(b[i]));
                asm volatile("v_min_i32_e32 %0, %1, %2" : "=v"(y) : "v"(b[i]), "v"(a[i]));
                asm volatile("v_min_i32_e32 %0, %1, %2" : "=v"(r) : "v"(c[i]), "v"(x));
            } else {  // v_add_u32 VOP2 only x3
                asm volatile("v_add_u32_e32 %0, %1, %2" : "=v"(x) : "v"(a[i]), "v"(b[i]));
                asm volatile("v_add_u32_e32 %0, %1, %2" : "=v"(y) : "v"(b[i]), "v"(a[i]));
                asm volatile("v_add_u32_e32 %0, %1, %2" : "=v"(r) : "v"(c[i]), "v"(x));
            }
            c[i] = r;
            a[i] ^= y;
        }
    }
    unsigned s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += c[i] + a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// Pair-packed adds: two u32 keys <= 0x7FFFFFFF per 64-bit register, so one 64-bit add yields two
// exact 32-bit sums.  MODE 0: v_lshl_add_u64 + v_min3_u32 (= two min-plus relaxations);
// MODE 1: v_lshl_add_u64 only; MODE 2: plain C++ u64 add + min3 (what the compiler emits).
template <int MODE>
__global__ void __launch_bounds__(256) k64(unsigned* out, unsigned seed) {
    unsigned long long p[8], q[8];
    unsigned c[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        p[i] = ((unsigned long long)(seed * (threadIdx.x + i) & 0x3FFFFFFF) << 32) | (seed ^ (threadIdx.x * 7 + i));
        q[i] = ((unsigned long long)(seed + i) << 32) | (threadIdx.x & 0xFFFF);
        c[i] = 0x7FFFFFFFu - i;
    }
    for (int it = 0; it < N_ITER; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            unsigned long long s;
            unsigned r;
            if constexpr (MODE == 0) {
                asm volatile("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(s) : "v"(p[i]), "v"(q[i]));
                asm volatile("v_min3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(c[i]), "v"((unsigned)s), "v"((unsigned)(s >> 32)));
            } else if constexpr (MODE == 1) {
                unsigned long long s0, s1;
                asm volatile("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(s0) : "v"(p[i]), "v"(q[i]));
                asm volatile("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(s1) : "v"(s0), "v"(q[i]));
                asm volatile("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(s) : "v"(s1), "v"(p[i]));
                r = (unsigned)s;
            } else {
                s = p[i] + q[i];
                asm volatile("v_min3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(c[i]), "v"((unsigned)s), "v"((unsigned)(s >> 32)));
            }
            c[i] = r;
            p[i] ^= (unsigned)s & 0xFFFu;
        }
    }
    unsigned sum = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) sum += c[i] + (unsigned)p[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = sum;
}

template <int MODE>
void run64(const char* name, int ninstr) {
    unsigned* out;
    hipMalloc(&out, 256 * 4096 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = 256 * 8;
    k64<MODE><<<blocks, 256>>>(out, 1);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) k64<MODE><<<blocks, 256>>>(out, r + 2);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double winst = 5.0 * blocks * 4 * (double)N_ITER * 8 * (ninstr + 1);  // + the xor
    const double per_simd_cycle = winst / (1024.0 * ms * 1e-3 * 2.4e9);
    printf("%-34s %8.3f ms  %.3f wave-instr/SIMD/cycle@2.4GHz (peak 0.5)\n", name, ms, per_simd_cycle);
    hipFree(out);
}

__global__ void check_min(unsigned* res) {
    // xorshift per thread; values spread over every exponent incl. denormals and 0
    unsigned x = 2463534242u ^ (blockIdx.x * 256 + threadIdx.x) * 2654435761u;
    unsigned bad = 0, n = 0;
    for (int i = 0; i < 64; ++i) {
        unsigned v[3];
        for (int j = 0; j < 3; ++j) {
            x ^= x << 13; x ^= x >> 17; x ^= x << 5;
            unsigned sh = x & 31;
            v[j] = (x >> sh) % 0x3FBFFFFFu * ((x >> 7) & 1 ? 2u : 1u);  // <= 0x7F7FFFFE
        }
        unsigned rf, ru;
        asm volatile("v_min3_f32 %0, %1, %2, %3" : "=v"(rf) : "v"(v[0]), "v"(v[1]), "v"(v[2]));
        asm volatile("v_min3_u32 %0, %1, %2, %3" : "=v"(ru) : "v"(v[0]), "v"(v[1]), "v"(v[2]));
        bad += rf != ru;
        ++n;
    }
    atomicAdd(&res[0], bad);
    atomicAdd(&res[1], n);
}

template <int MODE>
void run(const char* name, int ninstr) {
    unsigned* out;
    hipMalloc(&out, 256 * 4096 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = 256 * 8;  // 8 WGs of 4 waves per CU -> 8 waves per SIMD
    k<MODE><<<blocks, 256>>>(out, 1);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) k<MODE><<<blocks, 256>>>(out, r + 2);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    // wave-instructions issued: blocks * 4 waves * N_ITER * 8 chains * (ninstr + 1 xor)
    const double winst = 5.0 * blocks * 4 * (double)N_ITER * 8 * (ninstr + 1);
    const double per_simd_cycle = winst / (1024.0 * ms * 1e-3 * 2.4e9);  // at 2.4 GHz
    printf("%-34s %8.3f ms  %.3f wave-instr/SIMD/cycle@2.4GHz (peak 0.5)\n", name, ms, per_simd_cycle);
    hipFree(out);
}

int main() {
    {
        unsigned* z;
        hipMalloc(&z, 16);
        hipMemset(z, 0, 16);
        hipFree(z);
    }
    run<0>("add_clamp x2 + min3", 3);
    run<1>("add_e32 x2 + min3", 3);
    run<2>("add_e32 x2 + min_e32 x2", 4);
    run<3>("add_clamp x3", 3);
    run<4>("min3 x3", 3);
    run<5>("add_e32 x3", 3);
    run<6>("add_e32 x2 + min3_f32", 3);
    run<7>("min3_f32 x3", 3);
    run<8>("min_f32_e32 x3", 3);
    run<9>("min_u32_e32 x3", 3);
    run<10>("min_i32_e32 x3", 3);
    run64<0>("lshl_add_u64 + min3 (2 relax)", 2);
    run64<1>("lshl_add_u64 x3", 3);
    run64<2>("u64 '+' (compiler) + min3", 2);
    // exactness: v_min3_f32 on u32 bit patterns in [0, 2^31) incl. the denormal range
    unsigned *d;
    hipMalloc(&d, 4 * 3);
    hipMemset(d, 0, 12);
    hipLaunchKernelGGL(check_min, dim3(4096), dim3(256), 0, 0, d);
    unsigned h[3];
    hipMemcpy(h, d, 12, hipMemcpyDeviceToHost);
    printf("min3_f32 vs min3_u32 mismatches over 1M random triples (< 0x7F7FFFFF): %u (checked %u)\n", h[0], h[1]);
    return 0;
}
