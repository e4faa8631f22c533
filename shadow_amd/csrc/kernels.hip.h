// kernels.hip.h — HIP kernels (gfx950) of the dense routing-table path.
//
// Data layout in HBM (Vp = V rounded up to the FW tile, row-major, row stride Vp):
//   W   [Vp x Vp] K     lexicographic-min (latency) of all non-self-loop edges u->t,
//                        INF where there is none (diagonal INF).  Undirected edges fill
//                        both (u,t) and (t,u).            -> edge weight, mod.rs:333-340
//   WL  [Vp x Vp] u32   f32 bits of the min packet_loss among the min-latency parallel
//                        edges u->t (lexicographic PathProperties order, mod.rs:305-313)
//   D   [Vp x Vp] K     W with diagonal 0, then closed by blocked Floyd-Warshall.
//   PRED[n  x Vp] u32   per used source row: the unique tight predecessor of t, or MULTI
//   L   [n  x Vp] f32   left-fold loss per used source row (two buffers, Jacobi rounds)
// K = uint32_t (saturating add: exact for every distance < 2^32-1, certified on the host)
//   or uint64_t (INF = 2^62, exact for every distance < 2^62).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace srg {

constexpr uint32_t PRED_NONE = 0xFFFFFFFFu;   // t == s or t unreachable from s
constexpr uint32_t PRED_MULTI = 0xFFFFFFFEu;  // more than one tight predecessor

template <class K>
struct KeyOps;

template <>
struct KeyOps<uint32_t> {
    static constexpr uint32_t INF = 0xFFFFFFFFu;
    __device__ __forceinline__ static uint32_t add(uint32_t a, uint32_t b) {
        return __builtin_elementwise_add_sat(a, b);  // v_add_u32 ... clamp
    }
    __device__ __forceinline__ static uint32_t min2(uint32_t a, uint32_t b) { return a < b ? a : b; }
    __device__ __forceinline__ static uint32_t min3(uint32_t a, uint32_t b, uint32_t c) {
        // one v_min3_u32 (hipcc otherwise re-associates a min chain into a v_min tree:
        // 1.75 instead of 1.5 VALU ops per relaxation)
        uint32_t r;
        asm("v_min3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
        return r;
    }
};

template <>
struct KeyOps<uint64_t> {
    static constexpr uint64_t INF = 1ull << 62;
    __device__ __forceinline__ static uint64_t add(uint64_t a, uint64_t b) { return a + b; }
    __device__ __forceinline__ static uint64_t min2(uint64_t a, uint64_t b) { return a < b ? a : b; }
    __device__ __forceinline__ static uint64_t min3(uint64_t a, uint64_t b, uint64_t c) {
        return min2(min2(a, b), c);
    }
};

// Left-fold PathProperties::add on the loss (mod.rs:328): 1 - (1-a)*(1-b), each op rounded,
// no FMA contraction (the library is also compiled with -ffp-contract=off).
__device__ __forceinline__ float fold_loss(float path_loss, float one_minus_p) {
    float x = __fsub_rn(1.0f, path_loss);
    float y = __fmul_rn(x, one_minus_p);
    return __fsub_rn(1.0f, y);
}

// ---------------------------------------------------------------------------------------
// Tile geometry shared by the FW product kernels: a T x T output tile per 256-thread
// workgroup, 16 x 16 threads, each thread an M x M micro-tile (M = T/16) split in two
// halves so that every LDS/global vector access is 16 B per lane and conflict-free:
//   row(a) = (a < M/2) ? ty*M/2 + a : T/2 + ty*M/2 + (a - M/2)      (same for columns)
template <class K, int T>
struct Geo {
    static constexpr int M = T / 16;
    static constexpr int H = M / 2;       // elements per half (one 8- or 16-byte vector)
    static_assert(H * (int)sizeof(K) == 16 || H * (int)sizeof(K) == 8, "half = 8 or 16 bytes");
    __device__ __forceinline__ static int rc(int t, int a) {
        return (a < H) ? t * H + a : T / 2 + t * H + (a - H);
    }
};

template <class K, int N>
struct alignas(N * sizeof(K)) VecN {
    K v[N];
};
template <class K>
using Vec16 = VecN<K, 16 / sizeof(K)>;

template <class K, int N = 16 / sizeof(K)>
__device__ __forceinline__ VecN<K, N> ldv(const K* p) {
    return *reinterpret_cast<const VecN<K, N>*>(p);
}
template <class K, int N>
__device__ __forceinline__ void stv(K* p, const VecN<K, N>& v) {
    *reinterpret_cast<VecN<K, N>*>(p) = v;
}
template <class K>
__device__ __forceinline__ Vec16<K> ld16(const K* p) { return ldv<K>(p); }
template <class K>
__device__ __forceinline__ void st16(K* p, const Vec16<K>& v) { stv<K, 16 / sizeof(K)>(p, v); }

// ---------------------------------------------------------------------------------------
// Phase 1: close the pivot block D[kb][kb] (sequential k inside one workgroup).
// The T x T block lives in registers (M x M per thread).  Step k needs only row k and
// column k, so after updating, the owners of row k+1 / column k+1 publish them into a
// parity double-buffered LDS strip (step k reads buffer k&1, writes buffer (k+1)&1):
// one barrier per step and 2*T LDS words written instead of the whole block.
template <class K, int T>
__global__ void __launch_bounds__(256) fw_phase1(K* __restrict__ D, size_t ld, int kb) {
    using G = Geo<K, T>;
    constexpr int M = G::M;
    __shared__ __attribute__((aligned(16))) K prow[2][T];
    __shared__ __attribute__((aligned(16))) K pcol[2][T];
    const int tid = threadIdx.x, ty = tid >> 4, tx = tid & 15;
    K* base = D + (size_t)kb * T * ld + (size_t)kb * T;
    K c[M][M];
#pragma unroll
    for (int a = 0; a < M; ++a) {
        const int r = G::rc(ty, a);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            VecN<K, G::H> v = ldv<K, G::H>(base + (size_t)r * ld + G::rc(tx, h * G::H));
#pragma unroll
            for (int e = 0; e < G::H; ++e) c[a][h * G::H + e] = v.v[e];
        }
    }
    // publish row 0 / column 0
#pragma unroll
    for (int a = 0; a < M; ++a) {
        if (G::rc(ty, a) == 0) {
#pragma unroll
            for (int b = 0; b < M; ++b) prow[0][G::rc(tx, b)] = c[a][b];
        }
        if (G::rc(tx, a) == 0) {
#pragma unroll
            for (int b = 0; b < M; ++b) pcol[0][G::rc(ty, b)] = c[b][a];
        }
    }
    __syncthreads();
    for (int k = 0; k < T; ++k) {
        const int p = k & 1;
        K colk[M], rowk[M];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            VecN<K, G::H> vc = ldv<K, G::H>(&pcol[p][G::rc(ty, h * G::H)]);
            VecN<K, G::H> vr = ldv<K, G::H>(&prow[p][G::rc(tx, h * G::H)]);
#pragma unroll
            for (int e = 0; e < G::H; ++e) {
                colk[h * G::H + e] = vc.v[e];
                rowk[h * G::H + e] = vr.v[e];
            }
        }
#pragma unroll
        for (int a = 0; a < M; ++a)
#pragma unroll
            for (int b = 0; b < M; ++b) c[a][b] = KeyOps<K>::min2(c[a][b], KeyOps<K>::add(colk[a], rowk[b]));
        if (k + 1 < T) {
            const int q = (k + 1) & 1;
#pragma unroll
            for (int a = 0; a < M; ++a) {
                if (G::rc(ty, a) == k + 1) {
#pragma unroll
                    for (int b = 0; b < M; ++b) prow[q][G::rc(tx, b)] = c[a][b];
                }
                if (G::rc(tx, a) == k + 1) {
#pragma unroll
                    for (int b = 0; b < M; ++b) pcol[q][G::rc(ty, b)] = c[b][a];
                }
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int a = 0; a < M; ++a)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            VecN<K, G::H> v;
#pragma unroll
            for (int e = 0; e < G::H; ++e) v.v[e] = c[a][h * G::H + e];
            stv<K, G::H>(base + (size_t)G::rc(ty, a) * ld + G::rc(tx, h * G::H), v);
        }
}

// Stage a KC x T chunk of A^T (A rows i, columns k0..k0+KC) and of B (rows k0.., cols j)
// into LDS.  A rows may be gathered through `arow` (row index per tile row).
template <class K, int T, int KC>
__device__ __forceinline__ void stage_chunk(K* __restrict__ At, K* __restrict__ Bs,
                                            const K* __restrict__ A, const K* __restrict__ B,
                                            size_t ld, const uint32_t* arow_idx, int k0) {
    constexpr int VE = 16 / (int)sizeof(K);     // elements per 16-B vector
    constexpr int LDP = T + VE;                 // padded LDS row (keeps 16-B alignment)
    const int tid = threadIdx.x;
    // A^T: each thread reads 16 B along k of one row, scatters it transposed
    constexpr int AV = T * KC / VE;             // vectors in the A chunk
#pragma unroll
    for (int q = tid; q < AV; q += 256) {
        const int i = q / (KC / VE);
        const int kq = q % (KC / VE);
        const K* src = A + (size_t)arow_idx[i] * ld + k0 + kq * VE;
        Vec16<K> v = ld16(src);
#pragma unroll
        for (int e = 0; e < VE; ++e) At[(kq * VE + e) * LDP + i] = v.v[e];
    }
    constexpr int BV = KC * T / VE;
#pragma unroll
    for (int q = tid; q < BV; q += 256) {
        const int kk = q / (T / VE);
        const int jq = q % (T / VE);
        Vec16<K> v = ld16(B + (size_t)(k0 + kk) * ld + jq * VE);
        st16(Bs + kk * LDP + jq * VE, v);
    }
}

// Phase 2 / 3: C = min(C, A (x) B) over the kb pivot block (min-plus product), for the
// tiles (I, J) of a TileSet:  C = D[I][J],  A = D[I][kb],  B = D[kb][J].
//   row panel (I = kb):  A = D[kb][kb] (the closed pivot tile), B = C
//   col panel (J = kb):  A = C,  B = D[kb][kb]
//   phase 3:             I, J != kb
// With D[kb][kb] closed (phase 1) one product is exact for the panels; every product reads
// all of A and B before the tile is stored, so the in-place row/col panel is race-free.
//
// Staging: the k range is cut into KC-wide chunks held in a double-buffered LDS image
// (A transposed, B as is, rows padded by one 16-B vector).  Chunk i+1's global loads are
// issued into registers before chunk i is computed and written to the other LDS buffer
// after it (issue early / write late), so one barrier per chunk separates the phases.
template <class K, int T, int KC>
struct Stage {
    static constexpr int VE = 16 / (int)sizeof(K);  // elements per 16-B vector
    static constexpr int AV = T * KC / VE / 256;    // A vectors per thread per chunk
    static constexpr int BV = KC * T / VE / 256;    // B vectors per thread per chunk
    Vec16<K> a[AV], b[BV];
};

template <class K, int T, int KC>
__device__ __forceinline__ void stage_load(Stage<K, T, KC>& sg, const K* __restrict__ A, const K* __restrict__ B,
                                           size_t ld, const uint32_t* arow_idx, int k0) {
    using S = Stage<K, T, KC>;
    const int tid = threadIdx.x;
#pragma unroll
    for (int q = 0; q < S::AV; ++q) {
        const int v = tid + 256 * q;
        const int i = v / (KC / S::VE), kq = v % (KC / S::VE);
        sg.a[q] = ld16(A + (size_t)arow_idx[i] * ld + k0 + kq * S::VE);
    }
#pragma unroll
    for (int q = 0; q < S::BV; ++q) {
        const int v = tid + 256 * q;
        const int kk = v / (T / S::VE), jq = v % (T / S::VE);
        sg.b[q] = ld16(B + (size_t)(k0 + kk) * ld + jq * S::VE);
    }
}

template <class K, int T, int KC>
__device__ __forceinline__ void stage_store(const Stage<K, T, KC>& sg, K* __restrict__ At, K* __restrict__ Bs) {
    using S = Stage<K, T, KC>;
    constexpr int LDP = T + S::VE;
    const int tid = threadIdx.x;
#pragma unroll
    for (int q = 0; q < S::AV; ++q) {
        const int v = tid + 256 * q;
        const int i = v / (KC / S::VE), kq = v % (KC / S::VE);
#pragma unroll
        for (int e = 0; e < S::VE; ++e) At[(kq * S::VE + e) * LDP + i] = sg.a[q].v[e];
    }
#pragma unroll
    for (int q = 0; q < S::BV; ++q) {
        const int v = tid + 256 * q;
        const int kk = v / (T / S::VE), jq = v % (T / S::VE);
        st16(Bs + kk * LDP + jq * S::VE, sg.b[q]);
    }
}

// A TileSet is a rectangle of tiles minus at most two whole rows and two whole columns
// (pivot rows/columns handled elsewhere):  kept row y -> r0 + y, stepping over rx0 < rx1
// (-1 = none); kept column x likewise.  grid = (kept columns, kept rows).
struct TileSet {
    int r0, rx0, rx1;
    int c0, cx0, cx1;
};

__device__ __forceinline__ int tile_kept(int base, int idx, int x0, int x1) {
    int v = base + idx;
    if (x0 >= 0 && v >= x0) ++v;
    if (x1 >= 0 && v >= x1) ++v;
    return v;
}

template <class K, int T, int KC>
__global__ void __launch_bounds__(256) fw_product(K* __restrict__ D, size_t ld, int kb, TileSet ts) {
    using G = Geo<K, T>;
    constexpr int M = G::M;
    constexpr int VE = 16 / (int)sizeof(K);
    constexpr int LDP = T + VE;
    constexpr int BUF = 2 * KC * LDP;  // elements per LDS buffer (A^T + B)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    K* lds = reinterpret_cast<K*>(smem_raw);
    __shared__ uint32_t arow[T];

    const int I = tile_kept(ts.r0, (int)blockIdx.y, ts.rx0, ts.rx1);
    const int J = tile_kept(ts.c0, (int)blockIdx.x, ts.cx0, ts.cx1);
    K* C = D + (size_t)I * T * ld + (size_t)J * T;
    const K* A = D + (size_t)kb * T;                       // column block kb, rows via arow
    const K* B = D + (size_t)kb * T * ld + (size_t)J * T;  // row block kb, cols J
    const int tid = threadIdx.x, ty = tid >> 4, tx = tid & 15;
    if (tid < T) arow[tid] = I * T + tid;
    __syncthreads();

    Stage<K, T, KC> sg;
    stage_load<K, T, KC>(sg, A, B, ld, arow, 0);
    K c[M][M];
#pragma unroll
    for (int a = 0; a < M; ++a)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            VecN<K, G::H> v = ldv<K, G::H>(C + (size_t)G::rc(ty, a) * ld + G::rc(tx, h * G::H));
#pragma unroll
            for (int e = 0; e < G::H; ++e) c[a][h * G::H + e] = v.v[e];
        }
    stage_store<K, T, KC>(sg, lds, lds + KC * LDP);
    __syncthreads();
    constexpr int NCH = T / KC;
#pragma unroll 1
    for (int ch = 0; ch < NCH; ++ch) {
        const K* At = lds + (ch & 1) * BUF;
        const K* Bs = At + KC * LDP;
        if (ch + 1 < NCH) stage_load<K, T, KC>(sg, A, B, ld, arow, (ch + 1) * KC);  // issue early
#pragma unroll 4
        for (int kk = 0; kk < KC; kk += 2) {
            K a0[M], a1[M], b0[M], b1[M];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                VecN<K, G::H> va0 = ldv<K, G::H>(At + kk * LDP + G::rc(ty, h * G::H));
                VecN<K, G::H> va1 = ldv<K, G::H>(At + (kk + 1) * LDP + G::rc(ty, h * G::H));
                VecN<K, G::H> vb0 = ldv<K, G::H>(Bs + kk * LDP + G::rc(tx, h * G::H));
                VecN<K, G::H> vb1 = ldv<K, G::H>(Bs + (kk + 1) * LDP + G::rc(tx, h * G::H));
#pragma unroll
                for (int e = 0; e < G::H; ++e) {
                    a0[h * G::H + e] = va0.v[e];
                    a1[h * G::H + e] = va1.v[e];
                    b0[h * G::H + e] = vb0.v[e];
                    b1[h * G::H + e] = vb1.v[e];
                }
            }
#pragma unroll
            for (int a = 0; a < M; ++a)
#pragma unroll
                for (int b = 0; b < M; ++b)
                    c[a][b] = KeyOps<K>::min3(c[a][b], KeyOps<K>::add(a0[a], b0[b]),
                                              KeyOps<K>::add(a1[a], b1[b]));
        }
        if (ch + 1 < NCH) {  // write late into the other buffer
            K* Ant = lds + ((ch + 1) & 1) * BUF;
            stage_store<K, T, KC>(sg, Ant, Ant + KC * LDP);
        }
        __syncthreads();
    }
#pragma unroll
    for (int a = 0; a < M; ++a)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            VecN<K, G::H> v;
#pragma unroll
            for (int e = 0; e < G::H; ++e) v.v[e] = c[a][h * G::H + e];
            stv<K, G::H>(C + (size_t)G::rc(ty, a) * ld + G::rc(tx, h * G::H), v);
        }
}

// ---------------------------------------------------------------------------------------
// Tight-predecessor scan.  For used source row r (s = nodes[r]) and every column t:
//   tight(u) <=> D[s][u] + W[u][t] == D[s][t]   (Bellman equation of the closed D)
// PRED[r][t] = the tight u when exactly one exists, PRED_MULTI when several, PRED_NONE for
// t == s or D[s][t] == INF.  These u are exactly the predecessors whose (latency-equal)
// scores petgraph's Dijkstra compares by packet_loss (mod.rs:305-313 strict-< update).
template <class K, int T, int KC>
__global__ void __launch_bounds__(256) tight_scan(const K* __restrict__ D, const K* __restrict__ W,
                                                   size_t ld, const uint32_t* __restrict__ nodes,
                                                   uint32_t n, uint32_t* __restrict__ PRED) {
    using G = Geo<K, T>;
    constexpr int M = G::M;
    constexpr int VE = 16 / (int)sizeof(K);
    constexpr int LDP = T + VE;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    K* At = reinterpret_cast<K*>(smem_raw);
    K* Bs = At + KC * LDP;
    __shared__ uint32_t arow[T];
    const int tid = threadIdx.x, ty = tid >> 4, tx = tid & 15;
    const int r0 = blockIdx.y * T;           // used-row block
    const int J = blockIdx.x;                // column block
    if (tid < T) {
        uint32_t r = r0 + tid;
        arow[tid] = nodes[r < n ? r : n - 1];
    }
    __syncthreads();
    K dst[M][M];
    uint32_t cnt[M][M], last[M][M];
#pragma unroll
    for (int a = 0; a < M; ++a)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            VecN<K, G::H> v = ldv<K, G::H>(D + (size_t)arow[G::rc(ty, a)] * ld + (size_t)J * T + G::rc(tx, h * G::H));
#pragma unroll
            for (int e = 0; e < G::H; ++e) {
                dst[a][h * G::H + e] = v.v[e];
                cnt[a][h * G::H + e] = 0;
                last[a][h * G::H + e] = PRED_NONE;
            }
        }
    const size_t Vp = ld;
    for (size_t u0 = 0; u0 < Vp; u0 += KC) {
        __syncthreads();
        stage_chunk<K, T, KC>(At, Bs, D, W + (size_t)J * T, ld, arow, (int)u0);
        __syncthreads();
        for (int kk = 0; kk < KC; ++kk) {
            K av[M], bv[M];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                VecN<K, G::H> va = ldv<K, G::H>(At + kk * LDP + G::rc(ty, h * G::H));
                VecN<K, G::H> vb = ldv<K, G::H>(Bs + kk * LDP + G::rc(tx, h * G::H));
#pragma unroll
                for (int e = 0; e < G::H; ++e) {
                    av[h * G::H + e] = va.v[e];
                    bv[h * G::H + e] = vb.v[e];
                }
            }
            const uint32_t u = (uint32_t)(u0 + kk);
#pragma unroll
            for (int a = 0; a < M; ++a)
#pragma unroll
                for (int b = 0; b < M; ++b) {
                    const bool eq = KeyOps<K>::add(av[a], bv[b]) == dst[a][b];
                    cnt[a][b] += eq ? 1u : 0u;
                    last[a][b] = eq ? u : last[a][b];
                }
        }
    }
#pragma unroll
    for (int a = 0; a < M; ++a) {
        const int rr = r0 + G::rc(ty, a);
        if (rr >= (int)n) continue;
        const uint32_t s = arow[G::rc(ty, a)];
#pragma unroll
        for (int b = 0; b < M; ++b) {
            const uint32_t t = (uint32_t)(J * T + G::rc(tx, b));
            uint32_t p = cnt[a][b] == 1 ? last[a][b] : PRED_MULTI;
            if (t == s || dst[a][b] == KeyOps<K>::INF) p = PRED_NONE;
            if (cnt[a][b] == 0 && p != PRED_NONE) p = PRED_NONE;  // unreachable padding
            PRED[(size_t)rr * ld + t] = p;
        }
    }
}

}  // namespace srg
