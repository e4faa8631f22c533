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
// Phase 1: close the pivot block D[kb][kb] (the sequential k chain of FW; on the critical
// path of the multi-GPU schedule, so it is latency-optimised).
// 512 threads (2 waves per SIMD), thread (ty < 32, tx < 16) holds MR = T/32 rows x MC = T/16
// columns in registers.  The k steps run in groups of R = 4 per barrier: at the start of a
// group every thread reads the group's R pivot rows (its MC columns), R pivot columns (its
// MR rows) and the R x R pivot sub-block from LDS, replays the group's R steps on those
// cross values (tiny), and then folds all R steps into its own elements at once:
//   c = min(c, C_0 + R_0, ..., C_{R-1} + R_{R-1})   (C_i, R_i = step-i values; v_min3 pairs)
// which equals R sequential FW steps.  The owners then publish the next group's rows and
// columns into the other half of a double-buffered LDS strip.
template <class K, int T>
struct P1Geo {
    static constexpr int MR = T / 32, MC = T / 16;
    static constexpr int HR = MR / 2, HC = MC / 2;
    __device__ __forceinline__ static int row(int ty, int a) { return a < HR ? ty * HR + a : T / 2 + ty * HR + (a - HR); }
    __device__ __forceinline__ static int col(int tx, int b) { return b < HC ? tx * HC + b : T / 2 + tx * HC + (b - HC); }
};

template <class K, int T>
__global__ void __launch_bounds__(512) fw_phase1(K* __restrict__ D, size_t ld, int kb) {
    using G = P1Geo<K, T>;
    constexpr int MR = G::MR, MC = G::MC, HR = G::HR, HC = G::HC;
    constexpr int R = 4;
    __shared__ __attribute__((aligned(16))) K prow[2][R][T];  // prow[.][j][col] = D[k0+j][col]
    __shared__ __attribute__((aligned(16))) K pcol[2][R][T];  // pcol[.][j][row] = D[row][k0+j]
    const int tid = threadIdx.x, ty = tid >> 4, tx = tid & 15;
    K* base = D + (size_t)kb * T * ld + (size_t)kb * T;
    K c[MR][MC];
#pragma unroll
    for (int a = 0; a < MR; ++a)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            VecN<K, HC> v = ldv<K, HC>(base + (size_t)G::row(ty, a) * ld + G::col(tx, h * HC));
#pragma unroll
            for (int e = 0; e < HC; ++e) c[a][h * HC + e] = v.v[e];
        }
    auto publish = [&](int q, int k0) {
#pragma unroll
        for (int a = 0; a < MR; ++a) {
            const int r = G::row(ty, a) - k0;
            if (r >= 0 && r < R) {
#pragma unroll
                for (int b = 0; b < MC; ++b) prow[q][r][G::col(tx, b)] = c[a][b];
            }
        }
#pragma unroll
        for (int b = 0; b < MC; ++b) {
            const int j = G::col(tx, b) - k0;
            if (j >= 0 && j < R) {
#pragma unroll
                for (int a = 0; a < MR; ++a) pcol[q][j][G::row(ty, a)] = c[a][b];
            }
        }
    };
    publish(0, 0);
    __syncthreads();
    for (int g = 0; g < T / R; ++g) {
        const int q = g & 1, k0 = g * R;
        K Rv[R][MC], Cv[MR][R], Pv[R][R];
#pragma unroll
        for (int j = 0; j < R; ++j) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                VecN<K, HC> vr = ldv<K, HC>(&prow[q][j][G::col(tx, h * HC)]);
                VecN<K, HR> vc = ldv<K, HR>(&pcol[q][j][G::row(ty, h * HR)]);
#pragma unroll
                for (int e = 0; e < HC; ++e) Rv[j][h * HC + e] = vr.v[e];
#pragma unroll
                for (int e = 0; e < HR; ++e) Cv[h * HR + e][j] = vc.v[e];
            }
#pragma unroll
            for (int i = 0; i < R; ++i) Pv[j][i] = prow[q][j][k0 + i];
        }
        // replay the group's steps on the cross values
#pragma unroll
        for (int i = 0; i < R; ++i) {
#pragma unroll
            for (int x = i + 1; x < R; ++x)
#pragma unroll
                for (int b = 0; b < MC; ++b) Rv[x][b] = KeyOps<K>::min2(Rv[x][b], KeyOps<K>::add(Pv[x][i], Rv[i][b]));
#pragma unroll
            for (int y = i + 1; y < R; ++y)
#pragma unroll
                for (int a = 0; a < MR; ++a) Cv[a][y] = KeyOps<K>::min2(Cv[a][y], KeyOps<K>::add(Cv[a][i], Pv[i][y]));
#pragma unroll
            for (int x = i + 1; x < R; ++x)
#pragma unroll
                for (int y = i + 1; y < R; ++y) Pv[x][y] = KeyOps<K>::min2(Pv[x][y], KeyOps<K>::add(Pv[x][i], Pv[i][y]));
        }
        // fold the R steps into the own elements
#pragma unroll
        for (int a = 0; a < MR; ++a)
#pragma unroll
            for (int b = 0; b < MC; ++b) {
                K v = KeyOps<K>::min3(c[a][b], KeyOps<K>::add(Cv[a][0], Rv[0][b]), KeyOps<K>::add(Cv[a][1], Rv[1][b]));
                c[a][b] = KeyOps<K>::min3(v, KeyOps<K>::add(Cv[a][2], Rv[2][b]), KeyOps<K>::add(Cv[a][3], Rv[3][b]));
            }
        if (g + 1 < T / R) publish(q ^ 1, k0 + R);
        __syncthreads();
    }
#pragma unroll
    for (int a = 0; a < MR; ++a)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            VecN<K, HC> v;
#pragma unroll
            for (int e = 0; e < HC; ++e) v.v[e] = c[a][h * HC + e];
            stv<K, HC>(base + (size_t)G::row(ty, a) * ld + G::col(tx, h * HC), v);
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

// gridDim.z > 1 splits the pivot block's k range across workgroups (split-K): each split
// reduces its share and merges with atomicMin, which is exact because min is associative and
// commutative (used for the short launches on the multi-GPU critical path).
template <class K, int T, int KC>
__device__ __forceinline__ void fw_tile(K* __restrict__ D, size_t ld, int kb, int I, int J);

template <class K, int T, int KC>
__global__ void __launch_bounds__(256) fw_product(K* __restrict__ D, size_t ld, int kb, TileSet ts) {
    fw_tile<K, T, KC>(D, ld, kb, tile_kept(ts.r0, (int)blockIdx.y, ts.rx0, ts.rx1),
                      tile_kept(ts.c0, (int)blockIdx.x, ts.cx0, ts.cx1));
}

// Two tile sets in one launch (the pivot's row panel and column panel: they are independent
// once the pivot tile is closed, and each is a single short wave of workgroups, so one launch
// instead of two takes a tile latency off the FW critical path).  grid.x = na + nb tiles;
// set s is nc_s columns wide, tiles flattened row-major.
template <class K, int T, int KC>
__global__ void __launch_bounds__(256) fw_product_pair(K* __restrict__ D, size_t ld, int kb, TileSet a, int na,
                                                       int nca, TileSet b, int ncb) {
    int x = (int)blockIdx.x;
    const TileSet& t = x < na ? a : b;
    const int nc = x < na ? nca : ncb;
    if (x >= na) x -= na;
    fw_tile<K, T, KC>(D, ld, kb, tile_kept(t.r0, x / nc, t.rx0, t.rx1), tile_kept(t.c0, x % nc, t.cx0, t.cx1));
}

template <class K, int T, int KC>
__device__ __forceinline__ void fw_tile(K* __restrict__ D, size_t ld, int kb, int I, int J) {
    using G = Geo<K, T>;
    constexpr int M = G::M;
    constexpr int VE = 16 / (int)sizeof(K);
    constexpr int LDP = T + VE;
    constexpr int BUF = 2 * KC * LDP;  // elements per LDS buffer (A^T + B)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    K* lds = reinterpret_cast<K*>(smem_raw);
    __shared__ uint32_t arow[T];
    K* C = D + (size_t)I * T * ld + (size_t)J * T;
    const K* A = D + (size_t)kb * T;                       // column block kb, rows via arow
    const K* B = D + (size_t)kb * T * ld + (size_t)J * T;  // row block kb, cols J
    const int tid = threadIdx.x, ty = tid >> 4, tx = tid & 15;
    if (tid < T) arow[tid] = I * T + tid;
    __syncthreads();

    constexpr int NCH = T / KC;
    const int nsplit = (int)gridDim.z;
    const int ch0 = (int)blockIdx.z * NCH / nsplit, ch1 = ((int)blockIdx.z + 1) * NCH / nsplit;
    Stage<K, T, KC> sg;
    stage_load<K, T, KC>(sg, A, B, ld, arow, ch0 * KC);
    K c[M][M];
    if (nsplit == 1) {
#pragma unroll
        for (int a = 0; a < M; ++a)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                VecN<K, G::H> v = ldv<K, G::H>(C + (size_t)G::rc(ty, a) * ld + G::rc(tx, h * G::H));
#pragma unroll
                for (int e = 0; e < G::H; ++e) c[a][h * G::H + e] = v.v[e];
            }
    } else {
#pragma unroll
        for (int a = 0; a < M; ++a)
#pragma unroll
            for (int b = 0; b < M; ++b) c[a][b] = KeyOps<K>::INF;
    }
    stage_store<K, T, KC>(sg, lds, lds + KC * LDP);
    __syncthreads();
#pragma unroll 1
    for (int ch = ch0; ch < ch1; ++ch) {
        const K* At = lds + ((ch - ch0) & 1) * BUF;
        const K* Bs = At + KC * LDP;
        if (ch + 1 < ch1) stage_load<K, T, KC>(sg, A, B, ld, arow, (ch + 1) * KC);  // issue early
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
        if (ch + 1 < ch1) {  // write late into the other buffer
            K* Ant = lds + ((ch + 1 - ch0) & 1) * BUF;
            stage_store<K, T, KC>(sg, Ant, Ant + KC * LDP);
        }
        __syncthreads();
    }
    if (nsplit == 1) {
#pragma unroll
        for (int a = 0; a < M; ++a)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                VecN<K, G::H> v;
#pragma unroll
                for (int e = 0; e < G::H; ++e) v.v[e] = c[a][h * G::H + e];
                stv<K, G::H>(C + (size_t)G::rc(ty, a) * ld + G::rc(tx, h * G::H), v);
            }
    } else {
#pragma unroll
        for (int a = 0; a < M; ++a)
#pragma unroll
            for (int b = 0; b < M; ++b) atomicMin(C + (size_t)G::rc(ty, a) * ld + G::rc(tx, b), c[a][b]);
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
