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
// K = uint32_t (INF = 2^31-1: exact for every distance < INF, certified on the host)
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
    // INF = 2^31 - 1: every stored key is <= INF, so the sum of two keys never exceeds 2^32 - 2.
    // That lets the FW product add two packed keys per 64-bit add with no carry between the
    // halves (fw_tile_pk); the saturating add below then never saturates, and a used-row key
    // equal to INF (unreachable, or a path >= 2^31 - 1 ns) sends the build to the u64 keys.
    static constexpr uint32_t INF = 0x7FFFFFFFu;
    __device__ __forceinline__ static uint32_t add(uint32_t a, uint32_t b) {
        return __builtin_elementwise_add_sat(a, b);  // v_add_u32 ... clamp
    }
    // keys <= INF: the sum never wraps, so the FW tiles use the plain (VOP2, full-rate) add
    __device__ __forceinline__ static uint32_t add_nw(uint32_t a, uint32_t b) { return a + b; }
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
    __device__ __forceinline__ static uint64_t add_nw(uint64_t a, uint64_t b) { return a + b; }
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
template <class K, int T, int NTH = 512>
struct P1Geo {
    static constexpr int MR = T / (NTH / 16), MC = T / 16;
    static constexpr int HR = MR / 2, HC = MC / 2;
    __device__ __forceinline__ static int row(int ty, int a) { return a < HR ? ty * HR + a : T / 2 + ty * HR + (a - HR); }
    __device__ __forceinline__ static int col(int tx, int b) { return b < HC ? tx * HC + b : T / 2 + tx * HC + (b - HC); }
};

template <class K, int T, int NTH = 512>
__device__ __forceinline__ void phase1_body(K* __restrict__ base, size_t ld, int prio) {
    // prio: the chain runs beside the bulk tiles; a raised wave priority wins the VALU issue
    // arbitration on the SIMDs it shares with them (MI355X_MICROARCH.md, waves per SIMD)
    if (prio) __builtin_amdgcn_s_setprio(3);
    using G = P1Geo<K, T, NTH>;
    constexpr int MR = G::MR, MC = G::MC, HR = G::HR, HC = G::HC;
    static_assert(HR >= 1, "phase-1 geometry");
    constexpr int R = 4;
    __shared__ __attribute__((aligned(16))) K prow[2][R][T];  // prow[.][j][col] = D[k0+j][col]
    __shared__ __attribute__((aligned(16))) K pcol[2][R][T];  // pcol[.][j][row] = D[row][k0+j]
    const int tid = threadIdx.x, ty = tid >> 4, tx = tid & 15;
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
                for (int b = 0; b < MC; ++b) Rv[x][b] = KeyOps<K>::min2(Rv[x][b], KeyOps<K>::add_nw(Pv[x][i], Rv[i][b]));
#pragma unroll
            for (int y = i + 1; y < R; ++y)
#pragma unroll
                for (int a = 0; a < MR; ++a) Cv[a][y] = KeyOps<K>::min2(Cv[a][y], KeyOps<K>::add_nw(Cv[a][i], Pv[i][y]));
#pragma unroll
            for (int x = i + 1; x < R; ++x)
#pragma unroll
                for (int y = i + 1; y < R; ++y) Pv[x][y] = KeyOps<K>::min2(Pv[x][y], KeyOps<K>::add_nw(Pv[x][i], Pv[i][y]));
        }
        // fold the R steps into the own elements
#pragma unroll
        for (int a = 0; a < MR; ++a)
#pragma unroll
            for (int b = 0; b < MC; ++b) {
                K v = KeyOps<K>::min3(c[a][b], KeyOps<K>::add_nw(Cv[a][0], Rv[0][b]), KeyOps<K>::add_nw(Cv[a][1], Rv[1][b]));
                c[a][b] = KeyOps<K>::min3(v, KeyOps<K>::add_nw(Cv[a][2], Rv[2][b]), KeyOps<K>::add_nw(Cv[a][3], Rv[3][b]));
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

template <class K, int T, int NTH = 512>
__global__ void __launch_bounds__(NTH) fw_phase1(K* __restrict__ D, size_t ld, int kb, int prio) {
    phase1_body<K, T, NTH>(D + (size_t)kb * T * ld + (size_t)kb * T, ld, prio);
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
template <class K, int T, int KC, int PK>
__device__ __forceinline__ void fw_tile(K* __restrict__ D, size_t ld, int kb, int I, int J);

// PK (tile variant, SRG_OPT_FW_PACKED): 0 = add + min3 (any key); 2 = u32 keys only, the
// pair-packed tile below (fw_tile_pk) with 16-deep k-chunks and a register budget for 3 waves
// per SIMD (the other waves hide the LDS latency; LDS 33 KB per workgroup).  Variants with
// 32-deep chunks or an operand prefetch measured slower and were removed.
template <int PK>
constexpr int pk_kc() { return PK ? 16 : 32; }
template <int PK>
constexpr int pk_min_waves() { return PK ? 3 : 1; }  // waves per SIMD budgeted for

template <class K, int T, int KC, int PK>
__global__ void __launch_bounds__(256, pk_min_waves<PK>()) fw_product(K* __restrict__ D, size_t ld, int kb, TileSet ts) {
    fw_tile<K, T, KC, PK>(D, ld, kb, tile_kept(ts.r0, (int)blockIdx.y, ts.rx0, ts.rx1),
                          tile_kept(ts.c0, (int)blockIdx.x, ts.cx0, ts.cx1));
}

// Two tile sets in one launch (the pivot's row panel and column panel: they are independent
// once the pivot tile is closed, and each is a single short wave of workgroups, so one launch
// instead of two takes a tile latency off the FW critical path).  grid.x = na + nb tiles;
// set s is nc_s columns wide, tiles flattened row-major.
template <class K, int T, int KC, int PK>
__global__ void __launch_bounds__(256) fw_product_pair(K* __restrict__ D, size_t ld, int kb, TileSet a, int na,
                                                       int nca, TileSet b, int ncb) {
    int x = (int)blockIdx.x;
    const TileSet& t = x < na ? a : b;
    const int nc = x < na ? nca : ncb;
    if (x >= na) x -= na;
    fw_tile<K, T, KC, PK>(D, ld, kb, tile_kept(t.r0, x / nc, t.rx0, t.rx1), tile_kept(t.c0, x % nc, t.cx0, t.cx1));
}

// ---------------------------------------------------------------------------------------
// u32 keys, pair-packed (PK = true, the dominant kernel).  Every u32 key is <= INF = 2^31-1,
// so a sum of two keys is < 2^32 and one 64-bit add of two packed pairs
//     (x_k | x_{k+1} << 32) + (y_k | y_{k+1} << 32)
// yields both 32-bit sums exactly (no carry crosses the halves).  One v_lshl_add_u64 thus does
// the adds of two relaxations and one v_min3_u32 folds both into the accumulator: one
// full-rate and one half-rate VALU instruction per two relaxations, instead of two adds and a
// min3 (profiles/r01_valu_rate_microbench.txt).
// LDS image of a KC-deep chunk as k-pairs, rows of LDA = T + 2 pairs (16-B pad):
//     Ap[kp][i] = A[i][k0+2kp] | A[i][k0+2kp+1] << 32
//     Bp[kp][j] = B[k0+2kp][j] | B[k0+2kp+1][j] << 32
// Thread (ty, tx) owns rows pk_rc(ty, e) and columns pk_rc(tx, e), e < M = T/16: two adjacent
// rows/columns every 32, so one ds_read_b128 (two pairs) of 16 lanes covers 256 contiguous
// bytes (conflict-free; the A reads are 4-address broadcasts).
typedef unsigned long long u64p;

__device__ __forceinline__ u64p add_pairs(u64p x, u64p y) {
    u64p r;
    asm("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(r) : "v"(x), "v"(y));
    return r;
}

__device__ __forceinline__ int pk_rc(int t, int e) { return 32 * (e >> 1) + 2 * t + (e & 1); }

template <int T, int KC>
struct PkStage {
    static_assert(T % 32 == 0 && KC % 8 == 0, "pk tile");
    static constexpr int LDA = T + 2;                    // pairs per LDS row
    static constexpr int AV = T * KC / 4 / 256;          // A: 16-B vectors (4 k values) per thread
    static constexpr int BTN = (KC / 2) * (T / 4);       // B: pair-row tasks (two 16-B loads each)
    static constexpr int BT = (BTN + 255) / 256;         //    per thread (the last one maybe partial)
    static_assert(AV >= 1 && T * KC / 4 % 256 == 0, "pk staging");
    Vec16<uint32_t> a[AV], b0[BT], b1[BT];
};

template <int T, int KC>
__device__ __forceinline__ void pk_load(PkStage<T, KC>& sg, const uint32_t* __restrict__ A,
                                        const uint32_t* __restrict__ B, size_t ld, const uint32_t* arow, int k0) {
    using S = PkStage<T, KC>;
    const int tid = threadIdx.x;
#pragma unroll
    for (int q = 0; q < S::AV; ++q) {
        const int v = tid + 256 * q, i = v / (KC / 4), kq = v % (KC / 4);
        sg.a[q] = ld16(A + (size_t)arow[i] * ld + k0 + kq * 4);
    }
#pragma unroll
    for (int q = 0; q < S::BT; ++q) {
        const int v = tid + 256 * q, p = v / (T / 4), jq = v % (T / 4);
        if (S::BTN % 256 != 0 && v >= S::BTN) break;
        const uint32_t* r0 = B + (size_t)(k0 + 2 * p) * ld + jq * 4;
        sg.b0[q] = ld16(r0);
        sg.b1[q] = ld16(r0 + ld);
    }
}

template <int T, int KC>
__device__ __forceinline__ void pk_store(const PkStage<T, KC>& sg, u64p* __restrict__ Ap, u64p* __restrict__ Bp) {
    using S = PkStage<T, KC>;
    constexpr int LDA = S::LDA;
    const int tid = threadIdx.x;
#pragma unroll
    for (int q = 0; q < S::AV; ++q) {
        const int v = tid + 256 * q, i = v / (KC / 4), kq = v % (KC / 4);
        const uint32_t* x = sg.a[q].v;
        Ap[(2 * kq) * LDA + i] = (u64p)x[0] | ((u64p)x[1] << 32);
        Ap[(2 * kq + 1) * LDA + i] = (u64p)x[2] | ((u64p)x[3] << 32);
    }
#pragma unroll
    for (int q = 0; q < S::BT; ++q) {
        const int v = tid + 256 * q, p = v / (T / 4), jq = v % (T / 4);
        if (S::BTN % 256 != 0 && v >= S::BTN) break;
        const uint32_t* x = sg.b0[q].v;
        const uint32_t* y = sg.b1[q].v;
        VecN<u64p, 2> w0, w1;
        w0.v[0] = (u64p)x[0] | ((u64p)y[0] << 32);
        w0.v[1] = (u64p)x[1] | ((u64p)y[1] << 32);
        w1.v[0] = (u64p)x[2] | ((u64p)y[2] << 32);
        w1.v[1] = (u64p)x[3] | ((u64p)y[3] << 32);
        stv<u64p, 2>(Bp + p * LDA + jq * 4, w0);
        stv<u64p, 2>(Bp + p * LDA + jq * 4 + 2, w1);
    }
}

template <int T, int KC>
constexpr size_t pk_lds_bytes() {
    return (size_t)2 * KC * (T + 2) * sizeof(u64p);  // double-buffered Ap + Bp
}

template <int T, int KC>
__device__ __forceinline__ void fw_tile_pk(uint32_t* __restrict__ D, size_t ld, int kb, int I, int J) {
    using S = PkStage<T, KC>;
    constexpr int M = T / 16;
    constexpr int LDA = S::LDA;
    constexpr int BUF = KC * LDA;  // pairs per LDS buffer: Ap (KC/2 rows) then Bp (KC/2 rows)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    u64p* lds = reinterpret_cast<u64p*>(smem_raw);
    __shared__ uint32_t arow[T];
    uint32_t* C = D + (size_t)I * T * ld + (size_t)J * T;
    const uint32_t* A = D + (size_t)kb * T;                       // column block kb, rows via arow
    const uint32_t* B = D + (size_t)kb * T * ld + (size_t)J * T;  // row block kb, cols J
    const int tid = threadIdx.x, ty = tid >> 4, tx = tid & 15;
    if (tid < T) arow[tid] = I * T + tid;
    __syncthreads();

    constexpr int NCH = T / KC;
    const int nsplit = (int)gridDim.z;
    const int ch0 = (int)blockIdx.z * NCH / nsplit, ch1 = ((int)blockIdx.z + 1) * NCH / nsplit;
    S sg;
    pk_load<T, KC>(sg, A, B, ld, arow, ch0 * KC);
    uint32_t c[M][M];
    if (nsplit == 1) {
#pragma unroll
        for (int a = 0; a < M; ++a)
#pragma unroll
            for (int g = 0; g < M / 2; ++g) {
                VecN<uint32_t, 2> v = ldv<uint32_t, 2>(C + (size_t)pk_rc(ty, a) * ld + 32 * g + 2 * tx);
                c[a][2 * g] = v.v[0];
                c[a][2 * g + 1] = v.v[1];
            }
    } else {
#pragma unroll
        for (int a = 0; a < M; ++a)
#pragma unroll
            for (int b = 0; b < M; ++b) c[a][b] = KeyOps<uint32_t>::INF;
    }
    pk_store<T, KC>(sg, lds, lds + (KC / 2) * LDA);
    __syncthreads();
#pragma unroll 1
    for (int ch = ch0; ch < ch1; ++ch) {
        const u64p* Ap = lds + ((ch - ch0) & 1) * BUF;
        const u64p* Bp = Ap + (KC / 2) * LDA;
        if (ch + 1 < ch1) pk_load<T, KC>(sg, A, B, ld, arow, (ch + 1) * KC);  // issue early
        auto rd = [&](int kp, u64p* xa, u64p* xb) {
#pragma unroll
            for (int g = 0; g < M / 2; ++g) {
                VecN<u64p, 2> va = ldv<u64p, 2>(Ap + kp * LDA + 32 * g + 2 * ty);
                VecN<u64p, 2> vb = ldv<u64p, 2>(Bp + kp * LDA + 32 * g + 2 * tx);
                xa[2 * g] = va.v[0];
                xa[2 * g + 1] = va.v[1];
                xb[2 * g] = vb.v[0];
                xb[2 * g + 1] = vb.v[1];
            }
        };
        auto fold = [&](const u64p* xa, const u64p* xb) {
#pragma unroll
            for (int a = 0; a < M; ++a)
#pragma unroll
                for (int b = 0; b < M; ++b) {
                    const u64p s = add_pairs(xa[a], xb[b]);
                    c[a][b] = KeyOps<uint32_t>::min3(c[a][b], (uint32_t)s, (uint32_t)(s >> 32));
                }
        };
        // one register set: the other resident waves hide the LDS latency
#pragma unroll
        for (int kp = 0; kp < KC / 2; ++kp) {
            u64p ap[M], bp[M];
            rd(kp, ap, bp);
            fold(ap, bp);
        }
        if (ch + 1 < ch1) {  // write late into the other buffer
            u64p* An = lds + ((ch + 1 - ch0) & 1) * BUF;
            pk_store<T, KC>(sg, An, An + (KC / 2) * LDA);
        }
        __syncthreads();
    }
    if (nsplit == 1) {
#pragma unroll
        for (int a = 0; a < M; ++a)
#pragma unroll
            for (int g = 0; g < M / 2; ++g) {
                VecN<uint32_t, 2> v;
                v.v[0] = c[a][2 * g];
                v.v[1] = c[a][2 * g + 1];
                stv<uint32_t, 2>(C + (size_t)pk_rc(ty, a) * ld + 32 * g + 2 * tx, v);
            }
    } else {
#pragma unroll
        for (int a = 0; a < M; ++a)
#pragma unroll
            for (int b = 0; b < M; ++b) atomicMin(C + (size_t)pk_rc(ty, a) * ld + pk_rc(tx, b), c[a][b]);
    }
}

// ---------------------------------------------------------------------------------------
// Symmetric FW over line buffers (undirected graphs; one or several ranks).  W is symmetric, and
// so is D after every FW step (D[i][j] = min(D[i][j], D[i][k] + D[k][j]) maps symmetric to
// symmetric), so only the stored tiles (I <= J) of the row-major D are updated; the lower
// triangle is filled once at the end (mirror, or the multi-rank unpack).
// Every product reads its operands from the LINE BUFFER of the pivot L: nb tiles of T x T (row
// stride T), tile j = the stored tile (min(j, L), max(j, L)) -- line L of the triangle (row L
// and column L).  With that buffer
//     A = D[I][L] = tile I as stored if I <= L, else tile I read transposed
//     B = D[L][J] = tile J as stored if J >= L, else tile J read transposed
// and an operand is staged from either layout into the same k-pair LDS image:
//   row form  (element (x, k) at base + x*ld + k, 16 B along k)      = A plain / B transposed
//   col form  (element (x, k) at base + k*ld + x, two k-rows paired)  = A transposed / B plain
// The line buffer is the unit of exchange in the multi-rank schedule (one allgather per pivot,
// routing.hip fw_line_sym), and its tiles are contiguous 64-KB blocks for the bulk's operand reads.
__device__ __forceinline__ void tri_tile(int nb, int idx, int& I, int& J) {
    // idx -> (I, J), I <= J, row-major over the upper triangle: row I holds nb - I tiles
    const double b = 2.0 * nb + 1.0;
    int i = (int)((b - sqrt(b * b - 8.0 * (double)idx)) * 0.5);
    auto off = [&](int r) { return r * nb - r * (r - 1) / 2; };
    while (i > 0 && off(i) > idx) --i;
    while (i + 1 < nb && off(i + 1) <= idx) ++i;
    I = i;
    J = i + (idx - off(i));
}

template <int T, int KC>
struct SymOp {
    static constexpr int NV = T * KC / 4 / 256;  // 16-B vectors per thread per operand (either form)
    static_assert(T * KC / 4 % 256 == 0 && (KC / 2) * (T / 4) % 256 == 0, "sym staging");
    Vec16<uint32_t> r[NV];
};

template <int T, int KC>
__device__ __forceinline__ void sym_load(SymOp<T, KC>& o, const uint32_t* __restrict__ base, size_t ld, bool colform,
                                         int k0) {
    using S = SymOp<T, KC>;
    const int tid = threadIdx.x;
    if (!colform) {
#pragma unroll
        for (int q = 0; q < S::NV; ++q) {
            const int v = tid + 256 * q, x = v / (KC / 4), kq = v % (KC / 4);
            o.r[q] = ld16(base + (size_t)x * ld + k0 + kq * 4);
        }
    } else {
#pragma unroll
        for (int q = 0; q < S::NV / 2; ++q) {
            const int v = tid + 256 * q, p = v / (T / 4), xq = v % (T / 4);
            const uint32_t* r0 = base + (size_t)(k0 + 2 * p) * ld + xq * 4;
            o.r[2 * q] = ld16(r0);
            o.r[2 * q + 1] = ld16(r0 + ld);
        }
    }
}

template <int T, int KC>
__device__ __forceinline__ void sym_store(const SymOp<T, KC>& o, u64p* __restrict__ Xp, bool colform) {
    using S = SymOp<T, KC>;
    constexpr int LDA = T + 2;
    const int tid = threadIdx.x;
    if (!colform) {
#pragma unroll
        for (int q = 0; q < S::NV; ++q) {
            const int v = tid + 256 * q, x = v / (KC / 4), kq = v % (KC / 4);
            const uint32_t* e = o.r[q].v;
            Xp[(2 * kq) * LDA + x] = (u64p)e[0] | ((u64p)e[1] << 32);
            Xp[(2 * kq + 1) * LDA + x] = (u64p)e[2] | ((u64p)e[3] << 32);
        }
    } else {
#pragma unroll
        for (int q = 0; q < S::NV / 2; ++q) {
            const int v = tid + 256 * q, p = v / (T / 4), xq = v % (T / 4);
            const uint32_t* a = o.r[2 * q].v;
            const uint32_t* b = o.r[2 * q + 1].v;
            VecN<u64p, 2> w0, w1;
            w0.v[0] = (u64p)a[0] | ((u64p)b[0] << 32);
            w0.v[1] = (u64p)a[1] | ((u64p)b[1] << 32);
            w1.v[0] = (u64p)a[2] | ((u64p)b[2] << 32);
            w1.v[1] = (u64p)a[3] | ((u64p)b[3] << 32);
            stv<u64p, 2>(Xp + p * LDA + xq * 4, w0);
            stv<u64p, 2>(Xp + p * LDA + xq * 4 + 2, w1);
        }
    }
}

// C (TM x TM, row stride ldc) = min(C, A (x) B) with A = TM rows x TK (form acol), B = TK x TM
// columns (form bcol), both with row stride ldab; C2 (optional) receives a copy of the result.
// TM = 128: 256 threads x (8 x 8) micro-tiles (the bulk); TM = 64: (4 x 4) micro-tiles (the
// quadrant launches on the FW critical chain).  One v_lshl_add_u64 over packed k-pairs +
// v_min3_u32 per two relaxations (two v_add_u32 + v_min3_u32 measured slower in the tile: C3
// bulk launch 0.304 vs 0.242 ms, profiles/r02c/fw_fold.txt).  Every product reads all of A and
// B through LDS before C is stored; in-place line updates where A or B overlaps C across
// workgroups read old or new values of C's row, and both give the same result once the pivot
// is closed (min over k of C'[x][k] + P[k][y] = min over k of C[x][k] + P[k][y] for P closed).
// Epilogue functor epi(r, c, bits): the product's result, 8 bytes at element (r, c) of the tile (two
// u32 keys (r, c), (r, c + 1) here; one u64 key in fw_core_lb64), for destinations beyond C.
// STORE_C = false: C is only read (the result goes to the epilogue's destinations alone).
template <int TM, int TK, int KC, bool STORE_C = true, class Epi>
__device__ __forceinline__ void fw_core_lb_e(uint32_t* __restrict__ C, size_t ldc, const uint32_t* __restrict__ Ab,
                                             bool acol, const uint32_t* __restrict__ Bb, bool bcol, size_t ldab,
                                             Epi&& epi) {
    using S = SymOp<TM, KC>;
    constexpr int M = TM / 16;
    constexpr int LDA = TM + 2;
    constexpr int BUF = KC * LDA;
    constexpr int NCH = TK / KC;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    u64p* lds = reinterpret_cast<u64p*>(smem_raw);
    const int tid = threadIdx.x, ty = tid >> 4, tx = tid & 15;
    S sa, sb;
    sym_load<TM, KC>(sa, Ab, ldab, acol, 0);
    sym_load<TM, KC>(sb, Bb, ldab, bcol, 0);
    uint32_t c[M][M];
#pragma unroll
    for (int a = 0; a < M; ++a)
#pragma unroll
        for (int g = 0; g < M / 2; ++g) {
            VecN<uint32_t, 2> v = ldv<uint32_t, 2>(C + (size_t)pk_rc(ty, a) * ldc + 32 * g + 2 * tx);
            c[a][2 * g] = v.v[0];
            c[a][2 * g + 1] = v.v[1];
        }
    sym_store<TM, KC>(sa, lds, acol);
    sym_store<TM, KC>(sb, lds + (KC / 2) * LDA, bcol);
    __syncthreads();
#pragma unroll 1
    for (int ch = 0; ch < NCH; ++ch) {
        const u64p* Ap = lds + (ch & 1) * BUF;
        const u64p* Bp = Ap + (KC / 2) * LDA;
        if (ch + 1 < NCH) {  // issue early
            sym_load<TM, KC>(sa, Ab, ldab, acol, (ch + 1) * KC);
            sym_load<TM, KC>(sb, Bb, ldab, bcol, (ch + 1) * KC);
        }
#pragma unroll 2
        for (int kp = 0; kp < KC / 2; ++kp) {
            u64p ap[M], bp[M];
#pragma unroll
            for (int g = 0; g < M / 2; ++g) {
                VecN<u64p, 2> va = ldv<u64p, 2>(Ap + kp * LDA + 32 * g + 2 * ty);
                VecN<u64p, 2> vb = ldv<u64p, 2>(Bp + kp * LDA + 32 * g + 2 * tx);
                ap[2 * g] = va.v[0];
                ap[2 * g + 1] = va.v[1];
                bp[2 * g] = vb.v[0];
                bp[2 * g + 1] = vb.v[1];
            }
#pragma unroll
            for (int a = 0; a < M; ++a)
#pragma unroll
                for (int b = 0; b < M; b += 2) {
                    // two pair-adds, then their two v_min3: a v_min3 reading an add's result no
                    // longer follows it directly, which cost a hazard wait (s_nop) per pair; with
                    // the k-pair loop unrolled by 2 instead of fully (its hoisted LDS reads then fit
                    // the 168-VGPR budget: 156, no spill) the bulk launch runs 2 % faster
                    // (0.253-0.255 vs 0.258-0.262 ms, tools/gpu_r04v.sh)
                    const u64p s0 = add_pairs(ap[a], bp[b]);
                    const u64p s1 = add_pairs(ap[a], bp[b + 1]);
                    c[a][b] = KeyOps<uint32_t>::min3(c[a][b], (uint32_t)s0, (uint32_t)(s0 >> 32));
                    c[a][b + 1] = KeyOps<uint32_t>::min3(c[a][b + 1], (uint32_t)s1, (uint32_t)(s1 >> 32));
                }
        }
        if (ch + 1 < NCH) {  // write late into the other buffer
            u64p* An = lds + ((ch + 1) & 1) * BUF;
            sym_store<TM, KC>(sa, An, acol);
            sym_store<TM, KC>(sb, An + (KC / 2) * LDA, bcol);
        }
        __syncthreads();
    }
#pragma unroll
    for (int a = 0; a < M; ++a)
#pragma unroll
        for (int g = 0; g < M / 2; ++g) {
            VecN<uint32_t, 2> v;
            v.v[0] = c[a][2 * g];
            v.v[1] = c[a][2 * g + 1];
            if (STORE_C) stv<uint32_t, 2>(C + (size_t)pk_rc(ty, a) * ldc + 32 * g + 2 * tx, v);
            epi(pk_rc(ty, a), 32 * g + 2 * tx, (uint64_t)v.v[0] | ((uint64_t)v.v[1] << 32));
        }
}

template <int TM, int TK, int KC>
__device__ __forceinline__ void fw_core_lb(uint32_t* __restrict__ C, size_t ldc, const uint32_t* __restrict__ Ab,
                                           bool acol, const uint32_t* __restrict__ Bb, bool bcol, size_t ldab,
                                           uint32_t* __restrict__ C2, size_t ldc2) {
    fw_core_lb_e<TM, TK, KC>(C, ldc, Ab, acol, Bb, bcol, ldab, [&](int r, int cc, uint64_t bits) {
        if (C2) *reinterpret_cast<uint64_t*>(C2 + (size_t)r * ldc2 + cc) = bits;
    });
}

template <int T, int KC>
constexpr size_t lb_lds_bytes() { return (size_t)2 * KC * (T + 2) * sizeof(u64p); }

// ---- u64 keys (K = uint64_t, 64-tiles): the same products with one key per element ----------
// A staged operand chunk is X[k][x] (KC k-rows of TM keys, row stride TM + 2: 16-B aligned rows);
// the row form reads 16 B = two k of one x, the column form 16 B = two x of one k.
template <int TM, int KC>
struct SymOp64 {
    static constexpr int NV = TM * KC / 2 / 256;  // 16-B vectors per thread per operand
    static_assert(TM * KC / 2 % 256 == 0, "sym64 staging");
    Vec16<uint64_t> r[NV];
};

template <int TM, int KC>
__device__ __forceinline__ void sym_load64(SymOp64<TM, KC>& o, const uint64_t* __restrict__ base, size_t ld,
                                           bool colform, int k0) {
#pragma unroll
    for (int q = 0; q < SymOp64<TM, KC>::NV; ++q) {
        const int v = (int)threadIdx.x + 256 * q;
        if (!colform) {
            const int x = v / (KC / 2), kq = v % (KC / 2);
            o.r[q] = ld16(base + (size_t)x * ld + k0 + 2 * kq);
        } else {
            const int kk = v / (TM / 2), xq = v % (TM / 2);
            o.r[q] = ld16(base + (size_t)(k0 + kk) * ld + 2 * xq);
        }
    }
}

template <int TM, int KC>
__device__ __forceinline__ void sym_store64(const SymOp64<TM, KC>& o, uint64_t* __restrict__ X, bool colform) {
    constexpr int LDX = TM + 2;
#pragma unroll
    for (int q = 0; q < SymOp64<TM, KC>::NV; ++q) {
        const int v = (int)threadIdx.x + 256 * q;
        if (!colform) {
            const int x = v / (KC / 2), kq = v % (KC / 2);
            X[(2 * kq) * LDX + x] = o.r[q].v[0];
            X[(2 * kq + 1) * LDX + x] = o.r[q].v[1];
        } else {
            const int kk = v / (TM / 2), xq = v % (TM / 2);
            stv<uint64_t, 2>(X + kk * LDX + 2 * xq, o.r[q]);
        }
    }
}

// fw_core_lb for u64 keys (INF = 2^62: no sum wraps).  Thread (ty, tx) holds rows ty*M + i (its A
// reads are wave broadcasts: one 16-B read per two rows) and columns tx + 16 j (its B reads are 16
// lanes x 8 B contiguous: conflict-free).  Per k: M x M relaxations of a 64-bit add, a 64-bit
// compare and two selects (the u64 price of SURVEY §8d: 5 int32 ops).
template <int TM, int TK, int KC, bool STORE_C = true, class Epi>
__device__ __forceinline__ void fw_core_lb64_e(uint64_t* __restrict__ C, size_t ldc, const uint64_t* __restrict__ Ab,
                                               bool acol, const uint64_t* __restrict__ Bb, bool bcol, size_t ldab,
                                               Epi&& epi) {
    using S = SymOp64<TM, KC>;
    constexpr int M = TM / 16;
    constexpr int LDX = TM + 2;
    constexpr int BUF = 2 * KC * LDX;  // A and B chunks
    constexpr int NCH = TK / KC;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    uint64_t* lds = reinterpret_cast<uint64_t*>(smem_raw);
    const int tid = threadIdx.x, ty = tid >> 4, tx = tid & 15;
    S sa, sb;
    sym_load64<TM, KC>(sa, Ab, ldab, acol, 0);
    sym_load64<TM, KC>(sb, Bb, ldab, bcol, 0);
    uint64_t c[M][M];
#pragma unroll
    for (int i = 0; i < M; ++i)
#pragma unroll
        for (int j = 0; j < M; ++j) c[i][j] = C[(size_t)(ty * M + i) * ldc + tx + 16 * j];
    sym_store64<TM, KC>(sa, lds, acol);
    sym_store64<TM, KC>(sb, lds + KC * LDX, bcol);
    __syncthreads();
#pragma unroll 1
    for (int ch = 0; ch < NCH; ++ch) {
        const uint64_t* Ap = lds + (ch & 1) * BUF;
        const uint64_t* Bp = Ap + KC * LDX;
        if (ch + 1 < NCH) {  // issue early
            sym_load64<TM, KC>(sa, Ab, ldab, acol, (ch + 1) * KC);
            sym_load64<TM, KC>(sb, Bb, ldab, bcol, (ch + 1) * KC);
        }
#pragma unroll 2
        for (int k = 0; k < KC; ++k) {  // (a full unroll hoists every k's LDS reads: spills)
            uint64_t a[M], b[M];
            if constexpr (M >= 2) {
#pragma unroll
                for (int g = 0; g < M / 2; ++g) {
                    const VecN<uint64_t, 2> va = ldv<uint64_t, 2>(Ap + k * LDX + ty * M + 2 * g);
                    a[2 * g] = va.v[0];
                    a[2 * g + 1] = va.v[1];
                }
            } else {
                a[0] = Ap[k * LDX + ty];
            }
#pragma unroll
            for (int j = 0; j < M; ++j) b[j] = Bp[k * LDX + tx + 16 * j];
#pragma unroll
            for (int i = 0; i < M; ++i)
#pragma unroll
                for (int j = 0; j < M; ++j) {
                    const uint64_t s = a[i] + b[j];
                    c[i][j] = s < c[i][j] ? s : c[i][j];
                }
        }
        if (ch + 1 < NCH) {  // write late into the other buffer
            uint64_t* An = lds + ((ch + 1) & 1) * BUF;
            sym_store64<TM, KC>(sa, An, acol);
            sym_store64<TM, KC>(sb, An + KC * LDX, bcol);
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < M; ++i)
#pragma unroll
        for (int j = 0; j < M; ++j) {
            if (STORE_C) C[(size_t)(ty * M + i) * ldc + tx + 16 * j] = c[i][j];
            epi(ty * M + i, tx + 16 * j, c[i][j]);
        }
}

template <int TM, int TK, int KC>
__device__ __forceinline__ void fw_core_lb64(uint64_t* __restrict__ C, size_t ldc, const uint64_t* __restrict__ Ab,
                                             bool acol, const uint64_t* __restrict__ Bb, bool bcol, size_t ldab,
                                             uint64_t* __restrict__ C2, size_t ldc2) {
    fw_core_lb64_e<TM, TK, KC>(C, ldc, Ab, acol, Bb, bcol, ldab, [&](int r, int cc, uint64_t v) {
        if (C2) C2[(size_t)r * ldc2 + cc] = v;
    });
}

template <int T, int KC>
constexpr size_t lb_lds_bytes64() { return (size_t)2 * 2 * KC * (T + 2) * sizeof(uint64_t); }

// LDS of a line-buffer product of TM-tiles: pair-packed u32 or u64 keys
template <class K, int TM, int KC>
constexpr size_t lb_lds() { return sizeof(K) == 4 ? lb_lds_bytes<TM, KC>() : lb_lds_bytes64<TM, KC>(); }

// one product of the line-buffer schedule, for either key type, with an epilogue functor
template <class K, int TM, int TK, int KC, bool STORE_C = true, class Epi>
__device__ __forceinline__ void fw_core_e(K* __restrict__ C, size_t ldc, const K* __restrict__ Ab, bool acol,
                                          const K* __restrict__ Bb, bool bcol, size_t ldab, Epi&& epi) {
    if constexpr (sizeof(K) == 4) fw_core_lb_e<TM, TK, KC, STORE_C>(C, ldc, Ab, acol, Bb, bcol, ldab, epi);
    else fw_core_lb64_e<TM, TK, KC, STORE_C>(C, ldc, Ab, acol, Bb, bcol, ldab, epi);
}

// one product of the line-buffer schedule, for either key type
template <class K, int TM, int TK, int KC>
__device__ __forceinline__ void fw_core(K* __restrict__ C, size_t ldc, const K* __restrict__ Ab, bool acol,
                                        const K* __restrict__ Bb, bool bcol, size_t ldab, K* __restrict__ C2,
                                        size_t ldc2) {
    if constexpr (sizeof(K) == 4) fw_core_lb<TM, TK, KC>(C, ldc, Ab, acol, Bb, bcol, ldab, C2, ldc2);
    else fw_core_lb64<TM, TK, KC>(C, ldc, Ab, acol, Bb, bcol, ldab, C2, ldc2);
}

// ---- distribution of the stored tiles over G ranks (routing.hip fw_line_sym) ----------------
// Tile (I, J), I <= J, belongs to rank (I + J) mod G: every rank holds ~1/G of every row and of
// every LINE (line L's tile j is (min(j,L), max(j,L)), owner (j + L) mod G), so both the bulk of a
// pivot and the per-pivot line exchange are balanced.  A line buffer is laid out owner-major so
// that each rank's tiles of the line are one contiguous segment for the allgather:
//   slot(j) = base(owner) + (j - j0(owner)) / G,  j0(r) = (r - L) mod G,
//   count(r) = #{ j < nb : j = j0(r) mod G },  base(r) = sum_{r' < r} count(r')
struct LineMap {
    int nb, G;
    __host__ __device__ int j0(int r, int L) const { return ((r - L) % G + G) % G; }
    __host__ __device__ int count(int r, int L) const {
        const int a = j0(r, L);
        return a < nb ? (nb - 1 - a) / G + 1 : 0;
    }
    __host__ __device__ int base(int r, int L) const {
        int s = 0;
        for (int q = 0; q < r; ++q) s += count(q, L);
        return s;
    }
    __host__ __device__ int owner(int j, int L) const { return (j + L) % G; }
    __host__ __device__ int slot(int j, int L) const {
        const int r = owner(j, L);
        return base(r, L) + (j - j0(r, L)) / G;
    }
};

// Bulk of pivot L: this rank's stored tiles (triangle indices tiles[0 .. gridDim.x), -1 = none) except
// those in lines x0, x1 (the pivot's own line, final, and the next pivot's line, updated by the
// chain).  C in D (row stride ld), operands from line L's buffer.
// maxI: tiles of block-rows past it have not received their edges yet (the host entry's FW beside
// the H2D, routing.hip FwOverlap): skipped, they catch up on this pivot when they arrive.
template <class K, int T, int KC>
__global__ void __launch_bounds__(256, 3) fw_bulk_lb(K* __restrict__ D, size_t ld, const K* __restrict__ lb, int L,
                                                     int x0, int x1, LineMap lm, const int* __restrict__ tiles,
                                                     int maxI) {
    const int t = tiles[blockIdx.x];
    if (t < 0) return;  // (a slot past a short XCD run, routing.hip xcd_tile_order)
    int I, J;
    tri_tile(lm.nb, t, I, J);
    if (I == x0 || I == x1 || J == x0 || J == x1 || I > maxI) return;  // whole workgroup
    constexpr size_t TT = (size_t)T * T;
    fw_core<K, T, T, KC>(D + (size_t)I * T * ld + (size_t)J * T, ld, lb + lm.slot(I, L) * TT, I > L,
                         lb + lm.slot(J, L) * TT, J >= L, T, nullptr, 0);
}

// The bulk for launches below one round of the chip's slots (several ranks: C3 at G = 8 holds 395
// tiles per pivot against 768 slots): each tile as four 64 x 64 quadrants (grid (tiles, 4)), the
// quadrant products of fw_line_lb<S = 2>, so the launch fills the CUs.
template <class K, int T, int KC>
__global__ void __launch_bounds__(256, 4) fw_bulk_lb_q(K* __restrict__ D, size_t ld, const K* __restrict__ lb, int L,
                                                       int x0, int x1, LineMap lm, const int* __restrict__ tiles,
                                                       int maxI) {
    const int t = tiles[blockIdx.x];
    if (t < 0) return;
    int I, J;
    tri_tile(lm.nb, t, I, J);
    if (I == x0 || I == x1 || J == x0 || J == x1 || I > maxI) return;  // whole workgroup
    constexpr size_t TT = (size_t)T * T;
    constexpr int TM = T / 2;
    const int qi = (int)blockIdx.y >> 1, qj = (int)blockIdx.y & 1;
    const bool acol = I > L, bcol = J >= L;
    const K* Ab = lb + lm.slot(I, L) * TT + (acol ? (size_t)qi * TM : (size_t)qi * TM * T);
    const K* Bb = lb + lm.slot(J, L) * TT + (bcol ? (size_t)qj * TM : (size_t)qj * TM * T);
    fw_core<K, TM, T, KC>(D + ((size_t)I * T + (size_t)qi * TM) * ld + (size_t)J * T + qj * TM, ld, Ab, acol, Bb, bcol, T,
                          nullptr, 0);
}

// Late tiles (the host entry's FW beside the H2D, routing.hip FwOverlap; one rank, u32 keys): the
// tiles (I, J >= I) of block-row I, whose edges landed after the bulks of pivots [0, P) ran without
// them, catch up on pivots p in group blockIdx.y (pg pivots per group):
//     D(I, J) = min(D(I, J), min over p of LB(p)[I] (x) LB(p)[J]),
// LB(p) the FINAL line of p (kept for every pivot).  Blocked FW's bulk updates of a tile are
// independent of one another once the lines are final, so this is exactly the skipped work: one
// K = 128 pg product per workgroup, C in registers across its pivots, merged with atomicMin once
// (exact: min is associative; a read of D that already holds another group's contribution only
// lowers this product's operand C, never below the true result).  One atomicMin pass per pivot
// (pg = 1) cost ~10 ms of catch-up at C3.  I, J > p: both operands are stored tiles (p, I),
// (p, J), read in column form.
// (blockIdx.x enumerates the tiles (I, J >= I) of the block-rows I0, I0 + 1, ... row by row.)
template <int T>
__global__ void __launch_bounds__(256, 3) fw_catchup(uint32_t* __restrict__ D, size_t ld, const uint32_t* __restrict__ lball,
                                                     size_t lb_stride, int I0, int nb, int np, int pg) {
    constexpr int KC = 16;
    constexpr size_t TT = (size_t)T * T;
    using S = SymOp<T, KC>;
    constexpr int M = T / 16;
    constexpr int LDA = T + 2;
    constexpr int BUF = KC * LDA;
    constexpr int CPP = T / KC;  // chunks per pivot
    int I = I0, t = (int)blockIdx.x;
    while (t >= nb - I) t -= nb - I++;
    const int J = I + t, p0 = (int)blockIdx.y * pg, p1 = min(np, p0 + pg);
    if (p0 >= p1) return;
    uint32_t* C = D + (size_t)I * T * ld + (size_t)J * T;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    u64p* lds = reinterpret_cast<u64p*>(smem_raw);
    const int tid = threadIdx.x, ty = tid >> 4, tx = tid & 15;
    auto opA = [&](int p) { return lball + (size_t)p * lb_stride + (size_t)I * TT; };
    auto opB = [&](int p) { return lball + (size_t)p * lb_stride + (size_t)J * TT; };
    S sa, sb;
    sym_load<T, KC>(sa, opA(p0), T, true, 0);
    sym_load<T, KC>(sb, opB(p0), T, true, 0);
    uint32_t c[M][M];
#pragma unroll
    for (int a = 0; a < M; ++a)
#pragma unroll
        for (int g = 0; g < M / 2; ++g) {
            VecN<uint32_t, 2> v = ldv<uint32_t, 2>(C + (size_t)pk_rc(ty, a) * ld + 32 * g + 2 * tx);
            c[a][2 * g] = v.v[0];
            c[a][2 * g + 1] = v.v[1];
        }
    sym_store<T, KC>(sa, lds, true);
    sym_store<T, KC>(sb, lds + (KC / 2) * LDA, true);
    __syncthreads();
    const int nch = (p1 - p0) * CPP;
#pragma unroll 1
    for (int ch = 0; ch < nch; ++ch) {
        const u64p* Ap = lds + (ch & 1) * BUF;
        const u64p* Bp = Ap + (KC / 2) * LDA;
        if (ch + 1 < nch) {  // issue early
            const int pn = p0 + (ch + 1) / CPP, k0 = ((ch + 1) % CPP) * KC;
            sym_load<T, KC>(sa, opA(pn), T, true, k0);
            sym_load<T, KC>(sb, opB(pn), T, true, k0);
        }
#pragma unroll
        for (int kp = 0; kp < KC / 2; ++kp) {
            u64p ap[M], bp[M];
#pragma unroll
            for (int g = 0; g < M / 2; ++g) {
                VecN<u64p, 2> va = ldv<u64p, 2>(Ap + kp * LDA + 32 * g + 2 * ty);
                VecN<u64p, 2> vb = ldv<u64p, 2>(Bp + kp * LDA + 32 * g + 2 * tx);
                ap[2 * g] = va.v[0];
                ap[2 * g + 1] = va.v[1];
                bp[2 * g] = vb.v[0];
                bp[2 * g + 1] = vb.v[1];
            }
#pragma unroll
            for (int a = 0; a < M; ++a)
#pragma unroll
                for (int b = 0; b < M; b += 2) {  // (interleaved as in fw_core_lb_e)
                    const u64p s0 = add_pairs(ap[a], bp[b]);
                    const u64p s1 = add_pairs(ap[a], bp[b + 1]);
                    c[a][b] = KeyOps<uint32_t>::min3(c[a][b], (uint32_t)s0, (uint32_t)(s0 >> 32));
                    c[a][b + 1] = KeyOps<uint32_t>::min3(c[a][b + 1], (uint32_t)s1, (uint32_t)(s1 >> 32));
                }
        }
        if (ch + 1 < nch) {  // write late into the other buffer
            u64p* An = lds + ((ch + 1) & 1) * BUF;
            sym_store<T, KC>(sa, An, true);
            sym_store<T, KC>(sb, An + (KC / 2) * LDA, true);
        }
        __syncthreads();
    }
#pragma unroll
    for (int a = 0; a < M; ++a)
#pragma unroll
        for (int g = 0; g < M / 2; ++g) {
            uint32_t* q = C + (size_t)pk_rc(ty, a) * ld + 32 * g + 2 * tx;
            atomicMin(q, c[a][2 * g]);
            atomicMin(q + 1, c[a][2 * g + 1]);
        }
}

// Line launches of the FW critical chain, one (T/S) x (T/S) sub-tile of a line tile per
// workgroup (grid = (tiles, S*S)): S = 1 whole tiles (the throughput form, for one rank, whose chain
// hides behind the bulk), S = 2 quadrants, S = 4 32 x 32 sub-tiles (several ranks: the bulk shrinks
// with G and the chain is the critical path, so a line should take one small sub-tile's latency).
//   mode 0 (line K1 w.r.t. pivot L, this rank's tiles of line K1: j = j0 + G * blockIdx.x):
//          C = D tile (min(j,K1), max(j,K1)), operands from line L's buffer lbL; the result
//          also goes to lbK.  j == L is not updated (that tile, (L, K1), is final in line L):
//          it is copied from lbL, the same stored tile.
//   mode 1 (line K1 w.r.t. its own closed pivot, every tile j = blockIdx.x): C = lbK's tile,
//          operands from lbK; the result also goes to D when this rank owns the tile (rank g),
//          and the closed pivot tile j == K1 is copied back to D by its owner.
template <int S>
constexpr int line_kc() { return S == 1 ? 16 : S == 2 ? 32 : 64; }

template <class K, int T, int S>
__global__ void __launch_bounds__(256, S == 1 ? 3 : 2) fw_line_lb(K* __restrict__ D, size_t ld, const K* __restrict__ lbL,
                                                                  int L, K* __restrict__ lbK, int K1, int mode,
                                                                  LineMap lm, int g, int prio) {
    constexpr int TM = T / S;
    constexpr int KCL = line_kc<S>();
    constexpr size_t TT = (size_t)T * T;
    const int j = mode == 0 ? lm.j0(g, K1) + lm.G * (int)blockIdx.x : (int)blockIdx.x;
    const int q = (int)blockIdx.y, qi = q / S, qj = q % S;
    const int I = min(j, K1), J = max(j, K1);
    const bool own = lm.owner(j, K1) == g;
    K* Dt = D + (size_t)I * T * ld + (size_t)J * T;
    K* Lt = lbK + lm.slot(j, K1) * TT;
    auto copy_sub = [&](const K* src, size_t lds_, K* dst, size_t ldd) {
        constexpr int VE = 16 / (int)sizeof(K);
        src += (size_t)qi * TM * lds_ + qj * TM;
        dst += (size_t)qi * TM * ldd + qj * TM;
        for (int e = threadIdx.x; e < TM * TM / VE; e += 256) {
            const int r = e / (TM / VE), cv = e % (TM / VE);
            st16(dst + (size_t)r * ldd + cv * VE, ld16(src + (size_t)r * lds_ + cv * VE));
        }
    };
    if (mode == 1 && j == K1) {  // the closed pivot tile itself: back to D on its owner
        if (own) copy_sub(Lt, T, Dt, ld);
        return;
    }
    if (mode == 0 && j == L) {  // the final tile (L, K1) from line L's buffer
        copy_sub(lbL + lm.slot(K1, L) * TT, T, Lt, T);
        return;
    }
    if (prio) __builtin_amdgcn_s_setprio(3);  // the chain runs beside the bulk tiles (see fw_phase1)
    const K* lb = mode == 0 ? lbL : lbK;
    const int P = mode == 0 ? L : K1;
    const bool acol = I > P, bcol = J >= P;
    // A rows qi: row form advances rows, col form advances columns (and B likewise for columns qj)
    const K* Ab = lb + lm.slot(I, P) * TT + (acol ? (size_t)qi * TM : (size_t)qi * TM * T);
    const K* Bb = lb + lm.slot(J, P) * TT + (bcol ? (size_t)qj * TM : (size_t)qj * TM * T);
    Dt += (size_t)qi * TM * ld + qj * TM;
    Lt += (size_t)qi * TM * T + qj * TM;
    if (mode == 0) fw_core<K, TM, T, KCL>(Dt, ld, Ab, acol, Bb, bcol, T, Lt, T);
    else fw_core<K, TM, T, KCL>(Lt, T, Ab, acol, Bb, bcol, T, own ? Dt : nullptr, ld);
}

// Grid barrier among the launch's workgroups, which must all be resident together (a few small
// workgroups; no other kernel waits for them, so every one is eventually admitted).  Write-through
// form of the MI355X_MICROARCH.md hand-off (its "sc1 stores, sc1 loads" row): every byte handed
// across the barrier is stored and loaded with agent-scope (sc1) accesses, every wave drains its
// stores, and after a workgroup barrier one lane adds to the arrival counter and polls it
// (bounded: on a timeout it raises *timeout and the caller gives up; the host reports it).  No
// release / acquire fence: the release's L2 write-back (buffer_wbl2) also flushes whatever the
// FW bulk tiles beside this kernel have dirtied in the XCD's L2.
__device__ __forceinline__ bool grid_sync(uint32_t* cnt, uint32_t target, uint32_t* timeout, uint32_t* s_ok) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t ok = 1;
        for (uint32_t spins = 0; __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target; ++spins) {
            if (spins > (1u << 21) || __hip_atomic_load(timeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                __hip_atomic_store(timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        *s_ok = ok;
    }
    __syncthreads();
    return *s_ok != 0;
}

template <class K>
__device__ __forceinline__ void st_wt(K* p, K v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // a vector store, sc1
}

// Close the T x T pivot tile P (row stride T, inside a line buffer) in ONE launch: repeated
// squaring P <- min(P, P (x) P) in place, 16 x 16 outputs per workgroup, grid (T/16, T/16), the
// workgroups meeting at a grid barrier after every step and stopping after the first step that
// changed nothing (atlas pivot tiles: two changing steps and that one).  In place
// is exact: keys only decrease and every value read, old or new, is the length of a path inside
// the tile, so a step in which no workgroup changed anything read one consistent state and
// P = min(P, P (x) P) holds there: P is closed.  Eight steps (paths of 2^8 >= T hops) always
// suffice.  sync = {arrival counter, changed flag of steps 0 .. 7, ...} (16 words, zeroed before
// the launch).  Keys <= INF = 2^31 - 1: no sum wraps.  P is read and written write-through
// (grid_sync); the previous kernel's plain stores are visible at the launch boundary.  K = u64:
// keys <= INF = 2^62, the same.
// The closure's body for output block (by, bx) of nwg participating workgroups; A, B, sh: LDS
// scratch.
template <class K, int T>
__device__ __forceinline__ void close_body(K* __restrict__ P, uint32_t* __restrict__ sync, uint32_t* __restrict__ timeout,
                                           int by, int bx, uint32_t nwg, K (*A)[T + 1], K (*B)[17], uint32_t* sh) {
    uint32_t& s_chg = sh[0];
    uint32_t& s_ok = sh[1];
    uint32_t& s_more = sh[2];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int r0 = by * 16, c0 = bx * 16;
    // write-through (sc1, aux = 16) 16-B loads of the 16 rows and 16 columns this workgroup needs
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(P, (short)0, (int)(T * T * sizeof(K)), 0x00027000);
    constexpr int VE = 16 / (int)sizeof(K);  // keys per 16-B vector
    constexpr int NV = 16 * T / VE / 256;    // 16-B vectors per thread per operand
    static_assert(NV >= 1 && 16 * T / VE % 256 == 0, "closure staging");
    for (int step = 0; step < 8; ++step) {
        if (threadIdx.x == 0) s_chg = 0;
        typedef uint32_t v4u __attribute__((ext_vector_type(4)));
        v4u va[NV], vb[NV];
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            const int v = threadIdx.x + 256 * q;
            const int y = v / (T / VE), ka = v % (T / VE);    // A: row r0 + y, columns VE ka ..
            const int kk = v / (16 / VE), xb = v % (16 / VE);  // B: row kk, columns c0 + VE xb ..
            va[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(((r0 + y) * T + VE * ka) * sizeof(K)), 0, 16);
            vb[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)((kk * T + c0 + VE * xb) * sizeof(K)), 0, 16);
        }
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            const int v = threadIdx.x + 256 * q;
            const int y = v / (T / VE), ka = v % (T / VE), kk = v / (16 / VE), xb = v % (16 / VE);
            K ea[VE], eb[VE];
            __builtin_memcpy(ea, &va[q], 16);
            __builtin_memcpy(eb, &vb[q], 16);
#pragma unroll
            for (int e = 0; e < VE; ++e) {
                A[y][VE * ka + e] = ea[e];
                B[kk][VE * xb + e] = eb[e];
            }
        }
        __syncthreads();
        const K old = A[ty][c0 + tx];
        K v = old;
#pragma unroll 8
        for (int k = 0; k < T; k += 2) v = KeyOps<K>::min3(v, A[ty][k] + B[k][tx], A[ty][k + 1] + B[k + 1][tx]);
        if (v < old) {
            st_wt(&P[(size_t)(r0 + ty) * T + c0 + tx], v);
            s_chg = 1;
        }
        __syncthreads();
        if (threadIdx.x == 0 && s_chg) __hip_atomic_fetch_or(&sync[1 + step], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!grid_sync(&sync[0], nwg * (uint32_t)(step + 1), timeout, &s_ok)) return;
        if (threadIdx.x == 0) s_more = __hip_atomic_load(&sync[1 + step], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        if (!s_more) return;
    }
}

template <class K, int T>
__global__ void __launch_bounds__(256) fw_close_sq(K* __restrict__ P, uint32_t* __restrict__ sync,
                                                   uint32_t* __restrict__ timeout, int prio) {
    if (prio) __builtin_amdgcn_s_setprio(3);
    __shared__ K A[16][T + 1];
    __shared__ K B[T][17];
    __shared__ uint32_t sh[4];
    close_body<K, T>(P, sync, timeout, (int)blockIdx.y, (int)blockIdx.x, gridDim.x * gridDim.y, A, B, sh);
}

// lb[slot(j)] <- stored tile (min(j, L), max(j, L)) of D, j = blockIdx.x
template <class K, int T>
__global__ void __launch_bounds__(256) k_pack_line(const K* __restrict__ D, size_t ld, K* __restrict__ lb, int L,
                                                   LineMap lm) {
    constexpr int VE = 16 / (int)sizeof(K);
    const int j = (int)blockIdx.x, I = min(j, L), J = max(j, L);
    const K* src = D + (size_t)I * T * ld + (size_t)J * T;
    K* dst = lb + (size_t)lm.slot(j, L) * T * T;
    for (int e = threadIdx.x; e < T * T / VE; e += 256) {
        const int r = e / (T / VE), cv = e % (T / VE);
        st16(dst + (size_t)r * T + cv * VE, ld16(src + (size_t)r * ld + cv * VE));
    }
}

// Multi-rank end of FW: every rank packs its own stored tiles (triangle indices tiles[i]) into
// P[first + i] (T x T each; its segment of the allgather), and after the allgather every rank
// unpacks every tile t from P[slot[t]] into its row-major D, with the mirror (J, I) = (I, J)^T
// through 64 x 64 LDS transposes.
template <class K, int T>
__global__ void __launch_bounds__(256) k_pack_tiles(const K* __restrict__ D, size_t ld, int nb,
                                                    const int* __restrict__ tiles, size_t first, K* __restrict__ P) {
    constexpr int VE = 16 / (int)sizeof(K);
    int I, J;
    tri_tile(nb, tiles[blockIdx.x], I, J);
    const K* src = D + (size_t)I * T * ld + (size_t)J * T;
    K* dst = P + (first + blockIdx.x) * (size_t)T * T;
    for (int e = threadIdx.x; e < T * T / VE; e += 256) {
        const int r = e / (T / VE), cv = e % (T / VE);
        st16(dst + (size_t)r * T + cv * VE, ld16(src + (size_t)r * ld + cv * VE));
    }
}

template <class K, int T>
__global__ void __launch_bounds__(256) k_unpack_tiles(const K* __restrict__ P, const int* __restrict__ slot, int nb,
                                                      K* __restrict__ D, size_t ld) {
    int I, J;
    tri_tile(nb, (int)blockIdx.x, I, J);
    const K* src = P + (size_t)slot[blockIdx.x] * T * T;
    __shared__ K tile[64][65];
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int sb = 0; sb < (T / 64) * (T / 64); ++sb) {
        const int bi = sb / (T / 64), bj = sb % (T / 64);
        for (int r = ty; r < 64; r += 4) {
            const K v = src[(size_t)(bi * 64 + r) * T + bj * 64 + tx];
            tile[r][tx] = v;
            D[((size_t)I * T + bi * 64 + r) * ld + (size_t)J * T + bj * 64 + tx] = v;
        }
        __syncthreads();
        if (I != J)
            for (int r = ty; r < 64; r += 4)
                D[((size_t)J * T + bj * 64 + r) * ld + (size_t)I * T + bi * 64 + tx] = tile[tx][r];
        __syncthreads();
    }
}

// lower triangle <- transpose of the upper one, 64 x 64 blocks (bi > bj) through LDS
template <class K>
__global__ void __launch_bounds__(256) k_sym_mirror(K* __restrict__ D, size_t ld) {
    const uint32_t bi = blockIdx.y, bj = blockIdx.x;
    if (bi <= bj) return;
    __shared__ K tile[64][65];
    const uint32_t tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (uint32_t r = ty; r < 64; r += 4) tile[r][tx] = D[(size_t)(bj * 64 + r) * ld + bi * 64 + tx];
    __syncthreads();
    for (uint32_t r = ty; r < 64; r += 4) D[(size_t)(bi * 64 + r) * ld + bj * 64 + tx] = tile[tx][r];
}

template <class K, int T, int KC, int PK>
__device__ __forceinline__ void fw_tile(K* __restrict__ D, size_t ld, int kb, int I, int J) {
    if constexpr (PK != 0) {
        static_assert(sizeof(K) == 4, "pair-packed tiles need u32 keys");
        fw_tile_pk<T, KC>(reinterpret_cast<uint32_t*>(D), ld, kb, I, J);
        return;
    }
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
                    c[a][b] = KeyOps<K>::min3(c[a][b], KeyOps<K>::add_nw(a0[a], b0[b]),
                                              KeyOps<K>::add_nw(a1[a], b1[b]));
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
