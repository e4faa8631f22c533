// tight_v6.hip.h — entry-lane tight-predecessor scan (gfx950), the alternative to tight_v5.
//
// Same checks as tight_v5 (tight_sparse.hip.h): for every essential entry (u, t) and used source
// s, is D[s][u] + W[u][t] == D[s][t]?  tight_v5 puts SOURCES on the lanes and walks a uniform
// entry stream, so every entry pair pays two LDS address adds and two register-indexed moves of
// the target's -d for its 4 checks per lane (11 VALU per 4 checks, 5.6e9 VALU per C3 build,
// DESIGN.md §5).  Here ENTRIES are on the lanes: 16 lanes per entry, 4 entries per wave
// instruction, lane j of an entry holding sources 4j..4j+3 and 64+4j..64+4j+3 of the workgroup's
// 128.  -D of the whole 64-target tile sits in LDS beside the staged rows, so both operands are
// ds_read_b128 at a per-lane base + an immediate offset: per entry and lane 2 address adds,
// 8 add3, a min tree and one compare for 8 checks (~1.9 VALU per check against ~2.75).
//
// Banking: a ds_read_b128 is serviced in four 16-lane groups ({0-3,12-15,20-27}, {4-11,16-19,
// 28-31}, and the same + 32); each group holds 8 lanes of one entry and 8 of the next, whose
// 16-B columns cover complementary quarters of a 256-B bank line (rows 512 B apart), so the reads
// are conflict-free whatever rows u / targets t the four entries have.
//
// Hits (x = a + w - d == 0, ~1 check in 800 at C3: two groups in three have one) go to global
// memory as two no-return atomics, min into PRED (set to PRED_NONE before the scan) and max into
// PMAX (set to 0): exactly one hit <=> min == max, so k_v6_combine then turns min != max into
// PRED_MULTI.  (A CAS that returns the old value made each hit a global round trip the wave
// waited for: 47 ms per C3 build.)  The diagonal (t == s) and, for u32 keys, unreachable targets
// (d == INF) are never written, exactly as tight_v5 leaves them NONE.
// Records: per (64-target tile b, 32-row chunk k) the entries in target order, padded to whole
// 4-entry groups with w = INF (skipped in the hit path); rec = {a_off | d_off << 16, w}, the LDS
// byte offsets of the entry's row in the chunk buffer and of its target's -D row.  ent_w / ent_u /
// ent_b / the CSC lists are indexed by the same entry number (k_loss_rows reads them unchanged).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.hip.h"
#include "tight_sparse.hip.h"

namespace srg {

constexpr uint32_t V6_TT = 64;                      // targets per workgroup tile (one ESS word column)
constexpr uint32_t V6_UC = 32;                      // u rows per staged chunk
constexpr uint32_t V6_SB = 128;                     // sources per workgroup (= V5_SB: same DST, same cuts)
constexpr uint32_t V6_WAVES = 8;
constexpr uint32_t V6_ROW = V6_SB * 4;              // 512 B per staged row
constexpr uint32_t V6_BUF = V6_UC * V6_ROW;         // 16 KB per chunk buffer
constexpr uint32_t V6_ND = 2 * V6_BUF;              // -D tile at 32 KB
constexpr uint32_t V6_LDS = V6_ND + V6_TT * V6_ROW;  // 64 KB: two workgroups per CU
constexpr uint32_t V6_SLACK = 128;                  // records past the end (the loop reads two groups of 8 ahead)

// one wave per (tile b = 64-target column, chunk k), lane = target: entries per (b, k) rounded up to
// whole 4-entry groups, and indeg[t] for the CSC lists
__global__ void __launch_bounds__(256) k_v6_count(const unsigned long long* __restrict__ ess, uint32_t V,
                                                   uint32_t nw64, uint32_t nK, uint32_t* __restrict__ glen,
                                                   uint32_t* __restrict__ indeg) {
    const uint32_t lane = threadIdx.x & 63;
    const size_t wv = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
    if (wv >= (size_t)nw64 * nK) return;  // whole wave
    const uint32_t w64 = (uint32_t)(wv / nK), k = (uint32_t)(wv % nK);
    const uint32_t u0 = k * V6_UC, u1 = min(V, u0 + V6_UC);
    uint32_t c = 0;
    for (uint32_t u = u0; u < u1; ++u) c += (uint32_t)((ess[(size_t)u * nw64 + w64] >> lane) & 1ull);
    if (c) atomicAdd(&indeg[w64 * 64 + lane], c);
    uint32_t s = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) s += __shfl_xor(s, off, 64);
    if (lane == 0) glen[wv] = (s + 3) / 4 * 4;
}

// records + entry arrays + CSC lists, entries of a (b, k) in target order (lane order), then u
template <class K>
__global__ void __launch_bounds__(256) k_v6_fill(const unsigned long long* __restrict__ ess,
                                                  const K* __restrict__ W, const uint32_t* __restrict__ WL,
                                                  size_t ld, uint32_t V, uint32_t nw64, uint32_t nK,
                                                  const uint32_t* __restrict__ goff, const uint32_t* __restrict__ csc_off,
                                                  uint32_t* __restrict__ csc_fill, uint2* __restrict__ rec,
                                                  K* __restrict__ ent_w, uint32_t* __restrict__ ent_u,
                                                  float* __restrict__ ent_b, uint32_t* __restrict__ csc_ent) {
    const uint32_t lane = threadIdx.x & 63;
    const size_t wv = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
    if (wv >= (size_t)nw64 * nK) return;
    const uint32_t w64 = (uint32_t)(wv / nK), k = (uint32_t)(wv % nK);
    const uint32_t t = w64 * 64 + lane;
    const uint32_t u0 = k * V6_UC, u1 = min(V, u0 + V6_UC);
    uint32_t c = 0;
    for (uint32_t u = u0; u < u1; ++u) c += (uint32_t)((ess[(size_t)u * nw64 + w64] >> lane) & 1ull);
    uint32_t incl = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off, 64);
        if ((int)lane >= off) incl += y;
    }
    const uint32_t base = goff[wv];
    size_t e = (size_t)base + incl - c;
    const uint32_t cbase = t < V ? csc_off[t] : 0u;
    const uint32_t doff = lane * V6_ROW;
    for (uint32_t u = u0; u < u1; ++u) {
        if (!((ess[(size_t)u * nw64 + w64] >> lane) & 1ull)) continue;
        const K w = W[(size_t)u * ld + t];
        rec[e] = make_uint2(((u - u0) * V6_ROW) | (doff << 16), (uint32_t)w);
        ent_w[e] = w;
        ent_u[e] = u;
        ent_b[e] = __fsub_rn(1.0f, __uint_as_float(WL[(size_t)u * ld + t]));
        csc_ent[cbase + atomicAdd(&csc_fill[t], 1u)] = (uint32_t)e;
        ++e;
    }
    if (lane == 63)  // the list's group padding (w = INF: skipped by the hit path)
        for (size_t q = (size_t)base + incl; q < goff[wv + 1]; ++q) {
            rec[q] = make_uint2(0u, KeyOps<uint32_t>::INF);
            ent_w[q] = KeyOps<K>::INF;
            ent_u[q] = 0;
            ent_b[q] = 1.0f;
        }
}

// grid: 8 * 64 * ceil(nblk / 8) workgroups of 512 over the source blocks [c0, nbS), nblk =
// ceil(nbT / 8) * ceil((nbS - c0) / 8) blocks of 8 target tiles x 8 source blocks dealt to the XCDs
// in turn: an XCD holds one block at a time (2 workgroups per CU x 32 CUs), so each source block's
// staged rows are read 8 ways and each tile's records 8 ways out of that XCD's L2.
// u64 keys (inf_check = 0): DST and the record weights are the keys' low words (see tight_v5).
__global__ void __launch_bounds__(512, 2) tight_v6(const uint32_t* __restrict__ DST, size_t npad, uint32_t dst_bytes,
                                                    const uint32_t* __restrict__ nodes, uint32_t n, uint32_t nbT,
                                                    uint32_t nbS, uint32_t nK, uint32_t c0,
                                                    const uint32_t* __restrict__ goff, const uint2* __restrict__ rec,
                                                    uint32_t* __restrict__ PRED, uint32_t* __restrict__ PMAX, size_t ldp,
                                                    uint32_t inf_check) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[V6_LDS / 4];
    const uint32_t bid = blockIdx.x, xcd = bid & 7, slot = bid >> 3;
    const uint32_t blk = (slot >> 6) * 8 + xcd, nbb = (nbT + 7) / 8;
    const uint32_t b = (blk % nbb) * 8 + (slot & 7), c = c0 + (blk / nbb) * 8 + ((slot >> 3) & 7);
    if (c >= nbS || b >= nbT) return;  // whole workgroup
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(tid >> 6);
    const __amdgpu_buffer_rsrc_t rsrc = make_rsrc(DST, dst_bytes);
    unsigned char* lb = reinterpret_cast<unsigned char*>(lds);
    // -D of the tile: 64 rows x 512 B, 4 x 16 B per thread
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
        const uint32_t idx = tid + 512 * i, row = idx >> 5, col = (idx & 31) * 4;
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, ((b * V6_TT + row) * (uint32_t)npad + c * V6_SB + col) * 4u,
                                                             0, 0);
        *reinterpret_cast<uint4*>(lb + V6_ND + row * V6_ROW + col * 4) = make_uint4(0u - v[0], 0u - v[1], 0u - v[2], 0u - v[3]);
    }
    // chunk staging: 32 rows x 512 B, 2 x 16 B per thread
    const uint32_t srow = tid >> 5, scol = (tid & 31) * 4;
    uint4 sv[2];
    auto stage_load = [&](uint32_t k) {
#pragma unroll
        for (uint32_t i = 0; i < 2; ++i) {
            const uint32_t u = k * V6_UC + srow + 16 * i;
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (u * (uint32_t)npad + c * V6_SB + scol) * 4u, 0, 0);
            sv[i] = make_uint4(v[0], v[1], v[2], v[3]);  // rows past DST read 0 (range-checked)
        }
    };
    auto stage_store = [&](uint32_t buf) {
#pragma unroll
        for (uint32_t i = 0; i < 2; ++i)
            *reinterpret_cast<uint4*>(lb + buf * V6_BUF + (srow + 16 * i) * V6_ROW + scol * 4) = sv[i];
    };
    stage_load(0);
    stage_store(0);
    __syncthreads();
    const uint32_t j = lane & 15, es = lane >> 4;
    const uint32_t lane16 = j * 16;
    // the lane's 8 sources, for the diagonal test (columns past n are skipped: outside PRED)
    uint32_t snode[8];
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i) {
        const uint32_t sl = c * V6_SB + (i < 4 ? 4 * j + i : 64 + 4 * j + (i - 4));
        snode[i] = sl < n ? nodes[sl] : 0xFFFFFFFFu;
    }
    uint2 r0, r1;  // the wave's next two group records
    {
        const uint32_t g0 = (uint32_t)__builtin_amdgcn_readfirstlane(goff[(size_t)b * nK]) >> 2;
        r0 = rec[(size_t)(g0 + wave) * 4 + es];
        r1 = rec[(size_t)(g0 + wave + V6_WAVES) * 4 + es];
    }
    for (uint32_t k = 0; k < nK; ++k) {
        if (k + 1 < nK) stage_load(k + 1);  // issue early, write after the chunk
        const size_t q = (size_t)b * nK + k;
        const uint32_t g0 = (uint32_t)__builtin_amdgcn_readfirstlane(goff[q]) >> 2;
        const uint32_t g1 = (uint32_t)__builtin_amdgcn_readfirstlane(goff[q + 1]) >> 2;
        const uint32_t abase = (k & 1u) * V6_BUF + lane16, dbase = V6_ND + lane16;
        // one group: 4 entries x 128 sources; hits min / max into PRED / PMAX
        auto group = [&](const uint2 r, const uint32_t g) {
            const uint32_t ao = abase + (r.x & 0xFFFFu), dofs = dbase + (r.x >> 16), w = r.y;
            const uint4 a0 = *reinterpret_cast<const uint4*>(lb + ao);
            const uint4 a1 = *reinterpret_cast<const uint4*>(lb + ao + 256);
            const uint4 n0 = *reinterpret_cast<const uint4*>(lb + dofs);
            const uint4 n1 = *reinterpret_cast<const uint4*>(lb + dofs + 256);
            const uint32_t x[8] = {a0.x + n0.x + w, a0.y + n0.y + w, a0.z + n0.z + w, a0.w + n0.w + w,
                                   a1.x + n1.x + w, a1.y + n1.y + w, a1.z + n1.z + w, a1.w + n1.w + w};
            const uint32_t m = min(min(min(x[0], x[1]), min(x[2], x[3])), min(min(x[4], x[5]), min(x[6], x[7])));
            if (__builtin_expect(__ballot(m == 0) != 0, 0)) {
                // hits are ~1 lane in 64 and one of its 8 checks: walk them as scalars (readlane), one
                // single-lane atomic pair each, instead of 8 predicated per-lane passes
                const bool live = w != KeyOps<uint32_t>::INF;  // (w = INF: group padding)
                const uint32_t nd[8] = {n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, n1.z, n1.w};
#pragma unroll
                for (uint32_t i = 0; i < 8; ++i) {
                    unsigned long long hm = __ballot(live && x[i] == 0);
                    while (hm) {
                        const uint32_t L = (uint32_t)__builtin_ctzll(hm);
                        hm &= hm - 1;
                        const uint32_t jj = L & 15;
                        const uint32_t sl = c * V6_SB + (i < 4 ? 4 * jj + i : 64 + 4 * jj + (i - 4));
                        const uint32_t t = b * V6_TT + ((uint32_t)__builtin_amdgcn_readlane(r.x, L) >> 16) / V6_ROW;
                        const uint32_t sn = (uint32_t)__builtin_amdgcn_readlane(snode[i], L);
                        const uint32_t ndl = (uint32_t)__builtin_amdgcn_readlane(nd[i], L);
                        if (sl >= n || sn == t || (inf_check && ndl == 0u - KeyOps<uint32_t>::INF))
                            continue;  // (the diagonal and, u32 keys, unreachable targets stay NONE)
                        const uint32_t e = g * 4 + (L >> 4);
                        const size_t at = (size_t)sl * ldp + t;
                        if (lane == 0) {  // no-return atomics: nothing in the loop waits for them
                            __hip_atomic_fetch_min(PRED + at, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            __hip_atomic_fetch_max(PMAX + at, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        }
                    }
                }
            }
        };
        // the wave's groups g0 + wave, + 8, ...: two records in flight, each register reloaded right
        // after its group, unconditionally (no copies, and in-order counted waits: a conditional
        // reload made the compiler wait for every load at the loop top); the next chunk's first
        // two are issued before the barrier
        uint32_t g = g0 + wave;
        if (g < g1) {
            for (;;) {
                group(r0, g);
                r0 = rec[(size_t)(g + 2 * V6_WAVES) * 4 + es];  // (V6_SLACK past the end)
                g += V6_WAVES;
                if (g >= g1) break;
                group(r1, g);
                r1 = rec[(size_t)(g + 2 * V6_WAVES) * 4 + es];
                g += V6_WAVES;
                if (g >= g1) break;
            }
        }
        if (k + 1 < nK) {
            r0 = rec[(size_t)(g1 + wave) * 4 + es];  // (the next chunk's groups start at g1; V6_SLACK past the end)
            r1 = rec[(size_t)(g1 + wave + V6_WAVES) * 4 + es];
            stage_store((k + 1) & 1u);  // the other buffer: its readers (chunk k - 1) passed the last barrier
            __syncthreads();
        }
    }
}

// PRED = min hit, PMAX = max hit: two different hits -> PRED_MULTI (rows [0, nrows), targets < V)
__global__ void __launch_bounds__(256) k_v6_combine(uint32_t* __restrict__ PRED, const uint32_t* __restrict__ PMAX,
                                                     uint32_t nrows, uint32_t V, size_t ldp) {
    const uint32_t r = blockIdx.y;
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < V; t += gridDim.x * blockDim.x) {
        const size_t i = (size_t)r * ldp + t;
        const uint32_t p = PRED[i];
        if (p != PRED_NONE && PMAX[i] != p) PRED[i] = PRED_MULTI;
    }
    (void)nrows;
}

}  // namespace srg
