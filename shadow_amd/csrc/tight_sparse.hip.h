// tight_sparse.hip.h — tight-predecessor scan over the ESSENTIAL edges (gfx950).
//
// An edge (u,t) can be tight for some source s (D[s][u] + W[u][t] == D[s][t]) only if it is
// itself a shortest path: W[u][t] == D[u][t]  (else D[s][u]+W[u][t] > D[s][u]+D[u][t] >= D[s][t]).
// On Atlas-like graphs only ~8-15% of the V^2 edges are essential, so the scan walks them
// instead of all V^3 (s,u,t) triples.
//
// Layout (all in HBM):
//   DST [Vt x npad] u32  DST[u][r] = D[nodes[r]][u]  (sources on the fast axis -> lanes)
//   pair records per (128-target tile, 64-row u-chunk, 16-target wave slice), see tight_v5;
//   ent_w[e] = W[u][t] (exact key), ent_ub[e] = {u, bits of 1 - loss(u,t)} per entry e
//   csc_off[t] .. csc_off[t+1]: entry indices whose target is t (multi-predecessor slow path)
// Kernels: k_ess_mask (essential bitmask), k_build_dst, k_v5_count / k_v5_fill (records),
// tight_v5 (the scan), k_loss_rows (per-row left fold in LDS) and k_loss_round_sparse (the
// same fold in global memory, for rows too long for LDS).  Variants measured slower in rounds
// 1-2 (one source per lane, entry-vector batches, target runs, records in LDS, four sources
// per lane, ...) were removed; DESIGN.md keeps their measurements.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.hip.h"

namespace srg {

// ---- essential-edge extraction ---------------------------------------------------------
// ESS[u][w64] (u64): bit `lane` set <=> edge u -> t = 64*w64 + lane is essential.  Computed by
// the owner of row u (its rows of D are the only ones it has in the multi-GPU layout) and
// then all-gathered: V^2/8 bytes instead of the V^2 keys of D.
// One workgroup per row u (blockIdx.x = u - u0).  u32 keys: each lane reads 4 targets of W and of D
// as 16-B loads (a wave covers 4 words), its nibble ORed into the word of its 16-lane group by a
// 4-step butterfly; u64 keys: one target per lane and a ballot per word.  (A grid-stride loop over
// (u, word) pairs with a 64-bit division per word ran at ~1.6 TB/s, one word per wave at ~2.2.)
template <class K>
__global__ void __launch_bounds__(256) k_ess_mask(const K* __restrict__ W, const K* __restrict__ D, size_t ld,
                                                   uint32_t V, uint32_t u0, uint32_t u1, uint32_t nw64,
                                                   unsigned long long* __restrict__ ess) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t u = u0 + blockIdx.x;
    if (u >= u1) return;
    const K* Wu = W + (size_t)u * ld;
    const K* Du = D + (size_t)u * ld;
    unsigned long long* eu = ess + (size_t)u * nw64;
    if constexpr (sizeof(K) == 4) {
        // (ld is a multiple of 64 keys: a 16-B load below ld stays inside the padded row)
        for (uint32_t w0 = wave * 4; w0 < nw64; w0 += 16) {
            const uint32_t t = w0 * 64 + lane * 4;
            uint4 a = make_uint4(0u, 0u, 0u, 0u), d = make_uint4(1u, 1u, 1u, 1u);
            if (t < ld) {  // (the words past nw64 in this step: nothing read past the row)
                a = *reinterpret_cast<const uint4*>(Wu + t);
                d = *reinterpret_cast<const uint4*>(Du + t);
            }
            const uint32_t av[4] = {a.x, a.y, a.z, a.w}, dv[4] = {d.x, d.y, d.z, d.w};
            unsigned long long nib = 0;
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j)
                nib |= (unsigned long long)(t + j < V && t + j != u && av[j] != KeyOps<K>::INF && av[j] == dv[j]) << j;
            unsigned long long v = nib << (4 * (lane & 15));
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) v |= __shfl_xor(v, o, 64);
            const uint32_t w = w0 + (lane >> 4);
            if ((lane & 15) == 0 && w < nw64) eu[w] = v;
        }
    } else {
        for (uint32_t w0 = wave; w0 < nw64; w0 += 4) {
            const uint32_t t = w0 * 64 + lane;
            bool e = false;
            if (t < V && t != u) {
                const K w = Wu[t];
                e = (w != KeyOps<K>::INF) && (w == Du[t]);
            }
            const unsigned long long m = __ballot(e);
            if (lane == 0) eu[w0] = m;
        }
    }
}

// DST[u][r] = D[nodes[r]][u] for u < Vt, r < npad (r >= n -> nodes[n-1]); 64x64 LDS tiles.
template <class K>
__global__ void __launch_bounds__(256) k_build_dst(const K* __restrict__ D, size_t ld,
                                                    const uint32_t* __restrict__ nodes, uint32_t n,
                                                    K* __restrict__ DST, size_t npad) {
    __shared__ K tile[64][65];
    const uint32_t ub = blockIdx.x, rb = blockIdx.y;
    const uint32_t tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
    for (uint32_t i = ty; i < 64; i += 4) {
        uint32_t r = rb * 64 + i;
        const uint32_t s = nodes[r < n ? r : n - 1];
        tile[i][tx] = D[(size_t)s * ld + ub * 64 + tx];
    }
    __syncthreads();
    for (uint32_t j = ty; j < 64; j += 4) DST[(size_t)(ub * 64 + j) * npad + rb * 64 + tx] = tile[tx][j];
}

// ---- raw buffer resources ------------------------------------------------------------
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    // raw buffer: stride 0, num_records = bytes, gfx9 dword data format (0x00027000)
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00027000);
}

// ---- pair-lane LDS scan ----------------------------------------------------------------
// A workgroup owns 128 sources x V5_TT targets; lane l holds sources 2l and 2l+1, so ONE
// conflict-free ds_read_b64 (64 lanes x 8 B = the 512-B staged row) feeds two checks per lane:
// half the LDS cycles per check of a b32 row (§LDS table: b64 = 256 B/clk/CU).  Rows of a
// V5_UC-row u-chunk are staged into a double-buffered LDS ring (2 x 32 KB), one barrier per chunk.
// With D the exact closure, a + w >= d for every edge (u, t), so x = a + w - d (mod 2^32, with
// -d held per lane) is the true nonnegative slack and tight <=> x == 0: two v_add3 + a min per
// entry pair and source pair, one compare per pair of entries.  The entry stream of a
// (tile, chunk, wave) is a flat run of 16-B pair records {lo0 | tl << 16, w0, lo1, w1} (both
// entries of a pair share the target tl; odd runs end with a sentinel w = INF), read as 4-pair
// s_load_dwordx16 groups one group ahead, so the loop has no per-target trip counts; -d and the
// per-target state are 16-element register vectors read with the pair's uniform tl.  A hit
// (x == 0 in some lane: ~1 pair in 4) updates St[tl] = entry, or MULTI on a second hit.
constexpr uint32_t V5_WAVES = 8;                 // waves per workgroup
constexpr uint32_t V5_TW = 16;                   // targets per wave
constexpr uint32_t V5_TT = V5_WAVES * V5_TW;     // targets per workgroup tile (128)
constexpr uint32_t V5_UC = 64;                   // u rows per chunk: 64 x 512 B = 32 KB per buffer
constexpr uint32_t V5_SB = 128;                  // sources per workgroup (2 per lane)
constexpr uint32_t V5_SLACK = 256;               // entries past the end (tight_v5 reads one group ahead)

// one wave per (64-target window, chunk), lane = target: entries per (tile b, chunk k, target),
// pairs per (b, k, wave) rounded up to whole 4-pair groups, and indeg[t] for the CSC lists
__global__ void __launch_bounds__(256) k_v5_count(const unsigned long long* __restrict__ ess, uint32_t V,
                                                   uint32_t nw64, uint32_t nK, uint32_t* __restrict__ cnt,
                                                   uint32_t* __restrict__ glen, uint32_t* __restrict__ indeg) {
    const uint32_t lane = threadIdx.x & 63;
    const size_t wv = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
    if (wv >= (size_t)nw64 * nK) return;  // whole wave
    const uint32_t w64 = (uint32_t)(wv / nK), k = (uint32_t)(wv % nK);
    const uint32_t t = w64 * 64 + lane, b = t / V5_TT, tt = t % V5_TT;
    const uint32_t u0 = k * V5_UC, u1 = min(V, u0 + V5_UC);
    uint32_t c = 0;
    for (uint32_t u = u0; u < u1; ++u) c += (uint32_t)((ess[(size_t)u * nw64 + w64] >> lane) & 1ull);
    cnt[((size_t)b * nK + k) * V5_TT + tt] = c;
    if (c) atomicAdd(&indeg[t], c);
    uint32_t p = (c + 1) / 2;
#pragma unroll
    for (int off = 1; off < (int)V5_TW; off <<= 1) p += __shfl_xor(p, off, V5_TW);
    if ((lane % V5_TW) == 0) glen[((size_t)b * nK + k) * V5_WAVES + tt / V5_TW] = (p + 3) / 4 * 4;
}

// CSC positions without atomics: thread t walks the chunks k in order, pos[b][k][tt] = csc_off[t] +
// the entries of t in chunks before k (cnt from k_v5_count); k_v5_fill then stores each target's
// entries at consecutive positions (an atomicAdd per entry held every fill wave on its return)
__global__ void __launch_bounds__(256) k_v5_cscpos(const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ csc_off,
                                                    uint32_t NT, uint32_t nK, uint32_t* __restrict__ pos) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= NT) return;
    const uint32_t b = t / V5_TT, tt = t % V5_TT;
    uint32_t run = csc_off[t];
    for (uint32_t k = 0; k < nK; ++k) {
        const size_t i = ((size_t)b * nK + k) * V5_TT + tt;
        pos[i] = run;
        run += cnt[i];
    }
}

// records rec[e] = (lo | tl << 16, w) for entry e = 2 * pair + slot, plus ent_w / ent_ub
// (k_loss_rows) and the CSC lists (any order: the MULTI fold is a min)
// K = u64 (the u64-key path): records carry the low 32 bits of w (the scan then works on the
// low words of the keys, see tight_v5), ent_w the exact key (the loss pass's multi-predecessor
// check is exact).
template <class K>
__global__ void __launch_bounds__(256) k_v5_fill(const unsigned long long* __restrict__ ess,
                                                  const K* __restrict__ W, const uint32_t* __restrict__ WL,
                                                  size_t ld, uint32_t V, uint32_t nw64, uint32_t nK,
                                                  const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ goff,
                                                  const uint32_t* __restrict__ csc_pos,
                                                  uint2* __restrict__ rec, K* __restrict__ ent_w,
                                                  uint2* __restrict__ ent_ub, uint32_t* __restrict__ csc_ent) {
    const uint32_t lane = threadIdx.x & 63;
    const size_t wv = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
    if (wv >= (size_t)nw64 * nK) return;
    const uint32_t w64 = (uint32_t)(wv / nK), k = (uint32_t)(wv % nK);
    const uint32_t t = w64 * 64 + lane, b = t / V5_TT, tt = t % V5_TT, j = tt % V5_TW;
    const uint32_t c = cnt[((size_t)b * nK + k) * V5_TT + tt];
    const uint32_t p = (c + 1) / 2;
    uint32_t incl = p;
#pragma unroll
    for (int off = 1; off < (int)V5_TW; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off, V5_TW);
        if ((int)j >= off) incl += y;
    }
    const size_t g = ((size_t)b * nK + k) * V5_WAVES + tt / V5_TW;
    const uint32_t pbase = goff[g];
    size_t e = 2 * ((size_t)pbase + incl - p);
    const uint32_t u0 = k * V5_UC, u1 = min(V, u0 + V5_UC);
    uint32_t cp = csc_pos[((size_t)b * nK + k) * V5_TT + tt];  // (k_v5_cscpos)
    // eight rows per step: all their loads in flight before the stores (one row at a time, each
    // lane's dependent load -> store chain ran the kernel at ~0.4 TB/s)
    for (uint32_t ub = u0; ub < u1; ub += 8) {
        bool on[8];
        K wv[8];
        uint32_t lv[8];
#pragma unroll
        for (uint32_t q = 0; q < 8; ++q) {
            const uint32_t u = ub + q;
            on[q] = u < u1 && ((ess[(size_t)u * nw64 + w64] >> lane) & 1ull);
            if (on[q]) {
                wv[q] = W[(size_t)u * ld + t];
                lv[q] = WL[(size_t)u * ld + t];
            }
        }
#pragma unroll
        for (uint32_t q = 0; q < 8; ++q) {
            if (!on[q]) continue;
            const uint32_t u = ub + q;
            rec[e] = make_uint2(((u - u0) * 512u) | ((e & 1) ? 0u : (j << 16)), (uint32_t)wv[q]);  // the pair's target: first slot only
            ent_w[e] = wv[q];
            ent_ub[e] = make_uint2(u, __float_as_uint(__fsub_rn(1.0f, __uint_as_float(lv[q]))));
            csc_ent[cp++] = (uint32_t)e;
            ++e;
        }
    }
    if (c & 1u) {  // odd run: a sentinel second slot (w = INF is never tight on a reachable target)
        rec[e] = make_uint2(0u, KeyOps<uint32_t>::INF);
        ent_w[e] = KeyOps<K>::INF;
        ent_ub[e] = make_uint2(0u, __float_as_uint(1.0f));
    }
    if (j == V5_TW - 1) {  // the slice's group padding
        const uint32_t total = incl;
        for (size_t q = 2 * ((size_t)pbase + total); q < 2 * (size_t)goff[g + 1]; ++q) {
            rec[q] = make_uint2(0u, KeyOps<uint32_t>::INF);
            ent_w[q] = KeyOps<K>::INF;
            ent_ub[q] = make_uint2(0u, __float_as_uint(1.0f));
        }
    }
}

typedef uint32_t v16u_v5 __attribute__((ext_vector_type(16)));
struct alignas(64) V5Grp {
    uint32_t v[16];
};

// u64 keys (inf_check = 0): DST and the record weights hold the LOW 32 bits of the keys, and the
// test a + w == d runs mod 2^32.  That is exact in combination with the loss pass: the true tight
// predecessor of a reachable target always matches, so a single match IS it, and any false
// match (a + w - d a nonzero multiple of 2^32) adds a second one, i.e. PRED_MULTI, which
// k_loss_rows resolves with the exact u64 keys (DST / ent_w of type K).  Targets unreachable
// from the source are not used pairs (certified before the scan) and are no tight predecessor
// of a reachable target, so their entries are never read through a single match.
// grid: 8 * 32 * ceil(nblk / 8) workgroups of 512 for the source blocks [c0, nbS), nblk =
// ceil(nbTT / 4) * ceil((nbS - c0) / 8) blocks of 4 target tiles x 8 source blocks, dealt to the
// XCDs in turn.  XCD-aware: an XCD holds two such blocks at once (2 workgroups per CU), so every
// target tile's pair records are read by 8 workgroups together and every source block's staged
// rows by 4, and both come out of that XCD's L2 after the first read.  (With one source block per
// XCD the rows were shared 64 ways, but every record stream came from the Infinity Cache, and the
// scalar record loads are what each group waits for.)
__global__ void __launch_bounds__(512, 4) tight_v5(const uint32_t* __restrict__ DST, size_t npad, uint32_t dst_bytes,
                                                    const uint32_t* __restrict__ nodes, uint32_t n, uint32_t V,
                                                    uint32_t NT, uint32_t nbTT, uint32_t nbS, uint32_t nK, uint32_t c0,
                                                    const uint32_t* __restrict__ goff, const uint32_t* __restrict__ rec,
                                                    uint32_t* __restrict__ PRED, size_t ldp, uint32_t inf_check) {
    __shared__ __attribute__((aligned(16))) uint32_t rows[2 * V5_UC * V5_SB];  // 2 x 32 KB ring
    const uint32_t bid = blockIdx.x, xcd = bid & 7, slot = bid >> 3;
    const uint32_t blk = (slot >> 5) * 8 + xcd, nbb = (nbTT + 3) / 4;  // block of 4 tiles x 8 source blocks
    const uint32_t b = (blk % nbb) * 4 + (slot & 3), c = c0 + (blk / nbb) * 8 + ((slot >> 2) & 7);
    if (c >= nbS || b >= nbTT) return;  // whole workgroup: no barrier is left waiting
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t r0 = c * V5_SB + 2 * lane;  // this lane's two sources (columns of DST)
    const __amdgpu_buffer_rsrc_t rsrc = make_rsrc(DST, dst_bytes);
    const uint32_t t0 = b * V5_TT + wave * V5_TW;
    const bool active = t0 < NT;  // a wave past the targets still stages and syncs
    v16u_v5 ndl, ndh, stl, sth;
#pragma unroll
    for (uint32_t j = 0; j < V5_TW; ++j) {
        uint32_t dl = 0, dh = 0;
        if (active) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b64(rsrc, ((t0 + j) * (uint32_t)npad + r0) * 4u, 0, 0);
            dl = v[0];
            dh = v[1];
        }
        ndl[j] = 0u - dl;
        ndh[j] = 0u - dh;
        stl[j] = PRED_NONE;
        sth[j] = PRED_NONE;
    }
    // staging: 512 threads x 16 B = 16 rows per pass, 4 passes per 64-row chunk
    const uint32_t srow = tid >> 5, scol = (tid & 31) * 4;
    uint4 sv[4];
    auto stage_load = [&](uint32_t k) {
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) {
            const uint32_t u = k * V5_UC + srow + 16 * i;
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (u * (uint32_t)npad + c * V5_SB + scol) * 4u, 0, 0);
            sv[i] = make_uint4(v[0], v[1], v[2], v[3]);  // rows past DST read 0 (range-checked)
        }
    };
    auto stage_store = [&](uint32_t buf) {
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i)
            *reinterpret_cast<uint4*>(&rows[buf * (V5_UC * V5_SB) + (srow + 16 * i) * V5_SB + scol]) = sv[i];
    };
    stage_load(0);
    stage_store(0);
    __syncthreads();
    const unsigned char* lds = reinterpret_cast<const unsigned char*>(rows);
    for (uint32_t k = 0; k < nK; ++k) {
        if (k + 1 < nK) stage_load(k + 1);  // issue early, write after the chunk
        if (active) {
            const size_t q = ((size_t)b * nK + k) * V5_WAVES + wave;
            const uint32_t p0 = (uint32_t)__builtin_amdgcn_readfirstlane(goff[q]);
            const uint32_t p1 = (uint32_t)__builtin_amdgcn_readfirstlane(goff[q + 1]);
            const uint32_t vb = (k & 1u) * (V5_UC * V5_SB * 4u) + lane * 8u;
            // one 4-pair group: 8 staged-row reads, 16 checks per lane, the hit test
            auto group = [&](const V5Grp& cur, uint32_t p) {
                    uint2 A[8];
#pragma unroll
                    for (uint32_t i = 0; i < 4; ++i) {
                        A[2 * i] = *reinterpret_cast<const uint2*>(lds + vb + (cur.v[4 * i] & 0xFFFFu));
                        A[2 * i + 1] = *reinterpret_cast<const uint2*>(lds + vb + cur.v[4 * i + 2]);
                    }
#pragma unroll
                    for (uint32_t i = 0; i < 4; ++i) {
                        const uint32_t tl = cur.v[4 * i] >> 16;
                        const uint32_t dl = ndl[tl], dh = ndh[tl];
                        const uint32_t w0 = cur.v[4 * i + 1], w1 = cur.v[4 * i + 3];
                        const uint32_t x0l = A[2 * i].x + w0 + dl, x0h = A[2 * i].y + w0 + dh;
                        const uint32_t x1l = A[2 * i + 1].x + w1 + dl, x1h = A[2 * i + 1].y + w1 + dh;
                        const uint32_t m = min(min(x0l, x0h), min(x1l, x1h));
                        if (__builtin_expect(__ballot(m == 0) != 0, 0)) {
                            const uint32_t e0 = 2 * (p + i);
                            uint32_t sl = stl[tl], sh = sth[tl];
                            if (x0l == 0) sl = (sl == PRED_NONE) ? e0 : PRED_MULTI;
                            if (x1l == 0) sl = (sl == PRED_NONE) ? e0 + 1 : PRED_MULTI;
                            if (x0h == 0) sh = (sh == PRED_NONE) ? e0 : PRED_MULTI;
                            if (x1h == 0) sh = (sh == PRED_NONE) ? e0 + 1 : PRED_MULTI;
                            stl[tl] = sl;
                            sth[tl] = sh;
                        }
                    }
            };
            // two record groups in flight in two fixed SGPR sets, loop unrolled by 2: no 16-register
            // copy of the prefetched group per iteration and half the loop-counter work (both were
            // scalar instructions of the loop, which issues more SALU than the CU's one per cycle
            // covers at 16 waves: 1.73e9 SALU per C3 launch, profiles/r05/scan_v6/)
            if (p0 < p1) {
                V5Grp ga = *reinterpret_cast<const V5Grp*>(rec + 4 * (size_t)p0);
                V5Grp gb = *reinterpret_cast<const V5Grp*>(rec + 4 * (size_t)(p0 + 4));
                for (uint32_t p = p0;; p += 8) {
                    group(ga, p);
                    if (p + 4 >= p1) break;
                    ga = *reinterpret_cast<const V5Grp*>(rec + 4 * (size_t)(p + 8));
                    group(gb, p + 4);
                    if (p + 8 >= p1) break;
                    gb = *reinterpret_cast<const V5Grp*>(rec + 4 * (size_t)(p + 12));
                }
            }
        }
        if (k + 1 < nK) {
            stage_store((k + 1) & 1u);  // the other buffer: its readers (chunk k - 1) passed the last barrier
            __syncthreads();
        }
    }
    if (!active) return;
#pragma unroll
    for (uint32_t h = 0; h < 2; ++h) {
        const uint32_t r = r0 + h;
        if (r >= n) continue;
        const uint32_t s = nodes[r];
        uint32_t o[V5_TW];
#pragma unroll
        for (uint32_t j = 0; j < V5_TW; ++j) {
            const uint32_t t = t0 + j;
            const uint32_t nd = h ? ndh[j] : ndl[j];
            const uint32_t st = h ? sth[j] : stl[j];
            o[j] = (t >= V || t == s || (inf_check && nd == 0u - KeyOps<uint32_t>::INF)) ? PRED_NONE : st;
        }
        uint4* out = reinterpret_cast<uint4*>(PRED + (size_t)r * ldp + t0);
#pragma unroll
        for (uint32_t j = 0; j < V5_TW; j += 4) out[j / 4] = make_uint4(o[j], o[j + 1], o[j + 2], o[j + 3]);
    }
}

// PRED rows [r0, r1) -> PK[r][t] = {u, bits of 1 - loss(u,t)} of the single tight predecessor's
// entry, or {PRED_NONE / PRED_MULTI, 0}: the gather k_loss_rows would do per target, done here
// target tile by target tile.  A tile's entries are one contiguous run (~0.8 MB at C3), so with
// every workgroup of tile b on XCD b mod 8 (tiles taken in turn, all source blocks of a tile at
// once) the run stays in that XCD's L2; the loss pass's rows gather across every tile's entries
// (~62 MB at C3: Infinity-Cache misses, 680 us per launch there, 285 us on packed rows).
// Grid: 8 * ntile8 * nsb workgroups of 256 (ntile8 = ceil(nbTT / 8), nsb = source blocks of 128).
// (also counts the PRED_MULTI pairs it passes into *multi: the build's multi_pred_pairs)
__global__ void __launch_bounds__(256) k_pred_pack(const uint32_t* __restrict__ PRED, size_t ldp, uint32_t r0,
                                                   uint32_t r1, uint32_t NT, uint32_t nbTT, uint32_t nsb,
                                                   const uint2* __restrict__ ent_ub, uint2* __restrict__ PK,
                                                   unsigned long long* __restrict__ multi) {
    const uint32_t xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    const uint32_t b = xcd + 8 * (slot / nsb), sb = slot % nsb;
    if (b >= nbTT) return;
    const uint32_t tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8: 4 targets per thread
    const uint32_t t = b * V5_TT + tx * 4;
    const bool tv = t < NT;  // (tight_v5 writes targets < NT = V rounded up to 64; a multiple of 4)
    uint32_t nm = 0;
    // four rows per step: 16 gathers in flight per thread
    for (uint32_t i0 = ty; i0 < 128; i0 += 32) {
        uint32_t pv[4][4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t r = r0 + sb * 128 + i0 + 8 * k;
            uint4 p = make_uint4(PRED_NONE, PRED_NONE, PRED_NONE, PRED_NONE);
            if (tv && r < r1) p = *reinterpret_cast<const uint4*>(PRED + (size_t)r * ldp + t);
            pv[k][0] = p.x;
            pv[k][1] = p.y;
            pv[k][2] = p.z;
            pv[k][3] = p.w;
        }
        uint2 q[4][4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                q[k][j] = pv[k][j] < PRED_MULTI ? ent_ub[pv[k][j]] : make_uint2(pv[k][j], 0u);
                nm += pv[k][j] == PRED_MULTI;  // (rows past r1 hold PRED_NONE)
            }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t r = r0 + sb * 128 + i0 + 8 * k;
            if (!tv || r >= r1) break;
            uint4* o = reinterpret_cast<uint4*>(PK + (size_t)r * ldp + t);
            o[0] = make_uint4(q[k][0].x, q[k][0].y, q[k][1].x, q[k][1].y);
            o[1] = make_uint4(q[k][2].x, q[k][2].y, q[k][3].x, q[k][3].y);
        }
    }
    if (__ballot(nm != 0)) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) nm += __shfl_xor(nm, o, 64);
        if ((threadIdx.x & 63) == 0) atomicAdd(multi, (unsigned long long)nm);
    }
}

// Jacobi round of the left fold over the tight DAG, entries variant.
template <class K>
__global__ void k_loss_round_sparse(const uint32_t* __restrict__ PRED, size_t ldp, const K* __restrict__ DST,
                                    size_t npad, const uint32_t* __restrict__ nodes, uint32_t n, uint32_t V,
                                    const uint2* __restrict__ ent_ub, const K* __restrict__ ent_w,
                                    const uint32_t* __restrict__ csc_off,
                                    const uint32_t* __restrict__ csc_ent, const float* __restrict__ Lin,
                                    float* __restrict__ Lout, uint32_t* __restrict__ changed_flag) {
    const size_t total = (size_t)n * V;
    uint32_t changed = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = i / V, t = i - r * V;
        const uint32_t s = nodes[r];
        const uint32_t p = PRED[r * ldp + t];
        const float* Lrow = Lin + r * ldp;
        float v;
        if (t == s) {
            v = 0.0f;
        } else if (p == PRED_NONE) {
            v = 1.0f;
        } else if (p != PRED_MULTI) {
            const uint2 ub = ent_ub[p];
            v = fold_loss(Lrow[ub.x], __uint_as_float(ub.y));
        } else {
            const K dst = DST[t * npad + r];
            v = 1.0f;
            for (uint32_t k = csc_off[t]; k < csc_off[t + 1]; ++k) {
                const uint32_t e = csc_ent[k];
                const uint2 ub = ent_ub[e];
                if (KeyOps<K>::add(DST[(size_t)ub.x * npad + r], ent_w[e]) != dst) continue;
                const float cnd = fold_loss(Lrow[ub.x], __uint_as_float(ub.y));
                v = cnd < v ? cnd : v;
            }
        }
        Lout[r * ldp + t] = v;
        changed |= (v != Lrow[t]);
    }
    if (changed) atomicOr(changed_flag, 1u);
}

// Per-row left fold in LDS (one workgroup per used source row, Gauss-Seidel sweeps).
//   U[t] = tight predecessor u (or a marker), B[t] = 1 - loss(u,t), L[t] = path loss.
// Sweeps update L in place until a full sweep changes nothing: that state satisfies every
// L[t] = fold(L[U[t]], B[t]) at once, whose solution on the tight DAG is unique (induction on
// depth), so it equals Dijkstra's lexicographic scores (mod.rs:305-331).  Writes the used
// columns of the row straight into out_loss (diagonal = raw self-loop loss, mod.rs:216).
// Targets with several latency-tight predecessors (PRED_MULTI, rare) get their tight in-edges
// collected once, by the whole workgroup scanning the CSC list in parallel, into an LDS list the
// sweeps fold over; one thread walking ~V/10 CSC entries with two dependent global loads per
// entry in every sweep made such rows ~1 ms stragglers (every row-chunk launch waited for one).
// Overflow past LM_T targets / LM_E edges per target falls back to that per-thread walk.
constexpr uint32_t U_SELF = 0xFFFFFFFFu, U_NONE = 0xFFFFFFFEu, U_MULTI = 0xFFFFFFFDu;
constexpr uint32_t U_MLIST = 0xF0000000u;  // U_MLIST + i: multi target i of the LDS list
constexpr uint32_t LM_T = 32, LM_E = 16;
constexpr size_t loss_rows_lds(uint32_t V) { return (size_t)V * 12 + LM_T * (4 + 4 + LM_E * 8) + 16; }

// PK: PRED rows as tight_v5<true> writes them ({u, 1 - loss} or {marker, 0}, ldp uint2 per row)
template <class K, bool PK>
__global__ void __launch_bounds__(1024) k_loss_rows(const uint32_t* __restrict__ PRED, size_t ldp, uint32_t V,
                                                     const uint32_t* __restrict__ nodes, uint32_t n,
                                                     const uint2* __restrict__ ent_ub, const K* __restrict__ ent_w,
                                                     const K* __restrict__ DST, size_t npad,
                                                     const uint32_t* __restrict__ csc_off,
                                                     const uint32_t* __restrict__ csc_ent,
                                                     const float* __restrict__ self_loss,
                                                     const uint32_t* __restrict__ cols, uint32_t ncols,
                                                     const uint32_t* __restrict__ rowpos, float* __restrict__ out_loss,
                                                     uint32_t* __restrict__ max_sweeps, uint32_t row0) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    uint32_t* U = reinterpret_cast<uint32_t*>(smem_raw);
    float* Bf = reinterpret_cast<float*>(U + V);
    float* L = Bf + V;
    uint32_t* m_t = reinterpret_cast<uint32_t*>(L + V);  // [LM_T] multi targets
    uint32_t* m_n = m_t + LM_T;                          // [LM_T] tight in-edges collected
    uint32_t* m_u = m_n + LM_T;                          // [LM_T][LM_E] their sources
    float* m_b = reinterpret_cast<float*>(m_u + LM_T * LM_E);  // [LM_T][LM_E] 1 - loss
    __shared__ uint32_t changed, nm;
    const uint32_t r = row0 + blockIdx.x;  // launched in row chunks (host entry: D2H per chunk)
    const uint32_t s = nodes[r];
    const uint32_t* prow = PRED + (size_t)r * ldp * (PK ? 2 : 1);
    if (threadIdx.x == 0) nm = 0;
    if (threadIdx.x < LM_T) m_n[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < V; t += blockDim.x) {
        uint2 pk = make_uint2(0u, 0u);
        if constexpr (PK) pk = reinterpret_cast<const uint2*>(prow)[t];
        const uint32_t p = PK ? pk.x : prow[t];
        uint32_t u;
        float bb = 1.0f, l = 1.0f;
        if (t == s) {
            u = U_SELF;
            l = 0.0f;  // Dijkstra start score PathProperties::default()
        } else if (p == PRED_NONE) {
            u = U_NONE;
        } else if (p == PRED_MULTI) {
            const uint32_t i = atomicAdd(&nm, 1u);
            u = U_MULTI;
            if (i < LM_T) {
                m_t[i] = t;
                u = U_MLIST + i;
            }
        } else {
            const uint2 ub = PK ? pk : ent_ub[p];  // (one 8-B gather per target: u and 1 - loss together)
            u = ub.x;
            bb = __uint_as_float(ub.y);
        }
        U[t] = u;
        Bf[t] = bb;
        L[t] = l;
    }
    __syncthreads();
    const uint32_t nml = nm < LM_T ? nm : LM_T;
    for (uint32_t i = 0; i < nml; ++i) {  // whole workgroup per multi target
        const uint32_t t = m_t[i];
        const K dst = DST[(size_t)t * npad + r];
        for (uint32_t k = csc_off[t] + threadIdx.x; k < csc_off[t + 1]; k += blockDim.x) {
            const uint32_t e = csc_ent[k];
            const uint2 ub = ent_ub[e];
            const uint32_t uu = ub.x;
            if (KeyOps<K>::add(DST[(size_t)uu * npad + r], ent_w[e]) != dst) continue;
            const uint32_t j = atomicAdd(&m_n[i], 1u);
            if (j < LM_E) {
                m_u[i * LM_E + j] = uu;
                m_b[i * LM_E + j] = __uint_as_float(ub.y);
            }
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nml; i += blockDim.x)
        if (m_n[i] > LM_E) U[m_t[i]] = U_MULTI;  // too many tight in-edges: per-thread walk
    __syncthreads();
    uint32_t sweeps = 0;
    for (;;) {
        if (threadIdx.x == 0) changed = 0;
        __syncthreads();
        uint32_t ch = 0;
        for (uint32_t t = threadIdx.x; t < V; t += blockDim.x) {
            const uint32_t u = U[t];
            if (u >= U_MLIST) {
                if (u >= U_NONE) continue;
                float v = 1.0f;
                if (u == U_MULTI) {
                    // several latency-tight predecessors: min over them (in-edges of t)
                    const K dst = DST[(size_t)t * npad + r];
                    for (uint32_t k = csc_off[t]; k < csc_off[t + 1]; ++k) {
                        const uint32_t e = csc_ent[k];
                        const uint2 ub = ent_ub[e];
                        const uint32_t uu = ub.x;
                        if (KeyOps<K>::add(DST[(size_t)uu * npad + r], ent_w[e]) != dst) continue;
                        const float cnd = fold_loss(L[uu], __uint_as_float(ub.y));
                        v = cnd < v ? cnd : v;
                    }
                } else {
                    const uint32_t i = u - U_MLIST;
                    for (uint32_t j = 0; j < m_n[i]; ++j) {
                        const float cnd = fold_loss(L[m_u[i * LM_E + j]], m_b[i * LM_E + j]);
                        v = cnd < v ? cnd : v;
                    }
                }
                if (v != L[t]) {
                    L[t] = v;
                    ch = 1;
                }
                continue;
            }
            const float v = fold_loss(L[u], Bf[t]);
            if (v != L[t]) {
                L[t] = v;
                ch = 1;
            }
        }
        if (ch) changed = 1;  // benign race: every writer stores 1
        __syncthreads();
        ++sweeps;
        if (!changed) break;
        __syncthreads();
    }
    if (threadIdx.x == 0) atomicMax(max_sweeps, sweeps);
    const uint32_t p = rowpos[r];  // output row = position of s in the full `nodes` list
    float* orow = out_loss + (size_t)p * ncols;
    for (uint32_t j = threadIdx.x; j < ncols; j += blockDim.x) orow[j] = (j == p) ? self_loss[s] : L[cols[j]];
}

}  // namespace srg
