// tight_sparse.hip.h — tight-predecessor scan over the ESSENTIAL edges (gfx950).
//
// An edge (u,t) can be tight for some source s (D[s][u] + W[u][t] == D[s][t]) only if it is
// itself a shortest path: W[u][t] == D[u][t]  (else D[s][u]+W[u][t] > D[s][u]+D[u][t] >= D[s][t]).
// On Atlas-like graphs only ~8-15% of the V^2 edges are essential, so the scan walks them
// instead of all V^3 (s,u,t) triples.
//
// Layout (all in HBM):
//   DST [Vt x npad] K   DST[u][r] = D[nodes[r]][u]  (sources on the fast axis -> lanes)
//   target blocks of TB = 32 targets; the entries of block b are u-sorted and occupy
//   [eblk[b], eblk[b+1]), padded to a multiple of 64 with sentinels (w = INF, tl = 0, u = 0):
//     ent_ro[e] = u * npad * sizeof(K)   (byte offset of DST row u: a buffer-load soffset)
//     ent_w[e]  = W[u][t],  ent_tl[e] = t - 32*b,  ent_u[e] = u,  ent_b[e] = 1 - loss(u,t)
//   csc_off[t] .. csc_off[t+1]: entry indices whose target is t (multi-predecessor slow path)
//
// Scan (u32 keys): one 64-lane wave per (target block b, source block c), lane = source.
// d[tl] = D[s][32b+tl] is a register vector read with the wave-uniform tl (s_set_gpr_idx, no
// LDS, no copies); a hit (rare) updates St[tl][lane] in LDS under a vcc-skipped branch.  The
// entry stream arrives as coalesced 64-entry vector batches broadcast with v_readlane; every
// entry gets its own row load (u-sorted, so repeats hit L1) through a buffer load whose SGPR
// soffset is the precomputed row offset.  Loads are issued on a fully static schedule (two
// 32-entry halves, statically indexed row buffers) so every s_waitcnt is a compile-time count
// (vmcnt is in-order: a load issued under data-dependent control flow would drain the
// prefetch), and the per-entry work is VALU + v_readlane, not SALU (one scalar unit per CU).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "kernels.hip.h"

namespace srg {

constexpr uint32_t TB = 32;  // targets per block of the sparse scan

// ---- essential-edge extraction ---------------------------------------------------------
// ESS[u][w64] (u64): bit `lane` set <=> edge u -> t = 64*w64 + lane is essential.  Computed by
// the owner of row u (its rows of D are the only ones it has in the multi-GPU layout) and
// then all-gathered: V^2/8 bytes instead of the V^2 keys of D.
template <class K>
__global__ void __launch_bounds__(256) k_ess_mask(const K* __restrict__ W, const K* __restrict__ D, size_t ld,
                                                   uint32_t V, uint32_t u0, uint32_t u1, uint32_t nw64,
                                                   unsigned long long* __restrict__ ess) {
    const uint32_t lane = threadIdx.x & 63;
    const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
    const size_t nwaves = ((size_t)gridDim.x * blockDim.x) >> 6;
    const size_t total = (size_t)nw64 * (u1 - u0);
    for (size_t q = wave; q < total; q += nwaves) {
        const uint32_t u = u0 + (uint32_t)(q / nw64), w64 = (uint32_t)(q % nw64);
        const uint32_t t = w64 * 64 + lane;
        bool e = false;
        if (t < V && t != u) {
            const K w = W[(size_t)u * ld + t];
            e = (w != KeyOps<K>::INF) && (w == D[(size_t)u * ld + t]);
        }
        const unsigned long long m = __ballot(e);
        if (lane == 0) ess[(size_t)u * nw64 + w64] = m;
    }
}

__device__ __forceinline__ unsigned long long ess_mask(const unsigned long long* __restrict__ ess, uint32_t nw64,
                                                      uint32_t u, uint32_t w64) {
    return ess[(size_t)u * nw64 + w64];  // wave-uniform load
}

// cnt[b*V + u] = essential edges u -> block b;  indeg[t] for the CSC lists.
__global__ void __launch_bounds__(256) k_ess_count(const unsigned long long* __restrict__ ess, uint32_t V,
                                                    uint32_t nw64, uint32_t* __restrict__ cnt,
                                                    uint32_t* __restrict__ indeg) {
    const uint32_t lane = threadIdx.x & 63;
    const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
    const size_t nwaves = ((size_t)gridDim.x * blockDim.x) >> 6;
    const size_t total = (size_t)nw64 * V;
    for (size_t q = wave; q < total; q += nwaves) {
        const uint32_t w64 = (uint32_t)(q / V), u = (uint32_t)(q - (size_t)w64 * V);
        const unsigned long long m = ess_mask(ess, nw64, u, w64);
        if ((m >> lane) & 1ull) atomicAdd(&indeg[w64 * 64 + lane], 1u);
        if (lane == 0) {
            cnt[(size_t)(2 * w64) * V + u] = (uint32_t)__popcll(m & 0xFFFFFFFFull);
            cnt[(size_t)(2 * w64 + 1) * V + u] = (uint32_t)__popcll(m >> 32);
        }
    }
}

// Padded block bases: eblk[b] = sum_{b' < b} roundup64(total(b')), total from the raw scan.
__global__ void k_ess_blocks(const uint32_t* __restrict__ eoff, const uint32_t* __restrict__ cnt, uint32_t V,
                             uint32_t nb, uint32_t* __restrict__ eblk) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    uint64_t acc = 0;
    for (uint32_t b = 0; b < nb; ++b) {
        eblk[b] = (uint32_t)acc;
        const size_t last = (size_t)b * V + (V - 1);
        const uint64_t tot = (uint64_t)eoff[last] + cnt[last] - eoff[(size_t)b * V];
        acc += (tot + 63) / 64 * 64;
    }
    eblk[nb] = (uint32_t)acc;
}

template <class K>
__global__ void __launch_bounds__(256) k_ess_fill(const unsigned long long* __restrict__ ess,
                                                   const K* __restrict__ W, const uint32_t* __restrict__ WL,
                                                   size_t ld, uint32_t V,
                                                   uint32_t nw64, size_t npad, const uint32_t* __restrict__ eoff,
                                                   const uint32_t* __restrict__ eblk,
                                                   const uint32_t* __restrict__ csc_off,
                                                   uint32_t* __restrict__ csc_fill, uint32_t* __restrict__ ent_ro,
                                                   K* __restrict__ ent_w, uint32_t* __restrict__ ent_tl,
                                                   uint32_t* __restrict__ ent_u, float* __restrict__ ent_b,
                                                   uint32_t* __restrict__ csc_ent, const uint32_t* __restrict__ roff) {
    const uint32_t lane = threadIdx.x & 63;
    const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
    const size_t nwaves = ((size_t)gridDim.x * blockDim.x) >> 6;
    const size_t total = (size_t)nw64 * V;
    for (size_t q = wave; q < total; q += nwaves) {
        const uint32_t w64 = (uint32_t)(q / V), u = (uint32_t)(q - (size_t)w64 * V);
        const unsigned long long m = ess_mask(ess, nw64, u, w64);
        if (!((m >> lane) & 1ull)) continue;
        const uint32_t t = w64 * 64 + lane;
        const uint32_t hb = lane >> 5;  // which 32-target block of the window
        const uint32_t b = 2 * w64 + hb;
        const unsigned long long hm = hb ? (m >> 32) : (m & 0xFFFFFFFFull);
        const uint32_t tl = lane & 31u;
        const uint32_t rank = (uint32_t)__popcll(hm & ((1ull << tl) - 1ull));
        const size_t qb = (size_t)b * V + u;
        const uint32_t k = atomicAdd(&csc_fill[t], 1u);
        // block layout: u-sorted within the 32-target block; run layout: grouped by target
        const uint32_t e = roff ? roff[t] + k : eblk[b] + (eoff[qb] - eoff[(size_t)b * V]) + rank;
        ent_ro[e] = (uint32_t)((size_t)u * npad * sizeof(K));
        ent_w[e] = W[(size_t)u * ld + t];
        ent_tl[e] = tl;
        ent_u[e] = u;
        ent_b[e] = __fsub_rn(1.0f, __uint_as_float(WL[(size_t)u * ld + t]));
        csc_ent[csc_off[t] + k] = e;
    }
}

// Sentinel entries: the block padding [eblk[b] + tot(b), eblk[b+1]) and 256 entries past the
// end (the scan's batch loads run two batches ahead without guards).  grid = nb + 1 blocks.
template <class K>
__global__ void k_ess_pad(const uint32_t* __restrict__ eoff, const uint32_t* __restrict__ cnt,
                          const uint32_t* __restrict__ eblk, uint32_t V, uint32_t nb, uint32_t* __restrict__ ent_ro,
                          K* __restrict__ ent_w, uint32_t* __restrict__ ent_tl, uint32_t* __restrict__ ent_u,
                          float* __restrict__ ent_b) {
    const uint32_t b = blockIdx.x;
    uint32_t beg, end;
    if (b < nb) {
        const size_t last = (size_t)b * V + (V - 1);
        beg = eblk[b] + (eoff[last] + cnt[last] - eoff[(size_t)b * V]);
        end = eblk[b + 1];
    } else {
        beg = eblk[nb];
        end = beg + 256;
    }
    for (uint32_t e = beg + threadIdx.x; e < end; e += blockDim.x) {
        ent_ro[e] = 0;
        ent_w[e] = KeyOps<K>::INF;
        ent_tl[e] = 0;
        ent_u[e] = 0;
        ent_b[e] = 1.0f;
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

__device__ __forceinline__ void sparse_block_coords(uint32_t nbT, uint32_t& b, uint32_t& c) {
    // XCD-aware placement: workgroups bid, bid+8, ... share an XCD (round-robin dispatch), so
    // each XCD gets whole source blocks and re-reads the same DST columns from its own L2.
    const uint32_t bid = blockIdx.x;
    const uint32_t xcd = bid & 7, slot = bid >> 3;
    c = xcd + 8 * (slot / nbT);
    b = slot % nbT;
}

// ---- generic scan (u64 keys): LDS tile + LDS state, straightforward -------------------
template <class K>
__global__ void __launch_bounds__(64) tight_sparse(const K* __restrict__ DST, size_t npad,
                                                    const uint32_t* __restrict__ nodes, uint32_t n, uint32_t V,
                                                    uint32_t nbT, uint32_t nbS, const uint32_t* __restrict__ eblk,
                                                    const uint32_t* __restrict__ ent_u, const K* __restrict__ ent_w,
                                                    const uint32_t* __restrict__ ent_tl, uint32_t* __restrict__ PRED,
                                                    size_t ldp) {
    __shared__ K Dt[TB][64];
    __shared__ uint32_t St[TB][64];
    uint32_t b, c;
    sparse_block_coords(nbT, b, c);
    if (c >= nbS) return;
    const uint32_t lane = threadIdx.x;
    const uint32_t r = c * 64 + lane;
    const K* col = DST + c * 64 + lane;
    for (uint32_t tl = 0; tl < TB; ++tl) {
        Dt[tl][lane] = col[(size_t)(b * TB + tl) * npad];
        St[tl][lane] = PRED_NONE;
    }
    const uint32_t e0 = eblk[b], e1 = eblk[b + 1];
    uint32_t cur_u = 0xFFFFFFFFu;
    K a = 0;
    for (uint32_t e = e0; e < e1; ++e) {
        const uint32_t u = ent_u[e];
        if (u != cur_u) {
            cur_u = u;
            a = col[(size_t)u * npad];
        }
        const uint32_t tl = ent_tl[e];
        if (KeyOps<K>::add(a, ent_w[e]) == Dt[tl][lane]) {
            const uint32_t st = St[tl][lane];
            St[tl][lane] = (st == PRED_NONE) ? e : PRED_MULTI;
        }
    }
    if (r >= n) return;
    const uint32_t s = nodes[r];
    for (uint32_t tl = 0; tl < TB; ++tl) {
        const uint32_t t = b * TB + tl;
        uint32_t v = St[tl][lane];
        if (t >= V || t == s || Dt[tl][lane] == KeyOps<K>::INF) v = PRED_NONE;
        PRED[(size_t)r * ldp + t] = v;
    }
}

// ---- u32 scan: register tile, static load schedule (the hot variant) --------------------
typedef uint32_t v32u __attribute__((ext_vector_type(32)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    // raw buffer: stride 0, num_records = bytes, gfx9 dword data format (0x00027000)
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00027000);
}

#define SRG_HALF(ABUF, WV, TLV, LBASE, EBASE)                                                   \
    _Pragma("unroll") for (int j = 0; j < 32; ++j) {                                            \
        const uint32_t w_ = (uint32_t)__builtin_amdgcn_readlane((WV), (LBASE) + j);             \
        const uint32_t tl_ = (uint32_t)__builtin_amdgcn_readlane((TLV), (LBASE) + j);           \
        const uint32_t x_ = __builtin_elementwise_add_sat(ABUF[j], w_);                          \
        if (x_ == d[tl_]) {                                                                      \
            const uint32_t st_ = St[tl_][lane];                                                  \
            St[tl_][lane] = (st_ == PRED_NONE) ? (EBASE) + j : PRED_MULTI;                       \
        }                                                                                        \
    }
#define SRG_ROWS(ABUF, ROV, LBASE)                                                               \
    _Pragma("unroll") for (int j = 0; j < 32; ++j) {                                            \
        const uint32_t ro_ = (uint32_t)__builtin_amdgcn_readlane((ROV), (LBASE) + j);           \
        ABUF[j] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff, ro_, 0);                      \
    }

__global__ void __launch_bounds__(64) tight_sparse_u32(const uint32_t* __restrict__ DST, size_t npad,
                                                        uint32_t dst_bytes, const uint32_t* __restrict__ nodes,
                                                        uint32_t n, uint32_t V, uint32_t nbT, uint32_t nbS,
                                                        const uint32_t* __restrict__ eblk,
                                                        const uint32_t* __restrict__ ent_ro,
                                                        const uint32_t* __restrict__ ent_w,
                                                        const uint32_t* __restrict__ ent_tl,
                                                        uint32_t* __restrict__ PRED, size_t ldp) {
    __shared__ uint32_t St[TB][64];
    uint32_t b, c;
    sparse_block_coords(nbT, b, c);
    if (c >= nbS) return;
    const uint32_t lane = threadIdx.x;
    const uint32_t r = c * 64 + lane;
    const __amdgpu_buffer_rsrc_t rsrc = make_rsrc(DST, dst_bytes);
    const uint32_t voff = r * 4u;  // this lane's column
    v32u d;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        d[i] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff, (uint32_t)((b * TB + i) * npad * 4u), 0);
        St[i][lane] = PRED_NONE;
    }
    const uint32_t e_beg = eblk[b], e_end = eblk[b + 1];  // a multiple of 64 apart
    if (e_beg < e_end) {
        uint32_t roc = ent_ro[e_beg + lane], wc = ent_w[e_beg + lane], tlc = ent_tl[e_beg + lane];
        uint32_t ron = ent_ro[e_beg + 64 + lane], wn = ent_w[e_beg + 64 + lane], tln = ent_tl[e_beg + 64 + lane];
        uint32_t A0[32], A1[32];
        SRG_ROWS(A0, roc, 0)
        SRG_ROWS(A1, roc, 32)
        for (uint32_t e = e_beg; e < e_end; e += 64) {
            const uint32_t ro2 = ent_ro[e + 128 + lane], w2 = ent_w[e + 128 + lane], tl2 = ent_tl[e + 128 + lane];
            SRG_HALF(A0, wc, tlc, 0, e)
            SRG_ROWS(A0, ron, 0)
            SRG_HALF(A1, wc, tlc, 32, e + 32)
            SRG_ROWS(A1, ron, 32)
            roc = ron;
            wc = wn;
            tlc = tln;
            ron = ro2;
            wn = w2;
            tln = tl2;
        }
    }
    if (r >= n) return;
    const uint32_t s = nodes[r];
    uint32_t* out = PRED + (size_t)r * ldp + b * TB;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        const uint32_t t = b * TB + i;
        uint32_t v = St[i][lane];
        if (t >= V || t == s || d[i] == KeyOps<uint32_t>::INF) v = PRED_NONE;
        out[i] = v;
    }
}

// Variant with scalar entry loads: the entry index is wave-uniform, so (row offset, w, tl) are
// read with s_load into SGPRs (no v_readlane per entry); the hit test is a wave-uniform branch
// (one s_cbranch on the compare mask) and w enters the add as an SGPR operand.  Keys <= INF
// (2^31 - 1) so the plain add never wraps.  Same static load schedule: 32 row loads in flight,
// the next chunk's row for slot j issued right after slot j is consumed.
__global__ void __launch_bounds__(64) tight_sparse_u32_s(const uint32_t* __restrict__ DST, size_t npad,
                                                          uint32_t dst_bytes, const uint32_t* __restrict__ nodes,
                                                          uint32_t n, uint32_t V, uint32_t nbT, uint32_t nbS,
                                                          const uint32_t* __restrict__ eblk,
                                                          const uint32_t* __restrict__ ent_ro,
                                                          const uint32_t* __restrict__ ent_w,
                                                          const uint32_t* __restrict__ ent_tl,
                                                          uint32_t* __restrict__ PRED, size_t ldp) {
    __shared__ uint32_t St[TB][64];
    uint32_t b, c;
    sparse_block_coords(nbT, b, c);
    if (c >= nbS) return;
    const uint32_t lane = threadIdx.x;
    const uint32_t r = c * 64 + lane;
    const __amdgpu_buffer_rsrc_t rsrc = make_rsrc(DST, dst_bytes);
    const uint32_t voff = r * 4u;
    v32u d;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        d[i] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff, (uint32_t)((b * TB + i) * npad * 4u), 0);
        St[i][lane] = PRED_NONE;
    }
    const uint32_t e_beg = __builtin_amdgcn_readfirstlane(eblk[b]);
    const uint32_t e_end = __builtin_amdgcn_readfirstlane(eblk[b + 1]);  // a multiple of 64 apart
    if (e_beg < e_end) {
        // 16-entry groups as 64-B aligned uniform loads -> s_load_dwordx16 (e is a multiple of 32)
        struct alignas(64) U16 {
            uint32_t v[16];
        };
        auto ld16u = [](const uint32_t* p) { return *reinterpret_cast<const U16*>(p); };
        uint32_t A[32];
        {
            const U16 r0 = ld16u(ent_ro + e_beg), r1 = ld16u(ent_ro + e_beg + 16);
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                A[j] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff, r0.v[j], 0);
                A[16 + j] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff, r1.v[j], 0);
            }
        }
        for (uint32_t e = e_beg; e < e_end; e += 32) {
            const U16 w0 = ld16u(ent_w + e), w1 = ld16u(ent_w + e + 16);
            const U16 t0 = ld16u(ent_tl + e), t1 = ld16u(ent_tl + e + 16);
            const U16 n0 = ld16u(ent_ro + e + 32), n1 = ld16u(ent_ro + e + 48);  // next chunk / sentinel pad
#pragma unroll
            for (int j = 0; j < 32; ++j) {
                const uint32_t w = j < 16 ? w0.v[j] : w1.v[j - 16];
                const uint32_t tl = j < 16 ? t0.v[j] : t1.v[j - 16];
                const uint32_t nro = j < 16 ? n0.v[j] : n1.v[j - 16];
                const uint32_t x = A[j] + w;
                const bool hit = x == d[tl];
                if (__builtin_expect(__ballot(hit) != 0, 0)) {
                    if (hit) {
                        const uint32_t st = St[tl][lane];
                        St[tl][lane] = (st == PRED_NONE) ? e + j : PRED_MULTI;
                    }
                }
                A[j] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff, nro, 0);
            }
        }
    }
    if (r >= n) return;
    const uint32_t s = nodes[r];
    uint32_t* out = PRED + (size_t)r * ldp + b * TB;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        const uint32_t t = b * TB + i;
        uint32_t v = St[i][lane];
        if (t >= V || t == s || d[i] == KeyOps<uint32_t>::INF) v = PRED_NONE;
        out[i] = v;
    }
}

// ---- run layout (SRG_OPT_SCAN_VARIANT 2) -------------------------------------------------
// Entries grouped by TARGET: target t's essential in-arcs occupy [roff[t], roff[t] + indeg[t]),
// the run padded with sentinels to a multiple of RUN_CHUNK, runs of one 32-target block
// contiguous.  Every RUN_CHUNK-entry chunk then has ONE target, so the scan reads d[tl] once per
// chunk (instead of a register-indexed read per entry) and counts hits in registers with no
// per-entry branch; St is touched once per chunk, only when a lane hit.
constexpr uint32_t RUN_CHUNK = 16;

__global__ void k_run_len(const uint32_t* __restrict__ indeg, uint32_t V, uint32_t NT, uint32_t* __restrict__ rlen) {
    for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t <= NT; t += (size_t)gridDim.x * blockDim.x)
        rlen[t] = (t < V && t < NT) ? (indeg[t] + RUN_CHUNK - 1) / RUN_CHUNK * RUN_CHUNK : 0u;
}

template <class K>
__global__ void k_run_pad(const uint32_t* __restrict__ indeg, const uint32_t* __restrict__ roff, uint32_t V,
                          uint32_t NT, uint32_t* __restrict__ ent_ro, K* __restrict__ ent_w,
                          uint32_t* __restrict__ ent_tl, uint32_t* __restrict__ ent_u, float* __restrict__ ent_b) {
    for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t <= NT; t += (size_t)gridDim.x * blockDim.x) {
        const uint32_t beg = roff[t] + ((t < V && t < NT) ? indeg[t] : 0u);
        const uint32_t end = t < NT ? roff[t + 1] : roff[NT] + 256u;  // + tail read by the prefetch
        for (uint32_t e = beg; e < end; ++e) {
            ent_ro[e] = 0;
            ent_w[e] = KeyOps<K>::INF;
            ent_tl[e] = (uint32_t)(t % TB);
            ent_u[e] = 0;
            ent_b[e] = 1.0f;
        }
    }
}

// TBR targets per wave (16: the waves resident on one XCD then all work on the same source
// block, whose DST column block (V x 256 B) stays L2-resident)
template <uint32_t TBR>
__global__ void __launch_bounds__(64) tight_sparse_u32_runs(const uint32_t* __restrict__ DST, size_t npad,
                                                             uint32_t dst_bytes, const uint32_t* __restrict__ nodes,
                                                             uint32_t n, uint32_t V, uint32_t nbT, uint32_t nbS,
                                                             const uint32_t* __restrict__ roff,
                                                             const uint32_t* __restrict__ ent_ro,
                                                             const uint32_t* __restrict__ ent_w,
                                                             const uint32_t* __restrict__ ent_tl,
                                                             uint32_t* __restrict__ PRED, size_t ldp) {
    typedef uint32_t vdu __attribute__((ext_vector_type(TBR)));
    __shared__ uint32_t St[TBR][64];
    uint32_t b, c;
    sparse_block_coords(nbT, b, c);  // nbT = number of TBR-target blocks
    if (c >= nbS) return;
    const uint32_t lane = threadIdx.x;
    const uint32_t r = c * 64 + lane;
    const __amdgpu_buffer_rsrc_t rsrc = make_rsrc(DST, dst_bytes);
    const uint32_t voff = r * 4u;
    vdu d;
#pragma unroll
    for (uint32_t i = 0; i < TBR; ++i) {
        d[i] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff, (uint32_t)((b * TBR + i) * npad * 4u), 0);
        St[i][lane] = PRED_NONE;
    }
    const uint32_t e_beg = __builtin_amdgcn_readfirstlane(roff[b * TBR]);
    const uint32_t e_end = __builtin_amdgcn_readfirstlane(roff[b * TBR + TBR]);  // a multiple of RUN_CHUNK apart
    if (e_beg < e_end) {
        struct alignas(64) U16 {
            uint32_t v[RUN_CHUNK];
        };
        auto ld16u = [](const uint32_t* p) { return *reinterpret_cast<const U16*>(p); };
        uint32_t A[RUN_CHUNK];
        {
            const U16 r0 = ld16u(ent_ro + e_beg);
#pragma unroll
            for (uint32_t j = 0; j < RUN_CHUNK; ++j) A[j] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff, r0.v[j], 0);
        }
        for (uint32_t e = e_beg; e < e_end; e += RUN_CHUNK) {
            const U16 w0 = ld16u(ent_w + e);
            const U16 n0 = ld16u(ent_ro + e + RUN_CHUNK);  // the next chunk's rows (or the sentinel tail)
            const uint32_t tl = __builtin_amdgcn_readfirstlane(ent_tl[e]) % TBR;
            const uint32_t dd = d[tl];
            uint32_t cnt = 0, lastj = 0;
#pragma unroll
            for (uint32_t j = 0; j < RUN_CHUNK; ++j) {
                const bool hit = A[j] + w0.v[j] == dd;
                cnt += hit ? 1u : 0u;
                lastj = hit ? j : lastj;
                A[j] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff, n0.v[j], 0);
            }
            if (__ballot(cnt != 0)) {
                if (cnt) {
                    const uint32_t st = St[tl][lane];
                    St[tl][lane] = (st == PRED_NONE && cnt == 1) ? e + lastj : PRED_MULTI;
                }
            }
        }
    }
    if (r >= n) return;
    const uint32_t s = nodes[r];
    uint32_t* out = PRED + (size_t)r * ldp + b * TBR;
#pragma unroll
    for (uint32_t i = 0; i < TBR; ++i) {
        const uint32_t t = b * TBR + i;
        uint32_t v = St[i][lane];
        if (t >= V || t == s || d[i] == KeyOps<uint32_t>::INF) v = PRED_NONE;
        out[i] = v;
    }
}

// ---- LDS-staged scan (SRG_OPT_SCAN_VARIANT 3, the default) -------------------------------
// The gather scans above pull one 256-B DST row out of L2 per (entry, 64-source block): 7.8e10
// checks at C3 deliver 312 GB through the texture path, which caps them at ~4 clk per
// wave-entry.  Here a workgroup owns a 64-source block x LS_TT targets tile and walks the
// sources' DST columns in u-chunks of LS_UC rows staged ONCE into LDS (LS_UC x 256 B); every
// essential entry (u, t) of the tile's targets with u in the chunk then costs one conflict-free
// ds_read_b32 (lane = source) plus ~3.5 VALU ops:
//     m = min(m, (D[s][u] + w) ^ D[s][t])      -- m == 0 <=> some entry of the run is tight
// and only a run with a tight lane (rare: ~1 per (s, t) over all chunks) re-tests its entries
// for the count / the entry index.  Layout: entries grouped by (target tile b, u-chunk k,
// target), each (target, chunk) run padded with sentinels to a multiple of LS_R, so that a
// run has one target; per (b, k, target) the run count lives in ls_nr.
//   ent_lo[e] = (u - k*LS_UC) * 256   (LDS byte offset of u's staged row)
//   ent_w[e] = W[u][t], ent_u[e] = u, ent_b[e] = 1 - loss(u,t)   (shared with k_loss_rows)
// Roofline: LDS bytes, 256 B per wave-entry at 128 B/clk/CU.
constexpr uint32_t LS_WAVES = 8;               // waves per workgroup (512 threads)
constexpr uint32_t LS_TW = 32;                 // targets per wave (D[s][t] in a 32-register vector)
constexpr uint32_t LS_TT = LS_WAVES * LS_TW;   // targets per workgroup tile
constexpr uint32_t LS_UC = 128;                // u rows per staged chunk (32 KB of LDS)
constexpr uint32_t LS_R = 4;                   // entries per run granule

// per (target tile b, chunk k, target tt): entries / runs.  One wave per (64-target window,
// chunk), lane = target; also accumulates indeg[t] for the CSC lists.
__global__ void __launch_bounds__(256) k_ls_count(const unsigned long long* __restrict__ ess, uint32_t V,
                                                   uint32_t nw64, uint32_t nK, uint32_t* __restrict__ cnt,
                                                   uint32_t* __restrict__ nruns, uint32_t* __restrict__ rlen,
                                                   uint32_t* __restrict__ indeg) {
    const uint32_t lane = threadIdx.x & 63;
    const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
    if (wave >= (size_t)nw64 * nK) return;
    const uint32_t w64 = (uint32_t)(wave / nK), k = (uint32_t)(wave % nK);
    const uint32_t t = w64 * 64 + lane, b = t / LS_TT, tt = t % LS_TT;
    const uint32_t u0 = k * LS_UC, u1 = min(V, u0 + LS_UC);
    uint32_t c = 0;
    for (uint32_t u = u0; u < u1; ++u) c += (uint32_t)((ess[(size_t)u * nw64 + w64] >> lane) & 1ull);
    const size_t q = ((size_t)b * nK + k) * LS_TT + tt;
    cnt[q] = c;
    const uint32_t r = (c + LS_R - 1) / LS_R;
    nruns[q] = r;
    rlen[q] = r * LS_R;
    if (c) atomicAdd(&indeg[t], c);
}

// entries of (b, k, t) at roff[q]...: u-sorted, then sentinels (w = INF never tight).  The
// CSC list of t holds its entries in chunk order: rank = entries of t in chunks < k.
__global__ void __launch_bounds__(256) k_ls_fill(const unsigned long long* __restrict__ ess,
                                                  const uint32_t* __restrict__ W, const uint32_t* __restrict__ WL,
                                                  size_t ld, uint32_t V, uint32_t nw64, uint32_t nK,
                                                  const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ roff,
                                                  const uint32_t* __restrict__ csc_off, uint32_t* __restrict__ ent_lo,
                                                  uint32_t* __restrict__ ent_w, uint32_t* __restrict__ ent_u,
                                                  float* __restrict__ ent_b, uint32_t* __restrict__ csc_ent) {
    const uint32_t lane = threadIdx.x & 63;
    const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
    if (wave >= (size_t)nw64 * nK) return;
    const uint32_t w64 = (uint32_t)(wave / nK), k = (uint32_t)(wave % nK);
    const uint32_t t = w64 * 64 + lane, b = t / LS_TT, tt = t % LS_TT;
    const size_t qb = (size_t)b * nK * LS_TT + tt;
    const size_t q = qb + (size_t)k * LS_TT;
    uint32_t crank = 0;
    for (uint32_t k2 = 0; k2 < k; ++k2) crank += cnt[qb + (size_t)k2 * LS_TT];
    const uint32_t cbase = t < V ? csc_off[t] : 0u;
    const uint32_t u0 = k * LS_UC, u1 = min(V, u0 + LS_UC);
    uint32_t e = roff[q];
    for (uint32_t u = u0; u < u1; ++u) {
        if (!((ess[(size_t)u * nw64 + w64] >> lane) & 1ull)) continue;
        ent_lo[e] = (u - u0) * 256u;
        ent_w[e] = W[(size_t)u * ld + t];
        ent_u[e] = u;
        ent_b[e] = __fsub_rn(1.0f, __uint_as_float(WL[(size_t)u * ld + t]));
        csc_ent[cbase + crank++] = e;
        ++e;
    }
    const uint32_t end = roff[q] + (cnt[q] + LS_R - 1) / LS_R * LS_R;
    for (; e < end; ++e) {
        ent_lo[e] = 0;
        ent_w[e] = KeyOps<uint32_t>::INF;
        ent_u[e] = 0;
        ent_b[e] = 1.0f;
    }
}

typedef uint32_t v32u_ls __attribute__((ext_vector_type(32)));
struct alignas(16) LsWin {
    uint32_t v[16];
};
__device__ __forceinline__ LsWin ls_win(const uint32_t* p) { return *reinterpret_cast<const LsWin*>(p); }

// grid: 8 * nbTT * ceil(nbS / 8) workgroups (XCD-aware: the workgroups of one XCD share
// source blocks, so the staged DST column block stays in that XCD's L2).  PRED rows of the
// tile start as PRED_NONE; a target whose runs hold a tight entry for some lane (rare) is
// queued in LDS and resolved after the chunk: count + entry index, read-modify-write of
// PRED (only this workgroup owns those (source, target) pairs).
__global__ void __launch_bounds__(512, 2) tight_lds_u32(const uint32_t* __restrict__ DST, size_t npad,
                                                         uint32_t dst_bytes, const uint32_t* __restrict__ nodes,
                                                         uint32_t n, uint32_t V, uint32_t Vp, uint32_t nbTT,
                                                         uint32_t nbS, uint32_t nK, const uint32_t* __restrict__ nruns,
                                                         const uint32_t* __restrict__ roff,
                                                         const uint32_t* __restrict__ ent_lo,
                                                         const uint32_t* __restrict__ ent_w,
                                                         uint32_t* __restrict__ PRED, size_t ldp) {
    __shared__ __attribute__((aligned(16))) uint32_t chunk[LS_UC * 64];
    __shared__ uint32_t hitq[LS_WAVES][LS_TW][2];  // per wave: (target j, first entry) with a tight lane
    const uint32_t bid = blockIdx.x, xcd = bid & 7, slot = bid >> 3;
    const uint32_t c = xcd + 8 * (slot / nbTT), b = slot % nbTT;
    if (c >= nbS) return;  // whole workgroup: no barrier is left waiting
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t r = c * 64 + lane;
    const __amdgpu_buffer_rsrc_t rsrc = make_rsrc(DST, dst_bytes);
    const uint32_t voff = r * 4u;  // row offsets go into the VGPR offset: range-checked (rows past DST read 0)
    const uint32_t t0 = b * LS_TT + wave * LS_TW;
    const bool active = t0 < Vp;  // a wave past the padded width still stages and syncs
    const bool own_row = active && r < n;
    const uint32_t s = r < n ? nodes[r] : 0xFFFFFFFFu;
    uint32_t* out = PRED + (size_t)r * ldp + t0;
    v32u_ls dd;
#pragma unroll
    for (uint32_t j = 0; j < LS_TW; ++j)
        dd[j] = active ? __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff + (t0 + j) * (uint32_t)npad * 4u, 0, 0)
                       : KeyOps<uint32_t>::INF;
    if (own_row) {
        const uint4 none = make_uint4(PRED_NONE, PRED_NONE, PRED_NONE, PRED_NONE);
#pragma unroll
        for (uint32_t j = 0; j < LS_TW; j += 4) *reinterpret_cast<uint4*>(out + j) = none;
    }
    // staging: thread tid copies rows tid/16 + 32 i (i < LS_UC/32), 16 B at column (tid%16)*4
    constexpr uint32_t ROWS_PER_PASS = LS_WAVES * 64 / 16;
    constexpr uint32_t SR = LS_UC / ROWS_PER_PASS;
    const uint32_t srow = tid >> 4, scol = (tid & 15) * 4;
    uint4 sv[SR];
    auto stage_load = [&](uint32_t k) {
#pragma unroll
        for (uint32_t i = 0; i < SR; ++i) {
            const uint32_t u = k * LS_UC + srow + ROWS_PER_PASS * i;
            const uint32_t off = u * (uint32_t)npad * 4u + (c * 64 + scol) * 4u;
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0);  // rows >= V read 0
            sv[i] = make_uint4(v[0], v[1], v[2], v[3]);
        }
    };
    auto stage_store = [&]() {
#pragma unroll
        for (uint32_t i = 0; i < SR; ++i)
            *reinterpret_cast<uint4*>(&chunk[(srow + ROWS_PER_PASS * i) * 64 + scol]) = sv[i];
    };
    stage_load(0);
    stage_store();
    __syncthreads();
    const unsigned char* lrow = reinterpret_cast<const unsigned char*>(chunk) + lane * 4u;  // this source's column
    auto lds_ld = [&](uint32_t byte_off) { return *reinterpret_cast<const uint32_t*>(lrow + byte_off); };
    for (uint32_t k = 0; k < nK; ++k) {
        if (k + 1 < nK) stage_load(k + 1);  // issue early, write late
        if (active) {
            // per target: D[s][t] from the register vector (uniform index), a 16-entry window of
            // (ls_lo, w) in SGPRs, one scalar-load wait per target; up to 4 runs from the
            // window, longer runs (rare) in a loop.  m = 0 in a lane <=> a tight entry there.
            const size_t q0 = ((size_t)b * nK + k) * LS_TT + wave * LS_TW;
            const uint32_t* nrp = nruns + q0;
            uint32_t e_c = (uint32_t)__builtin_amdgcn_readfirstlane(roff[q0]);
            uint32_t nq = 0;
            for (uint32_t j = 0; j < LS_TW; ++j) {
                const uint32_t nr_c = nrp[j];
                if (nr_c) {
                    const LsWin lo_c = ls_win(ent_lo + e_c), w_c = ls_win(ent_w + e_c);
                    const uint32_t dj = dd[j];
                    uint32_t m = 0xFFFFFFFFu;
#pragma unroll
                    for (uint32_t i = 0; i < 4; ++i) {
                        if (nr_c > i) {
                            const uint32_t x0 = lds_ld(lo_c.v[4 * i]), x1 = lds_ld(lo_c.v[4 * i + 1]);
                            const uint32_t x2 = lds_ld(lo_c.v[4 * i + 2]), x3 = lds_ld(lo_c.v[4 * i + 3]);
                            m = min(m, min((x0 + w_c.v[4 * i]) ^ dj, (x1 + w_c.v[4 * i + 1]) ^ dj));
                            m = min(m, min((x2 + w_c.v[4 * i + 2]) ^ dj, (x3 + w_c.v[4 * i + 3]) ^ dj));
                        }
                    }
                    for (uint32_t ri = 4; ri < nr_c; ++ri) {
                        const uint32_t e = e_c + LS_R * ri;
                        const uint4 lo = *reinterpret_cast<const uint4*>(ent_lo + e);
                        const uint4 wv = *reinterpret_cast<const uint4*>(ent_w + e);
                        const uint32_t x0 = lds_ld(lo.x), x1 = lds_ld(lo.y), x2 = lds_ld(lo.z), x3 = lds_ld(lo.w);
                        m = min(m, min((x0 + wv.x) ^ dj, (x1 + wv.y) ^ dj));
                        m = min(m, min((x2 + wv.z) ^ dj, (x3 + wv.w) ^ dj));
                    }
                    if (__builtin_expect(__ballot(m == 0) != 0, 0)) {
                        if (lane == 0) {
                            hitq[wave][nq][0] = j;
                            hitq[wave][nq][1] = e_c;
                        }
                        ++nq;
                    }
                }
                e_c += LS_R * nr_c;
            }
            // resolve the queued targets: count the tight entries per lane, keep the entry index
            __builtin_amdgcn_wave_barrier();
            for (uint32_t qi = 0; qi < nq; ++qi) {
                const uint32_t j = hitq[wave][qi][0], e0 = hitq[wave][qi][1];
                const uint32_t runs = nrp[j];
                const uint32_t t = t0 + j;
                const uint32_t dj = __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff + t * (uint32_t)npad * 4u, 0, 0);
                uint32_t cnt = 0, last = 0;
                for (uint32_t ri = 0; ri < runs; ++ri) {
                    const uint32_t e = e0 + LS_R * ri;
                    const uint4 lo = *reinterpret_cast<const uint4*>(ent_lo + e);
                    const uint4 wv = *reinterpret_cast<const uint4*>(ent_w + e);
                    const uint32_t h0 = lds_ld(lo.x) + wv.x == dj, h1 = lds_ld(lo.y) + wv.y == dj;
                    const uint32_t h2 = lds_ld(lo.z) + wv.z == dj, h3 = lds_ld(lo.w) + wv.w == dj;
                    cnt += h0 + h1 + h2 + h3;
                    last = h3 ? e + 3 : h2 ? e + 2 : h1 ? e + 1 : h0 ? e : last;
                }
                if (cnt && own_row && t < V && t != s && dj != KeyOps<uint32_t>::INF) {
                    const uint32_t sj = out[j];
                    out[j] = (sj == PRED_NONE && cnt == 1) ? last : PRED_MULTI;
                }
            }
        }
        if (k + 1 < nK) {
            __syncthreads();  // every wave is done with chunk k
            stage_store();
            __syncthreads();
        }
    }
}

// Variant 4: the LDS-staged scan with the entry stream in VECTOR registers.  Variant 3 read
// each target's entries with scalar loads: one dependent scalar-cache round trip per target
// (the scalar cache misses on a 265 KB-per-workgroup stream) kept its waves parked ~70 % of the
// time (profiles/r02/scan_v3_lds_pmc.txt).  Here a wave loads its chunk's entries 64 at a time
// with coalesced vector loads, one batch ahead, and broadcasts each entry with v_readlane;
// the per-target run counts arrive the same way (lane j = target j).
__global__ void __launch_bounds__(512, 2) tight_lds_u32_rl(const uint32_t* __restrict__ DST, size_t npad,
                                                            uint32_t dst_bytes, const uint32_t* __restrict__ nodes,
                                                            uint32_t n, uint32_t V, uint32_t Vp, uint32_t nbTT,
                                                            uint32_t nbS, uint32_t nK,
                                                            const uint32_t* __restrict__ nruns,
                                                            const uint32_t* __restrict__ roff,
                                                            const uint32_t* __restrict__ ent_lo,
                                                            const uint32_t* __restrict__ ent_w,
                                                            uint32_t* __restrict__ PRED, size_t ldp) {
    __shared__ __attribute__((aligned(16))) uint32_t chunk[LS_UC * 64];
    __shared__ uint32_t hitq[LS_WAVES][LS_TW][2];
    const uint32_t bid = blockIdx.x, xcd = bid & 7, slot = bid >> 3;
    const uint32_t c = xcd + 8 * (slot / nbTT), b = slot % nbTT;
    if (c >= nbS) return;  // whole workgroup
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t r = c * 64 + lane;
    const __amdgpu_buffer_rsrc_t rsrc = make_rsrc(DST, dst_bytes);
    const uint32_t voff = r * 4u;  // row offsets in the VGPR offset: range-checked
    const uint32_t t0 = b * LS_TT + wave * LS_TW;
    const bool active = t0 < Vp;
    const bool own_row = active && r < n;
    const uint32_t s = r < n ? nodes[r] : 0xFFFFFFFFu;
    uint32_t* out = PRED + (size_t)r * ldp + t0;
    v32u_ls dd;
#pragma unroll
    for (uint32_t j = 0; j < LS_TW; ++j)
        dd[j] = active ? __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff + (t0 + j) * (uint32_t)npad * 4u, 0, 0)
                       : KeyOps<uint32_t>::INF;
    if (own_row) {
        const uint4 none = make_uint4(PRED_NONE, PRED_NONE, PRED_NONE, PRED_NONE);
#pragma unroll
        for (uint32_t j = 0; j < LS_TW; j += 4) *reinterpret_cast<uint4*>(out + j) = none;
    }
    constexpr uint32_t ROWS_PER_PASS = LS_WAVES * 64 / 16;
    constexpr uint32_t SR = LS_UC / ROWS_PER_PASS;
    const uint32_t srow = tid >> 4, scol = (tid & 15) * 4;
    uint4 sv[SR];
    auto stage_load = [&](uint32_t k) {
#pragma unroll
        for (uint32_t i = 0; i < SR; ++i) {
            const uint32_t u = k * LS_UC + srow + ROWS_PER_PASS * i;
            const uint32_t off = u * (uint32_t)npad * 4u + (c * 64 + scol) * 4u;
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0);
            sv[i] = make_uint4(v[0], v[1], v[2], v[3]);
        }
    };
    auto stage_store = [&]() {
#pragma unroll
        for (uint32_t i = 0; i < SR; ++i)
            *reinterpret_cast<uint4*>(&chunk[(srow + ROWS_PER_PASS * i) * 64 + scol]) = sv[i];
    };
    stage_load(0);
    stage_store();
    __syncthreads();
    const unsigned char* lrow = reinterpret_cast<const unsigned char*>(chunk) + lane * 4u;
    auto lds_ld = [&](uint32_t byte_off) { return *reinterpret_cast<const uint32_t*>(lrow + byte_off); };
    for (uint32_t k = 0; k < nK; ++k) {
        if (k + 1 < nK) stage_load(k + 1);  // issue early, write late
        if (active) {
            const size_t q0 = ((size_t)b * nK + k) * LS_TT + wave * LS_TW;
            const uint32_t nrv = lane < LS_TW ? nruns[q0 + lane] : 0u;
            uint32_t e = (uint32_t)__builtin_amdgcn_readfirstlane(roff[q0]);
            uint32_t eb = e & ~63u;  // entry batch base (the allocation has 256 entries of slack)
            uint32_t lo_c = ent_lo[eb + lane], w_c = ent_w[eb + lane];
            uint32_t lo_n = ent_lo[eb + 64 + lane], w_n = ent_w[eb + 64 + lane];
            uint32_t nq = 0;
            for (uint32_t j = 0; j < LS_TW; ++j) {
                const uint32_t runs = (uint32_t)__builtin_amdgcn_readlane((int)nrv, (int)j);
                if (!runs) continue;
                const uint32_t dj = dd[j];
                const uint32_t e_t = e;
                uint32_t m = 0xFFFFFFFFu;
                for (uint32_t ri = 0; ri < runs; ++ri, e += LS_R) {
                    if (e - eb >= 64) {  // next entry batch (a run never straddles one)
                        eb += 64;
                        lo_c = lo_n;
                        w_c = w_n;
                        lo_n = ent_lo[eb + 64 + lane];
                        w_n = ent_w[eb + 64 + lane];
                    }
                    const int i = (int)(e - eb);
                    const uint32_t l0 = (uint32_t)__builtin_amdgcn_readlane((int)lo_c, i);
                    const uint32_t l1 = (uint32_t)__builtin_amdgcn_readlane((int)lo_c, i + 1);
                    const uint32_t l2 = (uint32_t)__builtin_amdgcn_readlane((int)lo_c, i + 2);
                    const uint32_t l3 = (uint32_t)__builtin_amdgcn_readlane((int)lo_c, i + 3);
                    const uint32_t w0 = (uint32_t)__builtin_amdgcn_readlane((int)w_c, i);
                    const uint32_t w1 = (uint32_t)__builtin_amdgcn_readlane((int)w_c, i + 1);
                    const uint32_t w2 = (uint32_t)__builtin_amdgcn_readlane((int)w_c, i + 2);
                    const uint32_t w3 = (uint32_t)__builtin_amdgcn_readlane((int)w_c, i + 3);
                    const uint32_t x0 = lds_ld(l0), x1 = lds_ld(l1), x2 = lds_ld(l2), x3 = lds_ld(l3);
                    m = min(m, min((x0 + w0) ^ dj, (x1 + w1) ^ dj));
                    m = min(m, min((x2 + w2) ^ dj, (x3 + w3) ^ dj));
                }
                if (__builtin_expect(__ballot(m == 0) != 0, 0)) {
                    if (lane == 0) {
                        hitq[wave][nq][0] = j;
                        hitq[wave][nq][1] = e_t;
                    }
                    ++nq;
                }
            }
            // resolve the queued targets (rare): count the tight entries, keep the entry index
            __builtin_amdgcn_wave_barrier();
            for (uint32_t qi = 0; qi < nq; ++qi) {
                const uint32_t j = hitq[wave][qi][0], e0 = hitq[wave][qi][1];
                const uint32_t runs = nruns[q0 + j];
                const uint32_t t = t0 + j;
                const uint32_t dj = __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff + t * (uint32_t)npad * 4u, 0, 0);
                uint32_t cnt = 0, last = 0;
                for (uint32_t ri = 0; ri < runs; ++ri) {
                    const uint32_t e1 = e0 + LS_R * ri;
                    const uint4 lo = *reinterpret_cast<const uint4*>(ent_lo + e1);
                    const uint4 wv = *reinterpret_cast<const uint4*>(ent_w + e1);
                    const uint32_t h0 = lds_ld(lo.x) + wv.x == dj, h1 = lds_ld(lo.y) + wv.y == dj;
                    const uint32_t h2 = lds_ld(lo.z) + wv.z == dj, h3 = lds_ld(lo.w) + wv.w == dj;
                    cnt += h0 + h1 + h2 + h3;
                    last = h3 ? e1 + 3 : h2 ? e1 + 2 : h1 ? e1 + 1 : h0 ? e1 : last;
                }
                if (cnt && own_row && t < V && t != s && dj != KeyOps<uint32_t>::INF) {
                    const uint32_t sj = out[j];
                    out[j] = (sj == PRED_NONE && cnt == 1) ? last : PRED_MULTI;
                }
            }
        }
        if (k + 1 < nK) {
            __syncthreads();
            stage_store();
            __syncthreads();
        }
    }
}

// ---- pair-lane LDS scan (SRG_OPT_SCAN_VARIANT 5) ------------------------------------------
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
constexpr uint32_t V5_SLACK = 256;               // entries past the end (v5 reads one group ahead, v6 a 64-pair batch)

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

// records rec[e] = (lo | tl << 16, w) for entry e = 2 * pair + slot, plus ent_w / ent_u / ent_b
// (k_loss_rows) and the CSC lists (any order: the MULTI fold is a min)
// K = u64 (the u64-key path): records carry the low 32 bits of w (the scan then works on the
// low words of the keys, see tight_v5), ent_w the exact key (the loss pass's multi-predecessor
// check is exact).
template <class K>
__global__ void __launch_bounds__(256) k_v5_fill(const unsigned long long* __restrict__ ess,
                                                  const K* __restrict__ W, const uint32_t* __restrict__ WL,
                                                  size_t ld, uint32_t V, uint32_t nw64, uint32_t nK,
                                                  const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ goff,
                                                  const uint32_t* __restrict__ csc_off, uint32_t* __restrict__ csc_fill,
                                                  uint2* __restrict__ rec, K* __restrict__ ent_w,
                                                  uint32_t* __restrict__ ent_u, float* __restrict__ ent_b,
                                                  uint32_t* __restrict__ csc_ent) {
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
    const uint32_t cbase = t < V ? csc_off[t] : 0u;
    for (uint32_t u = u0; u < u1; ++u) {
        if (!((ess[(size_t)u * nw64 + w64] >> lane) & 1ull)) continue;
        const K w = W[(size_t)u * ld + t];
        rec[e] = make_uint2(((u - u0) * 512u) | ((e & 1) ? 0u : (j << 16)), (uint32_t)w);  // the pair's target: first slot only
        ent_w[e] = w;
        ent_u[e] = u;
        ent_b[e] = __fsub_rn(1.0f, __uint_as_float(WL[(size_t)u * ld + t]));
        csc_ent[cbase + atomicAdd(&csc_fill[t], 1u)] = (uint32_t)e;
        ++e;
    }
    if (c & 1u) {  // odd run: a sentinel second slot (w = INF is never tight on a reachable target)
        rec[e] = make_uint2(0u, KeyOps<uint32_t>::INF);
        ent_w[e] = KeyOps<K>::INF;
        ent_u[e] = 0;
        ent_b[e] = 1.0f;
    }
    if (j == V5_TW - 1) {  // the slice's group padding
        const uint32_t total = incl;
        for (size_t q = 2 * ((size_t)pbase + total); q < 2 * (size_t)goff[g + 1]; ++q) {
            rec[q] = make_uint2(0u, KeyOps<uint32_t>::INF);
            ent_w[q] = KeyOps<K>::INF;
            ent_u[q] = 0;
            ent_b[q] = 1.0f;
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
// grid: 8 * nbTT * ceil((nbS - c0) / 8) workgroups of 512 for the source blocks [c0, nbS)
// (XCD-aware: the workgroups of one XCD share the 128-source block, whose staged rows then come
// out of that XCD's L2)
__global__ void __launch_bounds__(512, 4) tight_v5(const uint32_t* __restrict__ DST, size_t npad, uint32_t dst_bytes,
                                                    const uint32_t* __restrict__ nodes, uint32_t n, uint32_t V,
                                                    uint32_t NT, uint32_t nbTT, uint32_t nbS, uint32_t nK, uint32_t c0,
                                                    const uint32_t* __restrict__ goff, const uint32_t* __restrict__ rec,
                                                    uint32_t* __restrict__ PRED, size_t ldp, uint32_t inf_check) {
    __shared__ __attribute__((aligned(16))) uint32_t rows[2 * V5_UC * V5_SB];  // 2 x 32 KB ring
    const uint32_t bid = blockIdx.x, xcd = bid & 7, slot = bid >> 3;
    const uint32_t c = c0 + xcd + 8 * (slot / nbTT), b = slot % nbTT;
    if (c >= nbS) return;  // whole workgroup: no barrier is left waiting
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
            if (p0 < p1) {
                V5Grp cur = *reinterpret_cast<const V5Grp*>(rec + 4 * (size_t)p0);
                for (uint32_t p = p0; p < p1; p += 4) {
                    const V5Grp nxt = *reinterpret_cast<const V5Grp*>(rec + 4 * (size_t)(p + 4));
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
                    cur = nxt;
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

// Variant 11: variant 5 with one hit test per 4-pair group.  v5's ISA checks each pair with its
// own v_cmp -> vcc -> s_cbranch (a VALU -> SALU round trip per pair that serialises the four
// independent pairs of a group); here the four pairs' slacks are computed first and one ballot
// of their min guards the (per-pair) state updates.
__global__ void __launch_bounds__(512, 4) tight_v11(const uint32_t* __restrict__ DST, size_t npad, uint32_t dst_bytes,
                                                    const uint32_t* __restrict__ nodes, uint32_t n, uint32_t V,
                                                    uint32_t NT, uint32_t nbTT, uint32_t nbS, uint32_t nK, uint32_t c0,
                                                    const uint32_t* __restrict__ goff, const uint32_t* __restrict__ rec,
                                                    uint32_t* __restrict__ PRED, size_t ldp, uint32_t inf_check) {
    __shared__ __attribute__((aligned(16))) uint32_t rows[2 * V5_UC * V5_SB];  // 2 x 32 KB ring
    const uint32_t bid = blockIdx.x, xcd = bid & 7, slot = bid >> 3;
    const uint32_t c = c0 + xcd + 8 * (slot / nbTT), b = slot % nbTT;
    if (c >= nbS) return;  // whole workgroup: no barrier is left waiting
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
            if (p0 < p1) {
                V5Grp cur = *reinterpret_cast<const V5Grp*>(rec + 4 * (size_t)p0);
                for (uint32_t p = p0; p < p1; p += 4) {
                    const V5Grp nxt = *reinterpret_cast<const V5Grp*>(rec + 4 * (size_t)(p + 4));
                    uint2 A[8];
#pragma unroll
                    for (uint32_t i = 0; i < 4; ++i) {
                        A[2 * i] = *reinterpret_cast<const uint2*>(lds + vb + (cur.v[4 * i] & 0xFFFFu));
                        A[2 * i + 1] = *reinterpret_cast<const uint2*>(lds + vb + cur.v[4 * i + 2]);
                    }
                    // all four pairs' slacks first (independent chains), one hit test per group
                    uint32_t X[4][4], mg = 0xFFFFFFFFu;
#pragma unroll
                    for (uint32_t i = 0; i < 4; ++i) {
                        const uint32_t tl = cur.v[4 * i] >> 16;
                        const uint32_t dl = ndl[tl], dh = ndh[tl];
                        const uint32_t w0 = cur.v[4 * i + 1], w1 = cur.v[4 * i + 3];
                        X[i][0] = A[2 * i].x + w0 + dl;
                        X[i][1] = A[2 * i].y + w0 + dh;
                        X[i][2] = A[2 * i + 1].x + w1 + dl;
                        X[i][3] = A[2 * i + 1].y + w1 + dh;
                        mg = min(mg, min(min(X[i][0], X[i][1]), min(X[i][2], X[i][3])));
                    }
                    if (__builtin_expect(__ballot(mg == 0) != 0, 0)) {
#pragma unroll
                        for (uint32_t i = 0; i < 4; ++i) {
                            const uint32_t m = min(min(X[i][0], X[i][1]), min(X[i][2], X[i][3]));
                            if (__ballot(m == 0) == 0) continue;
                            const uint32_t tl = cur.v[4 * i] >> 16;
                            const uint32_t e0 = 2 * (p + i);
                            uint32_t sl = stl[tl], sh = sth[tl];
                            if (X[i][0] == 0) sl = (sl == PRED_NONE) ? e0 : PRED_MULTI;
                            if (X[i][2] == 0) sl = (sl == PRED_NONE) ? e0 + 1 : PRED_MULTI;
                            if (X[i][1] == 0) sh = (sh == PRED_NONE) ? e0 : PRED_MULTI;
                            if (X[i][3] == 0) sh = (sh == PRED_NONE) ? e0 + 1 : PRED_MULTI;
                            stl[tl] = sl;
                            sth[tl] = sh;
                        }
                    }
                    cur = nxt;
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

// Variant 6: variant 5 with the record stream in VECTOR registers.  v5's 4-pair s_load groups
// cost one scalar-cache round trip per group that no other work covers (the s_waitcnt for a
// scalar load also drains every LDS read): 58 % of its wave cycles were waits
// (profiles/r02/pmc_v5).  Here each wave loads its chunk's records 64 pairs at a time with one
// coalesced 16-B-per-lane load, issued a whole chunk ahead (vmcnt is in order), and broadcasts
// pair j with four v_readlane; the rest of the pair's work is v5's.
__global__ void __launch_bounds__(512, 4) tight_v6(const uint32_t* __restrict__ DST, size_t npad, uint32_t dst_bytes,
                                                    const uint32_t* __restrict__ nodes, uint32_t n, uint32_t V,
                                                    uint32_t NT, uint32_t nbTT, uint32_t nbS, uint32_t nK, uint32_t c0,
                                                    const uint32_t* __restrict__ goff, const uint32_t* __restrict__ rec,
                                                    uint32_t* __restrict__ PRED, size_t ldp, uint32_t inf_check) {
    __shared__ __attribute__((aligned(16))) uint32_t rows[2 * V5_UC * V5_SB];  // 2 x 32 KB ring
    const uint32_t bid = blockIdx.x, xcd = bid & 7, slot = bid >> 3;
    const uint32_t c = c0 + xcd + 8 * (slot / nbTT), b = slot % nbTT;
    if (c >= nbS) return;  // whole workgroup
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t r0 = c * V5_SB + 2 * lane;
    const __amdgpu_buffer_rsrc_t rsrc = make_rsrc(DST, dst_bytes);
    const uint32_t t0 = b * V5_TT + wave * V5_TW;
    const bool active = t0 < NT;
    const uint4* rec4 = reinterpret_cast<const uint4*>(rec);
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
    const uint32_t srow = tid >> 5, scol = (tid & 31) * 4;
    uint4 sv[4];
    auto stage_load = [&](uint32_t k) {
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) {
            const uint32_t u = k * V5_UC + srow + 16 * i;
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (u * (uint32_t)npad + c * V5_SB + scol) * 4u, 0, 0);
            sv[i] = make_uint4(v[0], v[1], v[2], v[3]);
        }
    };
    auto stage_store = [&](uint32_t buf) {
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i)
            *reinterpret_cast<uint4*>(&rows[buf * (V5_UC * V5_SB) + (srow + 16 * i) * V5_SB + scol]) = sv[i];
    };
    auto slice = [&](uint32_t k, uint32_t& p0, uint32_t& p1) {
        const size_t q = ((size_t)b * nK + k) * V5_WAVES + wave;
        p0 = (uint32_t)__builtin_amdgcn_readfirstlane(goff[q]);
        p1 = (uint32_t)__builtin_amdgcn_readfirstlane(goff[q + 1]);
    };
    // loads are issued unconditionally (clamped indices) so that every wait is a counted vmcnt:
    // a load issued under a condition makes the compiler drain all of them
    stage_load(0);
    uint32_t p0, p1;
    slice(0, p0, p1);
    uint4 rc = rec4[p0 + lane];  // chunk 0's first 64 pairs (the array has slack past the end)
    stage_store(0);
    __syncthreads();
    const unsigned char* lds = reinterpret_cast<const unsigned char*>(rows);
    struct Pair {
        uint2 a0, a1;
        uint32_t h0, w0, w1;
    };
    for (uint32_t k = 0; k < nK; ++k) {
        const uint32_t kn = min(k + 1, nK - 1);
        stage_load(kn);
        uint32_t q0, q1;
        slice(kn, q0, q1);
        const uint4 rn = rec4[q0 + lane];  // the next chunk's first records, a whole chunk ahead
        const uint32_t vb = (k & 1u) * (V5_UC * V5_SB * 4u) + lane * 8u;
        auto fetch = [&](const uint4& r, int j) {
            Pair P;
            P.h0 = (uint32_t)__builtin_amdgcn_readlane((int)r.x, j);
            P.w0 = (uint32_t)__builtin_amdgcn_readlane((int)r.y, j);
            const uint32_t h1 = (uint32_t)__builtin_amdgcn_readlane((int)r.z, j);
            P.w1 = (uint32_t)__builtin_amdgcn_readlane((int)r.w, j);
            P.a0 = *reinterpret_cast<const uint2*>(lds + vb + (P.h0 & 0xFFFFu));
            P.a1 = *reinterpret_cast<const uint2*>(lds + vb + h1);
            return P;
        };
        auto check = [&](const Pair& P, uint32_t pair) {
            const uint32_t tl = P.h0 >> 16;
            const uint32_t dl = ndl[tl], dh = ndh[tl];
            const uint32_t x0l = P.a0.x + P.w0 + dl, x0h = P.a0.y + P.w0 + dh;
            const uint32_t x1l = P.a1.x + P.w1 + dl, x1h = P.a1.y + P.w1 + dh;
            const uint32_t m = min(min(x0l, x0h), min(x1l, x1h));
            if (__builtin_expect(__ballot(m == 0) != 0, 0)) {
                const uint32_t e0 = 2 * pair;
                uint32_t sl = stl[tl], sh = sth[tl];
                if (x0l == 0) sl = (sl == PRED_NONE) ? e0 : PRED_MULTI;
                if (x1l == 0) sl = (sl == PRED_NONE) ? e0 + 1 : PRED_MULTI;
                if (x0h == 0) sh = (sh == PRED_NONE) ? e0 : PRED_MULTI;
                if (x1h == 0) sh = (sh == PRED_NONE) ? e0 + 1 : PRED_MULTI;
                stl[tl] = sl;
                sth[tl] = sh;
            }
        };
        if (active && p1 > p0) {
            // the first 64 pairs: pair j + 1's LDS reads are in flight while pair j is checked
            const uint32_t np = min(64u, p1 - p0);  // a multiple of 4
            Pair cur = fetch(rc, 0);
            for (uint32_t g = 0; g < np; g += 4) {
#pragma unroll
                for (uint32_t i = 0; i < 4; ++i) {
                    const int jn = (int)min(g + i + 1, 63u);
                    const Pair nxt = fetch(rc, jn);
                    check(cur, p0 + g + i);
                    cur = nxt;
                }
            }
            // slices longer than 64 pairs (rare): the rest in line
            for (uint32_t base = p0 + 64; base < p1; base += 64) {
                const uint4 rx = rec4[base + lane];
                const uint32_t nx = min(64u, p1 - base);
                for (uint32_t j = 0; j < nx; ++j) check(fetch(rx, (int)j), base + j);
            }
        }
        p0 = q0;
        p1 = q1;
        rc = rn;
        if (k + 1 < nK) {
            stage_store((k + 1) & 1u);
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

// Variant 7: variant 5 with the record stream staged in LDS next to the rows.  v5 reads each
// 4-pair group with an s_load from the record array (L2 / Infinity Cache latency, one group
// ahead) and its s_waitcnt also drains the LDS row reads; here chunk k+1's rows AND records (the
// 8 wave slices of a chunk are one contiguous range) are copied into the other LDS buffers by
// LDS-DMA (global_load_lds, no staging registers) while chunk k is checked, so the loop issues
// only LDS reads.  The slice bounds (goff) of chunk k+2 are vector-loaded a chunk ahead; the
// end-of-chunk barrier drains every DMA.  Slices past V7_RC staged pairs read the rest with
// uniform vector loads.  V7_PIPE = 1: the next group's records are read behind the current
// group's rows.
constexpr uint32_t V7_RC = 448;  // staged pairs per chunk and buffer (7 waves x 64 lanes x 16 B)

template <int PIPE, int DBG = 0>
__global__ void __launch_bounds__(512, 4) tight_v7(const uint32_t* __restrict__ DST, size_t npad, uint32_t dst_bytes,
                                                    const uint32_t* __restrict__ nodes, uint32_t n, uint32_t V,
                                                    uint32_t NT, uint32_t nbTT, uint32_t nbS, uint32_t nK, uint32_t c0,
                                                    const uint32_t* __restrict__ goff, const uint32_t* __restrict__ rec,
                                                    uint32_t* __restrict__ PRED, size_t ldp, uint32_t inf_check) {
    __shared__ __attribute__((aligned(16))) uint32_t rows[2 * V5_UC * V5_SB];  // 2 x 32 KB ring
    __shared__ __attribute__((aligned(16))) uint4 recs[2 * V7_RC];             // 2 x 7 KB record ring
    const uint32_t bid = blockIdx.x, xcd = bid & 7, slot = bid >> 3;
    const uint32_t c = c0 + xcd + 8 * (slot / nbTT), b = slot % nbTT;
    if (c >= nbS) return;  // whole workgroup: no barrier is left waiting
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t r0 = c * V5_SB + 2 * lane;
    const __amdgpu_buffer_rsrc_t rsrc = make_rsrc(DST, dst_bytes);
    const uint32_t t0 = b * V5_TT + wave * V5_TW;
    const bool active = t0 < NT;
    const uint4* rec4 = reinterpret_cast<const uint4*>(rec);
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
    // lane j < 9 of every wave holds goff[(b*nK + k)*8 + j] of a chunk k
    auto go_load = [&](uint32_t k) { return goff[((size_t)b * nK + min(k, nK - 1)) * V5_WAVES + min(lane, V5_WAVES)]; };
    // LDS-DMA of chunk k's rows and records into buffer buf (lane-linear 1-KB pieces per wave)
    auto stage = [&](uint32_t k, uint32_t buf, uint32_t gk) {
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) {  // rows 2*wave + 16*i, +1: 512 B each
            const uint32_t u = k * V5_UC + 2 * wave + 16 * i + (lane >> 5);
            const uint32_t* src = DST + (size_t)min(u, V - 1) * npad + c * V5_SB + (lane & 31) * 4;
            __builtin_amdgcn_global_load_lds(src, &rows[buf * (V5_UC * V5_SB) + (2 * wave + 16 * i) * V5_SB], 16, 0, 0);
        }
        const uint32_t rbase = (uint32_t)__builtin_amdgcn_readlane((int)gk, 0);
        const uint32_t rend = (uint32_t)__builtin_amdgcn_readlane((int)gk, (int)V5_WAVES);
        const uint32_t rcnt = min(rend - rbase, V7_RC);
        if (wave * 64 < rcnt) {  // wave-uniform; lanes past rcnt copy a clamped (unused) record
            const uint32_t p = rbase + min(wave * 64 + lane, rcnt - 1);
            __builtin_amdgcn_global_load_lds(&rec4[p], &recs[buf * V7_RC + wave * 64], 16, 0, 0);
        }
    };
    uint32_t gcur = go_load(0);
    stage(0, 0, gcur);
    uint32_t gnext = go_load(1);
    __syncthreads();
    const unsigned char* lds = reinterpret_cast<const unsigned char*>(rows);
    for (uint32_t k = 0; k < nK; ++k) {
        const uint32_t buf = k & 1u;
        uint32_t gafter = 0;
        if (k + 1 < nK) {
            stage(k + 1, buf ^ 1u, gnext);  // the other buffers: their readers (chunk k - 1) passed the last barrier
            gafter = go_load(k + 2);
        }
        if (active && DBG != 1) {  // DBG (timing experiments only, wrong results): 1 = no pair loop
            const uint32_t base = (uint32_t)__builtin_amdgcn_readlane((int)gcur, 0);
            const uint32_t p0 = (uint32_t)__builtin_amdgcn_readlane((int)gcur, (int)wave);
            const uint32_t p1 = (uint32_t)__builtin_amdgcn_readlane((int)gcur, (int)wave + 1);
            const uint32_t vb = buf * (V5_UC * V5_SB * 4u) + lane * 8u;
            const uint4* rl = recs + buf * V7_RC;
            auto grp = [&](uint32_t p, uint4* R) {  // the 4 records of pair group p (uniform)
                const uint32_t li = p - base;
                if (li + 4 <= V7_RC) {
#pragma unroll
                    for (uint32_t i = 0; i < 4; ++i) R[i] = rl[li + i];
                } else {
#pragma unroll
                    for (uint32_t i = 0; i < 4; ++i) R[i] = rec4[p + i];
                }
            };
            auto check = [&](const uint4* R, const uint2* A, uint32_t p) {
#pragma unroll
                for (uint32_t i = 0; i < 4; ++i) {
                    const uint32_t tl = (uint32_t)__builtin_amdgcn_readfirstlane((int)R[i].x) >> 16;
                    const uint32_t dl = ndl[tl], dh = ndh[tl];
                    const uint32_t w0 = R[i].y, w1 = R[i].w;
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
            if (p0 < p1) {
                uint4 R[4];
                grp(p0, R);
                for (uint32_t p = p0; p < p1; p += 4) {
                    uint2 A[8];
#pragma unroll
                    for (uint32_t i = 0; i < 4; ++i) {
                        if constexpr (DBG == 2) {  // 2 = no row reads
                            A[2 * i] = make_uint2(R[i].x, R[i].z);
                            A[2 * i + 1] = make_uint2(R[i].z, R[i].x);
                        } else {
                            A[2 * i] = *reinterpret_cast<const uint2*>(lds + vb + (R[i].x & 0xFFFFu));
                            A[2 * i + 1] = *reinterpret_cast<const uint2*>(lds + vb + R[i].z);
                        }
                    }
                    if constexpr (PIPE) {
                        uint4 Rn[4];
                        grp(min(p + 4, p1 - 4), Rn);  // the next group's records behind the row reads
                        check(R, A, p);
#pragma unroll
                        for (uint32_t i = 0; i < 4; ++i) R[i] = Rn[i];
                    } else {
                        check(R, A, p);
                        if (p + 4 < p1) grp(p + 4, R);
                    }
                }
            }
        }
        gcur = gnext;
        gnext = gafter;
        if (k + 1 < nK) __syncthreads();  // drains the DMAs of chunk k + 1 (vmcnt) and orders the buffers
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

// Variant 9: variant 7's LDS staging with the per-pair scalar chain removed.  The timing
// decomposition of v7 put 9.6 of its 18.6 ms stage in the pair loop's own instruction chain, and
// v5's PMC counted 11.5 SALU instructions per pair (register indexing of the pair's target with
// s_set_gpr_idx, record copies, per-pair branches) against one scalar unit per CU.  Here the 16
// targets of a wave are a statically unrolled loop (their -d and state registers are plain
// operands), each target's pairs (its run of the slice, count from k_v5_count) a short dynamic
// loop two pairs at a time (both pairs' records and rows read before either is checked), and
// the hit test is one ballot per two pairs.
__global__ void __launch_bounds__(512, 4) tight_v9(const uint32_t* __restrict__ DST, size_t npad, uint32_t dst_bytes,
                                                    const uint32_t* __restrict__ nodes, uint32_t n, uint32_t V,
                                                    uint32_t NT, uint32_t nbTT, uint32_t nbS, uint32_t nK, uint32_t c0,
                                                    const uint32_t* __restrict__ goff, const uint32_t* __restrict__ rec,
                                                    const uint32_t* __restrict__ ecnt, uint32_t* __restrict__ PRED,
                                                    size_t ldp, uint32_t inf_check) {
    __shared__ __attribute__((aligned(16))) uint32_t rows[2 * V5_UC * V5_SB];  // 2 x 32 KB ring
    __shared__ __attribute__((aligned(16))) uint4 recs[2 * V7_RC];             // 2 x 7 KB record ring
    const uint32_t bid = blockIdx.x, xcd = bid & 7, slot = bid >> 3;
    const uint32_t c = c0 + xcd + 8 * (slot / nbTT), b = slot % nbTT;
    if (c >= nbS) return;  // whole workgroup: no barrier is left waiting
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t r0 = c * V5_SB + 2 * lane;
    const __amdgpu_buffer_rsrc_t rsrc = make_rsrc(DST, dst_bytes);
    const uint32_t t0 = b * V5_TT + wave * V5_TW;
    const bool active = t0 < NT;
    const uint4* rec4 = reinterpret_cast<const uint4*>(rec);
    uint32_t ndl[V5_TW], ndh[V5_TW], stl[V5_TW], sth[V5_TW];
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
    auto go_load = [&](uint32_t k) { return goff[((size_t)b * nK + min(k, nK - 1)) * V5_WAVES + min(lane, V5_WAVES)]; };
    // lane j < 16: entries of target t0 + j in chunk k
    auto cnt_load = [&](uint32_t k) {
        return ecnt[((size_t)b * nK + min(k, nK - 1)) * V5_TT + wave * V5_TW + (lane & (V5_TW - 1))];
    };
    auto stage = [&](uint32_t k, uint32_t buf, uint32_t gk) {
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) {
            const uint32_t u = k * V5_UC + 2 * wave + 16 * i + (lane >> 5);
            const uint32_t* src = DST + (size_t)min(u, V - 1) * npad + c * V5_SB + (lane & 31) * 4;
            __builtin_amdgcn_global_load_lds(src, &rows[buf * (V5_UC * V5_SB) + (2 * wave + 16 * i) * V5_SB], 16, 0, 0);
        }
        const uint32_t rbase = (uint32_t)__builtin_amdgcn_readlane((int)gk, 0);
        const uint32_t rend = (uint32_t)__builtin_amdgcn_readlane((int)gk, (int)V5_WAVES);
        const uint32_t rcnt = min(rend - rbase, V7_RC);
        if (wave * 64 < rcnt) {
            const uint32_t p = rbase + min(wave * 64 + lane, rcnt - 1);
            __builtin_amdgcn_global_load_lds(&rec4[p], &recs[buf * V7_RC + wave * 64], 16, 0, 0);
        }
    };
    uint32_t gcur = go_load(0), ccur = cnt_load(0);
    stage(0, 0, gcur);
    uint32_t gnext = go_load(1), cnext = cnt_load(1);
    __syncthreads();
    const unsigned char* lds = reinterpret_cast<const unsigned char*>(rows);
    for (uint32_t k = 0; k < nK; ++k) {
        const uint32_t buf = k & 1u;
        uint32_t gafter = 0, cafter = 0;
        if (k + 1 < nK) {
            stage(k + 1, buf ^ 1u, gnext);
            gafter = go_load(k + 2);
            cafter = cnt_load(k + 2);
        }
        if (active) {
            const uint32_t base = (uint32_t)__builtin_amdgcn_readlane((int)gcur, 0);
            uint32_t p = (uint32_t)__builtin_amdgcn_readlane((int)gcur, (int)wave);
            const uint32_t vb = buf * (V5_UC * V5_SB * 4u) + lane * 8u;
            const uint4* rl = recs + buf * V7_RC;
            auto rd = [&](uint32_t q) -> uint4 {  // record of pair q (uniform)
                const uint32_t li = q - base;
                return li < V7_RC ? rl[li] : rec4[q];
            };
#pragma unroll
            for (uint32_t j = 0; j < V5_TW; ++j) {
                const uint32_t np = ((uint32_t)__builtin_amdgcn_readlane((int)ccur, (int)j) + 1u) >> 1;
                const uint32_t pend = p + np;
                const uint32_t dl = ndl[j], dh = ndh[j];
                for (; p < pend; p += 2) {
                    const bool two = p + 1 < pend;
                    const uint4 R0 = rd(p), R1 = rd(two ? p + 1 : p);
                    const uint2 a00 = *reinterpret_cast<const uint2*>(lds + vb + (R0.x & 0xFFFFu));
                    const uint2 a01 = *reinterpret_cast<const uint2*>(lds + vb + R0.z);
                    const uint2 a10 = *reinterpret_cast<const uint2*>(lds + vb + (R1.x & 0xFFFFu));
                    const uint2 a11 = *reinterpret_cast<const uint2*>(lds + vb + R1.z);
                    const uint32_t y0l = a00.x + R0.y + dl, y0h = a00.y + R0.y + dh;
                    const uint32_t y1l = a01.x + R0.w + dl, y1h = a01.y + R0.w + dh;
                    uint32_t z0l = a10.x + R1.y + dl, z0h = a10.y + R1.y + dh;
                    uint32_t z1l = a11.x + R1.w + dl, z1h = a11.y + R1.w + dh;
                    if (!two) z0l = z0h = z1l = z1h = 1u;  // the second pair is the first again: no hit
                    const uint32_t m = min(min(min(y0l, y0h), min(y1l, y1h)), min(min(z0l, z0h), min(z1l, z1h)));
                    if (__builtin_expect(__ballot(m == 0) != 0, 0)) {
                        const uint32_t e0 = 2 * p, e1 = e0 + 2;
                        uint32_t sl = stl[j], sh = sth[j];
                        if (y0l == 0) sl = (sl == PRED_NONE) ? e0 : PRED_MULTI;
                        if (y1l == 0) sl = (sl == PRED_NONE) ? e0 + 1 : PRED_MULTI;
                        if (z0l == 0) sl = (sl == PRED_NONE) ? e1 : PRED_MULTI;
                        if (z1l == 0) sl = (sl == PRED_NONE) ? e1 + 1 : PRED_MULTI;
                        if (y0h == 0) sh = (sh == PRED_NONE) ? e0 : PRED_MULTI;
                        if (y1h == 0) sh = (sh == PRED_NONE) ? e0 + 1 : PRED_MULTI;
                        if (z0h == 0) sh = (sh == PRED_NONE) ? e1 : PRED_MULTI;
                        if (z1h == 0) sh = (sh == PRED_NONE) ? e1 + 1 : PRED_MULTI;
                        stl[j] = sl;
                        sth[j] = sh;
                    }
                }
                p = pend;
            }
        }
        gcur = gnext;
        gnext = gafter;
        ccur = cnext;
        cnext = cafter;
        if (k + 1 < nK) __syncthreads();  // drains the DMAs of chunk k + 1 (vmcnt) and orders the buffers
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

// Variant 10: variant 5 with FOUR sources per lane (256 per workgroup).  v5's time goes to the
// per-pair instruction chain (record -> target index -> -d -> adds -> min -> compare -> branch),
// whose cost does not depend on how many sources a lane checks; here one ds_read_b128 of the
// staged 1-KB row feeds four sources, so each pair's chain is paid for 8 checks per lane instead
// of 4, and the records are streamed once per 256 sources instead of per 128.  Same records as
// v5 (the row offset lo = (u - u0) * 512 is doubled for the 1-KB rows); the u-chunk ring is 2 x
// 64 KB (one workgroup per CU, 2 waves per SIMD).
constexpr uint32_t V10_SB = 256;  // sources per workgroup (4 per lane)
typedef uint32_t v16u_v10 __attribute__((ext_vector_type(16)));
__global__ void __launch_bounds__(512) tight_v10(const uint32_t* __restrict__ DST, size_t npad, uint32_t dst_bytes,
                                                  const uint32_t* __restrict__ nodes, uint32_t n, uint32_t V,
                                                  uint32_t NT, uint32_t nbTT, uint32_t nbS, uint32_t nK, uint32_t c0,
                                                  const uint32_t* __restrict__ goff, const uint32_t* __restrict__ rec,
                                                  uint32_t* __restrict__ PRED, size_t ldp, uint32_t inf_check) {
    extern __shared__ __attribute__((aligned(16))) uint32_t rows10[];  // 2 x V5_UC x V10_SB (128 KB)
    const uint32_t bid = blockIdx.x, xcd = bid & 7, slot = bid >> 3;
    const uint32_t c = c0 + xcd + 8 * (slot / nbTT), b = slot % nbTT;
    if (c >= nbS) return;  // whole workgroup: no barrier is left waiting
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t r0 = c * V10_SB + 4 * lane;  // this lane's four sources (columns of DST)
    const __amdgpu_buffer_rsrc_t rsrc = make_rsrc(DST, dst_bytes);
    const uint32_t t0 = b * V5_TT + wave * V5_TW;
    const bool active = t0 < NT;  // a wave past the targets still stages and syncs
    v16u_v10 nd0, nd1, nd2, nd3, s0, s1, s2, s3;
#pragma unroll
    for (uint32_t j = 0; j < V5_TW; ++j) {
        uint32_t d[4] = {0, 0, 0, 0};
        if (active) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, ((t0 + j) * (uint32_t)npad + r0) * 4u, 0, 0);
            d[0] = v[0];
            d[1] = v[1];
            d[2] = v[2];
            d[3] = v[3];
        }
        nd0[j] = 0u - d[0];
        nd1[j] = 0u - d[1];
        nd2[j] = 0u - d[2];
        nd3[j] = 0u - d[3];
        s0[j] = s1[j] = s2[j] = s3[j] = PRED_NONE;
    }
    // staging by LDS-DMA (no staging registers: the -d and state vectors need them): each wave
    // loads 8 of the chunk's 64 rows, one 1-KB row per instruction (16 B per lane)
    auto stage = [&](uint32_t k, uint32_t buf) {
#pragma unroll
        for (uint32_t i = 0; i < 8; ++i) {
            const uint32_t u = k * V5_UC + wave + 8 * i;  // rows >= V are never referenced by a record
            const uint32_t* src = DST + (size_t)min(u, V - 1) * npad + c * V10_SB + lane * 4;
            __builtin_amdgcn_global_load_lds(src, &rows10[buf * (V5_UC * V10_SB) + (wave + 8 * i) * V10_SB], 16, 0, 0);
        }
    };
    stage(0, 0);
    __syncthreads();  // drains the DMAs (vmcnt) and publishes the rows
    const unsigned char* lds = reinterpret_cast<const unsigned char*>(rows10);
    for (uint32_t k = 0; k < nK; ++k) {
        // the slice bounds are loaded before the next chunk's DMAs are issued, so waiting for
        // them (vmcnt is in order) does not wait for the DMAs
        const size_t q = ((size_t)b * nK + k) * V5_WAVES + wave;
        const uint32_t g0 = goff[q], g1 = goff[q + 1];
        if (k + 1 < nK) stage(k + 1, (k + 1) & 1u);  // the other buffer: its readers (chunk k - 1) passed the last barrier
        if (active) {
            const uint32_t p0 = (uint32_t)__builtin_amdgcn_readfirstlane(g0);
            const uint32_t p1 = (uint32_t)__builtin_amdgcn_readfirstlane(g1);
            const uint32_t vb = (k & 1u) * (V5_UC * V10_SB * 4u) + lane * 16u;
            if (p0 < p1) {
                V5Grp cur = *reinterpret_cast<const V5Grp*>(rec + 4 * (size_t)p0);
                for (uint32_t p = p0; p < p1; p += 4) {
                    const V5Grp nxt = *reinterpret_cast<const V5Grp*>(rec + 4 * (size_t)(p + 4));
                    uint4 A[8];
#pragma unroll
                    for (uint32_t i = 0; i < 4; ++i) {
                        A[2 * i] = *reinterpret_cast<const uint4*>(lds + vb + 2u * (cur.v[4 * i] & 0xFFFFu));
                        A[2 * i + 1] = *reinterpret_cast<const uint4*>(lds + vb + 2u * cur.v[4 * i + 2]);
                    }
#pragma unroll
                    for (uint32_t i = 0; i < 4; ++i) {
                        const uint32_t tl = cur.v[4 * i] >> 16;
                        const uint32_t d0 = nd0[tl], d1 = nd1[tl], d2 = nd2[tl], d3 = nd3[tl];
                        const uint32_t w0 = cur.v[4 * i + 1], w1 = cur.v[4 * i + 3];
                        const uint4 a = A[2 * i], e = A[2 * i + 1];
                        const uint32_t x00 = a.x + w0 + d0, x01 = a.y + w0 + d1, x02 = a.z + w0 + d2, x03 = a.w + w0 + d3;
                        const uint32_t x10 = e.x + w1 + d0, x11 = e.y + w1 + d1, x12 = e.z + w1 + d2, x13 = e.w + w1 + d3;
                        const uint32_t m = min(min(min(x00, x01), min(x02, x03)), min(min(x10, x11), min(x12, x13)));
                        if (__builtin_expect(__ballot(m == 0) != 0, 0)) {
                            const uint32_t e0 = 2 * (p + i);
                            uint32_t q0 = s0[tl], q1 = s1[tl], q2 = s2[tl], q3 = s3[tl];
                            if (x00 == 0) q0 = (q0 == PRED_NONE) ? e0 : PRED_MULTI;
                            if (x10 == 0) q0 = (q0 == PRED_NONE) ? e0 + 1 : PRED_MULTI;
                            if (x01 == 0) q1 = (q1 == PRED_NONE) ? e0 : PRED_MULTI;
                            if (x11 == 0) q1 = (q1 == PRED_NONE) ? e0 + 1 : PRED_MULTI;
                            if (x02 == 0) q2 = (q2 == PRED_NONE) ? e0 : PRED_MULTI;
                            if (x12 == 0) q2 = (q2 == PRED_NONE) ? e0 + 1 : PRED_MULTI;
                            if (x03 == 0) q3 = (q3 == PRED_NONE) ? e0 : PRED_MULTI;
                            if (x13 == 0) q3 = (q3 == PRED_NONE) ? e0 + 1 : PRED_MULTI;
                            s0[tl] = q0;
                            s1[tl] = q1;
                            s2[tl] = q2;
                            s3[tl] = q3;
                        }
                    }
                    cur = nxt;
                }
            }
        }
        if (k + 1 < nK) __syncthreads();  // drains chunk k + 1's DMAs and orders the buffers
    }
    if (!active) return;
#pragma unroll
    for (uint32_t h = 0; h < 4; ++h) {
        const uint32_t r = r0 + h;
        if (r >= n) continue;
        const uint32_t s = nodes[r];
        uint32_t o[V5_TW];
#pragma unroll
        for (uint32_t j = 0; j < V5_TW; ++j) {
            const uint32_t t = t0 + j;
            const uint32_t nd = h == 0 ? nd0[j] : h == 1 ? nd1[j] : h == 2 ? nd2[j] : nd3[j];
            const uint32_t st = h == 0 ? s0[j] : h == 1 ? s1[j] : h == 2 ? s2[j] : s3[j];
            o[j] = (t >= V || t == s || (inf_check && nd == 0u - KeyOps<uint32_t>::INF)) ? PRED_NONE : st;
        }
        uint4* out = reinterpret_cast<uint4*>(PRED + (size_t)r * ldp + t0);
#pragma unroll
        for (uint32_t j = 0; j < V5_TW; j += 4) out[j / 4] = make_uint4(o[j], o[j + 1], o[j + 2], o[j + 3]);
    }
}

// Jacobi round of the left fold over the tight DAG, entries variant.
template <class K>
__global__ void k_loss_round_sparse(const uint32_t* __restrict__ PRED, size_t ldp, const K* __restrict__ DST,
                                    size_t npad, const uint32_t* __restrict__ nodes, uint32_t n, uint32_t V,
                                    const uint32_t* __restrict__ ent_u, const K* __restrict__ ent_w,
                                    const float* __restrict__ ent_b, const uint32_t* __restrict__ csc_off,
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
            v = fold_loss(Lrow[ent_u[p]], ent_b[p]);
        } else {
            const K dst = DST[t * npad + r];
            v = 1.0f;
            for (uint32_t k = csc_off[t]; k < csc_off[t + 1]; ++k) {
                const uint32_t e = csc_ent[k];
                const uint32_t u = ent_u[e];
                if (KeyOps<K>::add(DST[(size_t)u * npad + r], ent_w[e]) != dst) continue;
                const float cnd = fold_loss(Lrow[u], ent_b[e]);
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

template <class K>
__global__ void __launch_bounds__(1024) k_loss_rows(const uint32_t* __restrict__ PRED, size_t ldp, uint32_t V,
                                                     const uint32_t* __restrict__ nodes, uint32_t n,
                                                     const uint32_t* __restrict__ ent_u,
                                                     const float* __restrict__ ent_b, const K* __restrict__ ent_w,
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
    const uint32_t* prow = PRED + (size_t)r * ldp;
    if (threadIdx.x == 0) nm = 0;
    if (threadIdx.x < LM_T) m_n[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < V; t += blockDim.x) {
        const uint32_t p = prow[t];
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
            u = ent_u[p];
            bb = ent_b[p];
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
            const uint32_t uu = ent_u[e];
            if (KeyOps<K>::add(DST[(size_t)uu * npad + r], ent_w[e]) != dst) continue;
            const uint32_t j = atomicAdd(&m_n[i], 1u);
            if (j < LM_E) {
                m_u[i * LM_E + j] = uu;
                m_b[i * LM_E + j] = ent_b[e];
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
                        const uint32_t uu = ent_u[e];
                        if (KeyOps<K>::add(DST[(size_t)uu * npad + r], ent_w[e]) != dst) continue;
                        const float cnd = fold_loss(L[uu], ent_b[e]);
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
