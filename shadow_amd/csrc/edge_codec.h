// edge_codec.h -- host side of the sequential-pair H2D codec (routing.hip codec_in).
//
// A row-ordered edge list (GML complete graphs: (i, i), (i, i+1), ..., (i, V-1), then row i+1)
// needs no endpoints over PCIe: an edge (s, d) that follows (s, d - 1) is implied, and only the
// others cross as exceptions (chunk-local index, src, dst).  The device rebuilds edge i of a chunk
// as (src, dst) = (es[j], ed[j] + i - ei[j]) for the last exception j with ei[j] <= i
// (k_decode_seq); the first edge of a chunk is always an exception.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace srg {

// Encodes edges [a, z) of a chunk (pointers at the chunk's first edge): narrows the latencies into
// hl, ORs endpoints / latencies into orx / orl (the caller's range checks) and appends exception
// triples to ex.  Returns false ("dense") once ex would exceed cap entries; the latencies and the
// checks still cover the whole slice then.  Blocks of 1 K edges: a vectorisable narrowing loop,
// a vectorisable exception-flag loop, then a scan of the flags 8 at a time (a branchy one-pass
// loop ran the host conversion at 7-9.5 ms for C3 against 5-7 ms for the u16 narrowing).
// Narrows lat[i] into hl[i] for i in [b0, b1) and ORs the latencies / endpoints into ol / ox.  The
// ring is only read by the DMA, so (clang) its 16-B lines are written non-temporally -- vector
// stores: scalar non-temporal stores (movnti) were measured 2.64 vs 1.99 ns/edge for plain
// stores, since they also stop the loop's vectorisation.  Plain loop under g++ (CPU tests).
inline void narrow_block(const uint32_t* src, const uint32_t* dst, const uint64_t* lat, uint32_t* hl, size_t b0,
                         size_t b1, uint64_t& ol, uint32_t& ox) {
    size_t i = b0;
#if defined(__clang__) && (defined(__x86_64__) || defined(__i386__))
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    typedef uint64_t v4q __attribute__((ext_vector_type(4)));
    for (; i < b1 && ((uintptr_t)(hl + i) & 15); ++i) {  // head up to a 16-B boundary of the ring
        ol |= lat[i];
        ox |= src[i] | dst[i];
        hl[i] = (uint32_t)lat[i];
    }
    v4q vol = 0;
    v4u vox = 0;
    for (; i + 4 <= b1; i += 4) {
        v4q l;
        v4u s, d;
        __builtin_memcpy(&l, lat + i, 32);
        __builtin_memcpy(&s, src + i, 16);
        __builtin_memcpy(&d, dst + i, 16);
        vol |= l;
        vox |= s | d;
        __builtin_nontemporal_store(__builtin_convertvector(l, v4u), reinterpret_cast<v4u*>(hl + i));
    }
    ol |= vol[0] | vol[1] | vol[2] | vol[3];
    ox |= vox[0] | vox[1] | vox[2] | vox[3];
#endif
    for (; i < b1; ++i) {
        ol |= lat[i];
        ox |= src[i] | dst[i];
        hl[i] = (uint32_t)lat[i];
    }
}

inline bool seq_encode_slice(const uint32_t* src, const uint32_t* dst, const uint64_t* lat, uint32_t* hl, size_t a,
                             size_t z, std::vector<uint32_t>& ex, size_t cap, uint32_t& orx, uint64_t& orl) {
    uint32_t ox = 0;
    uint64_t ol = 0;
    bool dense = false;
    // edge i is an exception unless it follows (src, dst - 1); a chunk's first edge always is
    auto exc = [&](size_t i) {
        if (dense) return;
        ex.push_back((uint32_t)i);
        ex.push_back(src[i]);
        ex.push_back(dst[i]);
        dense = ex.size() > cap;  // (then latencies and checks only)
    };
#if defined(__clang__) && (defined(__x86_64__) || defined(__i386__))
    // one pass: 4 edges per step, the narrowed latencies stored non-temporally (narrow_block), the
    // exception test on the same registers against the edges one back; a step with an exception
    // (C3: one in ~670 edges) records it in order.  (A separate flag pass over each 1 K block read
    // the endpoints twice: 1.9-2.2 ns per edge on one thread against 1.25 for the plain read.)
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    typedef uint64_t v4q __attribute__((ext_vector_type(4)));
    typedef int32_t v4i __attribute__((ext_vector_type(4)));
    size_t i = a;
    auto scalar = [&](size_t k) {
        ol |= lat[k];
        ox |= src[k] | dst[k];
        hl[k] = (uint32_t)lat[k];
        if (k == 0 || src[k] != src[k - 1] || dst[k] != dst[k - 1] + 1u) exc(k);
    };
    for (; i < z && (i == 0 || ((uintptr_t)(hl + i) & 15)); ++i) scalar(i);  // chunk start, 16-B boundary
    v4q vol = 0;
    v4u vox = 0;
    for (; i + 4 <= z; i += 4) {
        v4q l;
        v4u s, d, sp, dp;
        __builtin_memcpy(&l, lat + i, 32);
        __builtin_memcpy(&s, src + i, 16);
        __builtin_memcpy(&d, dst + i, 16);
        __builtin_memcpy(&sp, src + i - 1, 16);
        __builtin_memcpy(&dp, dst + i - 1, 16);
        vol |= l;
        vox |= s | d;
        __builtin_nontemporal_store(__builtin_convertvector(l, v4u), reinterpret_cast<v4u*>(hl + i));
        const v4i f = (s != sp) | (d != dp + 1u);
        if (__builtin_expect((f[0] | f[1] | f[2] | f[3]) != 0, 0))
            for (int q = 0; q < 4; ++q)
                if (f[q]) exc(i + q);
    }
    ol |= vol[0] | vol[1] | vol[2] | vol[3];
    ox |= vox[0] | vox[1] | vox[2] | vox[3];
    for (; i < z; ++i) scalar(i);
    __builtin_ia32_sfence();  // the non-temporal stores drained before the slot is handed to the DMA
#else
    constexpr size_t BLK = 1024;
    alignas(64) uint8_t fl[BLK + 8];
    for (size_t b0 = a; b0 < z; b0 += BLK) {
        const size_t b1 = b0 + BLK < z ? b0 + BLK : z, nb = b1 - b0;
        narrow_block(src, dst, lat, hl, b0, b1, ol, ox);
        if (dense) continue;
        size_t s0 = b0;
        if (b0 == 0) {
            fl[0] = 1;
            s0 = 1;
        }
        for (size_t i = s0; i < b1; ++i)
            fl[i - b0] = (uint8_t)((src[i] != src[i - 1]) | (dst[i] != dst[i - 1] + 1u));
        for (size_t k = nb; k < nb + 8; ++k) fl[k] = 0;
        for (size_t k = 0; k < nb && !dense; k += 8) {
            uint64_t w;
            __builtin_memcpy(&w, fl + k, 8);
            if (!w) continue;
            for (size_t q = k; q < k + 8 && q < nb; ++q)
                if (fl[q]) exc(b0 + q);
        }
    }
#endif
    orx |= ox;
    orl |= ol;
    return !dense;
}

}  // namespace srg
