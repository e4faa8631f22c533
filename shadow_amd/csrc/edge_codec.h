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
// ring stores bypass the cache (the DMA reads the ring; no read-for-ownership of its lines);
// plain stores under g++ (the CPU round-trip test)
#if defined(__clang__)
#define SRG_NT_STORE(v, p) __builtin_nontemporal_store((v), (p))
#else
#define SRG_NT_STORE(v, p) (*(p) = (v))
#endif

inline bool seq_encode_slice(const uint32_t* src, const uint32_t* dst, const uint64_t* lat, uint32_t* hl, size_t a,
                             size_t z, std::vector<uint32_t>& ex, size_t cap, uint32_t& orx, uint64_t& orl) {
    constexpr size_t BLK = 1024;
    alignas(64) uint8_t fl[BLK + 8];
    uint32_t ox = 0;
    uint64_t ol = 0;
    bool dense = false;
    for (size_t b0 = a; b0 < z; b0 += BLK) {
        const size_t b1 = b0 + BLK < z ? b0 + BLK : z, nb = b1 - b0;
        for (size_t i = b0; i < b1; ++i) {
            const uint64_t l = lat[i];
            SRG_NT_STORE((uint32_t)l, &hl[i]);
            ol |= l;
            ox |= src[i] | dst[i];
        }
        if (dense) continue;  // (latencies and checks only)
        // edge i is an exception unless it follows (src, dst - 1); a chunk's first edge always is
        size_t s0 = b0;
        if (b0 == 0) {
            fl[0] = 1;
            s0 = 1;
        }
        for (size_t i = s0; i < b1; ++i)
            fl[i - b0] = (uint8_t)((src[i] != src[i - 1]) | (dst[i] != dst[i - 1] + 1u));
        for (size_t k = nb; k < nb + 8; ++k) fl[k] = 0;
        for (size_t k = 0; k < nb; k += 8) {
            uint64_t w;
            __builtin_memcpy(&w, fl + k, 8);
            if (!w) continue;
            for (size_t q = k; q < k + 8 && q < nb; ++q) {
                if (!fl[q]) continue;
                const size_t i = b0 + q;
                ex.push_back((uint32_t)i);
                ex.push_back(src[i]);
                ex.push_back(dst[i]);
            }
            if (ex.size() > cap) {
                dense = true;
                break;
            }
        }
    }
    orx |= ox;
    orl |= ol;
    __builtin_ia32_sfence();  // the non-temporal stores drained before the slot is handed to the DMA
    return !dense;
}

}  // namespace srg
