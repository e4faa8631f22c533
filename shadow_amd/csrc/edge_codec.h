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
// checks still cover the whole slice then.
inline bool seq_encode_slice(const uint32_t* src, const uint32_t* dst, const uint64_t* lat, uint32_t* hl, size_t a,
                             size_t z, std::vector<uint32_t>& ex, size_t cap, uint32_t& orx, uint64_t& orl) {
    uint32_t ps = a ? src[a - 1] : 0u, pd = a ? dst[a - 1] : 0u;  // none before a chunk's first edge
    bool have = a > 0;
    for (size_t i = a; i < z; ++i) {
        const uint32_t x = src[i], y = dst[i];
        const uint64_t l = lat[i];
        orx |= x | y;
        orl |= l;
        hl[i] = (uint32_t)l;
        if (!(have && x == ps && y == pd + 1u)) {
            ex.push_back((uint32_t)i);
            ex.push_back(x);
            ex.push_back(y);
            if (ex.size() > cap) {
                for (size_t k = i + 1; k < z; ++k) {
                    const uint32_t x2 = src[k], y2 = dst[k];
                    const uint64_t l2 = lat[k];
                    orx |= x2 | y2;
                    orl |= l2;
                    hl[k] = (uint32_t)l2;
                }
                return false;
            }
        }
        ps = x;
        pd = y;
        have = true;
    }
    return true;
}

}  // namespace srg
