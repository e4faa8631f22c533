// events.hip.h — stretch row f4: one scheduling round's cross-host packet events,
// delivered and ordered the way Shadow's per-host event queues pop them (gfx950).
//
// Reference semantics, per event i (src_host -> dst_host, sent at send_ns):
//   Worker::send_packet (src/main/core/worker.rs:391-424)
//     delay   = RoutingInfo latency(src, dst)   -> the dense routing table, resident in HBM
//     deliver = max(send + delay, round_end)     (worker.rs:411-414; EmulatedTime add panics on
//                                                 overflow -> SRG_ERR_ARG here)
//     update_lowest_used_latency(delay)          (runahead.rs:61-116) -> min_used_latency
//     update_next_event_time(deliver)            (manager.rs:430-435, 459-464) -> min_next_event
//     push_packet_to_host(dst_host, deliver)     (worker.rs:644-654: one EventQueue per host)
//   EventQueue pop order (event_queue.rs:38-49): Event::partial_cmp (event.rs:84-155) = time,
//     then Packet < Local, then src_host_id, then src_host_event_id; two events equal in all of
//     these (different packets) have no order -> PanickingOrd unwrap panic -> SRG_ERR_EVENT_ORDER.
// The packet-drop draw (worker.rs:374-389) consumes each source host's RNG stream in program
// order and stays on the host.
//
// Device design: one pass computes deliver times and the batch's field ranges (min/max); the
// host then packs every event into one composite key of only the bits the batch uses
//     key = dst_host | deliver - t_min | src_host | event_id - id_min      (MSB ... LSB)
// in one or two 64-bit words, and an LSD radix sort (8-bit digits, stable per-digit scatter:
// per-tile histograms -> one scan -> wave-ballot ranks) orders the event indices.  A final pass
// derives the per-host offsets and detects equal adjacent keys.  HBM-bound integer work.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace srg {

struct EvReduce {
    unsigned long long t_min, t_max, id_min, id_max, lat_min;
    uint32_t dst_max, src_max, bad;  // bad: 1 host out of range, 2 node out of range, 4 time overflow
    uint32_t pad;
};

struct EvIn {
    uint64_t n;
    const uint32_t* src_node;
    const uint32_t* dst_node;
    const uint32_t* src_host;
    const uint32_t* dst_host;
    const uint64_t* send_ns;
    const uint64_t* event_id;
    const uint64_t* table;  // [tn x tn] routing latencies (row = source position)
    uint32_t tn;
    uint32_t num_hosts;
    uint64_t round_end;
};

template <class T>
__device__ __forceinline__ T wave_min(T v) {
    for (int off = 32; off; off >>= 1) {
        const T o = __shfl_xor(v, off, 64);
        v = o < v ? o : v;
    }
    return v;
}
template <class T>
__device__ __forceinline__ T wave_max(T v) {
    for (int off = 32; off; off >>= 1) {
        const T o = __shfl_xor(v, off, 64);
        v = o > v ? o : v;
    }
    return v;
}

__global__ void __launch_bounds__(256) k_ev_prep(EvIn in, uint64_t* __restrict__ deliver, EvReduce* red) {
    unsigned long long tmin = ~0ull, tmax = 0, imin = ~0ull, imax = 0, lmin = ~0ull;
    uint32_t dmax = 0, smax = 0, bad = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < in.n; i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t a = in.src_node[i], b = in.dst_node[i], dh = in.dst_host[i], sh = in.src_host[i];
        if (a >= in.tn || b >= in.tn) {
            bad |= 2;
            continue;
        }
        if (dh >= in.num_hosts) {
            bad |= 1;
            continue;
        }
        const uint64_t delay = in.table[(size_t)a * in.tn + b];
        const uint64_t s = in.send_ns[i];
        if (s > ~0ull - delay) {
            bad |= 4;
            continue;
        }
        uint64_t t = s + delay;
        t = t < in.round_end ? in.round_end : t;
        deliver[i] = t;
        const uint64_t id = in.event_id[i];
        tmin = t < tmin ? t : tmin;
        tmax = t > tmax ? t : tmax;
        imin = id < imin ? id : imin;
        imax = id > imax ? id : imax;
        lmin = delay < lmin ? delay : lmin;
        dmax = dh > dmax ? dh : dmax;
        smax = sh > smax ? sh : smax;
    }
    // wave, then workgroup reduction: one set of same-address atomics per workgroup (a grid of
    // ~2k workgroups), not per wave -- same-address atomics serialise at the memory side
    tmin = wave_min(tmin);
    tmax = wave_max(tmax);
    imin = wave_min(imin);
    imax = wave_max(imax);
    lmin = wave_min(lmin);
    dmax = wave_max(dmax);
    smax = wave_max(smax);
    __shared__ unsigned long long s64[5][4];
    __shared__ uint32_t s32[2][4];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s64[0][w] = tmin;
        s64[1][w] = tmax;
        s64[2][w] = imin;
        s64[3][w] = imax;
        s64[4][w] = lmin;
        s32[0][w] = dmax;
        s32[1][w] = smax;
    }
    if (bad) atomicOr(&red->bad, bad);  // invalid input only
    __syncthreads();
    if (threadIdx.x == 0) {
        const int nw = (int)(blockDim.x + 63) >> 6;
        for (int q = 1; q < nw; ++q) {
            s64[0][0] = min(s64[0][0], s64[0][q]);
            s64[1][0] = max(s64[1][0], s64[1][q]);
            s64[2][0] = min(s64[2][0], s64[2][q]);
            s64[3][0] = max(s64[3][0], s64[3][q]);
            s64[4][0] = min(s64[4][0], s64[4][q]);
            s32[0][0] = max(s32[0][0], s32[0][q]);
            s32[1][0] = max(s32[1][0], s32[1][q]);
        }
        atomicMin(&red->t_min, s64[0][0]);
        atomicMax(&red->t_max, s64[1][0]);
        atomicMin(&red->id_min, s64[2][0]);
        atomicMax(&red->id_max, s64[3][0]);
        atomicMin(&red->lat_min, s64[4][0]);
        atomicMax(&red->dst_max, s32[0][0]);
        atomicMax(&red->src_max, s32[1][0]);
    }
}

// Composite key layout: field f occupies bits [sh_f, sh_f + width_f) of the 128-bit (hi:lo) key.
struct EvKeyFmt {
    uint32_t sh_src, sh_t, sh_dst;
    uint64_t t_min, id_min;
};

__device__ __forceinline__ void or_bits(unsigned long long& lo, unsigned long long& hi, unsigned long long v,
                                        uint32_t sh) {
    if (sh >= 64) {
        hi |= v << (sh - 64);
        return;
    }
    lo |= v << sh;
    if (sh) hi |= v >> (64 - sh);
}

__device__ __forceinline__ unsigned long long get_bits(unsigned long long lo, unsigned long long hi, uint32_t sh) {
    if (sh >= 64) return hi >> (sh - 64);
    return sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
}

template <bool WIDE>
__global__ void __launch_bounds__(256) k_ev_keys(EvIn in, const uint64_t* __restrict__ deliver, EvKeyFmt f,
                                                 unsigned long long* __restrict__ klo, unsigned long long* __restrict__ khi,
                                                 uint32_t* __restrict__ idx) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < in.n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned long long lo = 0, hi = 0;
        or_bits(lo, hi, in.event_id[i] - f.id_min, 0);
        or_bits(lo, hi, in.src_host[i], f.sh_src);
        or_bits(lo, hi, deliver[i] - f.t_min, f.sh_t);
        or_bits(lo, hi, in.dst_host[i], f.sh_dst);
        klo[i] = lo;
        if (WIDE) khi[i] = hi;
        idx[i] = (uint32_t)i;
    }
}

constexpr int RS_THREADS = 256;
constexpr int RS_ROUNDS = 8;
constexpr int RS_TILE = RS_THREADS * RS_ROUNDS;  // 2048 keys per workgroup (40 KB of LDS staging when wide)

__device__ __forceinline__ uint32_t rs_digit(unsigned long long lo, unsigned long long hi, uint32_t p) {
    return (uint32_t)get_bits(lo, hi, p) & 0xFFu;
}

// per-tile digit counts, digit-major: hist[d * ntiles + tile]
template <bool WIDE>
__global__ void __launch_bounds__(RS_THREADS) k_rs_hist(const unsigned long long* __restrict__ klo,
                                                        const unsigned long long* __restrict__ khi, uint64_t n,
                                                        uint32_t p, uint32_t ntiles, uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * RS_TILE;
    // the high words only for a digit that reaches them (the last pass of a wide key): the other
    // passes read half the bytes
    const bool need_hi = WIDE && p + 8 > 64;
#pragma unroll 4
    for (int r = 0; r < RS_ROUNDS; ++r) {
        const size_t i = base + (size_t)r * RS_THREADS + threadIdx.x;
        if (i < n) atomicAdd(&h[rs_digit(p >= 64 ? 0ull : klo[i], need_hi ? khi[i] : 0ull, p)], 1u);
    }
    __syncthreads();
    hist[(size_t)threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];
}

// Stable scatter in two phases.  (1) Tile-local stable sort into LDS: a key's slot = the tile's
// exclusive count of smaller digits (scanned from its histogram) + earlier same-digit keys of the
// tile (earlier rounds, earlier waves of this round, lower lanes of this wave: 8 ballots match
// the digit).  (2) The staged keys leave in slot order: slot j of digit d goes to the digit's
// global run start + (j - tile base of d), so consecutive threads write consecutive addresses
// (runs of ~8 keys per digit per tile) instead of one scattered 8-B store per key, which ran the
// pass at 1.45 TB/s (276 us per 10^7 wide keys, profiles/r03e/).
template <bool WIDE>
__global__ void __launch_bounds__(RS_THREADS) k_rs_scatter(const unsigned long long* __restrict__ klo,
                                                           const unsigned long long* __restrict__ khi,
                                                           const uint32_t* __restrict__ idx,
                                                           unsigned long long* __restrict__ olo,
                                                           unsigned long long* __restrict__ ohi,
                                                           uint32_t* __restrict__ oidx, uint64_t n, uint32_t p,
                                                           uint32_t ntiles, const uint32_t* __restrict__ hist,
                                                           const uint32_t* __restrict__ offs) {
    __shared__ uint32_t gstart[256];   // global run start of each digit for this tile
    __shared__ uint32_t lbase[256];    // tile-local exclusive digit offsets
    __shared__ uint32_t run[256];      // tile-local next slot per digit
    __shared__ uint32_t wcnt[RS_THREADS / 64][256];
    __shared__ unsigned long long slo[RS_TILE];
    __shared__ unsigned long long shi[WIDE ? RS_TILE : 1];
    __shared__ uint32_t sidx[RS_TILE];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const size_t base = (size_t)blockIdx.x * RS_TILE;
    const uint32_t tn = (uint32_t)min((uint64_t)RS_TILE, n - base);
    gstart[tid] = offs[(size_t)tid * ntiles + blockIdx.x];
    // exclusive scan of the tile's 256 digit counts (one per thread): wave scans + wave totals
    const uint32_t cnt = hist[(size_t)tid * ntiles + blockIdx.x];
    uint32_t incl = cnt;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off, 64);
        if ((int)lane >= off) incl += y;
    }
    if (lane == 63) wcnt[0][w] = incl;
    __syncthreads();
    uint32_t wbase = 0;
    for (uint32_t q = 0; q < w; ++q) wbase += wcnt[0][q];
    lbase[tid] = wbase + incl - cnt;
    run[tid] = wbase + incl - cnt;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < RS_THREADS / 64; ++q) wcnt[q][tid] = 0;
    __syncthreads();
    const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;
    // every round's keys in flight at once (the rounds below only rank them)
    unsigned long long rlo[RS_ROUNDS], rhi[RS_ROUNDS];
    uint32_t rid[RS_ROUNDS];
#pragma unroll
    for (int r = 0; r < RS_ROUNDS; ++r) {
        const uint32_t li = (uint32_t)r * RS_THREADS + tid;
        rlo[r] = li < tn ? klo[base + li] : 0ull;
        rhi[r] = WIDE && li < tn ? khi[base + li] : 0ull;
        rid[r] = li < tn ? idx[base + li] : 0u;
    }
#pragma unroll
    for (int r = 0; r < RS_ROUNDS; ++r) {
        const uint32_t li = (uint32_t)r * RS_THREADS + tid;
        const bool valid = li < tn;
        const unsigned long long lo = rlo[r], hi = rhi[r];
        const uint32_t id = rid[r];
        const uint32_t d = valid ? rs_digit(lo, hi, p) : 0u;
        unsigned long long m = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1u;
            const unsigned long long bb = __ballot(valid && bit);
            m &= bit ? bb : ~bb;
        }
        const uint32_t rank = (uint32_t)__popcll(m & below);
        if (valid && rank == 0) wcnt[w][d] = (uint32_t)__popcll(m);
        __syncthreads();
        if (valid) {
            uint32_t pos = run[d] + rank;
            for (uint32_t q = 0; q < w; ++q) pos += wcnt[q][d];
            slo[pos] = lo;
            if (WIDE) shi[pos] = hi;
            sidx[pos] = id;
        }
        __syncthreads();
        uint32_t add = 0;
#pragma unroll
        for (int q = 0; q < RS_THREADS / 64; ++q) {
            add += wcnt[q][tid];
            wcnt[q][tid] = 0;
        }
        run[tid] += add;
        __syncthreads();
    }
    for (uint32_t j = tid; j < tn; j += RS_THREADS) {
        const unsigned long long lo = slo[j], hi = WIDE ? shi[j] : 0ull;
        const uint32_t d = rs_digit(lo, hi, p);
        const uint32_t pos = gstart[d] + (j - lbase[d]);
        olo[pos] = lo;
        if (WIDE) ohi[pos] = hi;
        oidx[pos] = sidx[j];
    }
}

// Sorted keys -> per-host offsets (empty hosts included) and the no-order check (equal keys).
template <bool WIDE>
__global__ void __launch_bounds__(256) k_ev_finish(const unsigned long long* __restrict__ klo,
                                                   const unsigned long long* __restrict__ khi, uint64_t n,
                                                   uint32_t sh_dst, uint32_t num_hosts, uint64_t* __restrict__ host_off,
                                                   uint32_t* __restrict__ flags) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const unsigned long long lo = klo[i], hi = WIDE ? khi[i] : 0ull;
        const uint32_t d = (uint32_t)get_bits(lo, hi, sh_dst);
        uint32_t h0 = 0;
        if (i) {
            const unsigned long long plo = klo[i - 1], phi = WIDE ? khi[i - 1] : 0ull;
            h0 = (uint32_t)get_bits(plo, phi, sh_dst) + 1;
            if (plo == lo && phi == hi) atomicOr(flags, 1u);
        }
        for (uint32_t h = h0; h <= d; ++h) host_off[h] = i;
        if (i == n - 1)
            for (uint32_t h = d + 1; h <= num_hosts; ++h) host_off[h] = n;
    }
}

}  // namespace srg
