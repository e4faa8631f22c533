// sparse_xcd_sim.cpp — sequential CPU model of k_sparse_xcd's step protocol (sparse_xcd.hip.h):
// per-step parity buffers (change bits, published push slices), owner-local pend bits, bucket
// releases as steps of their own, the chg_seq / pend_seq termination rule and the group step counter
// carried across batches.  Participants and their waves run one after another inside a step (the
// GPU runs them concurrently; any interleaving reaches the same fixpoint), so this checks the
// bookkeeping, not the concurrency.  Labels (latency << 32 | loss bits) are compared with a plain
// lexicographic Bellman-Ford fixpoint per source.  Not product code, not a checker of results.
//   usage: sparse_xcd_sim [V] [avg_deg] [participants] [delta_div] [batches] [seed]
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

typedef unsigned long long u64;
static const u64 INF = ~0ull;
static const int B = 8, WAVES = 16, MAXP = 64;

static float fold(float pl, float omp) {
    volatile float x = 1.0f - pl;
    volatile float y = x * omp;
    return 1.0f - y;
}
static u64 relax(u64 lu, uint32_t w, float b) {
    const uint32_t lat = (uint32_t)(lu >> 32);
    const uint64_t s = (uint64_t)lat + w;
    const uint32_t nl = s > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)s;
    float l;
    uint32_t lb = (uint32_t)lu;
    std::memcpy(&l, &lb, 4);
    const float loss = fold(l, b);
    uint32_t bits;
    std::memcpy(&bits, &loss, 4);
    return nl == 0xFFFFFFFFu ? INF : ((u64)nl << 32 | bits);
}

int main(int argc, char** argv) {
    const uint32_t V = argc > 1 ? atoi(argv[1]) : 3000;
    const int deg = argc > 2 ? atoi(argv[2]) : 8;
    const uint32_t P = argc > 3 ? atoi(argv[3]) : 3;
    const int ddiv = argc > 4 ? atoi(argv[4]) : 4;
    const uint32_t nbatch_run = argc > 5 ? atoi(argv[5]) : 6;
    std::mt19937_64 rng(argc > 6 ? atoi(argv[6]) : 1);
    // random undirected graph: a spanning path + random edges; latencies U{1..1000}, loss 50 % zero
    std::vector<uint32_t> es, ed, ew;
    std::vector<float> eb;
    for (uint32_t v = 1; v < V; ++v) es.push_back(v - 1), ed.push_back(v);
    for (uint64_t k = 0; k < (uint64_t)V * deg / 2; ++k) {
        uint32_t a = rng() % V, b = rng() % V;
        if (a != b) es.push_back(a), ed.push_back(b);
    }
    for (size_t k = 0; k < es.size(); ++k) {
        ew.push_back(1 + rng() % 1000);
        eb.push_back((rng() & 1) ? 1.0f : 1.0f - (float)((rng() % 1000) * 1e-5));
    }
    std::vector<uint32_t> off(V + 1, 0), src, w;
    std::vector<float> bb;
    for (size_t k = 0; k < es.size(); ++k) off[es[k] + 1]++, off[ed[k] + 1]++;
    for (uint32_t v = 0; v < V; ++v) off[v + 1] += off[v];
    src.resize(off[V]);
    w.resize(off[V]);
    bb.resize(off[V]);
    std::vector<uint32_t> cur(off.begin(), off.end() - 1);
    for (size_t k = 0; k < es.size(); ++k) {
        uint32_t i = cur[ed[k]]++;
        src[i] = es[k], w[i] = ew[k], bb[i] = eb[k];
        i = cur[es[k]]++;
        src[i] = ed[k], w[i] = ew[k], bb[i] = eb[k];
    }
    const uint32_t nw = (V + 63) / 64, NWT = P * WAVES;
    const uint64_t maxw = *std::max_element(ew.begin(), ew.end());
    const uint64_t delta = ddiv > 0 ? std::max<uint64_t>(1, maxw / ddiv) : ~0ull;
    std::vector<u64> L((size_t)V * B), chg[2] = {std::vector<u64>(nw), std::vector<u64>(nw)}, pend(nw);
    std::vector<u64> pub((size_t)2 * MAXP * nw);
    auto pubp = [&](int p, uint32_t r) { return &pub[((size_t)p * MAXP + r) * nw]; };
    std::vector<std::vector<u64>> lmark(P, std::vector<u64>(nw));
    uint32_t gs = 0, chg_seq = 0, pend_seq = 0;
    auto publish = [&](int p) {
        for (uint32_t r = 0; r < P; ++r)
            for (uint32_t i = 0; i < nw; ++i) pubp(p, r)[i] = lmark[r][i], lmark[r][i] = 0;
    };
    auto push = [&](uint32_t r, uint32_t v) {
        for (uint32_t k = off[v]; k < off[v + 1]; ++k) lmark[r][src[k] >> 6] |= 1ull << (src[k] & 63);
    };
    uint64_t pulls = 0, steps_total = 0;
    int bad = 0;
    for (uint32_t bt = 0; bt < nbatch_run; ++bt) {
        uint32_t S[B];
        for (int q = 0; q < B; ++q) S[q] = (uint32_t)((bt * 7919ull + q * 104729ull) % V);
        // init
        for (uint32_t r = 0; r < P; ++r)
            for (uint32_t wv = 0; wv < WAVES; ++wv)
                for (uint32_t wi = r * WAVES + wv; wi < nw; wi += NWT) {
                    u64 sb = 0;
                    for (uint32_t v = wi * 64; v < std::min(V, wi * 64 + 64); ++v)
                        for (int q = 0; q < B; ++q) L[(size_t)v * B + q] = v == S[q] ? 0 : INF;
                    for (int q = 0; q < B; ++q)
                        if (S[q] >> 6 == wi) sb |= 1ull << (S[q] & 63);
                    chg[(gs + 1) & 1][wi] = sb;
                    chg[gs & 1][wi] = 0;
                    pend[wi] = 0;
                }
        for (uint32_t r = 0; r < P; ++r)
            for (uint32_t qq = r; qq < (uint32_t)B; qq += P) push(r, S[qq]);
        publish(gs & 1);
        uint64_t bound = delta >= 0xFFFFFFFFull ? 0xFFFFFFFFull : delta;
        uint32_t last_rel = gs;
        for (;;) {
            const int p = gs & 1;
            bool s_chg = false, s_pend = false;
            for (uint32_t r = 0; r < P; ++r) {
                for (uint32_t wv = 0; wv < WAVES; ++wv) {
                    for (uint32_t wi = r * WAVES + wv; wi < nw; wi += NWT) {
                        u64 mk = 0;
                        for (uint32_t rr = 0; rr < P; ++rr) mk |= pubp(p, rr)[wi];
                        if (!mk) {
                            chg[p][wi] = 0;
                            continue;
                        }
                        u64 changed = 0, deferred = 0;
                        for (int i = 0; i < 64; ++i) {
                            if (!((mk >> i) & 1)) continue;
                            const uint32_t v = wi * 64 + i;
                            u64 best[B], old[B];
                            for (int q = 0; q < B; ++q) best[q] = old[q] = L[(size_t)v * B + q];
                            for (uint32_t k = off[v]; k < off[v + 1]; ++k) {
                                const uint32_t u = src[k];
                                if (!((chg[p ^ 1][u >> 6] >> (u & 63)) & 1)) continue;
                                ++pulls;
                                for (int q = 0; q < B; ++q) {
                                    const u64 lu = L[(size_t)u * B + q];
                                    const u64 c = lu == INF ? INF : relax(lu, w[k], bb[k]);
                                    best[q] = std::min(best[q], c);
                                }
                            }
                            bool dr = false, bd = false;
                            for (int q = 0; q < B; ++q)
                                if (best[q] < old[q]) {
                                    dr = true;
                                    bd |= (best[q] >> 32) < bound;
                                    L[(size_t)v * B + q] = best[q];
                                }
                            if (dr) (bd ? changed : deferred) |= 1ull << i;
                        }
                        chg[p][wi] = changed;
                        if (changed | deferred) {
                            const u64 pn = (pend[wi] | deferred) & ~changed;
                            pend[wi] = pn;
                            if (pn) s_pend = true;
                        }
                        if (changed) {
                            s_chg = true;
                            for (int i = 0; i < 64; ++i)
                                if ((changed >> i) & 1) push(r, wi * 64 + i);
                        }
                    }
                }
            }
            publish(p ^ 1);
            if (s_chg) chg_seq = std::max(chg_seq, gs + 1);
            if (s_pend) pend_seq = std::max(pend_seq, gs + 1);
            ++gs;
            ++steps_total;
            if (chg_seq >= gs) continue;
            if (pend_seq <= last_rel) break;
            bound = (delta >= 0xFFFFFFFFull || bound > 0xFFFFFFFFull - delta) ? 0xFFFFFFFFull : bound + delta;
            const int pr = gs & 1;
            for (uint32_t r = 0; r < P; ++r)
                for (uint32_t wv = 0; wv < WAVES; ++wv)
                    for (uint32_t wi = r * WAVES + wv; wi < nw; wi += NWT) {
                        const u64 bits = pend[wi];
                        chg[pr][wi] = bits;
                        pend[wi] = 0;
                        for (int i = 0; i < 64; ++i)
                            if ((bits >> i) & 1) push(r, wi * 64 + i);
                    }
            publish(pr ^ 1);
            ++gs;
            ++steps_total;
            last_rel = gs;
        }
        // reference: plain lexicographic Bellman-Ford per source
        for (int q = 0; q < B; ++q) {
            std::vector<u64> R(V, INF);
            R[S[q]] = 0;
            for (bool ch = true; ch;) {
                ch = false;
                for (uint32_t v = 0; v < V; ++v)
                    for (uint32_t k = off[v]; k < off[v + 1]; ++k) {
                        const u64 lu = R[src[k]];
                        if (lu == INF) continue;
                        const u64 c = relax(lu, w[k], bb[k]);
                        if (c < R[v]) R[v] = c, ch = true;
                    }
            }
            for (uint32_t v = 0; v < V; ++v)
                if (R[v] != L[(size_t)v * B + q]) ++bad;
        }
    }
    printf("{\"V\": %u, \"participants\": %u, \"batches\": %u, \"mismatches\": %d, \"steps_per_batch\": %.1f, "
           "\"pulls_per_arc\": %.2f}\n",
           V, P, nbatch_run, bad, (double)steps_total / nbatch_run, (double)pulls / nbatch_run / off[V]);
    return bad ? 1 : 0;
}
