// sparse2_sim.cpp — CPU model of the two-phase sparse schedule (latency-only delta-stepping, then
// the per-lane-ready loss fold over the tight arcs), to count label-row pulls per phase before the
// GPU kernel exists, and to check the fold's result against a lexicographic Dijkstra per lane.
// Exploration tool only; not product code, not a checker.  Input: CSR dumped by tools/sparse_sim.py
// (plus loss factors b = 1 - loss per arc in /tmp/ssim/b.bin).
//   usage: sparse2_sim <csr.bin> <b.bin> <order.bin> <delta> <nbatches> [stride] [check]
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <queue>
#include <vector>

static float fold(float l, float b) {
    volatile float x = 1.0f - l;
    volatile float y = x * b;
    return 1.0f - y;
}

int main(int argc, char** argv) {
    if (argc < 6) return 1;
    FILE* f = fopen(argv[1], "rb");
    uint32_t V, A;
    fread(&V, 4, 1, f);
    fread(&A, 4, 1, f);
    std::vector<uint32_t> off(V + 1), src(A), w(A);
    fread(off.data(), 4, V + 1, f);
    fread(src.data(), 4, A, f);
    fread(w.data(), 4, A, f);
    fclose(f);
    std::vector<float> bb(A);
    f = fopen(argv[2], "rb");
    fread(bb.data(), 4, A, f);
    fclose(f);
    std::vector<uint32_t> order(V);
    f = fopen(argv[3], "rb");
    fread(order.data(), 4, V, f);
    fclose(f);
    const uint32_t delta = (uint32_t)strtoul(argv[4], 0, 10);
    const int nb = atoi(argv[5]);
    const int stride = argc > 6 ? atoi(argv[6]) : 1;
    const int check = argc > 7 ? atoi(argv[7]) : 0;
    const int nhub = argc > 8 ? atoi(argv[8]) : 0;  // hub upper bounds as phase 1's initial labels
    const uint32_t INF = 0xFFFFFFFFu;
    const int NL = 64;
    const uint32_t nbatch = V / NL;
    std::vector<std::vector<uint32_t>> HD;  // exact distances from the nhub highest-degree vertices
    for (int h = 0; h < nhub; ++h) {
        static std::vector<uint32_t> hubs;
        if (hubs.empty()) {
            hubs.resize(V);
            for (uint32_t v = 0; v < V; ++v) hubs[v] = v;
            std::partial_sort(hubs.begin(), hubs.begin() + nhub, hubs.end(),
                              [&](uint32_t x, uint32_t y) { return off[x + 1] - off[x] > off[y + 1] - off[y]; });
        }
        std::vector<uint32_t> d(V, INF);
        std::priority_queue<std::pair<uint64_t, uint32_t>, std::vector<std::pair<uint64_t, uint32_t>>, std::greater<>> pq;
        d[hubs[h]] = 0;
        pq.push({0, hubs[h]});
        while (!pq.empty()) {
            auto [dd, u] = pq.top();
            pq.pop();
            if (dd != d[u]) continue;
            for (uint32_t k = off[u]; k < off[u + 1]; ++k) {
                const uint64_t nd = dd + w[k];
                if (nd < d[src[k]]) d[src[k]] = (uint32_t)nd, pq.push({nd, src[k]});
            }
        }
        HD.push_back(std::move(d));
    }
    std::vector<uint32_t> L((size_t)V * 64);
    std::vector<float> LO((size_t)V * 64);
    std::vector<uint64_t> tm(A), F(V), reach(V);
    std::vector<uint8_t> fprev(V), fcur(V), mark(V), mnext(V), pend(V);
    std::vector<uint64_t> cm(V), cmn(V), cmp(V);  // lanes changed in the last / this sweep / pending
    double p1_lines = 0, p1_scans = 0, p1_marked = 0, p1_hubscans = 0;
    double p1_pulls = 0, p1_sweeps = 0, p2_pulls = 0, p2_sweeps = 0, p2_scans = 0, tight_arcs = 0, tight_pairs = 0;
    long bad = 0;
    // fold pushes along tight arcs only (SIM_FILTER=1): t marks in-neighbour u (= out-neighbour,
    // undirected) only when the arc t -> u is tight in a lane t just completed
    const bool filt = getenv("SIM_FILTER") && atoi(getenv("SIM_FILTER"));
    std::vector<uint32_t> twin(A);
    for (uint32_t t = 0; t < V; ++t)
        for (uint32_t k = off[t]; k < off[t + 1]; ++k) {
            const uint32_t u = src[k];  // arc u -> t at k; its twin t -> u sits in u's list with src t
            uint32_t j = off[u];
            while (src[j] != t) ++j;
            twin[k] = j;
        }
    double p2_visits = 0, p2_useless = 0, p2_tscans = 0, p2_pushes = 0;
    for (int bi = 0; bi < nb; ++bi) {
        const uint32_t b = (uint32_t)((bi * (size_t)stride) % nbatch);
        std::fill(L.begin(), L.end(), INF);
        std::fill(fprev.begin(), fprev.end(), 0);
        std::fill(mark.begin(), mark.end(), 0);
        std::fill(pend.begin(), pend.end(), 0);
        std::fill(mnext.begin(), mnext.end(), 0);
        std::fill(fcur.begin(), fcur.end(), 0);
        std::fill(cm.begin(), cm.end(), 0);
        std::fill(cmn.begin(), cmn.end(), 0);
        std::fill(cmp.begin(), cmp.end(), 0);
        for (int l = 0; l < NL; ++l) {
            const uint32_t s = order[b * NL + l];
            L[(size_t)s * 64 + l] = 0;
            cm[s] |= 1ull << l;
            fprev[s] = 1;
            for (uint32_t k = off[s]; k < off[s + 1]; ++k) mark[src[k]] = 1;
        }
        if (nhub) {  // upper bounds through the hubs; every vertex evaluated from every in-arc first
            for (int l = 0; l < NL; ++l) {
                const uint32_t s = order[b * NL + l];
                for (uint32_t v = 0; v < V; ++v) {
                    uint64_t bst = v == s ? 0 : INF;
                    for (int h = 0; h < nhub; ++h) bst = std::min<uint64_t>(bst, (uint64_t)HD[h][s] + HD[h][v]);
                    L[(size_t)v * 64 + l] = (uint32_t)std::min<uint64_t>(bst, INF);
                }
            }
            std::fill(fprev.begin(), fprev.end(), 1);
            std::fill(mark.begin(), mark.end(), 1);
        }
        // ---- phase 1: latency-only pull sweeps with a bucket bound
        uint32_t bound = delta;
        for (;;) {
            bool any = false, anyp = false;
            for (uint32_t t = 0; t < V; ++t) {
                if (!mark[t]) continue;
                uint32_t* lt = &L[(size_t)t * 64];
                bool drop = false, below = false;
                p1_marked++;
                p1_scans += off[t + 1] - off[t];
                if (off[t + 1] - off[t] >= 64) p1_hubscans += off[t + 1] - off[t];
                for (uint32_t k = off[t]; k < off[t + 1]; ++k) {
                    const uint32_t u = src[k];
                    if (!fprev[u]) continue;
                    p1_pulls++;
                    p1_lines += ((cm[u] & 0xFFFFFFFFull) != 0) + ((cm[u] >> 32) != 0);
                    const uint32_t* lu = &L[(size_t)u * 64];
                    for (int l = 0; l < NL; ++l)
                        if (lu[l] != INF && lu[l] + w[k] < lt[l]) {
                            lt[l] = lu[l] + w[k];
                            cmp[t] |= 1ull << l;
                            drop = true;
                            below |= lt[l] < bound;
                        }
                }
                if (drop) {
                    if (below) {
                        fcur[t] = 1;
                        pend[t] = 0;
                        cmn[t] = cmp[t];
                        cmp[t] = 0;
                        any = true;
                        for (uint32_t k = off[t]; k < off[t + 1]; ++k) mnext[src[k]] = 1;
                    } else {
                        pend[t] = 1;
                    }
                }
            }
            ++p1_sweeps;
            for (uint32_t v = 0; v < V; ++v) {
                cm[v] = cmn[v];
                cmn[v] = 0;
                fprev[v] = fcur[v];
                fcur[v] = 0;
                mark[v] = mnext[v];
                mnext[v] = 0;
                anyp |= pend[v] != 0;
            }
            if (!any) {
                if (!anyp) break;
                bound = bound > INF - delta ? INF : bound + delta;
                for (uint32_t v = 0; v < V; ++v) {
                    if (pend[v]) cm[v] = cmp[v], cmp[v] = 0;
                    fprev[v] = pend[v];
                    if (pend[v])
                        for (uint32_t k = off[v]; k < off[v + 1]; ++k) mark[src[k]] = 1;
                    pend[v] = 0;
                }
            }
        }
        // ---- phase 2a: tight masks (one pull of D[u] per arc)
        for (uint32_t t = 0; t < V; ++t)
            for (uint32_t k = off[t]; k < off[t + 1]; ++k) {
                const uint32_t u = src[k];
                uint64_t m = 0;
                for (int l = 0; l < NL; ++l) {
                    const uint32_t a = L[(size_t)u * 64 + l], d = L[(size_t)t * 64 + l];
                    if (a != INF && (uint64_t)a + w[k] == d) m |= 1ull << l;
                }
                tm[k] = m;
                tight_arcs += m != 0;
                tight_pairs += __builtin_popcountll(m);
            }
        // ---- phase 2b: loss fold, a lane of t computed once all its tight preds are final
        std::fill(F.begin(), F.end(), 0);
        std::fill(mark.begin(), mark.end(), 0);
        std::fill(mnext.begin(), mnext.end(), 0);
        for (uint32_t v = 0; v < V; ++v) {
            uint64_t r = 0;
            for (int l = 0; l < NL; ++l) r |= (uint64_t)(L[(size_t)v * 64 + l] != INF) << l;
            reach[v] = r;
        }
        for (int l = 0; l < NL; ++l) {
            const uint32_t s = order[b * NL + l];
            F[s] |= 1ull << l;
            LO[(size_t)s * 64 + l] = 0.0f;
            for (uint32_t k = off[s]; k < off[s + 1]; ++k) mark[src[k]] = 1;
        }
        for (;;) {
            bool any = false;
            for (uint32_t t = 0; t < V; ++t) {
                if (!mark[t]) continue;
                const uint64_t nf = reach[t] & ~F[t];
                if (!nf) continue;
                uint64_t blocked = 0;
                p2_visits++;
                for (uint32_t k = off[t]; k < off[t + 1]; ++k) {
                    p2_scans++;
                    p2_tscans += tm[k] != 0;
                    blocked |= tm[k] & nf & ~F[src[k]];
                }
                const uint64_t comp = nf & ~blocked;
                if (!comp) { p2_useless++; continue; }
                float acc[64];
                for (int l = 0; l < 64; ++l) acc[l] = 2.0f;
                for (uint32_t k = off[t]; k < off[t + 1]; ++k) {
                    const uint64_t m = tm[k] & comp;
                    if (!m) continue;
                    p2_pulls++;
                    for (int l = 0; l < NL; ++l)
                        if ((m >> l) & 1) acc[l] = std::min(acc[l], fold(LO[(size_t)src[k] * 64 + l], bb[k]));
                }
                for (int l = 0; l < NL; ++l)
                    if ((comp >> l) & 1) LO[(size_t)t * 64 + l] = acc[l];
                F[t] |= comp;
                any = true;
                for (uint32_t k = off[t]; k < off[t + 1]; ++k)
                    if (!filt || (tm[twin[k]] & comp)) mnext[src[k]] = 1, p2_pushes++;
            }
            ++p2_sweeps;
            for (uint32_t v = 0; v < V; ++v) {
                mark[v] = mnext[v];
                mnext[v] = 0;
            }
            if (!any) break;
        }
        if (check && bi < check) {  // lexicographic Dijkstra per lane (petgraph semantics)
            for (int l = 0; l < NL; ++l) {
                const uint32_t s = order[b * NL + l];
                std::vector<uint64_t> dl(V, ~0ull);
                std::vector<float> dp(V, 0.0f);
                std::vector<uint8_t> vis(V, 0);
                typedef std::pair<std::pair<uint64_t, float>, uint32_t> E;
                std::priority_queue<E, std::vector<E>, std::greater<E>> pq;
                dl[s] = 0;
                pq.push({{0, 0.0f}, s});
                while (!pq.empty()) {
                    auto [sc, u] = pq.top();
                    pq.pop();
                    if (vis[u]) continue;
                    for (uint32_t k = off[u]; k < off[u + 1]; ++k) {  // undirected: out == in
                        const uint32_t t = src[k];
                        if (vis[t]) continue;
                        const std::pair<uint64_t, float> nx{sc.first + w[k], fold(sc.second, bb[k])};
                        if (dl[t] == ~0ull || nx < std::make_pair(dl[t], dp[t])) {
                            dl[t] = nx.first;
                            dp[t] = nx.second;
                            pq.push({nx, t});
                        }
                    }
                    vis[u] = 1;
                }
                for (uint32_t v = 0; v < V; ++v) {
                    if (dl[v] != L[(size_t)v * 64 + l]) ++bad;
                    else if (v != s && dp[v] != LO[(size_t)v * 64 + l]) ++bad;
                }
            }
        }
    }
    printf("{\"p1_scans_per_arc\": %.3f, \"p1_hub_scans_per_arc\": %.3f, \"p1_marked_per_vertex\": %.3f, \"p1_lines_per_arc\": %.3f, \"p1_pulls_per_arc\": %.3f, \"p1_sweeps\": %.2f, \"p2_pulls_per_arc\": %.3f, \"p2_sweeps\": %.2f, "
           "\"p2_scans_per_arc\": %.3f, \"tight_arc_frac\": %.3f, \"tight_lanes_per_tight_arc\": %.2f, \"mismatches\": %ld, \"p2_visits_per_vertex\": %.3f, \"p2_useless_frac\": %.3f, \"p2_tight_scans_per_arc\": %.3f, \"p2_pushes_per_arc\": %.3f}\n",
           p1_scans / nb / A, p1_hubscans / nb / A, p1_marked / nb / V, p1_lines / nb / A, p1_pulls / nb / A, p1_sweeps / nb, p2_pulls / nb / A, p2_sweeps / nb, p2_scans / nb / A, tight_arcs / nb / A,
           tight_pairs / std::max(1.0, tight_arcs), bad, p2_visits / nb / V, p2_useless / std::max(1.0, p2_visits), p2_tscans / nb / A, p2_pushes / nb / A);
    return 0;
}
