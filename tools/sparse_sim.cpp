// sparse_sim.cpp — CPU model of k_sparse_bf's sweep schedule (latency only), to compare batch
// compositions and bucket widths by the number of label-row pulls they cause, without a GPU.
// Not product code; not a checker.  Input: CSR dumped by tools/sparse_sim.py.
//   usage: sparse_sim <csr.bin> <order.bin> <delta> <nbatches> [stride]
#include <algorithm>
#include <cstdint>
#include <queue>
#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv) {
    if (argc < 5) return 1;
    FILE* f = fopen(argv[1], "rb");
    uint32_t V, A;
    fread(&V, 4, 1, f);
    fread(&A, 4, 1, f);
    std::vector<uint32_t> off(V + 1), src(A), w(A);
    fread(off.data(), 4, V + 1, f);
    fread(src.data(), 4, A, f);
    fread(w.data(), 4, A, f);
    fclose(f);
    FILE* g = fopen(argv[2], "rb");
    std::vector<uint32_t> order(V);
    fread(order.data(), 4, V, g);
    fclose(g);
    const uint32_t delta = (uint32_t)strtoul(argv[3], 0, 10);
    const int nb = atoi(argv[4]);
    const int stride = argc > 5 ? atoi(argv[5]) : 1;
    const int per_lane = argc > 6 ? atoi(argv[6]) : 0;
    const int gs_act = argc > 7 ? atoi(argv[7]) : 0;
    const int NL = argc > 8 ? atoi(argv[8]) : 64;  // sources per batch (lanes)  // 1: arcs from vertices changed earlier in this sweep are pulled too
    const int nhub = argc > 9 ? atoi(argv[9]) : 0;   // hub-bound initialisation: L = min_h D[h][s] + D[h][v]
    const uint32_t INF = 0xFFFFFFFFu;
    std::vector<std::vector<uint32_t>> HD;  // exact distances from the hubs (Dijkstra)
    if (nhub) {
        std::vector<uint32_t> deg(V), hubs(V);
        for (uint32_t v = 0; v < V; ++v) deg[v] = off[v + 1] - off[v], hubs[v] = v;
        std::partial_sort(hubs.begin(), hubs.begin() + nhub, hubs.end(), [&](uint32_t x, uint32_t y) { return deg[x] > deg[y]; });
        for (int h = 0; h < nhub; ++h) {
            std::vector<uint32_t> d(V, INF);
            std::priority_queue<std::pair<uint64_t, uint32_t>, std::vector<std::pair<uint64_t, uint32_t>>, std::greater<>> pq;
            d[hubs[h]] = 0;
            pq.push({0, hubs[h]});
            while (!pq.empty()) {
                auto [dd, u] = pq.top();
                pq.pop();
                if (dd != d[u]) continue;
                for (uint32_t k = off[u]; k < off[u + 1]; ++k) {  // undirected: in == out
                    const uint32_t t = src[k];
                    const uint64_t nd = dd + w[k];
                    if (nd < d[t]) d[t] = (uint32_t)nd, pq.push({nd, t});
                }
            }
            HD.push_back(std::move(d));
        }
    }
    std::vector<uint32_t> L((size_t)V * 64);
    std::vector<uint8_t> fprev(V), fcur(V), mark(V), mnext(V), pend(V);
    double tot_pulls = 0, tot_sweeps = 0, tot_lanechg = 0, tot_sectors = 0;
    const uint32_t nbatch = V / NL;
    for (int bi = 0; bi < nb; ++bi) {
        const uint32_t b = (uint32_t)((bi * (size_t)stride) % nbatch);
        for (size_t i = 0; i < L.size(); ++i) L[i] = INF;
        std::fill(fprev.begin(), fprev.end(), 0);
        std::fill(mark.begin(), mark.end(), 0);
        std::fill(pend.begin(), pend.end(), 0);
        std::fill(mnext.begin(), mnext.end(), 0);
        std::fill(fcur.begin(), fcur.end(), 0);
        for (int l = 0; l < NL; ++l) {
            uint32_t s = order[b * NL + l];
            L[(size_t)s * 64 + l] = 0;
            fprev[s] = 1;
            for (uint32_t k = off[s]; k < off[s + 1]; ++k) mark[src[k]] = 1;  // undirected: out == in
        }
        if (nhub) {  // upper bounds through the hubs; the first sweep evaluates every vertex from every in-arc
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
        uint32_t bound = delta;
        uint64_t pulls = 0, lanechg = 0, sectors = 0;
        int sweeps = 0;
        if (per_lane) {
            // per-lane buckets: a lane of u is pushed only when it changed since its last push and
            // is below the bound; a vertex row is pulled by its out-neighbours when any lane is pushed
            std::vector<uint64_t> dirty(V, 0), pm(V, 0);
            for (int l = 0; l < NL; ++l) dirty[order[b * NL + l]] |= 1ull << l;
            for (;;) {
                bool anyact = false, anydirty = false;
                for (uint32_t u = 0; u < V; ++u) {
                    uint64_t bl = 0;
                    if (dirty[u])
                        for (int l = 0; l < NL; ++l)
                            if (((dirty[u] >> l) & 1) && L[(size_t)u * 64 + l] < bound) bl |= 1ull << l;
                    pm[u] = bl;
                    anyact |= bl != 0;
                    anydirty |= dirty[u] != 0;
                }
                if (!anydirty) break;
                if (!anyact) {
                    bound = bound > INF - delta ? INF : bound + delta;
                    continue;
                }
                for (uint32_t u = 0; u < V; ++u) dirty[u] &= ~pm[u];
                for (uint32_t t = 0; t < V; ++t) {
                    bool m = false;
                    for (uint32_t k = off[t]; k < off[t + 1]; ++k) m |= pm[src[k]] != 0;
                    if (!m) continue;
                    pulls++;
                    uint32_t* lt = &L[(size_t)t * 64];
                    for (uint32_t k = off[t]; k < off[t + 1]; ++k) {
                        const uint32_t u = src[k];
                        if (!pm[u]) continue;
                        pulls++;
                        const uint32_t* lu = &L[(size_t)u * 64];
                        for (int l = 0; l < NL; ++l)
                            if (((pm[u] >> l) & 1) && lu[l] + w[k] < lt[l]) {
                                lt[l] = lu[l] + w[k];
                                dirty[t] |= 1ull << l;
                                lanechg++;
                            }
                    }
                }
                ++sweeps;
            }
            tot_pulls += pulls;
            tot_sweeps += sweeps;
            tot_lanechg += lanechg;
            continue;
        }
        std::vector<uint64_t> pmask(V, 0), cmask(V, 0);
        if (nhub) std::fill(pmask.begin(), pmask.end(), ~0ull);
        for (int l = 0; l < NL; ++l) pmask[order[b * NL + l]] |= 1ull << l;
        for (;;) {
            bool any = false, anyp = false;
            for (uint32_t t = 0; t < V; ++t) {
                if (!mark[t]) continue;
                uint32_t* lt = &L[(size_t)t * 64];
                uint32_t nl[64];
                for (int l = 0; l < NL; ++l) nl[l] = lt[l];
                pulls++;  // own row
                uint64_t need = 0;  // lanes pulled for t (changed in some pulled source)
                for (uint32_t k = off[t]; k < off[t + 1]; ++k) {
                    uint32_t u = src[k];
                    if (!fprev[u] && !(gs_act && fcur[u])) continue;
                    pulls++;
                    for (int sct = 0; sct < 8; ++sct) sectors += ((pmask[u] >> (8 * sct)) & 0xFF) != 0;
                    need |= pmask[u];
                    const uint32_t* lu = &L[(size_t)u * 64];
                    for (int l = 0; l < NL; ++l)
                        if (lu[l] != INF && lu[l] + w[k] < nl[l]) nl[l] = lu[l] + w[k];
                }
                for (int sct = 0; sct < 8; ++sct) sectors += ((need >> (8 * sct)) & 0xFF) != 0;  // own row, those lanes
                bool drop = false, below = false;
                for (int l = 0; l < NL; ++l)
                    if (nl[l] < lt[l]) {
                        drop = true;
                        lanechg++;
                        cmask[t] |= 1ull << l;
                        if (nl[l] < bound) below = true;
                        lt[l] = nl[l];
                    }
                if (drop) {
                    if (below) {
                        fcur[t] = 1;
                        pend[t] = 0;
                        any = true;
                        for (uint32_t k = off[t]; k < off[t + 1]; ++k) mnext[src[k]] = 1;
                    } else {
                        pend[t] = 1;
                    }
                }
            }
            ++sweeps;
            for (uint32_t v = 0; v < V; ++v) {
                // (lane masks: approximate -- a deferred vertex's lanes are counted when it changed)
                pmask[v] = fcur[v] ? cmask[v] : 0;
                cmask[v] = fcur[v] ? 0 : cmask[v];
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
                    pmask[v] = pend[v] ? cmask[v] : pmask[v];
                    if (pend[v]) cmask[v] = 0;
                    fprev[v] = pend[v];
                    if (pend[v])
                        for (uint32_t k = off[v]; k < off[v + 1]; ++k) mark[src[k]] = 1;
                    pend[v] = 0;
                }
            }
        }
        tot_pulls += pulls;
        tot_sweeps += sweeps;
        tot_lanechg += lanechg;
        tot_sectors += sectors;
    }
    printf("{\"pulls_per_arc\": %.3f, \"sweeps\": %.2f, \"lane_changes_per_vertex_lane\": %.3f, \"sectors_per_arc\": %.3f}\n",
           tot_pulls / nb / A, tot_sweeps / nb, tot_lanechg / nb / ((double)NL * V), tot_sectors / nb / A);
    return 0;
}
