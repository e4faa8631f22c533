// gml_write.cpp -- writes the GML text of a synthetic edge list (the same text as
// shadow_amd.synth.to_gml) for the ingest benchmark at C3 scale (≈4.5 GB).  Test/bench tool.
// usage: gml_write OUT.gml V DIRECTED < edges.bin   (edges.bin: E, then src u32[E], dst u32[E],
//        lat u64[E], loss f32[E], as written by tools/ingest/ingest_bench.py)
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

int main(int argc, char** argv) {
    if (argc != 4) return 2;
    const uint32_t V = (uint32_t)std::strtoul(argv[2], nullptr, 10);
    const int directed = std::atoi(argv[3]);
    uint64_t E = 0;
    if (std::fread(&E, 8, 1, stdin) != 1) return 3;
    std::vector<uint32_t> s(E), d(E);
    std::vector<uint64_t> l(E);
    std::vector<float> p(E);
    if (std::fread(s.data(), 4, E, stdin) != E || std::fread(d.data(), 4, E, stdin) != E ||
        std::fread(l.data(), 8, E, stdin) != E || std::fread(p.data(), 4, E, stdin) != E)
        return 4;
    FILE* f = std::fopen(argv[1], "wb");
    if (!f) return 5;
    std::vector<char> buf(1 << 24);
    std::setvbuf(f, buf.data(), _IOFBF, buf.size());
    std::fprintf(f, "graph [\n  directed %d", directed);
    for (uint32_t i = 0; i < V; ++i)
        std::fprintf(f, "\n  node [\n    id %u\n    host_bandwidth_up \"1 Gbit\"\n    host_bandwidth_down \"1 Gbit\"\n  ]", i);
    char ps[64];
    for (uint64_t e = 0; e < E; ++e) {
        std::snprintf(ps, sizeof ps, "%.9g", (double)p[e]);
        if (!std::strchr(ps, '.') && !std::strchr(ps, 'e') && !std::strstr(ps, "inf")) std::strcat(ps, ".0");
        std::fprintf(f, "\n  edge [\n    source %u\n    target %u\n    latency \"%llu ns\"\n    packet_loss %s\n  ]",
                     s[e], d[e], (unsigned long long)l[e], ps);
    }
    std::fprintf(f, "\n]\n");
    std::fclose(f);
    return 0;
}
