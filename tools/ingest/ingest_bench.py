"""Ingest at scale: write a synthetic graph's GML once (C3: ≈4.5 GB, the text
Shadow would read), parse it with srg_graph_parse_gml (NetworkGraph::parse, mod.rs:134-181),
time the parse, and check the parsed edge list equals the generator's.  Also times reading the
text with OMP_NUM_THREADS parser threads (chunked parallel parse, gml.cpp parse_impl).
usage: python tools/ingest/ingest_bench.py [--vertices 10000] [--graph atlas|ba]"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from shadow_amd import NetworkGraph, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--vertices", type=int, default=10000)
    ap.add_argument("--graph", choices=["atlas", "ba"], default="atlas")
    ap.add_argument("--dir", default=tempfile.gettempdir())
    args = ap.parse_args()
    here = os.path.dirname(os.path.abspath(__file__))
    exe = os.path.join(args.dir, "gml_write")
    subprocess.check_call(["g++", "-O2", "-o", exe, os.path.join(here, "gml_write.cpp")])
    V = args.vertices
    e = synth.atlas_like(V, seed=V) if args.graph == "atlas" else synth.barabasi_albert(V, 4, seed=V)
    path = os.path.join(args.dir, f"ingest_{args.graph}_{V}.gml")
    t0 = time.perf_counter()
    p = subprocess.Popen([exe, path, str(V), str(int(e.directed))], stdin=subprocess.PIPE)
    p.stdin.write(np.uint64(e.num_edges).tobytes())
    for a in (e.src, e.dst, e.latency_ns, e.packet_loss):
        p.stdin.write(np.ascontiguousarray(a).tobytes())
    p.stdin.close()
    assert p.wait() == 0
    t_write = time.perf_counter() - t0
    size = os.path.getsize(path)
    t0 = time.perf_counter()
    with open(path, "rb") as f:
        text = f.read()
    t_read = time.perf_counter() - t0
    t0 = time.perf_counter()
    g = NetworkGraph.parse(text)
    t_parse = time.perf_counter() - t0
    del text
    pe = g.edges
    same = (pe.num_vertices == V and np.array_equal(pe.src, e.src) and np.array_equal(pe.dst, e.dst)
            and np.array_equal(pe.latency_ns, e.latency_ns)
            and np.array_equal(pe.packet_loss.view(np.uint32), e.packet_loss.view(np.uint32)))
    os.remove(path)
    print(json.dumps({"what": "GML ingest (NetworkGraph::parse via srg_graph_parse_gml)", "graph": args.graph,
                      "vertices": V, "edges": int(e.num_edges), "gml_bytes": size, "write_s": round(t_write, 2),
                      "read_s": round(t_read, 2), "parse_s": round(t_parse, 2),
                      "parse_MBps": round(size / t_parse / 1e6, 1), "edge_list_equal": bool(same)}), flush=True)
    assert same


if __name__ == "__main__":
    main()
