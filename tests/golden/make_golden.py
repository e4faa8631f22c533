"""Generate tests/golden/*.json — golden vectors for the routing path.

Run from the repo root:  python tests/golden/make_golden.py

Each fixture holds an edge list (petgraph raw_edges order), the used nodes, and the
expected compute_shortest_paths output (or error code) computed by an INDEPENDENT
pure-Python restatement of petgraph 0.6.5 dijkstra + PathProperties (mod.rs:296-331) with
numpy float32 scalars (each op rounded, no FMA).  At generation time every fixture is also
checked against
  * networkx 3.4.2 all-pairs Dijkstra (latency),
  * the C++ oracle (oracle/oracle.cpp, both plumbing modes) -- latency AND loss bit-exact,
so three implementations agree on every committed vector.  reference_kats.json holds the
reference's own known-answer tests, transcribed from mod.rs:515-647 / units.rs:580-776.
"""
import heapq
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from shadow_amd import synth  # noqa: E402
from shadow_amd.graph import Edges  # noqa: E402

F = np.float32
ONE = F(1.0)


def pp_add(a, b):
    # mod.rs:322-331 -- numpy f32 scalar ops round individually
    return (a[0] + b[0], ONE - (ONE - a[1]) * (ONE - b[1]))


def dijkstra(V, directed, src, dst, lat, loss, start):
    """petgraph::algo::dijkstra restated (HashMap scores, visited set, strict-< update)."""
    adj = [[] for _ in range(V)]
    for e in range(len(src)):
        s, t = int(src[e]), int(dst[e])
        w = (int(lat[e]), F(loss[e]))
        adj[s].append((t, w))
        if not directed and s != t:
            adj[t].append((s, w))
    scores = {start: (0, F(0.0))}
    visited = set()
    heap = [(0, F(0.0), start)]
    while heap:
        l, p, node = heapq.heappop(heap)
        if node in visited:
            continue
        for t, w in adj[node]:
            if t in visited:
                continue
            ns = pp_add((l, p), w)
            old = scores.get(t)
            if old is None or ns < old:  # tuple order == PartialOrd (mod.rs:305-313)
                scores[t] = ns
                heapq.heappush(heap, (ns[0], ns[1], t))
        visited.add(node)
    return scores


def expected(edges, nodes):
    """compute_shortest_paths (mod.rs:183-228) -> (code, lat, loss)."""
    V = edges.num_vertices
    n = len(nodes)
    lat = np.zeros((n, n), dtype=np.uint64)
    loss = np.zeros((n, n), dtype=np.float32)
    filled = np.zeros((n, n), dtype=bool)
    pos = {v: i for i, v in enumerate(nodes)}
    for i, s in enumerate(nodes):
        sc = dijkstra(V, edges.directed, edges.src, edges.dst, edges.latency_ns, edges.packet_loss, s)
        for t, (l, p) in sc.items():
            if t in pos:
                lat[i, pos[t]] = l
                loss[i, pos[t]] = p
                filled[i, pos[t]] = True
    for i, v in enumerate(nodes):
        m = [e for e in range(edges.num_edges) if edges.src[e] == v and edges.dst[e] == v]
        if len(m) == 0:
            return 2, None, None
        if len(m) > 1:
            return 3, None, None
        lat[i, i] = edges.latency_ns[m[0]]
        loss[i, i] = edges.packet_loss[m[0]]
        filled[i, i] = True
    if not filled.all():
        return 4, None, None
    return 0, lat, loss


def nx_check(edges, nodes, lat):
    import networkx as nx
    G = nx.DiGraph() if edges.directed else nx.Graph()
    G.add_nodes_from(range(edges.num_vertices))
    for s, t, l in zip(edges.src.tolist(), edges.dst.tolist(), edges.latency_ns.tolist()):
        if s == t:
            continue
        if G.has_edge(s, t):
            l = min(l, G[s][t]["w"])
        G.add_edge(s, t, w=l)
    for i, s in enumerate(nodes):
        d = nx.single_source_dijkstra_path_length(G, s, weight="w")
        for j, t in enumerate(nodes):
            if i != j:
                assert d[t] == int(lat[i, j]), (s, t, d[t], lat[i, j])


def fixture(name, edges, nodes, note):
    code, lat, loss = expected(edges, nodes)
    # cross-check with the C++ oracle, both plumbing modes
    for mode in (0, 1):
        try:
            ol, of = oracle.compute_shortest_paths(edges.as_tuple(), nodes, mode=mode)
            ocode = 0
        except oracle.OracleError as e:
            ocode = e.code
        assert ocode == code, (name, mode, ocode, code)
        if code == 0:
            assert (ol == lat).all(), name
            assert (of.view(np.uint32) == loss.view(np.uint32)).all(), name
    if code == 0:
        nx_check(edges, nodes, lat)
    d = {
        "name": name, "note": note, "num_vertices": edges.num_vertices, "directed": bool(edges.directed),
        "src": edges.src.tolist(), "dst": edges.dst.tolist(),
        "latency_ns": [str(x) for x in edges.latency_ns.tolist()],
        "packet_loss_bits": edges.packet_loss.view(np.uint32).tolist(),
        "nodes": [int(x) for x in nodes], "expect_code": code,
    }
    if code == 0:
        d["expect_latency_ns"] = [str(x) for x in lat.ravel().tolist()]
        d["expect_packet_loss_bits"] = loss.view(np.uint32).ravel().tolist()
    return d


def main():
    fx = []
    rng = np.random.default_rng(20250220)
    # random graphs: ties (small latency ranges), parallel edges, directed/undirected
    cases = [
        ("undirected_ties", dict(V=20, density=0.3, seed=1, lat_hi=5)),
        ("undirected_ties_parallel", dict(V=24, density=0.25, seed=2, lat_hi=4, parallel=0.3)),
        ("directed_sparse", dict(V=30, density=0.15, seed=3, directed=True, lat_hi=1000)),
        ("directed_ties", dict(V=26, density=0.3, seed=4, directed=True, lat_hi=3)),
        ("undirected_dense", dict(V=40, density=0.9, seed=5, lat_hi=100000)),
        ("directed_dense_parallel", dict(V=32, density=0.7, seed=6, directed=True, lat_hi=50, parallel=0.2)),
        ("tiny_losses", dict(V=18, density=0.4, seed=7, lat_hi=6, loss_hi=1e-7)),
        ("high_losses", dict(V=18, density=0.4, seed=8, lat_hi=6, loss_hi=1.0, p_zero=0.0)),
    ]
    for name, kw in cases:
        kw = dict(kw)
        V = kw.pop("V")
        dens = kw.pop("density")
        seed = kw.pop("seed")
        g = synth.random_graph(V, dens, seed, **kw)
        nodes = list(range(V))
        fx.append(fixture(name, g, nodes, f"random_graph({V}, {dens}, {seed}, {kw})"))
    # subset of nodes in a scrambled (HashSet-like) order; intermediates are unused vertices
    g = synth.random_graph(36, 0.2, 9, lat_hi=20)
    nodes = rng.permutation(36)[:14].tolist()
    fx.append(fixture("subset_nodes", g, nodes, "14 of 36 vertices used, scrambled order"))
    # unused vertex WITHOUT a self-loop is fine; an unused unreachable vertex is fine
    V = 10
    src = list(range(8)) + [0, 1, 2, 3, 4, 5, 6, 8]
    dst = list(range(8)) + [1, 2, 3, 4, 5, 6, 7, 9]
    lat = [100 + i for i in range(8)] + [3, 4, 5, 6, 7, 8, 9, 1]
    loss = [0.0] * 8 + [0.01, 0.02, 0.0, 0.5, 0.0, 1e-3, 0.25, 0.0]
    e = Edges(V, src, dst, lat, loss, directed=False)
    fx.append(fixture("path_graph_unused_isolated", e, list(range(8)), "long path, isolated unused pair 8-9"))
    # equal-latency parallel edges with different losses, -0.0 loss, loss 1.0
    V = 4
    src = [0, 1, 2, 3, 0, 0, 0, 1, 2, 1, 0]
    dst = [0, 1, 2, 3, 1, 1, 1, 2, 3, 3, 3]
    lat = [1, 2, 3, 4, 10, 10, 10, 5, 5, 10, 20]
    loss = [0.0, -0.0, 1.0, 0.5, 0.3, 0.1, 0.2, 0.0, 1.0, -0.0, 0.05]
    e = Edges(V, src, dst, lat, loss, directed=True)
    fx.append(fixture("parallel_equal_latency", e, [0, 1, 2, 3], "parallel ties, -0.0, 1.0 losses"))
    # large latencies force the u64 key path on the GPU (distances >= 2^32)
    g = synth.random_graph(16, 0.3, 10, lat_lo=2**31, lat_hi=2**33, directed=True)
    fx.append(fixture("u64_latencies", g, list(range(16)), "latencies in [2^31, 2^33]"))
    # error cases (mod.rs:215-219)
    g = synth.random_graph(8, 0.5, 11, selfloops=False)
    fx.append(fixture("error_no_selfloop", g, list(range(8)), "no self-loops -> No edge connecting"))
    g = synth.random_graph(8, 0.5, 12)
    g2 = Edges(8, np.concatenate([g.src, [3]]), np.concatenate([g.dst, [3]]),
               np.concatenate([g.latency_ns, [7]]), np.concatenate([g.packet_loss, [0.0]]), directed=False)
    fx.append(fixture("error_multi_selfloop", g2, list(range(8)), "node 3 has two self-loops"))
    e = Edges(4, [0, 1, 2, 3, 0, 2], [0, 1, 2, 3, 1, 3], [1, 1, 1, 1, 5, 5], [0.0] * 6, directed=False)
    fx.append(fixture("error_unreachable", e, [0, 1, 2, 3], "two components -> assert panic"))

    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "routing_vectors.json")
    with open(out, "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "fixtures": fx}, f, separators=(",", ":"))
    print(f"wrote {len(fx)} fixtures to {out} ({os.path.getsize(out)} bytes)")


if __name__ == "__main__":
    main()
