"""CPU: pin the oracle (oracle/oracle.cpp) against the reference's KATs and the golden vectors."""
import numpy as np
import pytest

import oracle
from shadow_amd import NetworkGraph, PathProperties, synth
from helpers import bits_equal, fixture_edges, fixture_expect, kat_gml, load_kats, load_vectors


@pytest.mark.parametrize("directed", [True, False])
def test_kat_shortest_path(directed):
    """mod.rs:559-647 test_shortest_path through the oracle (both plumbing modes)."""
    kats = load_kats()["test_shortest_path"]
    exp = kats["expect_directed" if directed else "expect_undirected"]
    g = NetworkGraph.parse(kat_gml(directed))
    nodes = [g.node_id_to_index(i) for i in (0, 1, 2)]
    for mode in (0, 1):
        lat, _ = oracle.compute_shortest_paths(g.edges.as_tuple(), nodes, mode=mode)
        for k, v in exp.items():
            assert int(lat[int(k[0]), int(k[1])]) == v, (k, mode)


def test_kat_path_add():
    """mod.rs:515-529 test_path_add (tolerance 0.01) -- and the exact f32 value."""
    k = load_kats()["test_path_add"]
    lat, loss = oracle.path_add(tuple(k["a"]), tuple(k["b"]))
    assert lat == k["expect_latency"]
    assert abs(loss - k["expect_loss"]) < k["tolerance"]
    f = np.float32
    assert np.float32(loss) == f(1) - (f(1) - f(0.35)) * (f(1) - f(0.85))
    p = PathProperties(23, 0.35) + PathProperties(11, 0.85)
    assert p.latency_ns == 34 and np.float32(p.packet_loss) == np.float32(loss)


def test_path_properties_ordering():
    """PartialOrd is lexicographic (mod.rs:305-320)."""
    assert PathProperties(1, 0.9) < PathProperties(2, 0.0)
    assert PathProperties(2, 0.1) < PathProperties(2, 0.2)
    assert PathProperties(2, 0.0) == PathProperties(2, -0.0)


@pytest.mark.parametrize("fx", load_vectors(), ids=lambda f: f["name"])
def test_oracle_golden(fx):
    """The C++ oracle reproduces every committed golden vector bit-exactly."""
    e = fixture_edges(fx)
    if fx["expect_code"]:
        with pytest.raises(oracle.OracleError) as ei:
            oracle.compute_shortest_paths(e.as_tuple(), fx["nodes"], mode=0)
        assert ei.value.code == fx["expect_code"]
        return
    lat, loss = fixture_expect(fx)
    for mode in (0, 1, 2):
        ol, of = oracle.compute_shortest_paths(e.as_tuple(), fx["nodes"], mode=mode)
        assert np.array_equal(ol, lat)
        assert np.array_equal(of.view(np.uint32), loss)


@pytest.mark.parametrize("kw", [dict(V=300, density=0.3, seed=5, lat_hi=5, parallel=0.3),
                                dict(V=257, density=0.1, seed=6, directed=True, lat_hi=1000, loss_hi=1e-6),
                                dict(V=200, density=1.0, seed=8, lat_hi=3, parallel=0.5)],
                         ids=["ties_parallel", "directed_tiny_loss", "complete_ties"])
def test_oracle_matrix_mode_pinned(kw):
    """mode 2 (dense-matrix Dijkstra, the full-size checker) == mode 1 (petgraph heap Dijkstra)
    bit for bit on graphs with latency ties, parallel edges and tiny losses."""
    kw = dict(kw)
    V, d, s = kw.pop("V"), kw.pop("density"), kw.pop("seed")
    g = synth.random_graph(V, d, s, **kw)
    nodes = np.random.default_rng(s).permutation(V)[: V - 7].tolist()
    try:
        a = oracle.compute_shortest_paths(g.as_tuple(), nodes, mode=1)
    except oracle.OracleError as e1:
        with pytest.raises(oracle.OracleError) as e2:
            oracle.compute_shortest_paths(g.as_tuple(), nodes, mode=2)
        assert e2.value.code == e1.code
        return
    b = oracle.compute_shortest_paths(g.as_tuple(), nodes, mode=2)
    assert np.array_equal(a[0], b[0]) and bits_equal(a[1], b[1])


def test_oracle_rows_subset_matches_full():
    g = synth.random_graph(60, 0.2, 77, lat_hi=50)
    nodes = list(range(60))
    lat, loss = oracle.compute_shortest_paths(g.as_tuple(), nodes)
    rows = [3, 17, 59]
    rl, rs = oracle.compute_shortest_paths(g.as_tuple(), nodes, rows=rows)
    assert np.array_equal(rl, lat[rows]) and bits_equal(rs, loss[rows])


def test_oracle_latency_vs_networkx_c1_sample():
    """Latency of the C1 generator's graph vs networkx on sampled sources (no ties in weights)."""
    import networkx as nx
    e = synth.complete_random(200, seed=5)
    G = nx.Graph()
    for s, t, l in zip(e.src.tolist(), e.dst.tolist(), e.latency_ns.tolist()):
        if s != t:
            G.add_edge(s, t, w=l)
    nodes = list(range(200))
    rows = [0, 50, 199]
    lat, _ = oracle.compute_shortest_paths(e.as_tuple(), nodes, rows=rows)
    for r, s in enumerate(rows):
        d = nx.single_source_dijkstra_path_length(G, s, weight="w")
        for t in nodes:
            if t != s:
                assert d[t] == int(lat[r, t])


def test_direct_paths_oracle_kat():
    """get_direct_paths on the KAT graph: directed 1->2 has no edge -> error (mod.rs:266-268)."""
    g = NetworkGraph.parse(kat_gml(True))
    with pytest.raises(oracle.OracleError) as ei:
        oracle.get_direct_paths(g.edges.as_tuple(), [0, 1, 2])
    assert ei.value.code == 2 and "No edge connecting node 1 to 2" in ei.value.msg
    # complete graph: every pair has exactly one edge
    e = synth.complete_random(12, seed=3)
    lat, loss = oracle.get_direct_paths(e.as_tuple(), list(range(12)))
    assert lat[3, 5] == lat[5, 3]
