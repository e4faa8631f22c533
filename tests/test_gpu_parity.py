"""GPU parity: HIP path (through the C ABI) vs the oracle / golden vectors.  Bit-exact on
latency (u64) AND packet_loss (f32 bits) -- stricter than the north star's 1e-6 relative
loss tolerance, which is asserted too (LOSS_RTOL) so a tolerance regression is visible."""
import numpy as np
import pytest

import oracle
from shadow_amd import NetGraphError, NetworkGraph, Router, RoutingPanic, generate_routing_info, synth
from shadow_amd import _native as N
from shadow_amd.graph import Edges
from helpers import bits_equal, fixture_edges, fixture_expect, kat_gml, load_kats, load_vectors

pytestmark = pytest.mark.gpu
LOSS_RTOL = 1e-6  # north star: packet_loss within 1e-6 relative


def assert_parity(table, lat, loss):
    assert np.array_equal(table.latency_ns, lat), "latency_ns must be bit-exact"
    got = table.packet_loss.astype(np.float64)
    ref = np.asarray(loss, dtype=np.float32).astype(np.float64)
    assert np.all(np.abs(got - ref) <= LOSS_RTOL * np.abs(ref)), "packet_loss beyond 1e-6 relative"
    assert bits_equal(table.packet_loss, loss), "packet_loss not bit-exact"


@pytest.mark.parametrize("fx", load_vectors(), ids=lambda f: f["name"])
def test_golden_vectors(scan_router, fx):
    router = scan_router
    e = fixture_edges(fx)
    if fx["expect_code"]:
        with pytest.raises(NetGraphError) as ei:
            router.compute_shortest_paths(e, fx["nodes"])
        assert ei.value.code == fx["expect_code"]
        return
    lat, loss = fixture_expect(fx)
    t = router.compute_shortest_paths(e, fx["nodes"])
    assert_parity(t, lat, loss.view(np.float32))
    if fx["name"] == "u64_latencies":
        assert t.stats["path_kind"] == N.SRG_PATH_DENSE_U64


@pytest.mark.parametrize("directed", [True, False])
def test_kat_shortest_path_gpu(router, directed):
    """mod.rs:559-647 test_shortest_path, end to end: GML text -> HIP."""
    exp = load_kats()["test_shortest_path"]["expect_directed" if directed else "expect_undirected"]
    g = NetworkGraph.parse(kat_gml(directed))
    n0, n1, n2 = (g.node_id_to_index(i) for i in (0, 1, 2))
    sp = g.compute_shortest_paths([n0, n1, n2], router)
    assert len(sp) == 9
    for k, v in exp.items():
        a, b = (n0, n1, n2)[int(k[0])], (n0, n1, n2)[int(k[1])]
        assert sp[(a, b)].latency_ns == v


CASES = [
    dict(V=50, density=0.2, seed=101, lat_hi=8),
    dict(V=129, density=0.1, seed=102, directed=True, lat_hi=1000),
    dict(V=130, density=0.3, seed=103, lat_hi=3, parallel=0.3),
    dict(V=200, density=0.05, seed=104, directed=True, lat_hi=20, loss_hi=1e-6),
    dict(V=257, density=0.5, seed=105, lat_hi=10**8, lat_lo=10**6),
    dict(V=300, density=0.02, seed=106, lat_hi=50),
    dict(V=70, density=0.4, seed=107, directed=True, lat_lo=2**31, lat_hi=2**34),
]


@pytest.fixture(params=["sparse", "dense"])
def scan_router(request):
    """Both tight-scan variants: essential-edge (sparse) and all-triples (dense)."""
    r = Router(0)
    r.set_option(N.SRG_OPT_SPARSE_THRESHOLD, 1.0 if request.param == "sparse" else 0.0)
    r.expect_scan = N.SRG_SCAN_SPARSE if request.param == "sparse" else N.SRG_SCAN_DENSE
    yield r
    r.close()


@pytest.mark.parametrize("kw", CASES, ids=lambda k: f"V{k['V']}_s{k['seed']}")
def test_random_vs_oracle(scan_router, kw):
    router = scan_router
    kw = dict(kw)
    V, dens, seed = kw.pop("V"), kw.pop("density"), kw.pop("seed")
    g = synth.random_graph(V, dens, seed, **kw)
    nodes = list(range(V))
    try:
        lat, loss = oracle.compute_shortest_paths(g.as_tuple(), nodes)
    except oracle.OracleError as e:
        with pytest.raises(NetGraphError) as ei:
            router.compute_shortest_paths(g, nodes)
        assert ei.value.code == e.code
        return
    tab = router.compute_shortest_paths(g, nodes)
    assert tab.stats["scan_kind"] == router.expect_scan
    assert_parity(tab, lat, loss)


@pytest.mark.parametrize("kw", [dict(V=300, density=0.1, seed=111, lat_hi=40, parallel=0.1),
                                dict(V=390, density=0.2, seed=112, directed=True, lat_lo=10**6, lat_hi=10**8)],
                         ids=["ties", "directed_wide"])
def test_fw_kernels_match_oracle(router, kw):
    """The u32 FW tile kernels (pair-packed 64-bit adds; general FW on the directed graph, the
    symmetric line-buffer FW on the undirected one) are bit-exact; V not a multiple of the 128 tile
    exercises the padding."""
    r = Router(0)
    kw = dict(kw)
    V, dens, seed = kw.pop("V"), kw.pop("density"), kw.pop("seed")
    g = synth.random_graph(V, dens, seed, **kw)
    lat, loss = oracle.compute_shortest_paths(g.as_tuple(), list(range(V)))
    t = r.compute_shortest_paths(g, list(range(V)))
    assert t.stats["path_kind"] == N.SRG_PATH_DENSE_U32
    assert_parity(t, lat, loss)
    r.close()


def test_scan_matches_oracle():
    """The pair-lane tight scan (tight_v5) on ties, parallel edges and a directed graph, with
    scrambled node lists, forced onto the essential-entry path."""
    r = Router(0)
    r.set_option(N.SRG_OPT_SPARSE_THRESHOLD, 1.0)
    for kw in (dict(V=300, density=0.1, seed=121, lat_hi=30, parallel=0.2),
               dict(V=257, density=0.4, seed=122, directed=True, lat_lo=10**6, lat_hi=10**8)):
        kw = dict(kw)
        V, dens, seed = kw.pop("V"), kw.pop("density"), kw.pop("seed")
        g = synth.random_graph(V, dens, seed, **kw)
        nodes = np.random.default_rng(seed).permutation(V).tolist()
        lat, loss = oracle.compute_shortest_paths(g.as_tuple(), nodes)
        t = r.compute_shortest_paths(g, nodes)
        assert t.stats["scan_kind"] == N.SRG_SCAN_SPARSE
        assert_parity(t, lat, loss)
    r.close()


@pytest.mark.parametrize("V", [100, 200, 300, 1000])
def test_fw_symmetric_matches_general(V):
    """Undirected graphs: FW over the stored tiles I <= J (+ mirror) equals the general FW
    table bit for bit, at one, two, three and eight 128-tiles; and the oracle on V <= 300."""
    g = synth.atlas_like(V, seed=V + 7)
    nodes = np.random.default_rng(V).permutation(V).tolist()
    out = []
    for sym in (0, 1):  # general FW, symmetric FW
        r = Router(0)
        r.set_option(N.SRG_OPT_FW_SYMMETRIC, sym)
        t = r.compute_shortest_paths(g, nodes)
        assert t.stats["path_kind"] == N.SRG_PATH_DENSE_U32
        out.append(t)
        r.close()
    for o in out[1:]:
        assert np.array_equal(out[0].latency_ns, o.latency_ns)
        assert bits_equal(out[0].packet_loss, o.packet_loss)
    if V <= 300:
        lat, loss = oracle.compute_shortest_paths(g.as_tuple(), nodes)
        assert_parity(out[1], lat, loss)


@pytest.mark.parametrize("V,split", [(60, 0), (200, 0), (700, 1), (700, 2), (700, 4), (1500, 0)])
def test_fw_symmetric_u64_matches_general(V, split, monkeypatch):
    """u64 keys (nanosecond keys, SRG_LATENCY_UNIT=1, on latencies x 1000 so that used paths pass
    2^31 ns): the symmetric line-buffer FW on 64-tiles (fw_core_lb64, fw_close_sq<u64>) equals the
    general u64 FW bit for bit at one to 24 tiles and every line split; oracle rows pin it."""
    monkeypatch.setenv("SRG_LATENCY_UNIT", "1")
    g = synth.atlas_like(V, seed=V + 11)
    e = Edges(V, g.src, g.dst, g.latency_ns * np.uint64(1000), g.packet_loss, directed=False)
    nodes = np.random.default_rng(V).permutation(V).tolist()
    out = []
    for sym in (0, 1):
        r = Router(0)
        r.set_option(N.SRG_OPT_FW_SYMMETRIC, sym)
        if split:
            r.set_option(N.SRG_OPT_FW_LINE_SPLIT, split)
        t = r.compute_shortest_paths(e, nodes)
        assert t.stats["path_kind"] == N.SRG_PATH_DENSE_U64 and t.stats["latency_unit_ns"] == 1
        out.append(t)
        r.close()
    assert np.array_equal(out[0].latency_ns, out[1].latency_ns)
    assert bits_equal(out[0].packet_loss, out[1].packet_loss)
    rows = [0, V // 2, V - 1]
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), nodes, rows=rows, mode=2, nthreads=8)
    assert np.array_equal(out[1].latency_ns[rows], lat) and bits_equal(out[1].packet_loss[rows], loss)


def test_fw_stream_hops_events_match_values(monkeypatch):
    """The FW's two cross-stream hops per pivot as stream-value waits (a context alone on its
    device) and as events (SRG_STREAM_HOPS=events: several contexts per device, profilers) give
    the same table bit for bit, and the oracle's rows (routing.hip stream_hop)."""
    V = 1500
    g = synth.atlas_like(V, seed=91)
    nodes = list(range(V))
    out = []
    for hops in (None, "events"):
        if hops:
            monkeypatch.setenv("SRG_STREAM_HOPS", hops)
        else:
            monkeypatch.delenv("SRG_STREAM_HOPS", raising=False)
        r = Router(0)
        out.append(r.compute_shortest_paths(g, nodes))
        r.close()
    assert np.array_equal(out[0].latency_ns, out[1].latency_ns)
    assert bits_equal(out[0].packet_loss, out[1].packet_loss)
    rows = [0, 777, V - 1]
    lat, loss = oracle.compute_shortest_paths(g.as_tuple(), nodes, rows=rows, mode=2)
    assert np.array_equal(out[0].latency_ns[rows], lat) and bits_equal(out[0].packet_loss[rows], loss)


def test_scan_ragged_sources():
    """Several 128-source blocks, target tiles and u-chunks, with n and V off every block size and
    a used-node subset in random order (lanes past n, targets past V, sentinel pairs)."""
    r = Router(0)
    r.set_option(N.SRG_OPT_SPARSE_THRESHOLD, 1.0)
    g = synth.atlas_like(700, seed=1234)
    nodes = np.random.default_rng(7).permutation(700)[:333].tolist()
    lat, loss = oracle.compute_shortest_paths(g.as_tuple(), nodes)
    t = r.compute_shortest_paths(g, nodes)
    assert t.stats["scan_kind"] == N.SRG_SCAN_SPARSE
    assert_parity(t, lat, loss)
    r.close()


@pytest.mark.parametrize("lat_lo,lat_hi,kind",[(2**27, 2**28, "u32"), (2**29, 2**30 + 2**29, "u64")])
def test_u32_key_bound(router, lat_lo, lat_hi, kind):
    """u32 keys hold distances < INF = 2^31 - 1 (packed pair adds must not carry); longer used
    paths must be detected and rerun on u64 keys, bit-exact either way."""
    g = synth.random_graph(60, 0.08, 113, lat_lo=lat_lo, lat_hi=lat_hi)
    nodes = list(range(60))
    lat, loss = oracle.compute_shortest_paths(g.as_tuple(), nodes)
    t = router.compute_shortest_paths(g, nodes)
    exp = N.SRG_PATH_DENSE_U32 if kind == "u32" else N.SRG_PATH_DENSE_U64
    assert int(lat.max()) >= 2**31 - 1 if kind == "u64" else int(lat.max()) < 2**31 - 1
    assert t.stats["path_kind"] == exp
    assert_parity(t, lat, loss)


def test_subset_nodes_scrambled(scan_router):
    router = scan_router
    g = synth.random_graph(180, 0.1, 7, lat_hi=100)
    rng = np.random.default_rng(1)
    nodes = rng.permutation(180)[:77].tolist()
    lat, loss = oracle.compute_shortest_paths(g.as_tuple(), nodes)
    assert_parity(router.compute_shortest_paths(g, nodes), lat, loss)


def test_unused_isolated_vertex_keeps_u32(router):
    """certification covers used (row, column) pairs only, so an isolated UNUSED vertex
    (unreachable from everything) keeps the u32 keys; an isolated USED vertex with small
    latencies (max_lat * (V-1) < 2^31-1) is the reference's panic without a u64 rerun."""
    g = synth.atlas_like(300, seed=3)
    V = g.num_vertices + 1
    iso = Edges(V, np.r_[g.src, V - 1], np.r_[g.dst, V - 1], np.r_[g.latency_ns, 1_000_000],
                np.r_[g.packet_loss, 0.0], False)
    nodes = list(range(V - 1))
    lat, loss = oracle.compute_shortest_paths(iso.as_tuple(), nodes)
    t = router.compute_shortest_paths(iso, nodes)
    assert t.stats["path_kind"] == N.SRG_PATH_DENSE_U32
    assert_parity(t, lat, loss)
    small = synth.random_graph(100, 0.2, 5, lat_hi=10)
    iso2 = Edges(101, np.r_[small.src, 100], np.r_[small.dst, 100], np.r_[small.latency_ns, 7],
                 np.r_[small.packet_loss, 0.0], False)
    with pytest.raises(RoutingPanic):
        router.compute_shortest_paths(iso2, list(range(101)))


def test_latency_range_is_an_error(router, monkeypatch):
    """Documented divergence: when a used pair has no path below 2^62 latency
    units on a graph whose worst-case path sum reaches 2^62 units, the library returns
    SRG_ERR_LATENCY_RANGE, where the release build of the reference would wrap u64
    silently (mod.rs:327 `+` on u64, overflow checks off in src/Cargo.toml:56-61).  The Rust
    binding panics on it, like the `.unwrap()` of an overflowing unit conversion (mod.rs:336).
    With nanosecond keys (SRG_LATENCY_UNIT=1) a 2^61-ns pair of links is such a graph; with the
    latency unit (their gcd, 2^61) the same graph is 2 units of path and matches the reference."""
    big = 2 ** 61
    e = Edges(3, [0, 1, 2, 0, 1], [0, 1, 2, 1, 2], [1, 1, 1, big, big], [0.0] * 5, False)
    t = router.compute_shortest_paths(e, [0, 1, 2])
    assert t[(0, 2)].latency_ns == 2 ** 62 and t.stats["latency_unit_ns"] == big
    assert t.stats["path_kind"] == N.SRG_PATH_DENSE_U32
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), [0, 1, 2])
    assert_parity(t, lat, loss)
    monkeypatch.setenv("SRG_LATENCY_UNIT", "1")
    with pytest.raises(NetGraphError) as ei:
        router.compute_shortest_paths(e, [0, 1, 2])
    assert ei.value.code == N.SRG_ERR_LATENCY_RANGE
    ok = Edges(3, [0, 1, 2, 0, 1], [0, 1, 2, 1, 2], [1, 1, 1, 2 ** 40, 2 ** 40], [0.0] * 5, False)
    t = router.compute_shortest_paths(ok, [0, 1, 2])
    assert t[(0, 2)].latency_ns == 2 ** 41 and t.stats["path_kind"] == N.SRG_PATH_DENSE_U64
    assert t.stats["latency_unit_ns"] == 1
    # worst case max_lat * (V-1) >= 2^62, but no used shortest path comes near it (a "disabled"
    # 2^61-ns link beside a 2-hop route): the reference's Dijkstra succeeds, and so does this
    dis = Edges(3, [0, 1, 2, 0, 1, 0], [0, 1, 2, 1, 2, 2], [1, 1, 1, 1, 1, big], [0.0] * 6, False)
    t = router.compute_shortest_paths(dis, [0, 1, 2])
    assert t[(0, 2)].latency_ns == 2 and t[(2, 0)].latency_ns == 2
    lat, loss = oracle.compute_shortest_paths(dis.as_tuple(), [0, 1, 2])
    assert_parity(t, lat, loss)


def test_u64_edge_past_key_range_is_an_error(router, monkeypatch):
    """Documented deviation (include/shadow_routing.h SRG_ERR_LATENCY_RANGE): u64 keys hold
    distances below 2^62 units, so with nanosecond keys an edge of 2^63 ns + 1 counts as absent and
    the used pair it alone connects fails with SRG_ERR_LATENCY_RANGE, where the reference's u64
    Dijkstra returns it.  An edge of exactly 2^63 ns is one latency unit of 2^63 ns (the gcd of
    the non-self-loop latencies) and comes out as the reference's 2^63."""
    e = Edges(2, [0, 1, 0], [0, 1, 1], np.array([1000, 1000, 2 ** 63], dtype=np.uint64), [0.0, 0.0, 0.0], directed=False)
    t = router.compute_shortest_paths(e, [0, 1])
    assert t[(0, 1)].latency_ns == 2 ** 63 and t.stats["latency_unit_ns"] == 2 ** 63
    odd = Edges(2, [0, 1, 0, 0], [0, 1, 1, 1], np.array([1000, 1000, 2 ** 63 + 1, 2 ** 63 + 2], dtype=np.uint64),
                [0.0] * 4, directed=False)
    with pytest.raises(NetGraphError) as ei:
        router.compute_shortest_paths(odd, [0, 1])
    assert ei.value.code == N.SRG_ERR_LATENCY_RANGE
    monkeypatch.setenv("SRG_LATENCY_UNIT", "1")
    with pytest.raises(NetGraphError) as ei:
        router.compute_shortest_paths(e, [0, 1])
    assert ei.value.code == N.SRG_ERR_LATENCY_RANGE


def test_latency_unit_wrap_is_an_error(router):
    """with a latency unit the keys are small, but the outputs are key x unit ns.  Where
    a relaxation the reference's Dijkstra runs sums past 2^64 ns its release-build u64 `+` wraps
    (mod.rs:327) and its result is garbage; the library reports SRG_ERR_LATENCY_RANGE instead of a
    silently wrong table (k_wrap_edges).  Multi-hop paths with a unit >= 2^32 that stay below 2^64
    come out exact."""
    # 5-node path of 2^62-ns links: unit 2^62, key 1 per link; 0 -> 4 is 4 units = 2^64 ns
    p = Edges(5, list(range(5)) + [0, 1, 2, 3], list(range(5)) + [1, 2, 3, 4],
              np.array([1] * 5 + [2 ** 62] * 4, dtype=np.uint64), [0.0] * 9, False)
    with pytest.raises(NetGraphError) as ei:
        router.compute_shortest_paths(p, list(range(5)))
    assert ei.value.code == N.SRG_ERR_LATENCY_RANGE
    # ADVICE's triangle {2^63, 2^63, 3 * 2^62}: 2^63 + 2^63 wraps to 0 in the reference
    tri = Edges(3, [0, 1, 2, 0, 1, 0], [0, 1, 2, 1, 2, 2],
                np.array([1, 1, 1, 2 ** 63, 2 ** 63, 3 * 2 ** 62], dtype=np.uint64), [0.0] * 6, False)
    with pytest.raises(NetGraphError) as ei:
        router.compute_shortest_paths(tri, [0, 1, 2])
    assert ei.value.code == N.SRG_ERR_LATENCY_RANGE
    # unit 2^40 (>= 2^32), 3-hop shortest paths beside a long direct link: exact, u32 keys
    q = Edges(4, [0, 1, 2, 3, 0, 1, 2, 0], [0, 1, 2, 3, 1, 2, 3, 3],
              np.array([7, 7, 7, 7, 2 ** 40, 2 ** 40, 2 ** 41, 2 ** 43], dtype=np.uint64),
              np.array([0, 0, 0, 0, 0.01, 0.02, 0.0, 0.0], dtype=np.float32), False)
    t = router.compute_shortest_paths(q, [0, 1, 2, 3])
    assert t.stats["latency_unit_ns"] == 2 ** 40 and t.stats["path_kind"] == N.SRG_PATH_DENSE_U32
    assert t[(0, 3)].latency_ns == 2 ** 40 * 4
    lat, loss = oracle.compute_shortest_paths(q.as_tuple(), [0, 1, 2, 3])
    assert_parity(t, lat, loss)
    # a wrap-risk graph (max latency x V >= 2^64) whose relaxations all stay below 2^64: exact
    w = Edges(4, [0, 1, 2, 3, 0, 1, 2], [0, 1, 2, 3, 1, 2, 3],
              np.array([5, 5, 5, 5, 2 ** 61, 2 ** 61, 2 ** 62], dtype=np.uint64), [0.0] * 7, False)
    t = router.compute_shortest_paths(w, [0, 1, 2, 3])
    lat, loss = oracle.compute_shortest_paths(w.as_tuple(), [0, 1, 2, 3])
    assert t[(0, 3)].latency_ns == 2 ** 63
    assert_parity(t, lat, loss)


def test_deterministic_bytes(router):
    g = synth.random_graph(150, 0.2, 9, lat_hi=4, parallel=0.2)
    a = router.compute_shortest_paths(g, list(range(150)))
    b = router.compute_shortest_paths(g, list(range(150)))
    assert np.array_equal(a.latency_ns, b.latency_ns) and bits_equal(a.packet_loss, b.packet_loss)


def test_error_messages(router):
    g = NetworkGraph.parse(kat_gml(True))
    e = g.edges
    no_self = Edges(3, e.src[3:], e.dst[3:], e.latency_ns[3:], e.packet_loss[3:], True, e.node_ids)
    with pytest.raises(NetGraphError, match="No edge connecting node 0 to 0"):
        router.compute_shortest_paths(no_self, [0, 1, 2])
    two = Edges(3, np.r_[e.src, 1], np.r_[e.dst, 1], np.r_[e.latency_ns, 9], np.r_[e.packet_loss, 0.0], True, e.node_ids)
    with pytest.raises(NetGraphError, match="More than one edge connecting node 1 to 1"):
        router.compute_shortest_paths(two, [0, 1, 2])
    iso = Edges(4, [0, 1, 2, 3, 0], [0, 1, 2, 3, 1], [1, 1, 1, 1, 3], [0.0] * 5, False)
    with pytest.raises(RoutingPanic):
        router.compute_shortest_paths(iso, [0, 1, 2, 3])
    t = router.compute_shortest_paths(iso, [0, 1])     # unreachable unused vertices are fine
    assert t[(0, 1)].latency_ns == 3
    with pytest.raises(NetGraphError):
        router.compute_shortest_paths(iso, [0, 0])       # duplicate node


def test_direct_paths_vs_oracle(router):
    e = synth.complete_random(40, seed=11)
    nodes = list(np.random.default_rng(2).permutation(40)[:25])
    lat, loss = oracle.get_direct_paths(e.as_tuple(), nodes)
    t = router.get_direct_paths(e, nodes)
    assert np.array_equal(t.latency_ns, lat) and bits_equal(t.packet_loss, loss)
    g = NetworkGraph.parse(kat_gml(True))
    with pytest.raises(NetGraphError, match="No edge connecting node 1 to 2"):
        router.get_direct_paths(g.edges, [0, 1, 2])


def test_generate_routing_info_ids(router):
    """f1: generate_routing_info (sim_config.rs:425-462) through srg_routing_info_build -- a dense
    RoutingInfo keyed by GML id: path() by id (None for unknown ids), get_smallest_latency_ns over
    all entries incl. the diagonal (mod.rs:474-476), saturating packet counters (mod.rs:449-456),
    direct paths, and the reference's error context."""
    txt = synth.to_gml(synth.random_graph(20, 0.4, 3, lat_hi=9), node_ids=[100 + 3 * i for i in range(20)])
    g = NetworkGraph.parse(txt)
    ids = [157, 100, 130, 103]
    ri = generate_routing_info(g, set(ids), True, router)
    idx = [g.node_id_to_index(x) for x in ids]
    lat, loss = oracle.compute_shortest_paths(g.edges.as_tuple(), idx)
    for i, a in enumerate(ids):
        for j, b in enumerate(ids):
            p = ri.path(a, b)
            assert p.latency_ns == int(lat[i, j]) and np.float32(p.packet_loss) == loss[i, j]
    assert ri.path(100, 101) is None and ri.path(999, 100) is None
    assert ri.get_smallest_latency_ns() == int(lat.min())
    assert len(ri) == 16
    for _ in range(3):
        ri.increment_packet_count(100, 157)
    assert ri.packet_count(100, 157) == 3 and ri.packet_count(157, 100) == 0
    tl, tf, tid = ri.tables()
    assert sorted(tid.tolist()) == sorted(ids) and tl.shape == (4, 4)
    # use_shortest_path = false: direct edges; the KAT graph lacks 1->2 (mod.rs:266-268)
    kg = NetworkGraph.parse(kat_gml(True))
    with pytest.raises(NetGraphError, match="Failed to get the direct paths between graph nodes: No edge connecting"):
        generate_routing_info(kg, {0, 1, 2}, False, router)
    d = generate_routing_info(kg, {0, 1}, False, router)
    assert d.path(0, 1).latency_ns == 3 and d.path(1, 0).latency_ns == 5
    assert d.get_smallest_latency_ns() == 3
    with pytest.raises(NetGraphError, match="unwrap"):
        generate_routing_info(g, {100, 5}, True, router)  # id 5 is not a node (sim_config.rs:433)
    empty = generate_routing_info(g, set(), True, router)
    assert empty.get_smallest_latency_ns() is None and len(empty) == 0


def test_device_entry_matches_host(router):
    import torch
    from shadow_amd.device import DeviceGraph, compute_shortest_paths_device
    g = synth.atlas_like(300, seed=5)
    dg = DeviceGraph(g)
    nodes = torch.arange(300, dtype=torch.int32, device="cuda:0")
    ol = torch.empty((300, 300), dtype=torch.int64, device="cuda:0")
    os_ = torch.empty((300, 300), dtype=torch.float32, device="cuda:0")
    compute_shortest_paths_device(router, dg, nodes, ol, os_)
    torch.cuda.synchronize()
    t = router.compute_shortest_paths(g, list(range(300)))
    assert np.array_equal(ol.cpu().numpy().view(np.uint64), t.latency_ns)
    assert bits_equal(os_.cpu().numpy(), t.packet_loss)


@pytest.mark.parametrize("mode,groups", [(1, 0), (0, 0), (1, 1), (1, 2), (1, 7), (0, 3)])
def test_host_entry_early_rows_match_device(router, mode, groups):
    """Host entry with finished rows shipped while kernels run (table >= 64 MB: the caller's arrays
    are page-locked and filled by an SDMA engine (mode 1, default) or hipMemcpyAsync (0)) equals the device entry byte for byte, with the scan launched in
    `groups` source-block groups interleaved with the loss rows (0 = default 3, 1 = not
    interleaved, 7 = ragged groups); odd n makes the loss rows start off 16-B boundaries."""
    import torch
    from shadow_amd.device import DeviceGraph, compute_shortest_paths_device
    V = 2501
    g = synth.atlas_like(V, seed=77)
    router.set_option(N.SRG_OPT_D2H_MODE, mode)
    router.set_option(N.SRG_OPT_SCAN_GROUPS, groups)
    try:
        t = router.compute_shortest_paths(g, list(range(V)))
    finally:
        router.set_option(N.SRG_OPT_D2H_MODE, 1)
        router.set_option(N.SRG_OPT_SCAN_GROUPS, 0)
    # (latency rows as u32 keys widened on the host: 4 + 4 B per pair, else 8 + 4)
    assert t.stats["d2h_overlapped_bytes"] == V * V * (8 if t.stats["d2h_key_rows"] else 12)
    dg = DeviceGraph(g)
    nodes = torch.arange(V, dtype=torch.int32, device="cuda:0")
    ol = torch.empty((V, V), dtype=torch.int64, device="cuda:0")
    os_ = torch.empty((V, V), dtype=torch.float32, device="cuda:0")
    compute_shortest_paths_device(router, dg, nodes, ol, os_)
    torch.cuda.synchronize()
    assert np.array_equal(ol.cpu().numpy().view(np.uint64), t.latency_ns)
    assert bits_equal(os_.cpu().numpy(), t.packet_loss)


@pytest.mark.parametrize("shift,offset", [(32, 0), (32, 1), (40, 7), (0, 2 ** 33)])
def test_u64_low_word_scan(router, shift, offset, monkeypatch):
    """u64 keys: the pair-lane scan on the keys' low 32 bits equals the oracle.  Latencies that are multiples of 2^32 make every candidate
    match in the low words (false matches everywhere: the loss pass's exact multi-predecessor
    check must resolve them); with offsets the low words are informative again.  Nanosecond
    keys (SRG_LATENCY_UNIT=1): with the latency unit, the offset-free cases would be u32 keys."""
    monkeypatch.setenv("SRG_LATENCY_UNIT", "1")
    g = synth.random_graph(300, 0.08, 5 + shift, lat_lo=1, lat_hi=6, parallel=0.1)
    lat = g.latency_ns.astype(np.uint64) * np.uint64(2 ** shift) + np.uint64(offset)
    e = Edges(g.num_vertices, g.src, g.dst, lat, g.packet_loss, directed=False)
    nodes = list(range(300))
    try:
        ref_lat, ref_loss = oracle.compute_shortest_paths(e.as_tuple(), nodes)
    except oracle.OracleError as err:
        with pytest.raises(NetGraphError) as ei:
            router.compute_shortest_paths(e, nodes)
        assert ei.value.code == err.code
        return
    t = router.compute_shortest_paths(e, nodes)
    assert t.stats["path_kind"] == N.SRG_PATH_DENSE_U64
    assert_parity(t, ref_lat, ref_loss)


@pytest.mark.parametrize("algo", ["dense", "sparse"])
def test_latency_unit_keys(router, algo, monkeypatch):
    """Latency unit (routing.hip compute_device): keys count units of the gcd of the non-self-loop
    latencies.  Millisecond-granular latencies whose paths pass 2^31 ns keep u32 keys (dense FW
    or the sparse Bellman-Ford) and give the bytes of nanosecond keys (u64 FW), and the oracle's."""
    if algo == "dense":
        g = synth.atlas_like(700, seed=61)
    else:
        g = synth.random_graph(2100, 0.004, 62, lat_lo=1, lat_hi=200, parallel=0.1)
    lat = g.latency_ns.astype(np.uint64)
    if algo == "dense":  # multiples of 3 ms
        lat = np.maximum(lat // np.uint64(1000), np.uint64(1)) * np.uint64(3_000_000)
    else:  # multiples of 30 ms
        lat = lat * np.uint64(30_000_000)
    e = Edges(g.num_vertices, g.src, g.dst, lat, g.packet_loss, directed=False)
    nodes = list(range(0, g.num_vertices, 2)) if algo == "sparse" else list(range(g.num_vertices))
    if algo == "sparse":
        router.set_option(N.SRG_OPT_ALGORITHM, N.SRG_ALGO_SPARSE)
    try:
        t = router.compute_shortest_paths(e, nodes)
        monkeypatch.setenv("SRG_LATENCY_UNIT", "1")
        t1 = router.compute_shortest_paths(e, nodes)
    finally:
        router.set_option(N.SRG_OPT_ALGORITHM, N.SRG_ALGO_AUTO)
    assert int(t.latency_ns.max()) >= 2 ** 31  # past the nanosecond u32 keys
    unit = t.stats["latency_unit_ns"]
    assert unit % 3_000_000 == 0 and t1.stats["latency_unit_ns"] == 1
    want = N.SRG_PATH_SPARSE_U32 if algo == "sparse" else N.SRG_PATH_DENSE_U32
    want1 = N.SRG_PATH_SPARSE_U64 if algo == "sparse" else N.SRG_PATH_DENSE_U64
    assert t.stats["path_kind"] == want and t1.stats["path_kind"] == want1
    assert np.array_equal(t.latency_ns, t1.latency_ns) and bits_equal(t.packet_loss, t1.packet_loss)
    rows = [0, 1, len(nodes) - 1]
    rl, rs = oracle.compute_shortest_paths(e.as_tuple(), nodes, rows=rows, mode=2, nthreads=8)
    assert np.array_equal(t.latency_ns[rows], rl) and bits_equal(t.packet_loss[rows], rs)


def test_h2d_codec_matches_plain(router):
    """Host entry H2D codec (SRG_OPT_H2D_CODEC: u16 endpoints + u32 latencies over PCIe, widened on
    the device) gives the same bytes as the plain transfer; a latency >= 2^32 makes it fall back
    to the plain arrays (same result again), and oracle rows pin both."""
    V = 1500  # 1.12 M edges: past the codec's 2^20-edge threshold
    g = synth.atlas_like(V, seed=31)
    nodes = list(range(V))
    out = {}
    for codec in (1, 0):
        router.set_option(N.SRG_OPT_H2D_CODEC, codec)
        out[codec] = router.compute_shortest_paths(g, nodes)
    router.set_option(N.SRG_OPT_H2D_CODEC, 1)
    assert np.array_equal(out[0].latency_ns, out[1].latency_ns)
    assert bits_equal(out[0].packet_loss, out[1].packet_loss)
    rows = [0, 7, 1499]
    lat, loss = oracle.compute_shortest_paths(g.as_tuple(), nodes, rows=rows, mode=2, nthreads=8)
    assert np.array_equal(out[1].latency_ns[rows], lat) and bits_equal(out[1].packet_loss[rows], loss)
    # one edge of 2^33 ns (never on a shortest path): the codec cannot narrow it
    big = Edges(V, g.src, g.dst, g.latency_ns.copy(), g.packet_loss, directed=False)
    k = int(np.nonzero(big.src != big.dst)[0][5])
    big.latency_ns[k] = 2 ** 33
    t = router.compute_shortest_paths(big, nodes)
    router.set_option(N.SRG_OPT_H2D_CODEC, 0)
    t0 = router.compute_shortest_paths(big, nodes)
    router.set_option(N.SRG_OPT_H2D_CODEC, 1)
    assert np.array_equal(t.latency_ns, t0.latency_ns) and bits_equal(t.packet_loss, t0.packet_loss)


@pytest.mark.parametrize("order", ["rows", "rows_gaps", "shuffled_tail", "shuffled"])
def test_h2d_codec_sequential_pairs(router, monkeypatch, order):
    """Sequential-pair codec (routing.hip codec_in): a row-ordered edge list crosses PCIe as u32
    latencies + exceptions (row starts, gaps), decoded on the device (k_decode_seq); a chunk with
    more than 1/8 exceptions is re-narrowed to u16 endpoints, and the rest of the list with it.
    Every variant gives the plain transfer's bytes (SRG_CODEC_SEQ=0: u16 endpoints throughout;
    SRG_OPT_H2D_CODEC 0: plain)."""
    V = 2100 if order == "shuffled_tail" else 1600  # 2.2 M edges (two chunks) / 1.28 M
    g = synth.atlas_like(V, seed=41)
    src, dst, lat, loss = g.src.copy(), g.dst.copy(), g.latency_ns.copy(), g.packet_loss.copy()
    rng = np.random.default_rng(5)
    if order == "rows_gaps":  # ~5 % of the pairs missing: gaps are exceptions, still sequential mode
        keep = np.ones(len(src), dtype=bool)
        keep[V:] = rng.random(len(src) - V) > 0.05
        src, dst, lat, loss = src[keep], dst[keep], lat[keep], loss[keep]
    elif order == "shuffled_tail":  # chunk 0 in rows, chunk 1 shuffled: the switch mid-list
        head = 2 << 20
        perm = np.r_[np.arange(head), head + rng.permutation(len(src) - head)]
        src, dst, lat, loss = src[perm], dst[perm], lat[perm], loss[perm]
    elif order == "shuffled":
        perm = rng.permutation(len(src))
        src, dst, lat, loss = src[perm], dst[perm], lat[perm], loss[perm]
    e = Edges(V, src, dst, lat, loss, directed=False)
    nodes = list(range(V))
    monkeypatch.setenv("SRG_CODEC_SEQ", "1")
    t = router.compute_shortest_paths(e, nodes)
    monkeypatch.setenv("SRG_CODEC_SEQ", "0")
    t16 = router.compute_shortest_paths(e, nodes)
    monkeypatch.delenv("SRG_CODEC_SEQ")
    router.set_option(N.SRG_OPT_H2D_CODEC, 0)
    try:
        t0 = router.compute_shortest_paths(e, nodes)
    finally:
        router.set_option(N.SRG_OPT_H2D_CODEC, 1)
    for o in (t16, t0):
        assert np.array_equal(t.latency_ns, o.latency_ns) and bits_equal(t.packet_loss, o.packet_loss)
    rows = [0, 801, V - 1]
    rl, rs = oracle.compute_shortest_paths(e.as_tuple(), nodes, rows=rows, mode=2, nthreads=8)
    assert np.array_equal(t.latency_ns[rows], rl) and bits_equal(t.packet_loss[rows], rs)


def test_h2d_codec_host_slow_fallback(router, monkeypatch):
    """The codec's mid-transfer switch to plain arrays (taken when narrowing a chunk on the host
    is slower than shipping it plain; forced here after the first chunk) gives the same bytes."""
    V = 2100  # 2.2 M edges: two codec chunks
    g = synth.atlas_like(V, seed=33)
    nodes = list(range(V))
    monkeypatch.setenv("SRG_CODEC_SLOW_AFTER", "0")
    t = router.compute_shortest_paths(g, nodes)
    monkeypatch.delenv("SRG_CODEC_SLOW_AFTER")
    router.set_option(N.SRG_OPT_H2D_CODEC, 0)
    t0 = router.compute_shortest_paths(g, nodes)
    router.set_option(N.SRG_OPT_H2D_CODEC, 1)
    assert np.array_equal(t.latency_ns, t0.latency_ns) and bits_equal(t.packet_loss, t0.packet_loss)


@pytest.mark.slow
def test_c1_full_vs_oracle(router):
    """Config C1 (1000-vertex complete graph), every pair."""
    e = synth.complete_random(1000, seed=1001)
    nodes = list(range(1000))
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), nodes, nthreads=16)
    assert_parity(router.compute_shortest_paths(e, nodes), lat, loss)


C3_ROWS = 512  # >= 512 seeded sources checked against the oracle at C3


@pytest.mark.slow
def test_c3_bench_size_sampled_rows(router):
    """Config C3 at the bench's full size (10 000-vertex Atlas-like complete graph, the headline
    workload) through the device entry: C3_ROWS = 512 seeded oracle rows bit-exact (oracle mode 2,
    the dense-matrix Dijkstra pinned to the heap Dijkstra in test_oracle.py), plus
    size-independent properties over the whole 10^8-pair table (diagonal = self-loops,
    symmetric latency, every latency <= the direct edge, every loss in [0, 1])."""
    import torch
    from shadow_amd.device import DeviceGraph, compute_shortest_paths_device
    V = 10000
    e = synth.atlas_like(V, seed=V)
    dg = DeviceGraph(e)
    nodes_t = torch.arange(V, dtype=torch.int32, device="cuda:0")
    ol = torch.empty((V, V), dtype=torch.int64, device="cuda:0")
    os_ = torch.empty((V, V), dtype=torch.float32, device="cuda:0")
    st = compute_shortest_paths_device(router, dg, nodes_t, ol, os_)
    torch.cuda.synchronize()
    assert st["path_kind"] == N.SRG_PATH_DENSE_U32
    lat_t = ol.cpu().numpy().view(np.uint64)
    loss_t = os_.cpu().numpy()
    del ol, os_
    rows = np.random.default_rng(V).choice(V, C3_ROWS, replace=False).tolist()
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), list(range(V)), rows=rows, mode=2, nthreads=16)
    assert np.array_equal(lat_t[rows], lat)
    assert bits_equal(loss_t[rows], loss)
    assert np.array_equal(np.diag(lat_t), e.latency_ns[:V])
    off = ~np.eye(V, dtype=bool)
    assert np.array_equal(lat_t[off], lat_t.T[off])
    direct = np.full((V, V), np.iinfo(np.uint64).max, dtype=np.uint64)
    m = e.src != e.dst
    direct[e.src[m], e.dst[m]] = e.latency_ns[m]
    direct[e.dst[m], e.src[m]] = e.latency_ns[m]
    assert np.all(lat_t[off] <= direct[off])
    assert np.all((loss_t >= 0) & (loss_t <= 1))


@pytest.mark.slow
def test_c2_sampled_rows(router):
    """Config C2 (4096-vertex Atlas-like): full GPU matrix vs 512 seeded oracle rows (mode 2),
    plus size-independent properties (diagonal = self-loops, symmetric latency)."""
    e = synth.atlas_like(4096, seed=4096)
    nodes = list(range(4096))
    t = router.compute_shortest_paths(e, nodes)
    rows = np.random.default_rng(4096).choice(4096, 512, replace=False).tolist()
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), nodes, rows=rows, mode=2, nthreads=16)
    assert np.array_equal(t.latency_ns[rows], lat)
    assert bits_equal(t.packet_loss[rows], loss)
    assert np.array_equal(np.diag(t.latency_ns), e.latency_ns[:4096])
    off = ~np.eye(4096, dtype=bool)
    assert np.array_equal(t.latency_ns[off], t.latency_ns.T[off])


@pytest.mark.parametrize("kind", ["dense", "parallel", "u64", "sparse"])
def test_late_loss_matches_with_loss(router, kind):
    """Host entry with SRG_OPT_LATE_LOSS (the losses cross PCIe after the endpoints/latencies,
    beside the W build and FW; WL and the self-loop losses are built once they land) gives the
    bytes of the in-line transfer, on the dense u32 path (WL on the loss stream), with parallel
    edges (min loss among the min-latency ones), on the u64 rerun after a failed u32
    certification, and on the sparse path; oracle rows pin them."""
    V = 1500  # >= 2^20 edges: the codec (and so the late loss) is active
    if kind == "dense" or kind == "sparse":
        g = synth.atlas_like(V, seed=37)
    elif kind == "parallel":
        g = synth.random_graph(V, 0.9, 38, lat_lo=1, lat_hi=40, parallel=0.2)
    else:  # latencies in [2^31, 2^32): u32 keys first, certification fails, u64 rerun
        g = synth.random_graph(V, 0.95, 39, lat_lo=2 ** 31, lat_hi=2 ** 32 - 2)
    assert g.num_edges >= 1 << 20
    nodes = list(range(0, V, 3))
    if kind == "sparse":
        router.set_option(N.SRG_OPT_ALGORITHM, N.SRG_ALGO_SPARSE)
    out = {}
    try:
        for late in (0, 1):
            router.set_option(N.SRG_OPT_LATE_LOSS, late)
            out[late] = router.compute_shortest_paths(g, nodes)
    finally:
        router.set_option(N.SRG_OPT_LATE_LOSS, 1)
        router.set_option(N.SRG_OPT_ALGORITHM, N.SRG_ALGO_AUTO)
    want = {"dense": N.SRG_PATH_DENSE_U32, "parallel": N.SRG_PATH_DENSE_U32, "u64": N.SRG_PATH_DENSE_U64,
            "sparse": N.SRG_PATH_SPARSE_U32}[kind]
    assert out[1].stats["path_kind"] == want
    assert np.array_equal(out[0].latency_ns, out[1].latency_ns)
    assert bits_equal(out[0].packet_loss, out[1].packet_loss)
    rows = [0, 1, len(nodes) - 1]
    lat, loss = oracle.compute_shortest_paths(g.as_tuple(), nodes, rows=rows, mode=2, nthreads=8)
    assert np.array_equal(out[1].latency_ns[rows], lat) and bits_equal(out[1].packet_loss[rows], loss)


@pytest.mark.parametrize("entry", ["host", "device"])
def test_multi_pred_pairs_count(router, entry):
    """stats.multi_pred_pairs (counted by k_pred_pack on the per-row loss path) equals the number of
    used pairs (s, t), s != t, with two or more latency-tight essential in-edges, counted here from
    the oracle's latencies (ties forced by a 1..3 latency range)."""
    V = 300
    g = synth.random_graph(V, 0.05, 231, lat_hi=3, parallel=0.2)
    nodes = list(range(V))
    lat, _ = oracle.compute_shortest_paths(g.as_tuple(), nodes)
    D = lat.astype(np.int64)
    np.fill_diagonal(D, 0)
    W = np.full((V, V), np.iinfo(np.int64).max // 4, dtype=np.int64)
    m = g.src != g.dst
    s_, d_, w_ = g.src[m].astype(np.int64), g.dst[m].astype(np.int64), g.latency_ns[m].astype(np.int64)
    np.minimum.at(W, (s_, d_), w_)
    np.minimum.at(W, (d_, s_), w_)
    ess = W == D  # (u, t) essential: the edge is itself a shortest path
    expect = 0
    for s in range(V):
        tight = (D[s][:, None] + W == D[s][None, :]) & ess  # [u, t]
        cnt = tight.sum(axis=0)
        cnt[s] = 0
        expect += int((cnt >= 2).sum())
    if entry == "host":
        t = router.compute_shortest_paths(g, nodes)
        st = t.stats
    else:
        import torch
        from shadow_amd.device import DeviceGraph, compute_shortest_paths_device
        dev = torch.device("cuda", 0)
        ol = torch.empty((V, V), dtype=torch.int64, device=dev)
        os_ = torch.empty((V, V), dtype=torch.float32, device=dev)
        st = compute_shortest_paths_device(router, DeviceGraph(g), torch.arange(V, dtype=torch.int32, device=dev), ol, os_)
    assert st["scan_kind"] == N.SRG_SCAN_SPARSE
    assert expect > 0 and st["multi_pred_pairs"] == expect
