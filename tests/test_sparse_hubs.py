"""Sparse path with hub bounds (SRG_OPT_SPARSE_HUBS): the batches start from upper bounds through
the exact rows of the highest-degree vertices instead of INF; the fixpoint, and so every output
byte, must be the same as the oracle's (sparse.hip.h, k_hub_sweep / k_hub_ub)."""
import threading

import numpy as np
import pytest

import oracle
from shadow_amd import LocalGroup, NetGraphError, Router, RoutingPanic, synth
from shadow_amd import _native as N
from shadow_amd.graph import Edges
from helpers import bits_equal

pytestmark = pytest.mark.gpu


def hub_router(hubs, **opts):
    r = Router(0)
    r.set_option(N.SRG_OPT_ALGORITHM, N.SRG_ALGO_SPARSE)
    r.set_option(N.SRG_OPT_SPARSE_HUBS, hubs)
    for k, v in opts.items():
        r.set_option(getattr(N, "SRG_OPT_" + k), v)
    return r


def test_hub_option_validation():
    r = Router(0)
    for bad in (-128, 64, 100, 640):
        with pytest.raises(Exception):
            r.set_option(N.SRG_OPT_SPARSE_HUBS, bad)
    for ok in (0, 128, 256, 384, 512):
        r.set_option(N.SRG_OPT_SPARSE_HUBS, ok)
        assert r.get_option(N.SRG_OPT_SPARSE_HUBS) == ok
    r.close()


CASES = [
    dict(V=300, density=0.02, seed=206, lat_hi=50),
    dict(V=1000, density=0.004, seed=207, lat_hi=100),
    dict(V=1000, density=0.01, seed=211, lat_hi=3, parallel=0.3),
    dict(V=700, density=0.01, seed=212, lat_hi=1000, loss_hi=1e-6),
]


@pytest.mark.parametrize("hubs", [128, 256])
@pytest.mark.parametrize("kw", CASES, ids=lambda k: f"V{k['V']}_s{k['seed']}")
def test_hubs_random_vs_oracle(kw, hubs):
    kw = dict(kw)
    V, dens, seed = kw.pop("V"), kw.pop("density"), kw.pop("seed")
    g = synth.random_graph(V, dens, seed, **kw)
    nodes = list(range(V))
    r = hub_router(hubs)
    try:
        lat, loss = oracle.compute_shortest_paths(g.as_tuple(), nodes)
    except oracle.OracleError as e:
        with pytest.raises(NetGraphError) as ei:
            r.compute_shortest_paths(g, nodes)
        assert ei.value.code == e.code
        r.close()
        return
    t = r.compute_shortest_paths(g, nodes)
    assert t.stats["path_kind"] == N.SRG_PATH_SPARSE_U32
    assert t.stats["sparse_hubs"] == (hubs if V >= 2 * hubs else 0)
    assert np.array_equal(t.latency_ns, lat)
    assert bits_equal(t.packet_loss, loss)
    r.close()


@pytest.mark.parametrize("opts", [{}, {"SPARSE_DELTA_DIV": 8}, {"SPARSE_DELTA_DIV": 0}, {"SPARSE_GLOBAL_BITMAPS": 1}],
                         ids=["default", "delta8", "plain_bf", "global_bitmaps"])
@pytest.mark.parametrize("hubs", [128, 512])
def test_hubs_ba_sampled(hubs, opts):
    """C4's shape (Barabasi-Albert, m = 4), every node used, with buckets / plain BF / global bitmaps:
    seeded oracle rows, symmetric latency, the self-loop diagonal."""
    V = 4000
    e = synth.barabasi_albert(V, 4, seed=V + 3)
    r = hub_router(hubs, **opts)
    nodes = list(range(V))
    t = r.compute_shortest_paths(e, nodes)
    assert t.stats["path_kind"] == N.SRG_PATH_SPARSE_U32 and t.stats["sparse_hubs"] == hubs
    rows = np.random.default_rng(V).choice(V, 16, replace=False).tolist()
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), nodes, rows=rows, nthreads=16)
    assert np.array_equal(t.latency_ns[rows], lat) and bits_equal(t.packet_loss[rows], loss)
    off = ~np.eye(V, dtype=bool)
    assert np.array_equal(t.latency_ns[off], t.latency_ns.T[off])
    assert np.array_equal(np.diag(t.latency_ns), np.full(V, 1_000_000, dtype=np.uint64))
    r.close()


def test_hubs_match_no_hubs_bytes():
    """The same BA graph with and without hubs: every output byte equal (the fixpoint is unique)."""
    V = 3000
    e = synth.barabasi_albert(V, 3, seed=99)
    nodes = list(range(V))
    r0, r1 = hub_router(0), hub_router(256)
    t0 = r0.compute_shortest_paths(e, nodes)
    t1 = r1.compute_shortest_paths(e, nodes)
    assert t0.stats["sparse_hubs"] == 0 and t1.stats["sparse_hubs"] == 256
    assert np.array_equal(t0.latency_ns, t1.latency_ns) and bits_equal(t0.packet_loss, t1.packet_loss)
    r0.close()
    r1.close()


def test_hubs_subset_scrambled():
    """A scrambled subset of used nodes (batch lanes = used sources in locality order, padded)."""
    g = synth.barabasi_albert(1200, 3, seed=213)
    nodes = np.random.default_rng(4).permutation(1200)[:333].tolist()
    r = hub_router(128)
    lat, loss = oracle.compute_shortest_paths(g.as_tuple(), nodes)
    t = r.compute_shortest_paths(g, nodes)
    assert t.stats["sparse_hubs"] == 128
    assert np.array_equal(t.latency_ns, lat) and bits_equal(t.packet_loss, loss)
    r.close()


def test_hubs_directed_and_large_keys_skip():
    """Hubs apply to undirected u32 builds only: a directed graph and one with arcs >= 2^31 units run
    without them (and stay exact)."""
    r = hub_router(128)
    for g in (synth.random_graph(600, 0.03, 214, directed=True, lat_hi=100),
              synth.random_graph(400, 0.05, 215, lat_lo=2**31 + 1, lat_hi=2**31 + 1000)):
        nodes = list(range(g.num_vertices))
        try:
            lat, loss = oracle.compute_shortest_paths(g.as_tuple(), nodes)
        except oracle.OracleError as e:
            with pytest.raises(NetGraphError) as ei:
                r.compute_shortest_paths(g, nodes)
            assert ei.value.code == e.code
            continue
        t = r.compute_shortest_paths(g, nodes)
        assert t.stats["sparse_hubs"] == 0
        assert np.array_equal(t.latency_ns, lat) and bits_equal(t.packet_loss, loss)
    r.close()


def test_hubs_disconnected():
    """Two components: hub rows stay HUB_INF across them (no bound), used nodes in one component are
    exact, a used pair across them is the reference's panic."""
    a = synth.barabasi_albert(1500, 3, seed=5)
    V = 3000
    src = np.r_[a.src, a.src + 1500]
    dst = np.r_[a.dst, a.dst + 1500]
    e = Edges(V, src, dst, np.r_[a.latency_ns, a.latency_ns], np.r_[a.packet_loss, a.packet_loss], False)
    r = hub_router(256)
    with pytest.raises(RoutingPanic):
        r.compute_shortest_paths(e, [0, 1, 1500])
    nodes = list(range(1500, 3000))
    t = r.compute_shortest_paths(e, nodes)
    assert t.stats["sparse_hubs"] == 256
    rows = [0, 700, 1499]
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), nodes, rows=rows, nthreads=16)
    assert np.array_equal(t.latency_ns[rows], lat) and bits_equal(t.packet_loss[rows], loss)
    r.close()


@pytest.mark.parametrize("G", [2, 3])
def test_hubs_multi_rank(G):
    """Sources sharded over in-process ranks, each with its own bound rows: bit-exact vs the oracle."""
    e = synth.barabasi_albert(2500, 3, seed=78)
    nodes = np.random.default_rng(6).permutation(2500)[:900].tolist()
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), nodes, nthreads=16)
    group = LocalGroup(G)
    routers = [hub_router(128) for _ in range(G)]
    out = [None] * G
    for i, rt in enumerate(routers):
        rt.init_comm_local(group, i)

    def work(i):
        out[i] = routers[i].compute_shortest_paths(e, nodes)

    th = [threading.Thread(target=work, args=(i,)) for i in range(G)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=300)
    for t in out:
        assert t is not None and t.stats["sparse_hubs"] == 128
        assert np.array_equal(t.latency_ns, lat) and bits_equal(t.packet_loss, loss)
    for rt in routers:
        rt.close()
