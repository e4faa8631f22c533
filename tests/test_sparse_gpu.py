"""GPU parity of the sparse path (batched lexicographic Bellman-Ford, sparse.hip.h) against the
oracle: latency bit-exact, packet_loss bit-exact (the north star allows 1e-6 relative; the
lexicographic fixpoint is unique, so bits must match).  Forced on small random graphs (ties,
parallel edges, directed, tiny losses) and auto-selected on Barabasi-Albert graphs (C4 shape)."""
import threading

import numpy as np
import pytest

import oracle
from shadow_amd import LocalGroup, NetGraphError, Router, RoutingPanic, synth
from shadow_amd import _native as N
from shadow_amd.graph import Edges
from helpers import bits_equal

pytestmark = pytest.mark.gpu


@pytest.fixture
def bf_router():
    r = Router(0)
    r.set_option(N.SRG_OPT_ALGORITHM, N.SRG_ALGO_SPARSE)
    yield r
    r.close()


CASES = [
    dict(V=50, density=0.2, seed=201, lat_hi=8),
    dict(V=129, density=0.1, seed=202, directed=True, lat_hi=1000),
    dict(V=130, density=0.3, seed=203, lat_hi=3, parallel=0.3),
    dict(V=200, density=0.05, seed=204, directed=True, lat_hi=20, loss_hi=1e-6),
    dict(V=300, density=0.02, seed=206, lat_hi=50),
    dict(V=1000, density=0.004, seed=207, lat_hi=100),
]


@pytest.mark.parametrize("kw", CASES, ids=lambda k: f"V{k['V']}_s{k['seed']}")
def test_bf_random_vs_oracle(bf_router, kw):
    kw = dict(kw)
    V, dens, seed = kw.pop("V"), kw.pop("density"), kw.pop("seed")
    g = synth.random_graph(V, dens, seed, **kw)
    nodes = list(range(V))
    try:
        lat, loss = oracle.compute_shortest_paths(g.as_tuple(), nodes)
    except oracle.OracleError as e:
        with pytest.raises(NetGraphError) as ei:
            bf_router.compute_shortest_paths(g, nodes)
        assert ei.value.code == e.code
        return
    t = bf_router.compute_shortest_paths(g, nodes)
    assert t.stats["path_kind"] == N.SRG_PATH_SPARSE_U32
    assert np.array_equal(t.latency_ns, lat)
    assert bits_equal(t.packet_loss, loss)


@pytest.mark.parametrize("div", [1, 4, 16, 1000])
@pytest.mark.parametrize("kw", [CASES[1], CASES[2], CASES[3], dict(V=1000, density=0.01, seed=207, lat_hi=100, parallel=0.1)],
                         ids=lambda k: f"V{k['V']}_s{k['seed']}")
def test_bf_delta_buckets(bf_router, kw, div):
    """Delta-stepping buckets (deferred pushes) reach the same fixpoint bit for bit."""
    bf_router.set_option(N.SRG_OPT_SPARSE_DELTA_DIV, div)
    kw = dict(kw)
    V, dens, seed = kw.pop("V"), kw.pop("density"), kw.pop("seed")
    g = synth.random_graph(V, dens, seed, **kw)
    nodes = list(range(V))
    lat, loss = oracle.compute_shortest_paths(g.as_tuple(), nodes)
    t = bf_router.compute_shortest_paths(g, nodes)
    assert t.stats["path_kind"] == N.SRG_PATH_SPARSE_U32
    assert np.array_equal(t.latency_ns, lat) and bits_equal(t.packet_loss, loss)


@pytest.mark.parametrize("kw", [CASES[1], CASES[2], CASES[3], CASES[5]], ids=lambda k: f"V{k['V']}_s{k['seed']}")
def test_bf_global_bitmaps(bf_router, kw):
    """Vertex bitmaps in global memory (the layout for V beyond the LDS budget) are bit-exact."""
    bf_router.set_option(N.SRG_OPT_SPARSE_GLOBAL_BITMAPS, 1)
    kw = dict(kw)
    V, dens, seed = kw.pop("V"), kw.pop("density"), kw.pop("seed")
    g = synth.random_graph(V, dens, seed, **kw)
    nodes = list(range(V))
    try:
        lat, loss = oracle.compute_shortest_paths(g.as_tuple(), nodes)
    except oracle.OracleError as e:
        with pytest.raises(NetGraphError) as ei:
            bf_router.compute_shortest_paths(g, nodes)
        assert ei.value.code == e.code
        return
    t = bf_router.compute_shortest_paths(g, nodes)
    assert t.stats["path_kind"] == N.SRG_PATH_SPARSE_U32
    assert np.array_equal(t.latency_ns, lat) and bits_equal(t.packet_loss, loss)


def test_bf_unreachable_ms_latencies_no_fallback(bf_router):
    """an unreachable used pair with ms-scale latencies (max_lat * (V-1) >> 2^32) is the
    reference's panic straight from the sparse path (no saturated relaxation happened); an
    isolated UNUSED vertex does not disturb the sparse u32 result."""
    e = synth.barabasi_albert(3000, 4, seed=41)
    V = e.num_vertices + 1  # vertex 3000: isolated, only its self-loop
    iso = Edges(V, np.r_[e.src, V - 1], np.r_[e.dst, V - 1], np.r_[e.latency_ns, 1_000_000],
                np.r_[e.packet_loss, 0.0], False)
    with pytest.raises(RoutingPanic):
        bf_router.compute_shortest_paths(iso, list(range(V)))
    nodes = list(range(V - 1))
    t = bf_router.compute_shortest_paths(iso, nodes)
    assert t.stats["path_kind"] == N.SRG_PATH_SPARSE_U32
    rows = [0, 1234, 2999]
    lat, loss = oracle.compute_shortest_paths(iso.as_tuple(), nodes, rows=rows, nthreads=16)
    assert np.array_equal(t.latency_ns[rows], lat) and bits_equal(t.packet_loss[rows], loss)


def test_bf_delta_ba_sampled(bf_router):
    e = synth.barabasi_albert(3000, 4, seed=31)
    bf_router.set_option(N.SRG_OPT_SPARSE_DELTA_DIV, 8)
    nodes = list(range(3000))
    t = bf_router.compute_shortest_paths(e, nodes)
    rows = np.random.default_rng(31).choice(3000, 16, replace=False).tolist()
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), nodes, rows=rows, nthreads=16)
    assert np.array_equal(t.latency_ns[rows], lat) and bits_equal(t.packet_loss[rows], loss)


def test_bf_subset_scrambled(bf_router):
    g = synth.random_graph(400, 0.02, 208, lat_hi=60)
    nodes = np.random.default_rng(3).permutation(400)[:130].tolist()
    lat, loss = oracle.compute_shortest_paths(g.as_tuple(), nodes)
    t = bf_router.compute_shortest_paths(g, nodes)
    assert np.array_equal(t.latency_ns, lat) and bits_equal(t.packet_loss, loss)


def test_bf_unreachable_panics(bf_router):
    iso = Edges(4, [0, 1, 2, 3, 0], [0, 1, 2, 3, 1], [1, 1, 1, 1, 3], [0.0] * 5, False)
    with pytest.raises(RoutingPanic):
        bf_router.compute_shortest_paths(iso, [0, 1, 2, 3])
    t = bf_router.compute_shortest_paths(iso, [0, 1])
    assert t[(0, 1)].latency_ns == 3


def test_bf_large_latency_takes_wide_labels(bf_router):
    """Latencies whose sums pass 2^32: saturated u32 keys hand over to the wide (u64-key) labels."""
    g = synth.random_graph(120, 0.05, 209, lat_lo=2**30, lat_hi=2**31)
    nodes = list(range(120))
    lat, loss = oracle.compute_shortest_paths(g.as_tuple(), nodes)
    t = bf_router.compute_shortest_paths(g, nodes)
    assert t.stats["path_kind"] == N.SRG_PATH_SPARSE_U64
    assert int(lat.max()) >= 2 ** 32
    assert np.array_equal(t.latency_ns, lat) and bits_equal(t.packet_loss, loss)


@pytest.mark.parametrize("case", ["arcs_past_u32", "paths_past_u32", "delta"])
def test_ba_wide_labels(case):
    """A Barabasi-Albert graph with nanosecond latencies (unit 1) whose used paths pass 2^32 ns stays
    on the sparse path with u64 latency keys (SRG_PATH_SPARSE_U64): seeded oracle rows, symmetry,
    diagonal.  arcs_past_u32: single arcs above 2^32 (the u32 pass is skipped); paths_past_u32: arcs
    below 2^32, paths above (the u32 pass saturates and reruns wide); delta: with buckets."""
    V = 6000
    e0 = synth.barabasi_albert(V, 4, seed=V + 7)
    rng = np.random.default_rng(V)
    if case == "arcs_past_u32":
        lat = rng.integers(2 ** 32, 2 ** 34, size=len(e0.src), dtype=np.uint64) | np.uint64(1)
    else:
        lat = rng.integers(2 ** 29, 2 ** 31, size=len(e0.src), dtype=np.uint64) | np.uint64(1)
    lat[e0.src == e0.dst] = e0.latency_ns[e0.src == e0.dst]
    e = Edges(V, e0.src, e0.dst, lat, e0.packet_loss, directed=False)
    r = Router(0)
    if case == "delta":
        r.set_option(N.SRG_OPT_SPARSE_DELTA_DIV, 8)
    nodes = list(range(V))
    t = r.compute_shortest_paths(e, nodes)
    assert t.stats["path_kind"] == N.SRG_PATH_SPARSE_U64 and t.stats["latency_unit_ns"] == 1
    assert int(t.latency_ns.max()) >= 2 ** 32
    rows = rng.choice(V, 8, replace=False).tolist()
    rl, rs = oracle.compute_shortest_paths(e.as_tuple(), nodes, rows=rows, nthreads=16)
    assert np.array_equal(t.latency_ns[rows], rl) and bits_equal(t.packet_loss[rows], rs)
    off = ~np.eye(V, dtype=bool)
    assert np.array_equal(t.latency_ns[off], t.latency_ns.T[off])
    r.close()


@pytest.mark.parametrize("V", [3000, 12000])
def test_ba_auto_sparse_sampled(V):
    """C4 shape (Barabasi-Albert m=4): auto-dispatch picks the sparse path; full matrix vs
    seeded oracle rows, plus symmetric latency and the self-loop diagonal."""
    e = synth.barabasi_albert(V, 4, seed=V)
    r = Router(0)
    nodes = list(range(V))
    t = r.compute_shortest_paths(e, nodes)
    assert t.stats["path_kind"] == N.SRG_PATH_SPARSE_U32
    rows = np.random.default_rng(V).choice(V, 16, replace=False).tolist()
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), nodes, rows=rows, nthreads=16)
    assert np.array_equal(t.latency_ns[rows], lat)
    assert bits_equal(t.packet_loss[rows], loss)
    assert np.array_equal(np.diag(t.latency_ns), np.full(V, 1_000_000, dtype=np.uint64))
    off = ~np.eye(V, dtype=bool)
    assert np.array_equal(t.latency_ns[off], t.latency_ns.T[off])
    r.close()


@pytest.mark.slow
def test_c4_full_size_sampled_rows():
    """Config C4 at full size (barabasi_albert(50000, 4, seed=50000), all 50 000 nodes used; the
    2.5e9-pair table stays in HBM) through the device entry: 512 seeded oracle rows bit-exact
    (SURVEY §8d's gate),
    plus whole-table properties computed on the device: diagonal = the self-loops, symmetric
    latency, latency <= the direct edge on every arc, the Bellman inequality
    D[s][t] <= D[s][u] + w(u,t) over every source for 256 sampled arcs, loss in [0, 1]."""
    import torch
    from shadow_amd.device import DeviceGraph, compute_shortest_paths_device
    V = 50000
    dev = torch.device("cuda", 0)
    e = synth.barabasi_albert(V, 4, seed=V)
    dg = DeviceGraph(e)
    nodes_t = torch.arange(V, dtype=torch.int32, device=dev)
    ol = torch.empty((V, V), dtype=torch.int64, device=dev)
    os_ = torch.empty((V, V), dtype=torch.float32, device=dev)
    r = Router(0)
    st = compute_shortest_paths_device(r, dg, nodes_t, ol, os_)
    torch.cuda.synchronize()
    assert st["path_kind"] == N.SRG_PATH_SPARSE_U32
    rows = np.random.default_rng(V).choice(V, 512, replace=False)
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), list(range(V)), rows=rows.tolist(), nthreads=16)
    ri = torch.from_numpy(rows.astype(np.int64)).to(dev)
    assert np.array_equal(ol[ri].cpu().numpy().view(np.uint64), lat)
    assert bits_equal(os_[ri].cpu().numpy(), loss)
    idx = torch.arange(V, device=dev)
    assert bool((ol[idx, idx] == 1_000_000).all())
    B = 4096
    for i0 in range(0, V, B):
        i1 = min(V, i0 + B)
        assert torch.equal(ol[i0:i1], ol[:, i0:i1].t().contiguous()), f"latency not symmetric in rows {i0}:{i1}"
    m = e.src != e.dst
    s_ = torch.from_numpy(e.src[m].astype(np.int64)).to(dev)
    t_ = torch.from_numpy(e.dst[m].astype(np.int64)).to(dev)
    w_ = torch.from_numpy(e.latency_ns[m].view(np.int64)).to(dev)
    assert bool((ol[s_, t_] <= w_).all()) and bool((ol[t_, s_] <= w_).all())
    pick = torch.from_numpy(np.random.default_rng(1).choice(int(m.sum()), 256, replace=False)).to(dev)
    for k in pick.tolist():
        u, t, w = int(s_[k]), int(t_[k]), int(w_[k])
        col_t, col_u = ol[:, t].clone(), ol[:, u].clone()
        col_t[t] = 0  # the diagonal holds the self-loop, the Bellman inequality uses D[t][t] = 0
        col_u[u] = 0
        assert bool((col_t <= col_u + w).all()) and bool((col_u <= col_t + w).all())
    assert float(os_.min()) >= 0.0 and float(os_.max()) <= 1.0
    del ol, os_
    r.close()


@pytest.mark.parametrize("G", [2, 3])
def test_bf_multi_rank(G):
    e = synth.barabasi_albert(2500, 3, seed=77)
    nodes = np.random.default_rng(5).permutation(2500)[:900].tolist()
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), nodes, nthreads=16)
    group = LocalGroup(G)
    routers = [Router(0) for _ in range(G)]
    out = [None] * G
    for i, rt in enumerate(routers):
        rt.set_option(N.SRG_OPT_ALGORITHM, N.SRG_ALGO_SPARSE)
        rt.init_comm_local(group, i)

    def work(i):
        out[i] = routers[i].compute_shortest_paths(e, nodes)

    th = [threading.Thread(target=work, args=(i,)) for i in range(G)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=300)
    for i, t in enumerate(out):
        assert t is not None, f"rank {i} failed"
        assert np.array_equal(t.latency_ns, lat) and bits_equal(t.packet_loss, loss)
    for rt in routers:
        rt.close()
    group.close()
