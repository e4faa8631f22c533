"""Multi-rank routing build on ONE GPU: G ranks as threads of this process
attached to an in-process LocalGroup, each with its own context and full workspace.  Every
rank must end with exactly the single-GPU result (bit-exact latency and loss), for sorted,
scrambled and subset node lists, u32 and u64 keys, and with the output exchange off."""
import threading

import numpy as np
import pytest

import oracle
from shadow_amd import LocalGroup, MultiRouter, NetGraphError, Router, RoutingPanic, generate_routing_info, synth
from shadow_amd import _native as N
from helpers import bits_equal

pytestmark = pytest.mark.gpu


def run_ranks(G, edges, nodes, gather=True, threshold=None, shard=None):
    group = LocalGroup(G)
    routers = [Router(0) for _ in range(G)]
    for r, rt in enumerate(routers):
        rt.init_comm_local(group, r)
        assert rt.comm_size() == (G, r)
        if not gather:
            rt.set_option(N.SRG_OPT_GATHER_OUTPUT, 0)
        if threshold is not None:
            rt.set_option(N.SRG_OPT_SPARSE_THRESHOLD, threshold)
        if shard is not None:
            rt.set_option(N.SRG_OPT_EDGE_SHARD, shard)
    out, errs = [None] * G, [None] * G

    def work(r):
        try:
            out[r] = routers[r].compute_shortest_paths(edges, nodes)
        except Exception as e:  # noqa: BLE001
            errs[r] = e

    th = [threading.Thread(target=work, args=(r,)) for r in range(G)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    for rt in routers:
        rt.close()
    group.close()
    return out, errs


CASES = [
    dict(G=2, V=300, dens=0.05, seed=1, nodes="all"),
    dict(G=3, V=520, dens=0.02, seed=2, nodes="scrambled"),
    dict(G=4, V=700, dens=0.03, seed=3, nodes="subset"),
    dict(G=8, V=900, dens=0.01, seed=4, nodes="all"),
    dict(G=4, V=260, dens=0.2, seed=5, nodes="all", lat_lo=2**31, lat_hi=2**33),  # u64 keys
    dict(G=2, V=130, dens=0.3, seed=6, nodes="scrambled", threshold=0.0),        # dense scan
    dict(G=4, V=260, dens=0.2, seed=7, nodes="all", lat_lo=2**31, lat_hi=2**33, ms=True),  # latency unit
]


def node_list(kind, V, seed):
    rng = np.random.default_rng(seed)
    if kind == "all":
        return list(range(V))
    if kind == "scrambled":
        return rng.permutation(V).tolist()
    return sorted(rng.choice(V, size=V // 3, replace=False).tolist())


@pytest.mark.parametrize("c", CASES, ids=lambda c: f"G{c['G']}_V{c['V']}_{c['nodes']}")
def test_ranks_match_single_gpu(c):
    kw = {k: c[k] for k in ("lat_lo", "lat_hi") if k in c}
    e = synth.random_graph(c["V"], c["dens"], c["seed"], **kw)
    if c.get("ms"):  # millisecond multiples: u32 keys in units of the latencies' gcd on every rank
        e.latency_ns = e.latency_ns // np.uint64(10**6) * np.uint64(10**6)
    nodes = node_list(c["nodes"], c["V"], c["seed"])
    ref_router = Router(0)
    if c.get("threshold") is not None:
        ref_router.set_option(N.SRG_OPT_SPARSE_THRESHOLD, c["threshold"])
    ref = ref_router.compute_shortest_paths(e, nodes)
    ref_router.close()
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), nodes)
    assert np.array_equal(ref.latency_ns, lat) and bits_equal(ref.packet_loss, loss)
    out, errs = run_ranks(c["G"], e, nodes, threshold=c.get("threshold"))
    assert errs == [None] * c["G"], errs
    for r, t in enumerate(out):
        assert t.stats["nranks"] == c["G"] and t.stats["rank"] == r
        assert t.stats["path_kind"] == ref.stats["path_kind"]
        assert t.stats["latency_unit_ns"] == ref.stats["latency_unit_ns"]
        assert np.array_equal(t.latency_ns, lat), f"rank {r} latency"
        assert bits_equal(t.packet_loss, loss), f"rank {r} loss"
    assert sum(t.stats["local_sources"] for t in out) == len(nodes)


@pytest.mark.parametrize("kind", ["scrambled", "all"])
def test_ranks_without_exchange_fill_own_rows(kind):
    """Output exchange off: rank r routes the sources at positions [n r / G, n (r+1) / G) of the
    node list, whatever their order, and fills exactly those output rows; its min_latency_ns is the
    minimum over those rows only (RoutingInfo::get_smallest_latency_ns, mod.rs:474-476)."""
    e = synth.random_graph(400, 0.04, 11)
    nodes = node_list(kind, 400, 11)
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), nodes)
    out, errs = run_ranks(3, e, nodes, gather=False)
    assert errs == [None] * 3
    covered = np.zeros(len(nodes), dtype=bool)
    n = len(nodes)
    for r, t in enumerate(out):
        rows = list(range(n * r // 3, n * (r + 1) // 3))
        assert t.stats["local_sources"] == len(rows)
        assert np.array_equal(t.latency_ns[rows], lat[rows])
        assert bits_equal(t.packet_loss[rows], loss[rows])
        assert t.stats["min_latency_ns"] == int(lat[rows].min())
        covered[rows] = True
    assert covered.all()


def test_ranks_without_exchange_own_rows_page_locked():
    """Output exchange off with a table past the early-D2H threshold (n^2 x 12 B >= 64 MB): each
    rank page-locks only its own rows [n r / G, n (r+1) / G) of the caller's table and ships them
    while later kernels run (SDMA into the mapped rows); the rows equal the single-GPU table's."""
    V = 2400
    e = synth.atlas_like(V, seed=2400)
    nodes = node_list("scrambled", V, 12)
    ref_router = Router(0)
    ref = ref_router.compute_shortest_paths(e, nodes)
    ref_router.close()
    G = 3
    out, errs = run_ranks(G, e, nodes, gather=False)
    assert errs == [None] * G, errs
    n = len(nodes)
    for r, t in enumerate(out):
        rows = list(range(n * r // G, n * (r + 1) // G))
        assert np.array_equal(t.latency_ns[rows], ref.latency_ns[rows]), f"rank {r}"
        assert bits_equal(t.packet_loss[rows], ref.packet_loss[rows]), f"rank {r}"
        assert t.stats["d2h_overlapped_bytes"] == len(rows) * n * 12, f"rank {r}"
    rows = [0, n // 2, n - 1]
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), nodes, rows=rows, mode=2, nthreads=8)
    assert np.array_equal(ref.latency_ns[rows], lat) and bits_equal(ref.packet_loss[rows], loss)


def test_ranks_without_exchange_more_ranks_than_nodes():
    """n < G: some ranks own no source; they ship nothing and report no minimum."""
    e = synth.random_graph(150, 0.06, 14)
    nodes = [3, 77, 140]
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), nodes)
    out, errs = run_ranks(5, e, nodes, gather=False)
    assert errs == [None] * 5, errs
    for r, t in enumerate(out):
        rows = list(range(3 * r // 5, 3 * (r + 1) // 5))
        assert t.stats["local_sources"] == len(rows)
        if rows:
            assert np.array_equal(t.latency_ns[rows], lat[rows]) and bits_equal(t.packet_loss[rows], loss[rows])
            assert t.stats["min_latency_ns"] == int(lat[rows].min())
        else:
            assert t.stats["min_latency_ns"] == 2 ** 64 - 1


@pytest.mark.parametrize("G,shard", [(2, 1), (3, 1), (4, 0), (8, 1)])
def test_edge_sharded_host_entry(G, shard):
    """SRG_OPT_EDGE_SHARD: each rank ships only its 1/G slice of the edge list and the slices are
    exchanged between the ranks (default on from 4 ranks); every rank still gets the oracle's
    table.  E is not a multiple of G, so the slices are ragged."""
    e = synth.random_graph(350, 0.07, 20 + G, parallel=0.1)
    assert e.num_edges % G
    nodes = node_list("scrambled", 350, 20 + G)
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), nodes)
    out, errs = run_ranks(G, e, nodes, shard=shard)
    assert errs == [None] * G, errs
    for r, t in enumerate(out):
        assert np.array_equal(t.latency_ns, lat), f"rank {r} latency"
        assert bits_equal(t.packet_loss, loss), f"rank {r} loss"


@pytest.mark.parametrize("G,V,order", [(2, 2100, "rows"), (4, 3000, "rows"), (2, 2100, "shuffled")])
def test_edge_sharded_codec_slices(G, V, order):
    """Edge sharding with the H2D codec active on every rank's slice (>= 2^20 edges per slice): a
    row-ordered list crosses and is exchanged in the sequential-pair form (u32 latencies + row-start
    exceptions, decoded on every rank), a shuffled one in the u16 narrowing; both equal the
    single-GPU build."""
    e = synth.atlas_like(V, seed=V)
    if order == "shuffled":
        from shadow_amd.graph import Edges
        p = np.random.default_rng(V).permutation(e.num_edges)
        e = Edges(V, e.src[p], e.dst[p], e.latency_ns[p], e.packet_loss[p], False)
    assert e.num_edges >= G * (1 << 20) + 2
    nodes = list(range(0, V, 7))
    r1 = Router(0)
    ref = r1.compute_shortest_paths(e, nodes)
    r1.close()
    out, errs = run_ranks(G, e, nodes, shard=1)
    assert errs == [None] * G, errs
    for r, t in enumerate(out):
        assert np.array_equal(t.latency_ns, ref.latency_ns), f"rank {r} latency"
        assert bits_equal(t.packet_loss, ref.packet_loss), f"rank {r} loss"


def test_edge_sharded_bad_edge_on_one_slice():
    """An out-of-range endpoint in the last rank's slice: every rank reports the reference's
    error (the checks run on the exchanged whole list), none hangs."""
    from shadow_amd.graph import Edges
    g = synth.random_graph(200, 0.05, 21)
    dst = g.dst.copy()
    dst[-1] = 200  # only rank G-1 ships it
    e = Edges(200, g.src, dst, g.latency_ns, g.packet_loss, False)
    single = Router(0)
    with pytest.raises(NetGraphError) as ref:
        single.compute_shortest_paths(e, list(range(200)))
    single.close()
    out, errs = run_ranks(4, e, list(range(200)), shard=1)
    assert all(isinstance(x, NetGraphError) and x.code == ref.value.code for x in errs), errs


def test_ranks_agree_on_errors():
    """A panic-class error detected on one rank must surface on every rank (no hang)."""
    iso = synth.random_graph(300, 0.05, 12)
    # vertex 299 isolated: drop its edges except the self-loop
    keep = ((iso.src != 299) & (iso.dst != 299)) | (iso.src == iso.dst)
    from shadow_amd.graph import Edges
    e = Edges(300, iso.src[keep], iso.dst[keep], iso.latency_ns[keep], iso.packet_loss[keep], False)
    out, errs = run_ranks(3, e, list(range(300)))
    assert all(isinstance(x, RoutingPanic) for x in errs), errs


def test_rccl_single_rank():
    """RCCL backend bring-up on one GPU (nranks = 1): loads librccl, inits, computes."""
    e = synth.random_graph(200, 0.05, 13)
    r = Router(0)
    r.init_comm(1, 0, Router.comm_unique_id())
    assert r.comm_size() == (1, 0)
    t = r.compute_shortest_paths(e, list(range(200)))
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), list(range(200)))
    assert np.array_equal(t.latency_ns, lat) and bits_equal(t.packet_loss, loss)
    r.close()


@pytest.fixture(scope="module")
def c3_single():
    """Config C3 (atlas_like(10000, seed=10000)) built by one rank through the host entry exactly as
    the bench times it (edge list in host memory, FW beside the H2D, 1.2 GB table back): the
    reference table of the multi-rank tests, pinned to the oracle by test_c3_host_entry_oracle_rows."""
    e = synth.atlas_like(10000, seed=10000)
    r = Router(0)
    t = r.compute_shortest_paths(e, list(range(10000)))
    r.close()
    assert t.stats["path_kind"] == N.SRG_PATH_DENSE_U32
    return e, t


C3_ROWS = 512  # >= 512 seeded sources checked against the oracle at C3


@pytest.fixture(scope="module")
def c3_oracle_rows(c3_single):
    e, _ = c3_single
    rows = np.random.default_rng(10001).choice(10000, C3_ROWS, replace=False).tolist()
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), list(range(10000)), rows=rows, mode=2, nthreads=16)
    return rows, lat, loss


@pytest.mark.slow
def test_c3_host_entry_oracle_rows(c3_single, c3_oracle_rows):
    """The headline path itself at full size: the host entry with the FW beside the
    H2D -- what bench.py times and what Shadow's call site runs -- against C3_ROWS seeded oracle rows
    (mode 2, pinned to the heap Dijkstra in test_oracle.py), bit-exact, plus whole-table properties."""
    e, t = c3_single
    assert t.stats["fw_overlap_kept"] == 1 and t.stats["fw_overlap_pivots"] > 0, t.stats
    rows, lat, loss = c3_oracle_rows
    assert np.array_equal(t.latency_ns[rows], lat)
    assert bits_equal(t.packet_loss[rows], loss)
    V = 10000
    assert np.array_equal(np.diag(t.latency_ns), e.latency_ns[:V])
    off = ~np.eye(V, dtype=bool)
    assert np.array_equal(t.latency_ns[off], t.latency_ns.T[off])
    assert int(t.latency_ns[off].min()) >= int(e.latency_ns[V:].min())


@pytest.mark.slow
def test_c3_routing_info_full_size(c3_single, c3_oracle_rows):
    """Shadow's actual call at full C3 size: srg_routing_info_build (generate_routing_info +
    RoutingInfo, sim_config.rs:425-462) keeps the build's certified u32 latency keys; its tables equal
    the host-entry table everywhere and the oracle's rows, and path() / get_smallest_latency_ns()
    agree with them."""
    e, t = c3_single
    V = 10000
    ids = list(range(V))
    ri = generate_routing_info(e, ids)
    lt, ls, gid = ri.tables()
    assert np.array_equal(lt, t.latency_ns) and bits_equal(ls, t.packet_loss)
    rows, lat, loss = c3_oracle_rows
    assert np.array_equal(lt[rows], lat) and bits_equal(ls[rows], loss)
    rng = np.random.default_rng(3)
    for s, d in rng.integers(0, V, size=(64, 2)):
        p = ri.path(int(s), int(d))
        assert p.latency_ns == int(t.latency_ns[s, d]) and np.float32(p.packet_loss) == t.packet_loss[s, d]
    assert ri.get_smallest_latency_ns() == int(t.latency_ns.min())


@pytest.mark.slow
@pytest.mark.parametrize("G", [2, 8])
def test_c3_full_size_ranks_match_single_gpu(c3_single, G):
    """The multi-rank build at full C3 size (10 000 vertices, 5e7 edges): G in-process ranks on one
    GPU (row-block FW with per-pivot panel broadcasts, essential-mask exchange, output row
    exchange) -- every rank ends with the single-GPU table bit for bit."""
    e, ref = c3_single
    out, errs = run_ranks(G, e, list(range(10000)))
    assert errs == [None] * G, errs
    for r, t in enumerate(out):
        assert t.stats["nranks"] == G and t.stats["rank"] == r
        assert np.array_equal(t.latency_ns, ref.latency_ns), f"rank {r} latency"
        assert bits_equal(t.packet_loss, ref.packet_loss), f"rank {r} loss"
    assert sum(t.stats["local_sources"] for t in out) == 10000


# ---- srg_multi: one call, several GPUs (here: several ranks sharing the test box's one GPU) ----
@pytest.mark.parametrize("G,kw,kind", [
    (2, dict(V=700, dens=0.03, seed=41), "all"),
    (3, dict(V=520, dens=0.05, seed=42), "scrambled"),
    (8, dict(V=1100, dens=0.02, seed=43), "subset"),
    (4, dict(V=260, dens=0.2, seed=44, lat_lo=2**31, lat_hi=2**33), "all"),   # u64 keys
    (3, dict(V=300, dens=0.05, seed=45, directed=True), "scrambled"),         # general FW
    (2, dict(V=2000, dens=0.0, seed=46, algorithm="sparse"), "all"),          # sparse path (BA graph)
], ids=["G2", "G3_scrambled", "G8_subset", "G4_u64", "G3_directed", "G2_sparse"])
def test_multi_router_matches_oracle(G, kw, kind):
    """srg_multi_compute_shortest_paths: the whole table in the caller's arrays (every rank its own
    rows), equal to the oracle; stats aggregate the ranks (sources summed, min latency over all)."""
    kw = dict(kw)
    V, dens, seed = kw.pop("V"), kw.pop("dens"), kw.pop("seed")
    algo = kw.pop("algorithm", None)
    e = synth.barabasi_albert(V, 3, seed=seed) if algo == "sparse" else synth.random_graph(V, dens, seed, **kw)
    nodes = node_list(kind, V, seed)
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), nodes)
    m = MultiRouter([0] * G)
    assert len(m) == G
    if algo == "sparse":
        m.set_option(N.SRG_OPT_ALGORITHM, N.SRG_ALGO_SPARSE)
    t = m.compute_shortest_paths(e, nodes)
    m.close()
    assert t.stats["nranks"] == G and t.stats["local_sources"] == len(nodes)
    assert np.array_equal(t.latency_ns, lat) and bits_equal(t.packet_loss, loss)
    assert t.stats["min_latency_ns"] == int(lat.min())


def test_multi_router_big_table_registered_once():
    """A table past the early-D2H threshold (64 MB): the caller's arrays are page-locked once for
    all ranks and every rank ships its rows into them while later kernels run."""
    V = 2600
    e = synth.atlas_like(V, seed=2600)
    nodes = np.random.default_rng(5).permutation(V).tolist()
    r1 = Router(0)
    ref = r1.compute_shortest_paths(e, nodes)
    r1.close()
    m = MultiRouter([0, 0, 0])
    t = m.compute_shortest_paths(e, nodes)
    m.close()
    assert np.array_equal(t.latency_ns, ref.latency_ns) and bits_equal(t.packet_loss, ref.packet_loss)
    assert t.stats["d2h_overlapped_bytes"] == V * V * 12
    assert t.stats["ms_host_register"] >= 0


def test_multi_router_errors_agree():
    """A reference error (unreachable used pair -> the assert_eq! panic) surfaces once, from the
    one call, with the single-GPU code and message; the object stays usable afterwards."""
    iso = synth.random_graph(300, 0.05, 12)
    keep = ((iso.src != 299) & (iso.dst != 299)) | (iso.src == iso.dst)
    from shadow_amd.graph import Edges
    e = Edges(300, iso.src[keep], iso.dst[keep], iso.latency_ns[keep], iso.packet_loss[keep], False)
    m = MultiRouter([0, 0, 0, 0])
    with pytest.raises(RoutingPanic):
        m.compute_shortest_paths(e, list(range(300)))
    ok = synth.random_graph(200, 0.05, 13)
    lat, loss = oracle.compute_shortest_paths(ok.as_tuple(), list(range(200)))
    t = m.compute_shortest_paths(ok, list(range(200)))
    assert np.array_equal(t.latency_ns, lat) and bits_equal(t.packet_loss, loss)
    m.close()


def test_routing_info_multi_and_rank_guard():
    """srg_routing_info_build_multi builds the dense RoutingInfo with every rank; the per-rank
    srg_routing_info_build refuses a context that fills only its own rows."""
    e = synth.random_graph(250, 0.05, 15)
    ids = list(range(250))
    m = MultiRouter([0, 0])
    ri = generate_routing_info(e, ids, router=m)
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), ids)
    lt, ls, gid = ri.tables()
    assert np.array_equal(lt, lat) and bits_equal(ls, loss)
    assert ri.get_smallest_latency_ns() == int(lat.min())
    del ri  # the views keep the native tables alive
    import gc
    gc.collect()
    assert np.array_equal(lt, lat)
    m.close()
    group = LocalGroup(2)
    rt = Router(0)
    rt.init_comm_local(group, 0)
    rt.set_option(N.SRG_OPT_GATHER_OUTPUT, 0)
    with pytest.raises(NetGraphError) as ei:
        generate_routing_info(e, ids, router=rt)
    assert ei.value.code == N.SRG_ERR_ARG
    rt.close()
    group.close()


@pytest.mark.slow
def test_c4_multi_router_8_ranks():
    """Config C4 (barabasi_albert(50000, 4, seed=50000)) built by 8 ranks through srg_multi: each
    rank holds only its 6 250 rows on the device (3.75 GB) and ships them into the one 30 GB host
    table.  Every row's checksum equals the single-GPU device table's, and 512 seeded rows equal
    the oracle (mod.rs:190-208: independent per-source runs)."""
    import torch
    from shadow_amd.device import DeviceGraph, compute_shortest_paths_device
    V = 50000
    e = synth.barabasi_albert(V, 4, seed=V)
    dev = torch.device("cuda", 0)
    dg = DeviceGraph(e)
    nodes_t = torch.arange(V, dtype=torch.int32, device=dev)
    ol = torch.empty((V, V), dtype=torch.int64, device=dev)
    os_ = torch.empty((V, V), dtype=torch.float32, device=dev)
    r1 = Router(0)
    st = compute_shortest_paths_device(r1, dg, nodes_t, ol, os_)
    assert st["path_kind"] == N.SRG_PATH_SPARSE_U32
    ref_lat = ol.sum(dim=1).cpu().numpy()
    ref_loss = os_.view(torch.int32).to(torch.int64).sum(dim=1).cpu().numpy()
    del ol, os_, dg
    r1.close()
    torch.cuda.empty_cache()
    m = MultiRouter([0] * 8)
    t = m.compute_shortest_paths(e, np.arange(V, dtype=np.uint32))
    m.close()
    assert t.stats["path_kind"] == N.SRG_PATH_SPARSE_U32 and t.stats["local_sources"] == V
    got_lat = t.latency_ns.view(np.int64).sum(axis=1)
    got_loss = t.packet_loss.view(np.int32).astype(np.int64).sum(axis=1)
    assert np.array_equal(got_lat, ref_lat) and np.array_equal(got_loss, ref_loss)
    rows = np.random.default_rng(50000).choice(V, size=512, replace=False)
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), list(range(V)), rows=rows.tolist(), mode=1, nthreads=16)
    assert np.array_equal(t.latency_ns[rows], lat) and bits_equal(t.packet_loss[rows], loss)


@pytest.mark.slow
@pytest.mark.parametrize("G", [2, 8])
def test_c3_multi_router(c3_single, G):
    """Config C3 through srg_multi with G ranks: the distributed symmetric FW (line-buffer
    allgathers, packed-triangle exchange) and the position-split sources give the single-GPU
    table bit for bit, in the caller's one array."""
    e, ref = c3_single
    m = MultiRouter([0] * G)
    t = m.compute_shortest_paths(e, list(range(10000)))
    m.close()
    assert t.stats["nranks"] == G and t.stats["local_sources"] == 10000
    assert np.array_equal(t.latency_ns, ref.latency_ns)
    assert bits_equal(t.packet_loss, ref.packet_loss)
