"""Multi-rank routing build on ONE GPU: G ranks as threads of this process
attached to an in-process LocalGroup, each with its own context and full workspace.  Every
rank must end with exactly the single-GPU result (bit-exact latency and loss), for sorted,
scrambled and subset node lists, u32 and u64 keys, and with the output exchange off."""
import threading

import numpy as np
import pytest

import oracle
from shadow_amd import LocalGroup, NetGraphError, Router, RoutingPanic, synth
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
        assert np.array_equal(t.latency_ns, lat), f"rank {r} latency"
        assert bits_equal(t.packet_loss, loss), f"rank {r} loss"
    assert sum(t.stats["local_sources"] for t in out) == len(nodes)


@pytest.mark.parametrize("kind", ["scrambled", "all"])
def test_ranks_without_exchange_fill_own_rows(kind):
    """Output exchange off: each rank fills the rows of the sources it owns (with sorted nodes
    those rows are one block, and the host entry copies only that block to the caller)."""
    e = synth.random_graph(400, 0.04, 11)
    nodes = node_list(kind, 400, 11)
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), nodes)
    out, errs = run_ranks(3, e, nodes, gather=False)
    assert errs == [None] * 3
    covered = np.zeros(len(nodes), dtype=bool)
    T = 128
    nb = (400 + T - 1) // T
    for r, t in enumerate(out):
        lo, hi = r * nb // 3 * T, (r + 1) * nb // 3 * T
        rows = [i for i, v in enumerate(nodes) if lo <= v < hi]
        assert np.array_equal(t.latency_ns[rows], lat[rows])
        assert bits_equal(t.packet_loss[rows], loss[rows])
        covered[rows] = True
    assert covered.all()


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


def test_edge_sharded_codec_slices():
    """Edge sharding with the H2D codec active on every rank's slice (>= 2^20 edges per slice):
    the exchanged widened slices equal the single-GPU build."""
    e = synth.atlas_like(2100, seed=2100)
    assert e.num_edges >= 2 * (1 << 20) + 2
    nodes = list(range(0, 2100, 7))
    r1 = Router(0)
    ref = r1.compute_shortest_paths(e, nodes)
    r1.close()
    out, errs = run_ranks(2, e, nodes, shard=1)
    assert errs == [None] * 2, errs
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
    """Config C3 (atlas_like(10000, seed=10000)) built by one rank: the reference table."""
    e = synth.atlas_like(10000, seed=10000)
    r = Router(0)
    t = r.compute_shortest_paths(e, list(range(10000)))
    r.close()
    assert t.stats["path_kind"] == N.SRG_PATH_DENSE_U32
    return e, t


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
