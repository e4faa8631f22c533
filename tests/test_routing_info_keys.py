"""RoutingInfo (mod.rs:428-477, sim_config.rs:425-462) kept in the build's certified u32 latency keys
(srg_routing_info_build, one rank): path() widens key x latency unit exactly, the diagonal is the raw
self-loop latency, get_smallest_latency_ns covers both, tables() gives the widened u64 view -- all
equal to the u64 host-entry table.  Builds that need u64 keys keep a u64 table (table_keys = 0)."""
import numpy as np
import pytest

from shadow_amd import Router, generate_routing_info, synth
from shadow_amd import _native as N
from shadow_amd.graph import Edges

pytestmark = pytest.mark.gpu


def check(e, ids, expect_keys, router=None):
    r = router or Router(0)
    t = r.compute_shortest_paths(e, ids)
    ri = generate_routing_info(e, ids, True, r)
    assert ri.stats["table_keys"] == expect_keys
    tl, tf, tid = ri.tables()
    pos = {int(x): i for i, x in enumerate(tid.tolist())}
    order = [pos[i] for i in ids]
    assert np.array_equal(tl[np.ix_(order, order)], t.latency_ns)
    assert np.array_equal(tf[np.ix_(order, order)].view(np.uint32), t.packet_loss.view(np.uint32))
    rng = np.random.default_rng(1)
    for _ in range(200):
        a, b = rng.choice(len(ids), 2)
        p = ri.path(ids[a], ids[b])
        assert p.latency_ns == int(t.latency_ns[a, b]) and np.float32(p.packet_loss) == t.packet_loss[a, b]
    a = int(rng.integers(len(ids)))
    assert ri.path(ids[a], ids[a]).latency_ns == int(t.latency_ns[a, a])  # raw self-loop
    assert ri.get_smallest_latency_ns() == int(t.latency_ns.min())
    return ri


def test_keys_ms_unit_graph():
    """Millisecond latencies (unit 10^6 ns): keys count ms, the self-loops are sub-ms (not multiples
    of the unit) -- the diagonal must come from the raw self-loop latencies."""
    e = synth.random_graph(400, 0.1, 5, lat_lo=1, lat_hi=300)
    lat = e.latency_ns * np.uint64(10 ** 6)
    lat[e.src == e.dst] = 123_457  # raw self-loop latency, not a multiple of the unit
    g = Edges(400, e.src, e.dst, lat, e.packet_loss, False)
    ri = check(g, list(range(0, 400, 2)), 1)
    assert ri.get_smallest_latency_ns() == 123_457


def test_keys_large_dense_table():
    """C2-sized atlas table through the early-D2H path (u32 rows shipped while the scan runs)."""
    e = synth.atlas_like(2600, seed=26)
    ids = np.random.default_rng(3).permutation(2600).tolist()
    check(e, ids, 1)


def test_keys_sparse_path():
    """Sparse graphs (V >= 2048, batched Bellman-Ford) write the key table from the sparse kernel."""
    e = synth.barabasi_albert(3000, 3, seed=30)
    r = Router(0)
    t = r.compute_shortest_paths(e, list(range(3000)))
    assert t.stats["path_kind"] == N.SRG_PATH_SPARSE_U32
    check(e, list(range(0, 3000, 3)), 1, r)


def test_u64_build_keeps_u64_table(monkeypatch):
    """Nanosecond keys with paths past 2^31 units run on u64 keys: the table stays u64."""
    monkeypatch.setenv("SRG_LATENCY_UNIT", "1")
    e = synth.random_graph(300, 0.1, 7, lat_lo=2 ** 31, lat_hi=2 ** 33)
    check(e, list(range(300)), 0)


def test_pool_recycles_page_locked_tables():
    """srg_routing_info_build's tables come from the context's pinned-table pool: freeing a RoutingInfo
    returns them (still page-locked), the next build into them skips the prefault + page-locking and
    writes the same table."""
    e = synth.atlas_like(2600, seed=26)
    ids = list(range(2600))
    r = Router(0)
    assert r.get_option(N.SRG_OPT_TABLE_POOL_IDLE_BYTES) == 0
    ri = generate_routing_info(e, ids, True, r)
    assert ri.stats["table_keys"] == 1 and ri.stats["ms_host_register"] >= 0
    tl, tf, _ = ri.tables()
    tl, tf = tl.copy(), tf.copy()
    ri.close()
    idle = r.get_option(N.SRG_OPT_TABLE_POOL_IDLE_BYTES)
    assert idle >= 2 * 2600 * 2600 * 4
    ri = generate_routing_info(e, ids, True, r)
    assert r.get_option(N.SRG_OPT_TABLE_POOL_IDLE_BYTES) == 0  # both tables taken again
    assert ri.stats["ms_host_register"] < 2.0, ri.stats["ms_host_register"]  # (~12 ms when registering)
    tl2, tf2, _ = ri.tables()
    assert np.array_equal(tl2, tl) and np.array_equal(tf2.view(np.uint32), tf.view(np.uint32))
    ri.close()
    r.set_option(N.SRG_OPT_TABLE_POOL_BYTES, 0)  # trims the idle tables
    assert r.get_option(N.SRG_OPT_TABLE_POOL_IDLE_BYTES) == 0
    ri = generate_routing_info(e, ids, True, r)
    ri.close()
    assert r.get_option(N.SRG_OPT_TABLE_POOL_IDLE_BYTES) == 0
    r.close()


def test_pool_keeps_one_idle_pair_by_default():
    """Without a byte cap the pool keeps only the most recently freed table pair: two RoutingInfos freed
    leave the idle bytes of one (page-locked host memory stays bounded per context)."""
    e = synth.atlas_like(2600, seed=26)
    ids = list(range(2600))
    r = Router(0)
    a = generate_routing_info(e, ids, True, r)
    b = generate_routing_info(e, ids, True, r)
    a.close()
    one = r.get_option(N.SRG_OPT_TABLE_POOL_IDLE_BYTES)
    assert one >= 2 * 2600 * 2600 * 4
    b.close()
    assert r.get_option(N.SRG_OPT_TABLE_POOL_IDLE_BYTES) == one
    r.close()


def test_routing_info_outlives_its_router():
    """A RoutingInfo owns its pooled tables past srg_destroy of the context that built them."""
    e = synth.atlas_like(2600, seed=27)
    r = Router(0)
    t = r.compute_shortest_paths(e, list(range(0, 2600, 1)))
    ri = generate_routing_info(e, list(range(2600)), True, r)
    r.close()
    rng = np.random.default_rng(2)
    for _ in range(100):
        a, b = rng.choice(2600, 2)
        assert ri.path(int(a), int(b)).latency_ns == int(t.latency_ns[a, b])
    tl, _, _ = ri.tables()
    assert np.array_equal(tl, t.latency_ns)
    ri.close()


def test_create_timing_options():
    """srg_create's HIP-runtime part and its own part are reported (read-only options)."""
    r = Router(0)
    rt = r.get_option(N.SRG_OPT_CREATE_MS_RUNTIME)
    lib = r.get_option(N.SRG_OPT_CREATE_MS_LIBRARY)
    assert rt >= 0 and lib > 0
    with pytest.raises(Exception):
        r.set_option(N.SRG_OPT_CREATE_MS_RUNTIME, 1)
    r.close()


def test_host_entry_key_rows_u64_fallback(monkeypatch):
    """The host entry's u64 output ships a dense u32 build's latency rows as keys (d2h_key_rows = 1);
    a build that needs u64 keys ships u64 rows instead (d2h_key_rows = 0).  Both equal the device
    entry."""
    from shadow_amd.device import DeviceGraph, compute_shortest_paths_device
    import torch
    r = Router(0)
    for big in (False, True):
        if big:
            monkeypatch.setenv("SRG_LATENCY_UNIT", "1")
            e0 = synth.atlas_like(2500, seed=25)
            e = Edges(e0.num_vertices, e0.src, e0.dst, e0.latency_ns * np.uint64(2 ** 20), e0.packet_loss, False)
        else:
            e = synth.atlas_like(2500, seed=25)
        t = r.compute_shortest_paths(e, list(range(2500)))
        assert t.stats["d2h_key_rows"] == (0 if big else 1), t.stats
        assert t.stats["path_kind"] == (N.SRG_PATH_DENSE_U64 if big else N.SRG_PATH_DENSE_U32)
        g = DeviceGraph(e, "cuda:0")
        ol = torch.empty((2500, 2500), dtype=torch.int64, device="cuda:0")
        os_ = torch.empty((2500, 2500), dtype=torch.float32, device="cuda:0")
        compute_shortest_paths_device(r, g, torch.arange(2500, dtype=torch.int32, device="cuda:0"), ol, os_)
        torch.cuda.synchronize()
        assert np.array_equal(ol.cpu().numpy().view(np.uint64), t.latency_ns)
        assert np.array_equal(os_.cpu().numpy().view(np.uint32), t.packet_loss.view(np.uint32))
    r.close()
