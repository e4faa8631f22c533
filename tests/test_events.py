"""Stretch row f4: one round's packet-event batch (events.hip.h) -- oracle checks on CPU, GPU
parity (bit-exact order, deliver times, per-host offsets, min next event / min used latency)
against the restatement of worker.rs:391-424 / event.rs:84-155 / manager.rs:459-464."""
import numpy as np
import pytest

import oracle
from shadow_amd import events as ev


def numpy_reference(batch, table, num_hosts, round_end):
    """Independent statement: deliver = max(send + table[src, dst], round_end); order =
    lexicographic (dst_host, deliver, src_host, event_id)."""
    lat = table[batch["src_node"].astype(np.int64), batch["dst_node"].astype(np.int64)]
    deliver = np.maximum(batch["send_time_ns"].astype(np.uint64) + lat, np.uint64(round_end))
    order = np.lexsort((batch["src_event_id"], batch["src_host"], deliver, batch["dst_host"]))
    off = np.searchsorted(batch["dst_host"][order], np.arange(num_hosts + 1), side="left").astype(np.uint64)
    return deliver, order.astype(np.uint32), off, int(deliver.min()), int(lat.min())


def rand_batch(n, H, tn, seed, id_span=10**6, t_span=10**6):
    rng = np.random.default_rng(seed)
    b = dict(src_node=rng.integers(0, tn, n, dtype=np.uint32), dst_node=rng.integers(0, tn, n, dtype=np.uint32),
             src_host=rng.integers(0, H, n, dtype=np.uint32), dst_host=rng.integers(0, H, n, dtype=np.uint32),
             send_time_ns=(10**12 + rng.integers(0, t_span, n, dtype=np.uint64)).astype(np.uint64))
    # unique (src_host, event_id): ids = per-position unique values spread over id_span
    b["src_event_id"] = (rng.permutation(max(n, 1))[:n].astype(np.uint64) * max(1, id_span // max(n, 1)) + 5)
    table = rng.integers(10**5, 10**7, (tn, tn), dtype=np.uint64)
    return b, table


def test_oracle_matches_numpy():
    b, table = rand_batch(3000, 41, 17, 1)
    re = 10**12 + 400_000
    got = oracle.order_packet_events(b, table, 41, re)
    exp = numpy_reference(b, table, 41, re)
    for g, e in zip(got, exp):
        assert np.array_equal(np.asarray(g), np.asarray(e))


def test_oracle_kat():
    """Hand-checked: host 1 receives three packets; two are delivered at the round end (tie on
    time -> src_host decides, then the event id); host 0 and host 2 stay empty."""
    table = np.array([[5, 7], [9, 3]], dtype=np.uint64)
    b = dict(src_node=np.array([0, 1, 0], np.uint32), dst_node=np.array([1, 0, 1], np.uint32),
             src_host=np.array([4, 2, 4], np.uint32), dst_host=np.array([1, 1, 1], np.uint32),
             send_time_ns=np.array([100, 100, 95], np.uint64), src_event_id=np.array([8, 3, 7], np.uint64))
    deliver, order, off, mn, ml = oracle.order_packet_events(b, table, 3, 104)
    assert deliver.tolist() == [107, 109, 104]   # 100+7, 100+9, max(95+7, 104)
    assert order.tolist() == [2, 0, 1]
    assert off.tolist() == [0, 0, 3, 3] and mn == 104 and ml == 7


def test_oracle_unordered_panics():
    table = np.array([[5]], dtype=np.uint64)
    b = dict(src_node=np.zeros(2, np.uint32), dst_node=np.zeros(2, np.uint32), src_host=np.array([3, 3], np.uint32),
             dst_host=np.zeros(2, np.uint32), send_time_ns=np.array([10, 10], np.uint64),
             src_event_id=np.array([1, 1], np.uint64))
    with pytest.raises(oracle.OracleError) as e:
        oracle.order_packet_events(b, table, 1, 0)
    assert e.value.code == 3


def test_synthetic_round_shape():
    b, re = ev.synthetic_round(20000, 500, 64, seed=3)
    key = np.lexsort((b["send_time_ns"], b["src_host"]))
    # per-source event ids are 1.. in send order (Host::get_new_event_id)
    s, i = b["src_host"][key], b["src_event_id"][key]
    first = np.r_[True, s[1:] != s[:-1]]
    assert np.all(i[first] == 1) and np.all(np.diff(i.astype(np.int64))[~first[1:]] == 1)
    assert b["send_time_ns"].max() < re


# ---------------------------------------------------------------------------------------- GPU
@pytest.fixture
def gpu_router():
    from shadow_amd import Router
    r = Router(0)
    yield r
    r.close()


def check(router, b, table, H, re):
    got = ev.order_packet_events(router, b, table, H, re)
    exp = oracle.order_packet_events(b, table, H, re)
    assert np.array_equal(got[0], exp[0]), "deliver times"
    assert np.array_equal(got[1], exp[1]), "order"
    assert np.array_equal(got[2], exp[2]), "host offsets"
    if len(b["send_time_ns"]):
        assert got[3]["min_next_event_ns"] == exp[3] and got[3]["min_used_latency_ns"] == exp[4]
    return got[3]


@pytest.mark.gpu
@pytest.mark.parametrize("n,H,tn,seed,id_span,t_span", [
    (1, 3, 2, 1, 10, 10),
    (1000, 7, 5, 2, 10**4, 10**3),            # narrow key, many ties on time
    (70000, 3000, 40, 3, 10**6, 10**7),       # one-word key, several tiles
    (200000, 100, 30, 4, 2**45, 2**40),       # key wider than 64 bits (two words)
])
def test_gpu_events_vs_oracle(gpu_router, n, H, tn, seed, id_span, t_span):
    b, table = rand_batch(n, H, tn, seed, id_span, t_span)
    res = check(gpu_router, b, table, H, 10**12 + t_span // 3)
    if id_span > 2**40:
        assert res["key_bits"] > 64


@pytest.mark.gpu
def test_gpu_events_empty_and_synthetic(gpu_router):
    b, table = rand_batch(0, 5, 3, 5)
    d, o, off, res = ev.order_packet_events(gpu_router, b, table, 5, 0)
    assert len(d) == 0 and off.tolist() == [0] * 6 and res["min_next_event_ns"] == 2**64 - 1
    b, re = ev.synthetic_round(300000, 10000, 256, seed=7)
    table = np.random.default_rng(8).integers(10**6, 10**8, (256, 256), dtype=np.uint64)
    check(gpu_router, b, table, 10000, re)


@pytest.mark.gpu
def test_gpu_events_routing_table(gpu_router):
    """The latency table is a RoutingInfo built on the GPU (f1 dense backing store)."""
    from shadow_amd import synth
    g = synth.random_graph(60, 0.2, 9, lat_lo=10**5, lat_hi=10**7)
    t = gpu_router.compute_shortest_paths(g, list(range(60)))
    b, re = ev.synthetic_round(50000, 60, 60, seed=9, runahead=2 * 10**6)
    b["src_node"], b["dst_node"] = b["src_host"].copy(), b["dst_host"].copy()
    check(gpu_router, b, t.latency_ns, 60, re)


@pytest.mark.gpu
def test_gpu_events_errors(gpu_router):
    b, table = rand_batch(500, 9, 4, 6)
    b["src_event_id"][7] = b["src_event_id"][3]
    b["src_host"][7], b["dst_host"][7] = b["src_host"][3], b["dst_host"][3]
    b["src_node"][7], b["dst_node"][7], b["send_time_ns"][7] = b["src_node"][3], b["dst_node"][3], b["send_time_ns"][3]
    with pytest.raises(ev.EventOrderError):
        ev.order_packet_events(gpu_router, b, table, 9, 0)
    b, table = rand_batch(50, 9, 4, 7)
    b["dst_host"][4] = 9
    with pytest.raises(Exception):
        ev.order_packet_events(gpu_router, b, table, 9, 0)


@pytest.mark.gpu
@pytest.mark.slow
def test_gpu_events_c5_full_size(gpu_router):
    """Config C5 at full size: the bench's 10^7-event round (synthetic_round(1e7, 10 000 hosts,
    seed 7)) against a 10k x 10k routing table, every output compared with the oracle."""
    n, H = 10**7, 10000
    b, re = ev.synthetic_round(n, H, H, seed=7)
    table = np.random.default_rng(7).integers(10**6, 10**8, (H, H), dtype=np.uint64)
    res = check(gpu_router, b, table, H, re)
    assert res["key_bits"] > 0
