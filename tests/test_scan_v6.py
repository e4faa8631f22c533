"""tight_v6 (entry lanes, tight_v6.hip.h) against tight_v5 (source lanes, tight_sparse.hip.h): the
same tight-predecessor table, hence the same multi-predecessor count and bit-identical outputs, on
the graphs the scan tests cover -- atlas tables through the host entry's interleaved scan groups,
random graphs with parallel edges, ms-unit keys, u64 keys scanned on their low words (false
matches everywhere), a scrambled node subset and a directed graph.  tight_v5 itself is
pinned to the oracle by test_gpu_parity.py / test_multi_gpu.py."""
import numpy as np
import pytest

from shadow_amd import Router, synth
from shadow_amd import _native as N
from shadow_amd.graph import Edges

pytestmark = pytest.mark.gpu


def both(e, nodes, opts=()):
    out = []
    for k in (5, 6):
        r = Router(0)
        r.set_option(N.SRG_OPT_SCAN_KERNEL, k)
        for o, v in opts:
            r.set_option(o, v)
        out.append(r.compute_shortest_paths(e, nodes))
        r.close()
    a, b = out
    assert a.stats["scan_kind"] == N.SRG_SCAN_SPARSE and b.stats["scan_kind"] == N.SRG_SCAN_SPARSE
    assert a.stats["multi_pred_pairs"] == b.stats["multi_pred_pairs"]
    assert a.stats["essential_edges"] == b.stats["essential_edges"]
    assert np.array_equal(a.latency_ns, b.latency_ns)
    assert np.array_equal(a.packet_loss.view(np.uint32), b.packet_loss.view(np.uint32))
    return a, b


@pytest.mark.parametrize("V,seed", [(300, 1), (1000, 2), (2501, 3)])
def test_v6_atlas(V, seed):
    both(synth.atlas_like(V, seed=seed), list(range(V)))


def test_v6_random_parallel_edges():
    e = synth.random_graph(700, 0.05, 11, lat_lo=1, lat_hi=20, parallel=0.2)
    both(e, list(range(700)))


def test_v6_ms_units_and_subset():
    e = synth.random_graph(900, 0.08, 12, lat_lo=1, lat_hi=300)
    g = Edges(900, e.src, e.dst, e.latency_ns * np.uint64(10 ** 6), e.packet_loss, False)
    nodes = np.random.default_rng(4).permutation(900)[:611].tolist()
    both(g, nodes)


@pytest.mark.parametrize("shift,offset", [(32, 0), (32, 1), (0, 2 ** 33)])
def test_v6_u64_low_words(shift, offset, monkeypatch):
    monkeypatch.setenv("SRG_LATENCY_UNIT", "1")
    g = synth.random_graph(300, 0.08, 5 + shift, lat_lo=1, lat_hi=6, parallel=0.1)
    lat = g.latency_ns.astype(np.uint64) * np.uint64(2 ** shift) + np.uint64(offset)
    a, b = both(Edges(300, g.src, g.dst, lat, g.packet_loss, False), list(range(300)))
    assert a.stats["path_kind"] == N.SRG_PATH_DENSE_U64


def test_v6_directed():
    e = synth.random_graph(640, 0.06, 13, lat_lo=1, lat_hi=50, directed=True)
    both(e, list(range(640)))
