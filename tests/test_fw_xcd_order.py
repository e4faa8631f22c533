"""The symmetric FW bulk launched in XCD Z-order runs (SRG_OPT_FW_XCD_ORDER = 1, routing.hip
xcd_tile_order) computes the same closure as triangle order: bit-identical tables through the host
entry (with and without the FW beside the H2D) and on a simulated rank of a 3-rank group."""
import numpy as np
import pytest

from shadow_amd import Router, synth
from shadow_amd import _native as N

pytestmark = pytest.mark.gpu


def run(e, nodes, order, opts=()):
    r = Router(0)
    r.set_option(N.SRG_OPT_FW_XCD_ORDER, order)
    for o, v in opts:
        r.set_option(o, v)
    t = r.compute_shortest_paths(e, nodes)
    r.close()
    return t


@pytest.mark.parametrize("V,overlap", [(3000, 1), (3000, 0), (1100, 0)])
def test_xcd_order_matches(V, overlap):
    e = synth.atlas_like(V, seed=V + 5)
    a = run(e, list(range(V)), 0, ((N.SRG_OPT_FW_OVERLAP, overlap),))
    b = run(e, list(range(V)), 1, ((N.SRG_OPT_FW_OVERLAP, overlap),))
    assert a.stats["path_kind"] == N.SRG_PATH_DENSE_U32
    assert np.array_equal(a.latency_ns, b.latency_ns)
    assert np.array_equal(a.packet_loss.view(np.uint32), b.packet_loss.view(np.uint32))
