"""debug: the overlap build at V=2048 after other tests ran in the same process"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from shadow_amd import Router, synth  # noqa: E402
from shadow_amd import _native as N  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ov,step", [(1, 0), (0, 0), (1, -1), (1, 0)])
def test_ov(ov, step):
    e = synth.atlas_like(2048, seed=31)
    r = Router(0)
    r.set_option(N.SRG_OPT_FW_OVERLAP, ov)
    r.set_option(N.SRG_OPT_FW_STEP, step)
    os.environ["SRG_DEBUG_OVERLAP"] = "1"
    t = r.compute_shortest_paths(e, list(range(2048)))
    del os.environ["SRG_DEBUG_OVERLAP"]
    r.close()
    z = int((t.latency_ns == 0).sum())
    print(f"ov={ov} step={step} zeros={z} stats={t.stats}", flush=True)
    assert z == 0
