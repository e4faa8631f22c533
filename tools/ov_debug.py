"""FW beside the H2D at several sizes: overlap on vs off, byte comparison and the first differing
entries (debugging aid).  usage: SRG_DEBUG_OVERLAP=1 python tools/ov_debug.py V [V ...]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shadow_amd import Router, synth  # noqa: E402
from shadow_amd import _native as N  # noqa: E402


def build(e, nodes, ov, step=-1):
    r = Router(0)
    r.set_option(N.SRG_OPT_FW_OVERLAP, ov)
    if step != -1:
        r.set_option(N.SRG_OPT_FW_STEP, step)
    try:
        return r.compute_shortest_paths(e, nodes)
    finally:
        r.close()


extra = Router(0) if os.environ.get("OV_EXTRA_CTX") else None  # a second context: event stream hops
for V in [int(x) for x in sys.argv[1:]]:
    e = synth.atlas_like(V, seed=31 if V == 2048 else V + 1)
    nodes = list(range(V))
    for step in (-1, 0):
        t1 = build(e, nodes, 1, step)
        t0 = build(e, nodes, 0, step)
        bad = np.argwhere(t1.latency_ns != t0.latency_ns)
        print(f"V={V} step={step} kind={t1.stats['path_kind']} bad={len(bad)} zeros1={(t1.latency_ns == 0).sum()} "
              f"zeros0={(t0.latency_ns == 0).sum()} first={bad[:4].tolist()}", flush=True)
