import os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np
from shadow_amd import Router, synth
V = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
e = synth.atlas_like(V, seed=V)
nodes = np.arange(V, dtype=np.uint32)
lat = np.zeros((V, V), np.uint64); loss = np.zeros((V, V), np.float32)
for it in range(3):
    r = Router(0)
    for k in range(2):
        t = r.compute_shortest_paths(e, nodes, lat, loss)
        print("router", it, "call", k, "kept", t.stats["fw_overlap_kept"], "pivots", t.stats["fw_overlap_pivots"], "h2d", round(t.stats["ms_h2d"], 2), "total", round(t.stats["ms_total"], 2), flush=True)
    r.close()
