"""Debug probe: tight-predecessor vertices of scan variants 2 and 3 on small graphs (SRG_DEBUG_PRED)."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from shadow_amd import Router, synth
from shadow_amd import _native as N
from helpers import load_vectors, fixture_edges

cases = [("golden_undirected_ties", [f for f in load_vectors() if f["name"] == "undirected_ties"][0])]
for name, fx in cases:
    e = fixture_edges(fx)
    nodes = fx["nodes"]
    res = {}
    for v in (2, 3):
        r = Router(0)
        r.set_option(N.SRG_OPT_SPARSE_THRESHOLD, 1.0)
        r.set_option(N.SRG_OPT_SCAN_VARIANT, v)
        os.environ["SRG_DEBUG_PRED"] = f"/tmp/pred{v}.bin"
        t = r.compute_shortest_paths(e, nodes)
        res[v] = np.fromfile(f"/tmp/pred{v}.bin", dtype=np.int32).reshape(len(nodes), -1)
        r.close()
    d = np.argwhere(res[2] != res[3])
    print(name, "V", e.num_vertices, "n", len(nodes), "diffs", len(d))
    for r_, t_ in d[:40]:
        print(" row", r_, "src", nodes[r_], "t", t_, "v2", res[2][r_, t_], "v3", res[3][r_, t_])
