"""Full (unsampled) CPU baselines for the small configs, on the GPU box's host cores:
C1 (complete_random(1000)) and C2 (atlas_like(4096)): every source through the
reference-equivalent pipeline (oracle mode 0: HashMap-score petgraph Dijkstra + linear
nodes.contains + per-source HashMaps merged into one, mod.rs:190-208) and through the CPU-best
dense-matrix Dijkstra (mode 2).  Prints one JSON line per config."""
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import oracle  # noqa: E402
from bench import cpu_info  # noqa: E402
from shadow_amd import synth  # noqa: E402


def _heartbeat():
    t0 = time.perf_counter()
    while True:
        time.sleep(30)
        print(f"... {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)


def main():
    threading.Thread(target=_heartbeat, daemon=True).start()
    info = cpu_info()
    th = info["threads"]
    cfgs = [("C1", lambda: synth.complete_random(1000, seed=1001)), ("C2", lambda: synth.atlas_like(4096, seed=4096))]
    only = sys.argv[1:] or None
    for name, make in cfgs:
        if only and name not in only:
            continue
        e = make()
        V = e.num_vertices
        nodes = np.arange(V, dtype=np.uint32)
        out = {"config": name, "vertices": V, "edges": int(e.num_edges), **info}
        for mode, label in ((0, "reference_equivalent"), (2, "cpu_best_dense_matrix")):
            t0 = time.perf_counter()
            t, setup = oracle.time_sources_mode(e.as_tuple(), nodes, nodes, nthreads=th, mode=mode)
            wall = time.perf_counter() - t0
            out[label] = {"seconds": round(t, 3), "setup_s": round(setup, 3), "wall_s": round(wall, 3),
                          "source_SSSPs_per_s": round(V / t, 3), "sources": V, "extrapolated": False}
            print(f"{name} mode {mode}: {t:.2f}s", file=sys.stderr, flush=True)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
