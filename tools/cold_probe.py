"""Cold-call breakdown of the C3 host entry (what Shadow's one call per simulation pays,
sim_config.rs:137-141): srg_create, the first build on never-touched output arrays (as the
Rust binding's vec![0u64; n*n] hands them over), and the same on pre-faulted arrays; with the
host page-locking time the library reports (stats.ms_host_register).  Prints one JSON line.
usage: python tools/cold_probe.py [V]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    from shadow_amd import Router, synth
    V = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    e = synth.atlas_like(V, seed=V)
    nodes = np.arange(V, dtype=np.uint32)
    out = {"V": V}
    try:
        with open("/sys/kernel/mm/transparent_hugepage/enabled") as f:
            out["thp"] = f.read().strip()
    except OSError:
        out["thp"] = None
    t0 = time.perf_counter()
    torch.cuda.init()  # the HIP runtime itself (any first HIP call pays it)
    out["hip_init_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
    t0 = time.perf_counter()
    r = Router(0)
    out["create_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
    for label in ("first_fresh", "second_fresh", "prefaulted", "steady"):
        lat = np.empty((V, V), dtype=np.uint64)
        loss = np.empty((V, V), dtype=np.float32)
        if label in ("prefaulted", "steady"):
            t1 = time.perf_counter()
            lat.fill(0)
            loss.fill(0)
            out["prefault_numpy_ms"] = round((time.perf_counter() - t1) * 1e3, 1)
        if label == "steady":
            r.compute_shortest_paths(e, nodes, lat, loss)
        t1 = time.perf_counter()
        res = r.compute_shortest_paths(e, nodes, lat, loss)
        ms = (time.perf_counter() - t1) * 1e3
        out[label] = {"ms": round(ms, 1), "ms_host_register": round(res.stats.get("ms_host_register", -1), 1),
                      "ms_total": round(res.stats.get("ms_total", -1), 1), "ms_h2d": round(res.stats.get("ms_h2d", -1), 1),
                      "ms_d2h": round(res.stats.get("ms_d2h", -1), 1)}
        del lat, loss
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
