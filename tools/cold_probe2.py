"""Cold-call breakdown, round 4 (SRG_DEBUG_CREATE / SRG_DEBUG_CODEC print the library's own steps):
HIP runtime init, srg_create, then the first C3 host entry on never-touched arrays and a second one.
usage: SRG_DEBUG_CREATE=1 SRG_DEBUG_CODEC=1 python tools/cold_probe2.py [V]"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    from shadow_amd import Router, synth
    V = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    e = synth.atlas_like(V, seed=V)
    nodes = np.arange(V, dtype=np.uint32)
    out = {"V": V}
    hip = ctypes.CDLL("libamdhip64.so")
    t0 = time.perf_counter()
    n = ctypes.c_int()
    hip.hipGetDeviceCount(ctypes.byref(n))
    out["hip_init_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
    t0 = time.perf_counter()
    r = Router(0)
    out["create_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
    for label in ("first_fresh", "second_fresh"):
        lat = np.empty((V, V), dtype=np.uint64)
        loss = np.empty((V, V), dtype=np.float32)
        t1 = time.perf_counter()
        res = r.compute_shortest_paths(e, nodes, lat, loss)
        ms = (time.perf_counter() - t1) * 1e3
        out[label] = {"ms": round(ms, 1), **{k: round(v, 2) for k, v in res.stats.items() if k.startswith("ms_")}}
        del lat, loss
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
