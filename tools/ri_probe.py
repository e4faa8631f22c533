"""RoutingInfo build times on C3 (what Shadow's call site runs, sim_config.rs:425-462): the first
build on a fresh context, then several more, with every srg_stats time of each build.
usage: python tools/ri_probe.py [V] [builds]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from shadow_amd import Router, generate_routing_info, synth
    V = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    e = synth.atlas_like(V, seed=V)
    ids = list(range(V))
    r = Router(0)
    res = []
    for i in range(nb):
        t0 = time.perf_counter()
        ri = generate_routing_info(e, ids, True, r)
        ms = (time.perf_counter() - t0) * 1e3
        st = ri.stats
        res.append({"ms": round(ms, 1), "keys": st.get("table_keys"),
                    **{k: round(v, 2) for k, v in st.items() if k.startswith("ms_")}})
        ri.close()
    r.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
