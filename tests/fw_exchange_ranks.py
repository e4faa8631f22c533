"""Child process of tests/test_fw_exchange.py: G in-process ranks on device 0 running the symmetric FW
with the DEVICE-SIDE line exchange (SRG_OPT_FW_STEP = 2: the chain's k_line_xchg stores each rank's
line segments into its peers' line buffers and raises arrival words, xchg.hip.h).  Ranks sharing a GPU
need a hardware queue each for that (one rank's in-kernel wait must not sit in front of a peer's
launch), so the parent starts this script with GPU_MAX_HW_QUEUES = 16.  Prints one JSON line: per
case, whether every rank matched the single-GPU build and the oracle bit for bit."""
import json
import os
import sys
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle  # noqa: E402
from shadow_amd import LocalGroup, Router, synth  # noqa: E402
from shadow_amd import _native as N  # noqa: E402


def bits_equal(a, b):
    return np.array_equal(np.asarray(a, dtype=np.float32).view(np.uint32), np.asarray(b, dtype=np.float32).view(np.uint32))


def run(G, e, nodes, split, step=2):
    group = LocalGroup(G)
    routers = [Router(0) for _ in range(G)]
    for r, rt in enumerate(routers):
        rt.init_comm_local(group, r)
        rt.set_option(N.SRG_OPT_FW_STEP, step)
        if split:
            rt.set_option(N.SRG_OPT_FW_LINE_SPLIT, split)
    out, errs = [None] * G, [None] * G

    def work(r):
        try:
            out[r] = routers[r].compute_shortest_paths(e, nodes)
        except Exception as ex:  # noqa: BLE001
            errs[r] = repr(ex)

    th = [threading.Thread(target=work, args=(r,)) for r in range(G)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    for rt in routers:
        rt.close()
    group.close()
    return out, errs


def main():
    cases = [
        dict(G=2, V=700, seed=11, split=0),
        dict(G=3, V=900, seed=17, split=2),
        dict(G=4, V=1500, seed=18, split=0),
        dict(G=4, V=1100, seed=13, split=4),
        dict(G=2, V=400, seed=19, split=0, u64=True),
    ]
    res = []
    for c in cases:
        kw = dict(lat_lo=2 ** 31, lat_hi=2 ** 33) if c.get("u64") else {}
        e = synth.random_graph(c["V"], 0.05, c["seed"], **kw)
        nodes = list(range(c["V"]))
        ref = Router(0)
        ref.set_option(N.SRG_OPT_FW_STEP, 0)
        t0 = ref.compute_shortest_paths(e, nodes)
        ref.close()
        lat, loss = oracle.compute_shortest_paths(e.as_tuple(), nodes)
        out, errs = run(c["G"], e, nodes, c["split"])
        ok = all(x is None for x in errs) and all(
            np.array_equal(t.latency_ns, t0.latency_ns) and bits_equal(t.packet_loss, t0.packet_loss)
            and np.array_equal(t.latency_ns, lat) and bits_equal(t.packet_loss, loss) for t in out if t is not None)
        diag = []
        for t in out:
            if t is None:
                continue
            bad = np.argwhere(t.latency_ns != lat)
            diag.append({"lat_bad": int(len(bad)), "loss_bad": int((t.packet_loss.view(np.uint32) != loss.view(np.uint32)).sum()),
                         "rows": sorted(set(int(x) for x in bad[:, 0]))[:8], "cols": sorted(set(int(x) for x in bad[:, 1]))[:8]})
        res.append({"case": c, "ok": bool(ok), "errors": errs, "path_kind": t0.stats["path_kind"], "diag": diag})
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
