"""Host<->HBM transfer rates on the GPU box (design input for the host entry).

Measures, for the C3 sizes (1.0 GB of edge list in, 1.2 GB of routing table out):
pageable vs pinned H2D / D2H through torch (hipMemcpyAsync), and the cost of pinning an
existing pageable buffer (hipHostRegister) -- the options a host entry has when the caller's
buffers are ordinary Rust Vecs.
"""
import json
import time

import numpy as np
import torch


def rate(fn, nbytes, reps=3):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return {"ms": round(best * 1e3, 2), "GBps": round(nbytes / best / 1e9, 2)}


def main():
    dev = torch.device("cuda", 0)
    out = {}
    for name, nb in (("edges_1GB", 10**9), ("table_1.2GB", 12 * 10**8)):
        n = nb // 4
        host = np.ones(n, dtype=np.float32)
        th = torch.from_numpy(host)
        d = torch.empty(n, dtype=torch.float32, device=dev)
        pin = torch.empty(n, dtype=torch.float32, pin_memory=True)
        pin.fill_(1.0)
        r = {}
        r["h2d_pageable"] = rate(lambda: d.copy_(th, non_blocking=False), nb)
        r["h2d_pinned"] = rate(lambda: d.copy_(pin, non_blocking=True), nb)
        r["d2h_pageable"] = rate(lambda: th.copy_(d, non_blocking=False), nb)
        r["d2h_pinned"] = rate(lambda: pin.copy_(d, non_blocking=True), nb)
        # pin the existing pageable buffer in place
        cr = torch.cuda.cudart()
        t0 = time.perf_counter()
        rc = cr.cudaHostRegister(th.data_ptr(), nb, 0)
        t1 = time.perf_counter()
        r["host_register_ms"] = round((t1 - t0) * 1e3, 2)
        r["host_register_rc"] = int(rc) if not isinstance(rc, tuple) else int(rc[0])
        r["h2d_registered"] = rate(lambda: d.copy_(th, non_blocking=True), nb)
        r["d2h_registered"] = rate(lambda: th.copy_(d, non_blocking=True), nb)
        t0 = time.perf_counter()
        cr.cudaHostUnregister(th.data_ptr())
        r["host_unregister_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
        # host memcpy pageable -> pinned (bounce-buffer cost), single thread
        t0 = time.perf_counter()
        pin.numpy()[:] = host
        r["host_memcpy_GBps_1thr"] = round(nb / (time.perf_counter() - t0) / 1e9, 2)
        out[name] = r
        del d, pin, th, host
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
