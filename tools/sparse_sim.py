"""Drive tools/sparse_sim.cpp (CPU model of the sparse sweep schedule): dump C4's in-arc CSR and
candidate source orders (batch compositions), then print row pulls per arc for each.
Exploration tool only; not product code, not a checker."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from shadow_amd import synth  # noqa: E402


def csr(e):
    m = e.src != e.dst
    s, d, w = e.src[m], e.dst[m], np.minimum(e.latency_ns[m], 2**32 - 2).astype(np.uint32)
    s2, d2 = np.concatenate([s, d]), np.concatenate([d, s])
    w2 = np.concatenate([w, w])
    o = np.argsort(d2, kind="stable")
    off = np.zeros(e.num_vertices + 1, np.uint32)
    np.add.at(off, d2 + 1, 1)
    return np.cumsum(off).astype(np.uint32), s2[o].astype(np.uint32), w2[o]


def bfs_tree_preorder(off, src, V, root):
    parent = np.full(V, -1, np.int64)
    parent[root] = root
    q = [root]
    order = []
    children = [[] for _ in range(V)]
    while q:
        nq = []
        for u in q:
            for k in range(off[u], off[u + 1]):
                v = int(src[k])
                if parent[v] < 0:
                    parent[v] = u
                    children[u].append(v)
                    nq.append(v)
        q = nq
    st = [root]
    while st:
        u = st.pop()
        order.append(u)
        st.extend(reversed(children[u]))
    return np.array(order, np.uint32)


def main():
    V = int(sys.argv[1]) if len(sys.argv) > 1 else 50000
    e = synth.barabasi_albert(V, 4, seed=V)
    off, src, w = csr(e)
    os.makedirs("/tmp/ssim", exist_ok=True)
    with open("/tmp/ssim/csr.bin", "wb") as f:
        np.array([V, len(src)], np.uint32).tofile(f)
        off.tofile(f)
        src.tofile(f)
        w.tofile(f)
    exe = "/tmp/ssim/sim"
    subprocess.check_call(["g++", "-O3", "-march=native", "-std=c++17", "-o", exe, os.path.join(ROOT, "tools/sparse_sim.cpp")])
    deg = np.diff(off)
    orders = {
        "identity": np.arange(V, dtype=np.uint32),
        "random": np.random.default_rng(1).permutation(V).astype(np.uint32),
        "bfs_preorder": bfs_tree_preorder(off, src, V, int(np.argmax(deg))),
        "degree_desc": np.argsort(-deg, kind="stable").astype(np.uint32),
    }
    maxw = int(w.max())
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    divs = [int(x) for x in (sys.argv[3].split(",") if len(sys.argv) > 3 else ["1"])]
    names = sys.argv[4].split(",") if len(sys.argv) > 4 else list(orders)
    for name in names:
        o = orders[name]
        o.tofile("/tmp/ssim/order.bin")
        for div in divs:
            r = subprocess.run([exe, "/tmp/ssim/csr.bin", "/tmp/ssim/order.bin", str(maxw // div), str(nb), "61", os.environ.get("PER_LANE", "0"),
                                os.environ.get("GS_ACT", "0"), os.environ.get("LANES", "64"), os.environ.get("HUBS", "0")],
                               capture_output=True, text=True)
            print(name, "delta=max/%d" % div, r.stdout.strip(), flush=True)


if __name__ == "__main__":
    main()
