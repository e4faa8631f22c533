"""Seeded synthetic graphs for the benchmark / parity configs (BASELINE.json).

All generators return a shadow_amd.Edges in GML edge order: every node's self-loop first
(Shadow requires exactly one per used node, mod.rs:215-216), then the other edges.
numpy PCG64 (np.random.default_rng(seed)) is the generator; streams are consumed in a fixed
order so a (config, seed) pair always yields the same graph.

  C1  complete_random(1000, seed=1001)    lat U{1e6..1e8} ns, loss 50% 0.0 else U(0, 0.05)
  C2  atlas_like(4096, seed=4096)         points on a sphere, lat = round(1e6*(2+d_km/100)*U(0.9,1.6))
  C3  atlas_like(10000, seed=10000)       same generator, 10k vertices (the bench workload)
  C4  barabasi_albert(50000, 4, seed=50000)  sparse, avg degree ~8, lat U{1e6..5e7}
"""
import numpy as np

from .graph import Edges

EARTH_RADIUS_KM = 6371.0


def _selfloops(V, rng, lo=500_000, hi=5_000_000, fixed=None):
    src = np.arange(V, dtype=np.uint32)
    if fixed is not None:
        lat = np.full(V, fixed, dtype=np.uint64)
    else:
        lat = rng.integers(lo, hi + 1, size=V, dtype=np.uint64)
    return src, src.copy(), lat, np.zeros(V, dtype=np.float32)


def _loss(rng, m, p_zero, hi):
    u = rng.random(m)
    v = rng.uniform(0.0, hi, size=m).astype(np.float32)
    return np.where(u < p_zero, np.float32(0.0), v).astype(np.float32)


def complete_random(V=1000, seed=1001, lat_lo=1_000_000, lat_hi=100_000_000, loss_hi=0.05):
    """C1: complete undirected graph with uniform random latency / loss."""
    rng = np.random.default_rng(seed)
    s0, d0, l0, p0 = _selfloops(V, rng)
    iu, ju = np.triu_indices(V, 1)
    m = len(iu)
    lat = rng.integers(lat_lo, lat_hi + 1, size=m, dtype=np.uint64)
    loss = _loss(rng, m, 0.5, loss_hi)
    return Edges(V, np.concatenate([s0, iu.astype(np.uint32)]), np.concatenate([d0, ju.astype(np.uint32)]),
                 np.concatenate([l0, lat]), np.concatenate([p0, loss]), directed=False)


def atlas_like(V=4096, seed=4096, p_zero=0.7, loss_hi=0.01):
    """C2/C3: Tor-atlas-like complete graph; multiplicative noise violates the triangle
    inequality so some shortest paths are multi-hop (about 12-15% of direct edges are
    shortest paths at V=800-1600)."""
    rng = np.random.default_rng(seed)
    s0, d0, l0, p0 = _selfloops(V, rng)
    z = rng.normal(size=(V, 3))
    z /= np.linalg.norm(z, axis=1, keepdims=True)
    m = V * (V - 1) // 2
    src = np.empty(m, dtype=np.uint32)
    dst = np.empty(m, dtype=np.uint32)
    lat = np.empty(m, dtype=np.uint64)
    loss = np.empty(m, dtype=np.float32)
    k = 0
    for i in range(V - 1):
        j = np.arange(i + 1, V)
        c = np.clip(z[j] @ z[i], -1.0, 1.0)
        d_km = EARTH_RADIUS_KM * np.arccos(c)
        noise = rng.uniform(0.9, 1.6, size=len(j))
        lat[k:k + len(j)] = np.round(1e6 * (2.0 + d_km / 100.0) * noise).astype(np.uint64)
        loss[k:k + len(j)] = _loss(rng, len(j), p_zero, loss_hi)
        src[k:k + len(j)] = i
        dst[k:k + len(j)] = j
        k += len(j)
    return Edges(V, np.concatenate([s0, src]), np.concatenate([d0, dst]), np.concatenate([l0, lat]),
                 np.concatenate([p0, loss]), directed=False)


def barabasi_albert(V=50000, m=4, seed=50000, lat_lo=1_000_000, lat_hi=50_000_000, loss_hi=0.02):
    """C4: preferential attachment (each new vertex links to m distinct earlier vertices
    chosen proportionally to degree, networkx-style repeated-nodes list), undirected."""
    rng = np.random.default_rng(seed)
    s0, d0, l0, p0 = _selfloops(V, rng, fixed=1_000_000)
    E = (V - m) * m
    src = np.empty(E, dtype=np.uint32)
    dst = np.empty(E, dtype=np.uint32)
    repeated = np.empty(2 * E, dtype=np.int64)  # endpoint multiset (degree-proportional)
    nrep = 0
    targets = list(range(m))
    k = 0
    for v in range(m, V):
        src[k:k + m] = v
        dst[k:k + m] = targets
        k += m
        repeated[nrep:nrep + m] = targets
        repeated[nrep + m:nrep + 2 * m] = v
        nrep += 2 * m
        chosen = set()
        while len(chosen) < m:
            chosen.add(int(repeated[rng.integers(0, nrep)]))
        targets = sorted(chosen)
    lat = rng.integers(lat_lo, lat_hi + 1, size=E, dtype=np.uint64)
    loss = _loss(rng, E, 0.5, loss_hi)
    return Edges(V, np.concatenate([s0, src]), np.concatenate([d0, dst]), np.concatenate([l0, lat]),
                 np.concatenate([p0, loss]), directed=False)


def random_graph(V, density, seed, directed=False, lat_lo=1, lat_hi=1000, loss_hi=0.3, p_zero=0.3,
                 parallel=0.0, selfloops=True):
    """Small random graphs for parity tests (parallel edges, ties with small lat ranges)."""
    rng = np.random.default_rng(seed)
    src, dst = [], []
    if selfloops:
        src += list(range(V))
        dst += list(range(V))
    mask = rng.random((V, V)) < density
    np.fill_diagonal(mask, False)
    if not directed:
        mask = np.triu(mask, 1)
    ii, jj = np.nonzero(mask)
    src += ii.tolist()
    dst += jj.tolist()
    npar = int(parallel * len(ii))
    if npar:
        pick = rng.integers(0, len(ii), size=npar)
        src += ii[pick].tolist()
        dst += jj[pick].tolist()
    E = len(src)
    lat = rng.integers(lat_lo, lat_hi + 1, size=E, dtype=np.uint64)
    loss = _loss(rng, E, p_zero, loss_hi)
    if selfloops:
        loss[:V] = _loss(rng, V, 0.5, loss_hi)
    return Edges(V, np.asarray(src, dtype=np.uint32), np.asarray(dst, dtype=np.uint32), lat, loss,
                 directed=directed)


def to_gml(edges, bandwidth="1 Gbit", node_ids=None):
    """GML text for an edge list (latency as "<n> ns", packet_loss as a float token)."""
    V = edges.num_vertices
    ids = node_ids if node_ids is not None else (edges.node_ids if edges.node_ids is not None else range(V))
    ids = [int(x) for x in ids]
    out = ["graph [", f"  directed {1 if edges.directed else 0}"]
    for i in range(V):
        out.append(f"  node [\n    id {ids[i]}\n    host_bandwidth_up \"{bandwidth}\"\n"
                   f"    host_bandwidth_down \"{bandwidth}\"\n  ]")
    for s, d, l, p in zip(edges.src.tolist(), edges.dst.tolist(), edges.latency_ns.tolist(),
                          edges.packet_loss.tolist()):
        ps = "%.9g" % p
        if "." not in ps and "e" not in ps and "inf" not in ps:
            ps += ".0"  # an int token would be a parse error ("not a float", mod.rs:96)
        out.append(f"  edge [\n    source {ids[s]}\n    target {ids[d]}\n    latency \"{l} ns\"\n"
                   f"    packet_loss {ps}\n  ]")
    out.append("]")
    return "\n".join(out) + "\n"
