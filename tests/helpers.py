"""Shared helpers for the routing tests (fixture loading, KAT graph text)."""
import json
import os

import numpy as np

from shadow_amd.graph import Edges

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_vectors():
    with open(os.path.join(GOLDEN, "routing_vectors.json")) as f:
        return json.load(f)["fixtures"]


def load_kats():
    with open(os.path.join(GOLDEN, "reference_kats.json")) as f:
        return json.load(f)


def fixture_edges(fx):
    return Edges(fx["num_vertices"], fx["src"], fx["dst"], np.array([int(x) for x in fx["latency_ns"]], dtype=np.uint64),
                 np.array(fx["packet_loss_bits"], dtype=np.uint32).view(np.float32), directed=fx["directed"])


def fixture_expect(fx):
    n = len(fx["nodes"])
    lat = np.array([int(x) for x in fx["expect_latency_ns"]], dtype=np.uint64).reshape(n, n)
    loss = np.array(fx["expect_packet_loss_bits"], dtype=np.uint32).reshape(n, n)
    return lat, loss


def kat_gml(directed):
    g = load_kats()["test_shortest_path"]["graph"]
    lines = ["graph [", f"  directed {1 if directed else 0}"]
    for v in g["nodes"]:
        lines += ["  node [", f"    id {v}", "  ]"]
    for s, t, lat in g["edges"]:
        lines += ["  edge [", f"    source {s}", f"    target {t}", f"    latency \"{lat}\"", "  ]"]
    lines.append("]")
    return "\n".join(lines)


def edge_gml(latency=None, packet_loss=None, jitter=None, extra=""):
    """Two-node graph whose 0->1 edge carries the given raw attribute tokens."""
    attrs = []
    if latency is not None:
        attrs.append(f"    latency {latency}")
    if jitter is not None:
        attrs.append(f"    jitter {jitter}")
    if packet_loss is not None:
        attrs.append(f"    packet_loss {packet_loss}")
    body = "\n".join(attrs)
    return (f"graph [\n  node [\n    id 0\n  ]\n  node [\n    id 1\n  ]\n"
            f"  edge [\n    source 0\n    target 1\n{body}\n  ]\n{extra}]\n")


def bits_equal(a, b):
    return np.array_equal(np.asarray(a, dtype=np.float32).view(np.uint32), np.asarray(b, dtype=np.float32).view(np.uint32))
