"""load_network_graph / read_xz / tilde_expansion (mod.rs:480-509, utility/mod.rs:223-245).
tests/golden/graph-compressed.gml is the data file of the reference's src/test/compressed-graph
test; like its CMakeLists.txt the test xz-compresses it and loads it back."""
import lzma
import os

import pytest

from shadow_amd import NetGraphError, NetworkGraph
from shadow_amd.ingest import ONE_GBIT_SWITCH_GRAPH, load_network_graph, tilde_expansion

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURE = os.path.join(HERE, "golden", "graph-compressed.gml")


def test_xz_file_roundtrip(tmp_path):
    raw = open(FIXTURE, "rb").read()
    p = tmp_path / "graph-compressed.gml.xz"
    p.write_bytes(lzma.compress(raw, format=lzma.FORMAT_XZ))
    text = load_network_graph({"type": "gml", "file": {"path": str(p), "compression": "xz"}})
    assert text == raw.decode()
    g = NetworkGraph.parse(text)
    assert g.num_nodes() == 1 and g.edges.latency_ns.tolist() == [1_000_000]


def test_plain_file_and_inline(tmp_path):
    raw = open(FIXTURE).read()
    assert load_network_graph({"type": "gml", "file": {"path": FIXTURE, "compression": None}}) == raw
    assert load_network_graph({"type": "gml", "inline": raw}) == raw
    assert load_network_graph({"type": "1_gbit_switch"}) == ONE_GBIT_SWITCH_GRAPH


def test_errors(tmp_path):
    with pytest.raises(NetGraphError, match="Failed to open file"):
        load_network_graph({"type": "gml", "file": {"path": str(tmp_path / "none.xz"), "compression": "xz"}})
    bad = tmp_path / "bad.xz"
    bad.write_bytes(b"not xz at all")
    with pytest.raises(NetGraphError, match="Failed to decompress file"):
        load_network_graph({"type": "gml", "file": {"path": str(bad), "compression": "xz"}})
    with pytest.raises(NetGraphError, match="Failed to read file"):
        load_network_graph({"type": "gml", "file": {"path": str(tmp_path / "none.gml"), "compression": None}})


def test_tilde_expansion(monkeypatch):
    monkeypatch.setenv("HOME", "/h/me")
    assert tilde_expansion("~/a/b.gml") == "/h/me/a/b.gml"
    assert tilde_expansion("~bob/g.gml") == "/home/bob/g.gml"
    assert tilde_expansion("~+/g.gml") == "~+/g.gml"
    assert tilde_expansion("/abs/g.gml") == "/abs/g.gml"
