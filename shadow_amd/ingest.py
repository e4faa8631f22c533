"""Graph source loading: the text that NetworkGraph.parse consumes.

Mirrors, on the host side of the boundary:
  load_network_graph   src/main/network/graph/mod.rs:495-509  (file / xz file / inline / built-in)
  read_xz              mod.rs:480-492  (lzma_rs::xz_decompress of the whole file, then UTF-8)
  tilde_expansion      src/main/utility/mod.rs:223-245
  ONE_GBIT_SWITCH_GRAPH  src/main/core/configuration.rs:1355-1368

`graph_options` has the shape of Shadow's `network.graph` config section (GraphOptions, serde):
    {"type": "gml", "file": {"path": "...", "compression": None | "xz"}}
    {"type": "gml", "inline": "graph [ ... ]"}
    {"type": "1_gbit_switch"}
xz decoding uses liblzma through Python's lzma module (the reference uses the lzma-rs crate,
absent here; both implement the xz container format, so the decoded bytes are identical).
"""
import lzma
import os

from . import _native as N
from .graph import NetGraphError

ONE_GBIT_SWITCH_GRAPH = """graph [
  directed 0
  node [
    id 0
    host_bandwidth_up "1 Gbit"
    host_bandwidth_down "1 Gbit"
  ]
  edge [
    source 0
    target 0
    latency "1 ms"
    packet_loss 0.0
  ]
]"""


def tilde_expansion(path):
    """utility/mod.rs:223-245: "~/x" -> $HOME/x, "~user/x" -> /home/user/x, "~+"/"~-" unchanged."""
    if path.startswith("~"):
        x = path[1:]
        prefix, _, remainder = x.partition("/")
        if prefix == "":
            home = os.environ.get("HOME")
            if home is not None:
                return os.path.join(home, remainder)
        elif prefix[0] in "+-":
            pass  # not supported
        else:
            return os.path.join("/home", prefix, remainder)
    return path


def read_xz(path):
    """mod.rs:480-492: open, xz-decompress the whole file, decode UTF-8."""
    try:
        f = open(path, "rb")
    except OSError as e:
        raise NetGraphError(N.SRG_ERR_PARSE, f'Failed to open file: "{path}": {e}') from e
    with f:
        try:
            data = lzma.LZMADecompressor(format=lzma.FORMAT_XZ).decompress(f.read())
        except lzma.LZMAError as e:
            raise NetGraphError(N.SRG_ERR_PARSE, f"Failed to decompress file: {e}") from e
    try:
        return data.decode("utf-8")
    except UnicodeDecodeError as e:
        raise NetGraphError(N.SRG_ERR_PARSE, str(e)) from e


def load_network_graph(graph_options):
    """mod.rs:495-509: the GML text of the configured graph."""
    kind = graph_options.get("type", "gml")
    if kind == "1_gbit_switch":
        return ONE_GBIT_SWITCH_GRAPH
    if kind != "gml":
        raise NetGraphError(N.SRG_ERR_ARG, f"unknown graph type {kind!r}")
    if "inline" in graph_options:
        return graph_options["inline"]
    src = graph_options["file"]
    path = tilde_expansion(src["path"])
    if src.get("compression") is None:
        try:
            with open(path, "rb") as f:
                return f.read().decode("utf-8")
        except (OSError, UnicodeDecodeError) as e:
            raise NetGraphError(N.SRG_ERR_PARSE, f"Failed to read file: {src['path']}: {e}") from e
    if src["compression"] == "xz":
        return read_xz(path)
    raise NetGraphError(N.SRG_ERR_ARG, f"unknown compression {src['compression']!r}")
