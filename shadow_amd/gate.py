"""Go/no-go gate for a multi-device build before anything is timed.

The reference returns a whole table or an error (``assert_eq!(paths.len(), nodes.len().pow(2))``,
``src/main/network/graph/mod.rs:219``); a multi-device schedule that produced a wrong table would
otherwise still print a number.  ``compare_builds`` runs small builds through the multi-device
router and through one GPU and accepts the multi-device path only if every case agrees bit for bit
(latency and loss) and neither raises.  The cases cover the three schedules a rank group runs: the
general dense FW, the symmetric line-buffer FW with its per-pivot exchange, and the sparse path.
Pure host logic: the CPU tests drive it with stand-in builders.
"""
import numpy as np


def gate_cases():
    from . import synth
    return [
        ("dense-random", synth.random_graph(300, 0.05, 1234, lat_hi=1000)),
        ("atlas-symmetric-fw", synth.atlas_like(1200, seed=12)),
        ("sparse-ba", synth.barabasi_albert(3000, 4, seed=3000)),
    ]


def compare_builds(build_multi, build_single, cases):
    """build_*(edges, nodes) -> object with ``latency_ns`` (uint64 n x n) and ``packet_loss``
    (float32 n x n).  Returns (True, None) or (False, reason)."""
    for name, g in cases:
        nodes = np.arange(g.num_vertices, dtype=np.uint32)
        try:
            got = build_multi(g, nodes)
            ref = build_single(g, nodes)
        except Exception as e:  # noqa: BLE001 -- any failure is a no-go, reported by name
            return False, f"{name}: {type(e).__name__}: {e}"
        gl, rl = np.asarray(got.latency_ns), np.asarray(ref.latency_ns)
        if gl.shape != rl.shape or not np.array_equal(gl, rl):
            bad = int((gl != rl).sum()) if gl.shape == rl.shape else -1
            return False, f"{name}: latency differs from the single-GPU build ({bad} pairs)"
        gp = np.asarray(got.packet_loss, dtype=np.float32).view(np.uint32)
        rp = np.asarray(ref.packet_loss, dtype=np.float32).view(np.uint32)
        if gp.shape != rp.shape or not np.array_equal(gp, rp):
            bad = int((gp != rp).sum()) if gp.shape == rp.shape else -1
            return False, f"{name}: packet_loss differs from the single-GPU build ({bad} pairs)"
    return True, None
