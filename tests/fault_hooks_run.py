"""Fault-injection regressions, run by tests/test_fw_overlap.py::test_fault_hooks_in_the_test_build in a
child process whose SRG_LIB_PATH names the TEST build of the library (libshadow_routing_testhooks.so,
compiled with -DSRG_TEST_HOOKS; the product library refuses SRG_OPT_TEST_FAULT).  Prints "ok".

1. Stale FW sync words (SRG_OPT_TEST_FAULT = 2; round 4's all-zero tables): the FW sync words hold a
   recycled allocation's nonzero values and the line buffers are zero when a build starts.  The chain
   stream must not read them before this build's reset: with the value hops on the table still equals
   the oracle, through the FW beside the H2D and through the FW after the H2D.
2. Impossible table (SRG_OPT_TEST_FAULT = 1): a closed matrix overwritten with zeros after FW (what a
   lost synchronisation produced in round 4) must fail the build with SRG_ERR_INTERNAL, never come
   back with rc = 0; the same context then builds correctly (guards.h in k_certify)."""
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import oracle  # noqa: E402
from helpers import bits_equal  # noqa: E402
from shadow_amd import HipError, Router, synth  # noqa: E402
from shadow_amd import _native as N  # noqa: E402


def captured_stderr(fn):
    """fn() with the process's fd 2 sent to a file (the library writes its diagnostics there)."""
    sys.stderr.flush()
    saved = os.dup(2)
    with tempfile.TemporaryFile(mode="w+b") as f:
        os.dup2(f.fileno(), 2)
        try:
            out = fn()
        finally:
            os.dup2(saved, 2)
            os.close(saved)
        f.seek(0)
        return out, f.read().decode(errors="replace")


def stale_sync_words(overlap):
    V = 2100
    e = synth.atlas_like(V, seed=31)
    nodes = list(range(V))

    def run():
        r = Router(0)
        r.set_option(N.SRG_OPT_FW_OVERLAP, overlap)
        r.set_option(N.SRG_OPT_TEST_FAULT, 2)
        try:
            return r.compute_shortest_paths(e, nodes)
        finally:
            r.close()

    t, err = captured_stderr(run)
    if overlap:
        assert "fw-overlap: ok=1" in err, err
    assert int((t.latency_ns == 0).sum()) == 0
    rows = [0, 1, V // 2, V - 1]
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), nodes, rows=rows, mode=2)
    assert np.array_equal(t.latency_ns[rows], lat) and bits_equal(t.packet_loss[rows], loss)


def impossible_table(overlap):
    V = 2100
    e = synth.atlas_like(V, seed=32)
    nodes = list(range(0, V, 2))
    r = Router(0)
    r.set_option(N.SRG_OPT_FW_OVERLAP, overlap)
    r.set_option(N.SRG_OPT_TEST_FAULT, 1)
    try:
        r.compute_shortest_paths(e, nodes)
        raise AssertionError("a zeroed FW matrix came back as a table")
    except HipError as ex:
        assert ex.code == N.SRG_ERR_INTERNAL and "impossible" in str(ex), str(ex)
    r.set_option(N.SRG_OPT_TEST_FAULT, 0)
    t = r.compute_shortest_paths(e, nodes)
    r.close()
    rows = [0, len(nodes) - 1]
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), nodes, rows=rows, mode=2)
    assert np.array_equal(t.latency_ns[rows], lat) and bits_equal(t.packet_loss[rows], loss)


def main():
    assert os.environ.get("SRG_LIB_PATH", "").endswith("libshadow_routing_testhooks.so")
    for ov in (1, 0):
        stale_sync_words(ov)
        print(f"stale sync words, overlap {ov}: ok", flush=True)
        impossible_table(ov)
        print(f"impossible table, overlap {ov}: ok", flush=True)
    print("ok", flush=True)


if __name__ == "__main__":
    main()
