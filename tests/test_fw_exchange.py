"""The symmetric line-buffer FW's per-pivot hand-offs (routing.hip SymFw, xchg.hip.h):
  * the two cross-stream hops per pivot (value hops: one-wave set / wait kernels on signal memory,
    the default for a context alone on its device; or events, SRG_STREAM_HOPS=events) must give the
    same bytes, on the FW after the H2D and beside it;
  * the chain's device-side line exchange between in-process ranks (SRG_OPT_FW_STEP = 2: peer stores +
    arrival words, k_line_xchg) must give the one-rank table, in a child process whose ranks each get
    a hardware queue;
  * SRG_OPT_FW_STEP = 1 (round 4's fused one-launch-per-pivot FW, measured slower and removed) is
    refused."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle
from shadow_amd import Router, synth
from shadow_amd import _native as N
from helpers import bits_equal

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def build(e, nodes, overlap, hops, monkeypatch):
    if hops == "events":
        monkeypatch.setenv("SRG_STREAM_HOPS", "events")
    r = Router(0)
    r.set_option(N.SRG_OPT_FW_OVERLAP, overlap)
    try:
        return r.compute_shortest_paths(e, nodes)
    finally:
        r.close()
        monkeypatch.delenv("SRG_STREAM_HOPS", raising=False)


@pytest.mark.parametrize("overlap", [1, 0])
def test_value_hops_match_event_hops(overlap, monkeypatch):
    """An atlas-like complete graph (multi-hop shortest paths, 16 pivots): value hops vs event hops,
    bytes equal, and the oracle's rows."""
    e = synth.atlas_like(2048, seed=31)
    nodes = list(range(2048))
    tv = build(e, nodes, overlap, "values", monkeypatch)
    te = build(e, nodes, overlap, "events", monkeypatch)
    assert np.array_equal(tv.latency_ns, te.latency_ns) and bits_equal(tv.packet_loss, te.packet_loss)
    rows = [0, 777, 2047]
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), nodes, rows=rows, mode=2)
    assert np.array_equal(tv.latency_ns[rows], lat) and bits_equal(tv.packet_loss[rows], loss)


def test_fused_step_option_refused():
    r = Router(0)
    try:
        assert N.lib().srg_set_option(r._h, N.SRG_OPT_FW_STEP, 1.0) == N.SRG_ERR_ARG
        for v in (-1, 0, 2):
            assert N.lib().srg_set_option(r._h, N.SRG_OPT_FW_STEP, float(v)) == N.SRG_OK
    finally:
        r.close()


def test_device_exchange_ranks():
    """2-4 in-process ranks on one GPU, line segments exchanged device-side (peer stores + arrival
    words, k_line_xchg on the chain's stream): every rank bit-exact vs the one-rank build and the
    oracle."""
    env = dict(os.environ)
    env["GPU_MAX_HW_QUEUES"] = "16"
    p = subprocess.run([sys.executable, "-u", os.path.join(HERE, "fw_exchange_ranks.py")], env=env, capture_output=True,
                       text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    bad = [(r["case"], r["errors"], [(d["lat_bad"], d["loss_bad"], d["rows"][:4]) for d in r["diag"]]) for r in res if not r["ok"]]
    assert not bad, bad
