"""The fused FW step (shadow_amd/csrc/fw_step.hip.h): one launch per pivot carrying the pivot's bulk and
the next pivot's chain (line w.r.t. the pivot, exchange, closure, line w.r.t. itself).  It must give
the same bytes as the two-stream schedule (SRG_OPT_FW_STEP = 0) and the oracle: on one rank, on the
u64 keys, at every line split and bulk split, and with several in-process ranks exchanging their line
segments inside the launch (a child process whose ranks each get a hardware queue)."""
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


def build(e, nodes, step, split=0, env=None, monkeypatch=None):
    r = Router(0)
    r.set_option(N.SRG_OPT_FW_STEP, step)
    if split:
        r.set_option(N.SRG_OPT_FW_LINE_SPLIT, split)
    if env and monkeypatch:
        for k, v in env.items():
            monkeypatch.setenv(k, v)
    t = r.compute_shortest_paths(e, nodes)
    if env and monkeypatch:
        for k in env:
            monkeypatch.delenv(k)
    r.close()
    return t


@pytest.mark.parametrize("kw", [dict(V=300, dens=0.1, seed=201, lat_hi=40, parallel=0.1),
                                dict(V=1000, dens=0.05, seed=202),
                                dict(V=777, dens=0.2, seed=203, lat_lo=2 ** 31, lat_hi=2 ** 33)],
                         ids=["ties", "v1000", "u64"])
@pytest.mark.parametrize("sb", ["1", "2"])
def test_fused_one_rank_matches_two_stream(kw, sb, monkeypatch):
    kw = dict(kw)
    V, dens, seed = kw.pop("V"), kw.pop("dens"), kw.pop("seed")
    e = synth.random_graph(V, dens, seed, **kw)
    nodes = np.random.default_rng(seed).permutation(V).tolist()
    t0 = build(e, nodes, 0)
    t1 = build(e, nodes, 1, env={"SRG_FW_SB": sb}, monkeypatch=monkeypatch)
    assert t1.stats["path_kind"] == t0.stats["path_kind"]
    assert np.array_equal(t1.latency_ns, t0.latency_ns) and bits_equal(t1.packet_loss, t0.packet_loss)
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), nodes)
    assert np.array_equal(t1.latency_ns, lat) and bits_equal(t1.packet_loss, loss)


@pytest.mark.parametrize("split", [2, 4])
def test_fused_atlas_line_splits(split):
    """An atlas-like complete graph (multi-hop shortest paths, many pivots) at both line splits."""
    e = synth.atlas_like(2048, seed=31)
    nodes = list(range(2048))
    t0 = build(e, nodes, 0)
    t1 = build(e, nodes, 1, split=split)
    assert np.array_equal(t1.latency_ns, t0.latency_ns) and bits_equal(t1.packet_loss, t0.packet_loss)
    rows = [0, 777, 2047]
    lat, loss = oracle.compute_shortest_paths(e.as_tuple(), nodes, rows=rows, mode=2)
    assert np.array_equal(t1.latency_ns[rows], lat) and bits_equal(t1.packet_loss[rows], loss)


def test_fused_device_exchange_ranks():
    """2-4 in-process ranks on one GPU, line segments exchanged device-side (peer stores + arrival
    flags) inside the fused launch and by the two-stream chain's exchange launch: every rank bit-exact
    vs the one-rank build and the oracle."""
    env = dict(os.environ)
    env["GPU_MAX_HW_QUEUES"] = "16"
    p = subprocess.run([sys.executable, "-u", os.path.join(HERE, "fw_step_ranks.py")], env=env, capture_output=True,
                       text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    bad = [(r["case"], r["errors"], [(d["lat_bad"], d["loss_bad"], d["rows"][:4]) for d in r["diag"]]) for r in res if not r["ok"]]
    assert not bad, bad
