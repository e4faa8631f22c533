"""CPU tests of the multi-device go/no-go gate (shadow_amd.gate) that bench.py runs before timing a
rank group (bench_multi) -- the host logic only, with stand-in builders (no GPU).  The reference's
contract it enforces: a table is whole or an error (mod.rs:219)."""
import numpy as np
import pytest

from shadow_amd import gate
from shadow_amd.graph import PathTable


def _table(g, nodes, bump_lat=None, bump_loss=None):
    n = len(nodes)
    rng = np.random.default_rng(g.num_vertices)
    lat = rng.integers(1, 1000, size=(n, n), dtype=np.uint64)
    loss = rng.random((n, n), dtype=np.float32)
    if bump_lat:
        lat[bump_lat] += np.uint64(1)
    if bump_loss:
        loss[bump_loss] = np.nextafter(loss[bump_loss], np.float32(2))
    return PathTable(nodes, lat, loss)


@pytest.fixture(scope="module")
def cases():
    return gate.gate_cases()


def test_cases_cover_dense_symmetric_and_sparse(cases):
    names = [n for n, _ in cases]
    assert names == ["dense-random", "atlas-symmetric-fw", "sparse-ba"]
    g = dict(cases)
    assert not g["atlas-symmetric-fw"].directed and g["atlas-symmetric-fw"].num_vertices > 1024  # > 8 tiles
    sp = g["sparse-ba"]
    arcs = 2 * int((sp.src != sp.dst).sum())
    assert sp.num_vertices >= 2048 and arcs * 32 < sp.num_vertices ** 2  # choose_sparse takes it


def test_equal_builds_pass(cases):
    assert gate.compare_builds(_table, _table, cases) == (True, None)


def test_one_latency_off_fails_with_the_case_name(cases):
    def bad(g, nodes):
        return _table(g, nodes, bump_lat=(3, 7) if g.num_vertices == 3000 else None)
    ok, why = gate.compare_builds(bad, _table, cases)
    assert not ok and why.startswith("sparse-ba: latency differs") and "(1 pairs)" in why


def test_one_loss_ulp_off_fails(cases):
    def bad(g, nodes):
        return _table(g, nodes, bump_loss=(0, 1))
    ok, why = gate.compare_builds(bad, _table, cases)
    assert not ok and why.startswith("dense-random: packet_loss differs")


def test_raising_build_fails(cases):
    def boom(g, nodes):
        raise RuntimeError("hipErrorPeerAccessUnsupported")
    ok, why = gate.compare_builds(boom, _table, cases)
    assert not ok and "RuntimeError" in why and "dense-random" in why


def test_shape_mismatch_fails(cases):
    def short(g, nodes):
        return _table(g, nodes[:-1])
    ok, why = gate.compare_builds(short, _table, cases)
    assert not ok and "latency differs" in why
