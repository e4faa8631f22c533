"""CPU check of the sequential-pair H2D encoder (shadow_amd/csrc/edge_codec.h, used by
routing.hip codec_in): tests/cpp/edge_codec_roundtrip.cpp encodes complete-graph edge lists in
both GML orders and with gaps, split into worker slices and chunks as codec_in splits them,
decodes them with k_decode_seq's formula and compares; a shuffled list must report "dense"."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_sequential_pair_encoder_roundtrip(tmp_path):
    exe = tmp_path / "edge_codec_roundtrip"
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), os.path.join(HERE, "cpp", "edge_codec_roundtrip.cpp")],
                   check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("ok ")
