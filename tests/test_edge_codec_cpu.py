"""CPU check of the sequential-pair H2D encoder (shadow_amd/csrc/edge_codec.h, used by
routing.hip codec_in): tests/cpp/edge_codec_roundtrip.cpp encodes complete-graph edge lists in
both GML orders and with gaps, split into worker slices and chunks as codec_in splits them,
decodes them with k_decode_seq's formula and compares; a shuffled list must report "dense"."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


CLANG = "/opt/rocm/lib/llvm/bin/clang++"


# clang++ builds the product's encoder (one fused vector pass, non-temporal ring stores: what
# hipcc compiles into the library); g++ the portable block form
@pytest.mark.parametrize("cxx", ["g++", CLANG])
def test_sequential_pair_encoder_roundtrip(tmp_path, cxx):
    if shutil.which(cxx) is None and not os.path.exists(cxx):
        pytest.skip(f"{cxx} not available")
    exe = tmp_path / "edge_codec_roundtrip"
    subprocess.run([cxx, "-O2", "-std=c++17", "-o", str(exe), os.path.join(HERE, "cpp", "edge_codec_roundtrip.cpp")],
                   check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("ok ")
