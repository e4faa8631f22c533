"""CPU check of the impossible-result guard (shadow_amd/csrc/guards.h, applied by k_certify):
tests/cpp/guard_check.cpp feeds it a zeroed table (the all-zero result of round 4's value-hop race,
which must be flagged -> SRG_ERR_INTERNAL), a valid closure (must pass), an entry lowered below the
smallest edge (flagged) and unreachable entries (left to the certification).  The GPU side of the
same guard: tests/test_gpu_parity.py::test_impossible_table_is_an_error."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_guard_flags_zeroed_table(tmp_path):
    exe = tmp_path / "guard_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), os.path.join(HERE, "cpp", "guard_check.cpp")],
                   check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "ok"
