"""The byte-parallel cutter's field converter (``csv_swar_field16``, ops/csrc/hip/csv_parse_dev.h)
against the byte-walking fast path (``csv_field_fast``): same accepted set, same bits, over 4.2 M
random fields of 1-16 bytes (the device header compiled as host C++ with clang)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = "/opt/rocm/lib/llvm/bin/clang++"


@pytest.mark.skipif(not os.path.exists(CLANG) and shutil.which("clang++") is None, reason="needs clang++")
def test_swar16_matches_fast_path(tmp_path):
    cc = CLANG if os.path.exists(CLANG) else "clang++"
    exe = str(tmp_path / "swar16")
    r = subprocess.run([cc, "-O2", "-std=c++17", "-I", os.path.join(ROOT, "net/jgp/labs/sparkdq4ml_amd/ops/csrc/hip"),
                        os.path.join(ROOT, "tests/native/swar16_check.cpp"), "-o", exe],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    run = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert run.returncode == 0, run.stdout[-3000:]
    assert "swar16 ok" in run.stdout
