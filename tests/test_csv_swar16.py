"""The byte-parallel cutter's field converters (``csv_swar_field16``, ``csv_field_r16`` /
``csv_field_r8``, ops/csrc/hip/csv_parse_dev.h) against the byte-walking fast path
(``csv_field_fast``): same accepted set, same bits, over 4.2 M random fields of 1-16 bytes; and
the division-free m / 10^k they share (the device header compiled as host C++ with clang)."""
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


@pytest.mark.skipif(not os.path.exists(CLANG) and shutil.which("clang++") is None, reason="needs clang++")
def test_div_pow10_is_correctly_rounded(tmp_path):
    """The division-free m / 10^k of every fast-path number (m < 10^9, k <= 9) equals the IEEE
    quotient (a stride of 1.03e8 cases; the full 1e10 sweep passed offline)."""
    cc = CLANG if os.path.exists(CLANG) else "clang++"
    exe = str(tmp_path / "divp10")
    r = subprocess.run([cc, "-O2", "-ffp-contract=off", "-std=c++17", "-I",
                        os.path.join(ROOT, "net/jgp/labs/sparkdq4ml_amd/ops/csrc/hip"),
                        os.path.join(ROOT, "tests/native/div_pow10_check.cpp"), "-o", exe],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    run = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert run.returncode == 0 and "div_pow10 ok" in run.stdout, run.stdout[-3000:]
