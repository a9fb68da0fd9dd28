"""Host runtime library under AddressSanitizer + UndefinedBehaviorSanitizer: the
C++ solvers, WLS driver and CSV scanner are compiled together with a native self-test and run
here on the CPU (GPU ASan / xnack are not available on this pool, so sanitizers cover host code)."""
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "net", "jgp", "labs", "sparkdq4ml_amd", "ops", "csrc", "host")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_library_under_asan_ubsan(tmp_path):
    srcs = [s for s in glob.glob(os.path.join(HOST, "*.cpp")) if not s.endswith("module.cpp")]
    exe = str(tmp_path / "host_selftest")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", "-I", HOST, os.path.join(ROOT, "tests", "native", "host_selftest.cpp"),
           *srcs, "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    run = subprocess.run([exe, ROOT], capture_output=True, text=True, timeout=600, env=env)
    assert run.returncode == 0, (run.stdout + run.stderr)[-4000:]
    assert "host selftest ok" in run.stdout
