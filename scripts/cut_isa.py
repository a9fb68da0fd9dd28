"""Dump the generated wide-row cutter kernel (ops/scancut.py) of the BASELINE shape and its gfx950
ISA on the CPU, for instruction counting of the field-conversion loop.

    python scripts/cut_isa.py --features 32 --out /tmp/cut32   # -> cut32.hip, cut32.s
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--features", type=int, default=32)
    ap.add_argument("--max-line", type=int, default=0, help="default: 10 bytes per field")
    ap.add_argument("--out", default="/tmp/cut")
    a = ap.parse_args(argv)
    from test_scancut_codegen import _cut_source

    from net.jgp.labs.sparkdq4ml_amd import SparkSession

    spark = SparkSession.builder().master("local[1]").getOrCreate()
    src = _cut_source(spark, a.features, False, max_line=a.max_line or None)
    with open(a.out + ".hip", "w") as f:
        f.write("#include <hip/hip_runtime.h>\n" + src)
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only",
                        "-S", a.out + ".hip", "-o", a.out + ".s"], capture_output=True, text=True)
    if r.returncode:
        print(r.stderr[-4000:])
        return 1
    print(a.out + ".s")
    return 0


if __name__ == "__main__":
    sys.exit(main())
