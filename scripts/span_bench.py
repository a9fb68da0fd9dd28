#!/usr/bin/env python3
"""``filter(col = 'text')`` over a device string column (``csv_span_eq``: the spans' bytes are
compared in HBM, the column's strings are never built) on the csv_strings_bench file
(``id,name,x,ts,"q"``, ``--rows`` rows).  The file is loaded once; each repetition re-runs the
filter + count action.  Prints one JSON line with ms per action.

    python scripts/span_bench.py [--rows 1e7] [--reps 10]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1e7)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args(argv)
    import torch

    from csv_strings_bench import make_csv
    from net.jgp.labs.sparkdq4ml_amd import SparkSession, col

    path = os.path.join(os.environ.get("TMPDIR", tempfile.gettempdir()), f"dq4ml_span_{int(a.rows)}.csv")
    n = make_csv(path, int(a.rows))
    spark = SparkSession.builder().master("mi355x[*]").config("dq4ml.csv.deviceThresholdBytes", "0").getOrCreate()
    df = spark.read().option("inferSchema", "true").csv(path)
    want = df.filter(col("_c1") == "word").count()  # warm-up (and the kernel's first launch)
    torch.cuda.synchronize()
    prof = None
    if os.environ.get("SPAN_PROFILE"):  # host-side cProfile of the timed actions
        import cProfile

        prof = cProfile.Profile()
        prof.enable()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        got = df.filter(col("_c1") == "word").count()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / a.reps
    if prof is not None:
        import pstats

        prof.disable()
        pstats.Stats(prof).sort_stats("cumulative").print_stats(35)
    print(json.dumps({"rows": n, "matches": int(got), "ms_per_action": round(ms, 4), "csv_bytes": os.path.getsize(path),
                      "check": int(got) == int(want)}), flush=True)
    spark.stop()


if __name__ == "__main__":
    main()
