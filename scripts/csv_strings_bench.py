#!/usr/bin/env python3
"""Device vs host scan of a CSV with string, quoted and timestamp columns (round 4: device string
columns, ``csv_scan.h`` kind 4; timestamps, kind 5).  One file of ``--rows`` rows
``id,name,x,ts,"q"``; per variant the wall time of ``load`` (the eager scan: types + columns),
of building the string column's Python values on first read, and of a re-read of the cached file
(the type hint: one pass).  Prints one JSON line.

    python scripts/csv_strings_bench.py [--rows 1e7]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def make_csv(path: str, n: int):
    import numpy as np

    rng = np.random.default_rng(3)
    names = [b'plain', b'"a,b"', b'"x""y"', b'caf\xc3\xa9', b'"p\\"q"', b'', b'word', b'"12"']
    block = []
    for i in range(1000):
        ts = b"2019-%02d-%02d %02d:%02d:%02d" % (1 + i % 12, 1 + i % 28, i % 24, i % 60, (7 * i) % 60)
        block.append(b"%d,%s,%.4f,%s,\"%.2f\"" % (i, names[i % len(names)], rng.normal(), ts, rng.normal() * 10))
    reps = max(1, n // 1000)
    with open(path, "wb") as f:
        body = b"\r".join(block)
        for k in range(reps):
            f.write(body if k == 0 else b"\r" + body)
    return reps * 1000


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1e7)
    a = ap.parse_args(argv)
    import torch

    from net.jgp.labs.sparkdq4ml_amd import SparkSession
    from net.jgp.labs.sparkdq4ml_amd.ops import csvscan
    from net.jgp.labs.sparkdq4ml_amd.runtime import filecache

    d = tempfile.mkdtemp(prefix="csvstr", dir=os.environ.get("TMPDIR", "/tmp"))
    p = os.path.join(d, "s.csv")
    n = make_csv(p, int(a.rows))
    nbytes = os.path.getsize(p)
    out = {"rows": n, "bytes": nbytes}
    for name, thresh in (("device", "0"), ("host", str(1 << 50))):
        s = SparkSession.getActiveSession()
        if s is not None:
            s.stop()
        filecache.clear()
        spark = SparkSession.builder().master("mi355x[*]").config("dq4ml.csv.deviceThresholdBytes", thresh).getOrCreate()
        b0 = csvscan.STATS["device_scans"]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        df = spark.read().option("inferSchema", "true").csv(p)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        col = df._plan.table.columns[1]
        vals = col.values
        t2 = time.perf_counter()
        df2 = spark.read().option("inferSchema", "true").csv(p)
        cnt = df2.count()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        out[name] = {"load_s": t1 - t0, "strings_s": t2 - t1, "reread_count_s": t3 - t2,
                     "device_scan": csvscan.STATS["device_scans"] > b0, "types": [t for _, t in df.dtypes],
                     "count": cnt, "first": vals[:3]}
        spark.stop()
        del df, df2, col, vals
    out["load_speedup"] = out["host"]["load_s"] / out["device"]["load_s"]
    print(json.dumps(out), flush=True)
    os.remove(p)
    os.rmdir(d)


if __name__ == "__main__":
    main()
