#!/usr/bin/env python3
"""Host issue time vs device time of one asynchronous ``LinearRegression.fit`` (SURVEY §7e.6:
at small d a fit is ~0.13 ms of HBM streaming per 1.25e7-row shard, so host overhead decides
strong scaling).  For each row count: the time to ISSUE K fits (no synchronisation), the time
until they complete, and the per-fit host cost measured on a tiny table (device time ~0).

    python scripts/host_overhead.py [--rows 1.25e7,1e5] [--steps 200]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="1.25e7,1e5")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--d", type=int, default=32)
    a = ap.parse_args(argv)
    import torch

    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, SparkSession
    from net.jgp.labs.sparkdq4ml_amd.parallel import comm

    comm.init()
    spark = SparkSession.builder().master("mi355x[*]").config("dq4ml.fit.async", "true").getOrCreate()
    dev = spark.device
    for r in a.rows.split(","):
        n = int(float(r))
        g = torch.Generator(device=dev).manual_seed(5)
        X = torch.randn(a.d, n, generator=g, device=dev).to(torch.bfloat16)
        y = torch.linspace(-1, 1, a.d, device=dev) @ X.float() + 0.5
        df = spark.createDataFrame({"features": X, "label": y})
        lr = LinearRegression(solver="normal", gramDtype="bf16")
        for _ in range(10):
            m = lr.fit(df)
        m.coefficients  # noqa: B018 (sync)
        torch.cuda.synchronize()
        prof = os.environ.get("HOSTOV_PROFILE")  # write a cProfile summary of the issue loop here
        if prof:
            import cProfile
            import io
            import pstats

            pr = cProfile.Profile()
            pr.enable()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            m = lr.fit(df)
        t1 = time.perf_counter()
        if prof:
            pr.disable()
            buf = io.StringIO()
            st = pstats.Stats(pr, stream=buf)
            st.sort_stats("tottime").print_stats(45)
            st.sort_stats("cumulative").print_stats(60)
            with open(f"{prof}.{n}.txt", "w") as f:
                f.write(buf.getvalue())
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(json.dumps({"rows": n, "steps": a.steps, "issue_us_per_fit": (t1 - t0) / a.steps * 1e6,
                          "total_us_per_fit": (t2 - t0) / a.steps * 1e6,
                          "forced_collectives": os.environ.get("DQ4ML_FORCE_COLLECTIVES", "0")}), flush=True)
    comm.shutdown()


if __name__ == "__main__":
    main()
