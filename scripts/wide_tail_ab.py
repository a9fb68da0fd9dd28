#!/usr/bin/env python3
"""Same-process A/B of the asynchronous wide fit's tail stream (models/regression.py
``_WIDE_TAIL``): "high" = a high-priority side stream, "queue" = a normal-priority stream on a
hardware queue of its own (CU-masked over every CU).  Rows x 4096 fp8, alternating blocks of
fits, ms per fit per block.

    python scripts/wide_tail_ab.py [--rows 1.25e6] [--fits 20] [--reps 3]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1.25e6)
    ap.add_argument("--fits", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch

    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, SparkSession
    from net.jgp.labs.sparkdq4ml_amd.models import regression
    from net.jgp.labs.sparkdq4ml_amd.ops import device, native
    from net.jgp.labs.sparkdq4ml_amd.ops.layout import TiledWide

    spark = SparkSession.builder().master("mi355x[*]").config("dq4ml.fit.async", "true").getOrCreate()
    d, n, eb = 4096, int(a.rows), 8
    h = native.hip()
    buf = torch.empty(int(h.wide_tiled_bytes(eb, d, n)), dtype=torch.uint8, device="cuda")
    per_row = buf.numel() // (((n + 63) // 64) * 64)
    scale = torch.full((d,), 4.5 / 448.0, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(1)
    beta = torch.linspace(-1.0, 1.0, d, device="cuda")
    y = torch.empty(n, dtype=torch.float32, device="cuda")
    chunk = max(64, (int(2e8) // d) // 64 * 64)
    for r0 in range(0, n, chunk):
        r1 = min(n, r0 + chunk)
        xc = torch.randn(d, r1 - r0, generator=g, device="cuda")
        y[r0:r1] = beta @ xc + 0.5
        lo = r0 * per_row
        device.pack_wide([xc], eb, None, inv_scale=1.0 / scale, out=buf[lo:lo + ((r1 - r0 + 63) // 64) * 64 * per_row],
                         shift=None)
    df = spark.createDataFrame({"features": TiledWide(buf, d, n, eb, scale), "label": y})
    lr = LinearRegression(solver="normal", gramDtype="fp8", regParam=0.01, elasticNetParam=0.0)
    out = []
    for rep in range(a.reps):
        for mode in ("high", "queue"):
            regression._WIDE_TAIL = mode
            for _ in range(3):
                lr.fit(df)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.fits):
                m = lr.fit(df)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / a.fits * 1e3
            m.coefficients  # resolve the last fit
            out.append({"rep": rep, "tail": mode, "ms_per_fit": ms})
            print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
