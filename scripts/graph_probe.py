#!/usr/bin/env python3
"""Would a captured HIP graph shorten the strong-scaling shard's fit?  The replayed fit's Gram
pass (``TiledGramPlan.launch``: the tall bf16 kernel + its fold + the un-shift) is captured once
with ``torch.cuda.CUDAGraph`` (a hipGraph on ROCm) and replayed, against the same launches issued
directly.  Prints host issue and device time per pass for both (1.25e7 x 32 bf16 by default).

    python scripts/graph_probe.py [--rows 1.25e7] [--steps 400]
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
    ap.add_argument("--rows", type=float, default=1.25e7)
    ap.add_argument("--d", type=int, default=32)
    ap.add_argument("--steps", type=int, default=400)
    a = ap.parse_args(argv)
    import torch

    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, SparkSession

    spark = SparkSession.builder().master("mi355x[*]").config("dq4ml.fit.async", "true").getOrCreate()
    dev = spark.device
    n, d = int(a.rows), a.d
    g = torch.Generator(device=dev).manual_seed(5)
    X = torch.randn(d, n, generator=g, device=dev).to(torch.bfloat16)
    y = torch.linspace(-1, 1, d, device=dev) @ X.float() + 0.5
    df = spark.createDataFrame({"features": X, "label": y})
    lr = LinearRegression(solver="normal", gramDtype="bf16")
    for _ in range(3):
        m = lr.fit(df)
    m.coefficients  # noqa: B018 (sync)
    plan = df.__dict__["_fit_replays"][lr.uid].plan
    s = torch.cuda.Stream(dev)
    torch.cuda.synchronize()

    def direct(k):
        with torch.cuda.stream(s):
            for _ in range(k):
                plan.launch(s.cuda_stream, False)

    direct(5)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    direct(a.steps)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    res = {"direct_issue_us": 1e6 * (t1 - t0) / a.steps, "direct_us": 1e6 * (t2 - t0) / a.steps}

    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        plan.launch(s.cuda_stream, False)  # (warm the allocator on the capture stream)
    torch.cuda.synchronize()
    with torch.cuda.graph(graph, stream=s):
        out = plan.launch(torch.cuda.current_stream().cuda_stream, False)
    torch.cuda.synchronize()
    ref = plan.launch(torch.cuda.current_stream().cuda_stream, False)
    graph.replay()
    torch.cuda.synchronize()
    res["graph_matches_direct"] = bool(torch.equal(out, ref))
    for _ in range(5):
        graph.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        graph.replay()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    res.update(graph_issue_us=1e6 * (t1 - t0) / a.steps, graph_us=1e6 * (t2 - t0) / a.steps, rows=n, d=d,
               steps=a.steps)
    print(json.dumps(res), flush=True)
    spark.stop()


if __name__ == "__main__":
    sys.exit(main())
