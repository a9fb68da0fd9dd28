"""In-process A/B of the asynchronous fit tail: serial vs side-stream overlap
(``dq4ml.fit.overlapTail``), alternating rounds so clocks/thermal drift hit both equally."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from net.jgp.labs.sparkdq4ml_amd import LinearRegression, SparkSession  # noqa: E402

n = int(float(os.environ.get("N", "1.25e7")))
steps = int(os.environ.get("STEPS", "30"))
spark = SparkSession.builder().master("mi355x[*]").config("dq4ml.fit.async", "true").getOrCreate()
X = torch.randn(32, n, device="cuda").to(torch.bfloat16)
y = torch.randn(n, device="cuda")
df = spark.createDataFrame({"features": X, "label": y})
lr = LinearRegression(solver="normal", gramDtype="bf16")
res = {"false": [], "true": []}
for rnd in range(6):
    for mode in ("false", "true"):
        spark.conf.set("dq4ml.fit.overlapTail", mode)
        for _ in range(3):
            lr.fit(df)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            m = lr.fit(df)
        torch.cuda.synchronize()
        res[mode].append((time.perf_counter() - t0) / steps * 1e6)
        m.coefficients
for mode, v in res.items():
    v = sorted(v)
    print(f"n={n} overlapTail={mode}: median {v[len(v) // 2]:.1f} us  min {v[0]:.1f}  max {v[-1]:.1f}")
