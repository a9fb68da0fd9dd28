"""Where does a GPU LinearRegression.fit step spend host time? (cProfile + event timing)"""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from net.jgp.labs.sparkdq4ml_amd import LinearRegression, SparkSession  # noqa: E402
from net.jgp.labs.sparkdq4ml_amd.ops import device  # noqa: E402

n = int(float(os.environ.get("N", "1.25e7")))
spark = SparkSession.builder().master("mi355x[*]").getOrCreate()
X = torch.randn(32, n, device="cuda").to(torch.bfloat16)
y = torch.randn(n, device="cuda")
df = spark.createDataFrame({"features": X, "label": y})
lr = LinearRegression(solver="normal", gramDtype="bf16")
T = df._table().column("features").values
for _ in range(5):
    lr.fit(df)
torch.cuda.synchronize()


def t(fn, reps=50):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


print(f"n={n}")
print("gram_stats (launch+kernels) us", t(lambda: device.gram_stats(T, y, None, None, "bf16")))
print("gram_stats + D2H us", t(lambda: device.gram_stats(T, y, None, None, "bf16").cpu()))
print("fit us", t(lambda: lr.fit(df)))
pr = cProfile.Profile()
pr.enable()
for _ in range(50):
    lr.fit(df)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
