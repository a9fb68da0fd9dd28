"""f64 Gram statistics throughput (Spark-parity dtype) for small d: skinny VALU vs MFMA path."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from net.jgp.labs.sparkdq4ml_amd.ops import device  # noqa: E402

n = int(float(os.environ.get("N", "1e8")))
for d in (1, 2, 4, 8, 9, 16, 32):
    X = torch.randn(d, n, device="cuda", dtype=torch.float64)
    y = torch.randn(n, device="cuda", dtype=torch.float64)
    for _ in range(2):
        device.gram_stats(X, y, None, None, "fp64")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        device.gram_stats(X, y, None, None, "fp64")
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 5 * 1e3
    gb = (d + 1) * n * 8 / 1e9
    print(f"d={d:3d} n={n:.0e}: {ms:8.3f} ms  {gb / ms:6.2f} TB/s", flush=True)
    del X, y
