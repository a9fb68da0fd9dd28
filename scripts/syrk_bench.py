"""Wide exact SYRK (``gram_syrk.hip``) timing vs the library GEMM it replaced.

For each (d, n, dtype, compute): our one-pass augmented SYRK (``device.gram_stats``) against
``X @ X.T`` on hipBLAS in the same precision (a full square GEMM, without the side sums), CUDA
events, median of REPS after a warm-up.  Prints one JSON line per case."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from net.jgp.labs.sparkdq4ml_amd.ops import device  # noqa: E402

REPS = int(os.environ.get("REPS", "5"))
CASES = os.environ.get("CASES", "4096:1000000:f64:fp64,1024:4000000:f64:fp64,256:20000000:f64:fp64,"
                                "4096:1000000:f32:fp32,1024:4000000:f32:fp32,300:10000000:f32:fp64").split(",")


def timed(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(REPS):
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


for case in CASES:
    d, n, dt, comp = case.split(":")
    d, n = int(d), int(n)
    dtype = {"f64": torch.float64, "f32": torch.float32, "bf16": torch.bfloat16}[dt]
    g = torch.Generator(device="cuda").manual_seed(d)
    X = torch.randn(d, n, generator=g, device="cuda", dtype=torch.float32).to(dtype)
    y = torch.randn(n, generator=g, device="cuda", dtype=torch.float64)
    ours = timed(lambda: device.gram_stats(X, y, None, None, comp))
    lib_dt = torch.float64 if comp == "fp64" else torch.float32
    Xl = X.to(lib_dt)
    lib = timed(lambda: Xl @ Xl.t())
    useful = float(n) * d * (d + 1)  # upper triangle, 2 flop per MAC
    print(json.dumps({"d": d, "n": n, "x": dt, "compute": comp, "ours_ms": ours, "hipblas_full_gemm_ms": lib,
                      "ours_useful_tflops": useful / ours / 1e9, "speedup_vs_hipblas": lib / ours}), flush=True)
    del X, Xl, y
    torch.cuda.empty_cache()
