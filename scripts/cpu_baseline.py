#!/usr/bin/env python3
"""CPU reference throughput for the headline metric (the reference publishes no
numbers and neither Java nor Spark runs here, so the CPU point is a torch-CPU normal-equation
pipeline on the same synthetic shape, labelled as such): rows/s of one f64 normal-equation
``LinearRegression`` fit — XᵀX, Xᵀy, column sums, Cholesky solve — over n x 32 f32 features on
the host's cores (the box's CPU share: 16 threads).

    OMP_NUM_THREADS=16 python scripts/cpu_baseline.py [--rows 2e7] [--reps 3]
"""
from __future__ import annotations

import argparse
import json
import os
import time


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=2e7)
    ap.add_argument("--d", type=int, default=32)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16")))
    a = ap.parse_args(argv)
    import torch

    torch.set_num_threads(a.threads)
    n, d = int(a.rows), a.d
    g = torch.Generator().manual_seed(3)
    X = torch.randn(n, d, generator=g, dtype=torch.float32)
    beta = torch.linspace(-2, 2, d)
    y = X @ beta + 0.5 + 0.1 * torch.randn(n, generator=g)

    def fit():
        Xd = X.to(torch.float64)
        yd = y.to(torch.float64)
        G = Xd.T @ Xd
        b = Xd.T @ yd
        s = Xd.sum(0)
        sy = yd.sum()
        # centered normal equations with intercept (Spark's fitIntercept standardization path)
        mu, my = s / n, sy / n
        A = G / n - torch.outer(mu, mu)
        rhs = b / n - mu * my
        coef = torch.linalg.solve(A + 1e-12 * torch.eye(d, dtype=torch.float64), rhs)
        return coef, my - mu @ coef

    fit()
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        coef, icpt = fit()
        ts.append(time.perf_counter() - t0)
    t = sorted(ts)[len(ts) // 2]
    print(json.dumps({"metric": "rows/sec LinearRegression.fit (torch CPU f64 normal equations, reference point)",
                      "rows": n, "d": d, "threads": a.threads, "s_per_fit": t, "rows_per_s": n / t,
                      "coef_max_abs_err": float((coef.float() - beta).abs().max()), "intercept": float(icpt)}))


if __name__ == "__main__":
    main()
