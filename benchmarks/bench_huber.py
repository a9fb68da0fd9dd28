#!/usr/bin/env python3
"""Huber regression (``LinearRegression(loss="huber")``, Spark 2.4's L-BFGS-B over the Huber
objective): ms per fit and per cost evaluation, the device optimizer (``huber_qn.hip``: pass ->
all-reduce -> control kernel, no host read per evaluation) against the host-steered one
(``--host``: the same algorithm in ``models/lbfgsb.py``, one D2H read per evaluation).

Synthetic rows: N(0,1) features, a linear model with N(0, 0.2) noise, every 37th label shifted
by +25 (the outliers the Huber loss exists for).

    python benchmarks/bench_huber.py [--rows 1e7] [--features 16] [--dtype f32|bf16|fp8] [--host]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from harness import check_world, emit, self_launch, timed, world_info  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--rows", type=float, default=1e7, help="global rows (strong scaling)")
    ap.add_argument("--features", type=int, default=16)
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16", "fp8"])
    ap.add_argument("--max-iter", type=int, default=100)
    ap.add_argument("--host", action="store_true", help="the host-steered optimizer (dq4ml.huber.device=false)")
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args(argv)
    rc = self_launch(a.gpus, __file__, argv)
    if rc is not None:
        return rc
    import numpy as np
    import torch

    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, SparkSession
    from net.jgp.labs.sparkdq4ml_amd.ops import device
    from net.jgp.labs.sparkdq4ml_amd.parallel import comm

    comm.init()
    if not check_world(a.gpus):
        return 2
    rank, world = comm.rank(), comm.world_size()
    spark = SparkSession.builder().appName("bench-huber").master("local[*]") \
        .config("dq4ml.huber.device", "false" if a.host else "true").getOrCreate()
    dev = spark.device
    d, total = a.features, int(a.rows)
    if dev.type != "cuda":
        total = min(total, 20_000 * world)
    n = total // world if rank < world - 1 else total - (world - 1) * (total // world)
    g = torch.Generator(device=dev).manual_seed(97 + rank)
    X = torch.randn(d, n, generator=g, device=dev)
    beta = torch.linspace(-1.0, 2.0, d, device=dev)
    y = (beta @ X + 0.7 + 0.2 * torch.randn(n, generator=g, device=dev)).double()
    y[::37] += 25.0
    if a.dtype != "f32" and dev.type == "cuda":
        X = device.pack_wide([X], 8 if a.dtype == "fp8" else 16, None, shift=None)
    df = spark.createDataFrame({"features": X, "label": y})
    lr = LinearRegression(loss="huber", maxIter=a.max_iter, tol=1e-6)
    last = {}

    def step():
        m = lr.fit(df)
        m.coefficients  # (a pending fit resolves here)
        last["m"] = m
        return m

    elapsed, model = timed(step, a.steps, a.warmup, dev)
    m = last["m"]
    evals = getattr(m, "_huber_evaluations", None)
    hist = np.asarray(m.summary.objectiveHistory)
    err = float(np.abs(np.asarray(m.coefficients.toArray()) - beta.double().cpu().numpy()).max())
    ms = elapsed / a.steps * 1e3
    emit({"metric": "ms per LinearRegression(loss=huber).fit", "value": ms, "unit": "ms", "n_gpus": world,
          "steps": a.steps, "warmup": a.warmup, "ms_per_step": ms, "higher_is_better": False, "scaling": "strong",
          "vs_baseline": None, "dtype": a.dtype, "data": "synthetic (N(0,1) features, 1/37 outlier labels)",
          "config": {"model": f"LinearRegression(huber, l-bfgs-b) d={d}", "global_batch": total, "seq_len": d,
                     "parallelism": f"dp{world}", "optimizer": "host" if a.host else "device",
                     "states": int(hist.size), "evaluations": evals,
                     "us_per_evaluation": (ms * 1e3 / evals) if evals else None, "coef_max_abs_err": err},
          **world_info(dev)}, a.json_out)
    comm.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
