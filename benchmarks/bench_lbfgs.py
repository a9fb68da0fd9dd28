#!/usr/bin/env python3
"""Squared-loss l-bfgs path: ``LinearRegression(solver="auto")`` with
numFeatures > 4096 -> Spark's l-bfgs switch.  One step = one full fit: the summarizer pass (feature
moments), then per cost evaluation the two ``lsq.hip`` passes over the HBM-resident shard (margins,
then Σ w·diff·x) + one (d + 1)-f64 RCCL all-reduce, Breeze L-BFGS state on the device.

Default shape: 1e6 rows x 16384 features, bf16 wide fragment layout (32.8 GB), L2 0.01.  Features
are stream-ingested into the layout (the matrix never exists in f32).

    python benchmarks/bench_lbfgs.py [--rows 1e6] [--features 16384] [--dtype bf16|fp8] [--gpus N]
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
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--rows", type=float, default=1e6, help="global rows (strong scaling)")
    ap.add_argument("--features", type=int, default=16384)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"])
    ap.add_argument("--reg", type=float, default=0.01)
    ap.add_argument("--enet", type=float, default=0.0)
    ap.add_argument("--max-iter", type=int, default=100)
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args(argv)
    rc = self_launch(a.gpus, __file__, argv)
    if rc is not None:
        return rc
    import time

    import numpy as np
    import torch

    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, SparkSession
    from net.jgp.labs.sparkdq4ml_amd.ops import device, native
    from net.jgp.labs.sparkdq4ml_amd.ops.layout import TiledWide
    from net.jgp.labs.sparkdq4ml_amd.parallel import comm

    comm.init()
    if not check_world(a.gpus):
        return 2
    rank, world = comm.rank(), comm.world_size()
    spark = SparkSession.builder().appName("bench-lbfgs").master("local[*]").getOrCreate()
    dev = spark.device
    d, total = a.features, int(a.rows)
    if dev.type != "cuda":  # host-engine rehearsal of the launcher / JSON contract: small dense shape
        d, total = min(d, 4200), min(total, 1000 * world)
    n = total // world if rank < world - 1 else total - (world - 1) * (total // world)
    eb = 8 if a.dtype == "fp8" else 16
    if dev.type != "cuda":
        g = torch.Generator().manual_seed(97 + rank)
        beta = torch.linspace(-1.0, 1.0, d)
        X = torch.randn(d, n, generator=g, dtype=torch.float64)
        y = (beta.double() @ X + 0.5 + 0.1 * torch.randn(n, generator=g, dtype=torch.float64)).float()
        buf = X
    else:
        X, y, beta, buf = _ingest(d, n, eb, rank, dev, native, device, TiledWide)
    df = spark.createDataFrame({"features": X, "label": y})
    lr = LinearRegression(solver="auto", regParam=a.reg, elasticNetParam=a.enet, maxIter=a.max_iter)
    elapsed, model = timed(lambda: lr.fit(df), a.steps, a.warmup, dev)
    coef = np.asarray(model.coefficients.toArray())
    err = float(np.abs(coef - beta.double().cpu().numpy()).max())
    evals = getattr(model, "_qn_evaluations", None)  # the device fit (lsq_qn.hip) counts its data passes
    host_steered = None
    if evals is not None and os.environ.get("DQ4ML_BENCH_AB", "1") != "0":
        # same-process A/B: the round-3 host-steered optimizer over the two-pass evaluations
        os.environ["DQ4ML_LSQ_QN"] = "0"
        try:
            el2, m2 = timed(lambda: lr.fit(df), 1, 0, dev)
        finally:
            os.environ.pop("DQ4ML_LSQ_QN", None)
        host_steered = {"ms_per_fit": el2 * 1e3, "iterations": int(m2.summary.totalIterations),
                        "coef_max_abs_diff_vs_device": float(np.abs(np.asarray(m2.coefficients.toArray()) - coef).max())}
    # one two-pass evaluation alone (margins + columns + fold: the host-steered path's), per-pass bandwidth
    from net.jgp.labs.sparkdq4ml_amd.ops import kernels

    P = kernels.lsq_passes(X, y, None, None)
    cf = torch.randn(d, device=dev, dtype=torch.float64) * 1e-3
    off = torch.zeros(1, dtype=torch.float64, device=dev)
    P.evaluate(cf, off, 1.0)
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    sync()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        P.evaluate(cf, off, 1.0)
    sync()
    eval_ms = (time.perf_counter() - t0) / reps * 1e3
    xbytes = buf.numel() * buf.element_size()
    ms = elapsed / a.steps * 1e3
    info = world_info(dev)
    emit({"metric": f"rows/sec LinearRegression.fit, l-bfgs path {total:.0e}x{d} {a.dtype} (SURVEY K9/X4)",
          "value": total * a.steps / elapsed, "unit": "rows/s", "n_gpus": world, "steps": a.steps,
          "warmup": a.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "strong",
          "vs_baseline": None, "dtype": a.dtype if dev.type == "cuda" else "fp64",
          "data": "synthetic (N(0,1) features, random-init coefficients)",
          "config": {"model": f"LinearRegression(solver=auto -> l-bfgs, L2 {a.reg}, enet {a.enet}) d={d}",
                     "global_batch": total, "seq_len": d, "parallelism": f"dp{world}", "rows_per_gpu": n,
                     "iterations": int(model.summary.totalIterations), "solver": model.summary.solver,
                     "coef_max_abs_err": err, "eval_ms": eval_ms,
                     "device_fit_evaluations": evals,
                     "device_fit_ms_per_evaluation": (ms / (evals + 1)) if evals else None,
                     "host_steered": host_steered,
                     "eval_hbm_TBps": 2 * xbytes / (eval_ms * 1e-3) / 1e12, "x_bytes_per_gpu": xbytes},
          **info}, a.json_out)
    comm.shutdown()
    return 0


def _ingest(d, n, eb, rank, dev, native, device, TiledWide):
    """Stream the synthetic rows straight into the wide fragment layout (64-row-aligned chunks)."""
    import torch

    h = native.hip()
    buf = torch.empty(int(h.wide_tiled_bytes(eb, d, n)), dtype=torch.uint8, device=dev)
    per_row = buf.numel() // (((n + 63) // 64) * 64)
    scale = torch.full((d,), 4.5 / 448.0, device=dev)
    g = torch.Generator(device=dev).manual_seed(97 + rank)
    beta = torch.linspace(-1.0, 1.0, d, device=dev)
    y = torch.empty(n, dtype=torch.float32, device=dev)
    chunk = max(64, (int(2e8) // d) // 64 * 64)
    for r0 in range(0, n, chunk):
        r1 = min(n, r0 + chunk)
        xc = torch.randn(d, r1 - r0, generator=g, device=dev)
        y[r0:r1] = beta @ xc + 0.5 + 0.1 * torch.randn(r1 - r0, generator=g, device=dev)
        lo = r0 * per_row
        device.pack_wide([xc], eb, None, inv_scale=(1.0 / scale) if eb == 8 else None,
                         out=buf[lo:lo + ((r1 - r0 + 63) // 64) * 64 * per_row], shift=None)
        del xc
    return TiledWide(buf, d, n, eb, scale if eb == 8 else None), y, beta, buf


if __name__ == "__main__":
    sys.exit(main())
