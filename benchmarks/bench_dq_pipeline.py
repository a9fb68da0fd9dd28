#!/usr/bin/env python3
"""BASELINE.json config #4: DQ pipeline (null / range UDF filters) + VectorAssembler +
LinearRegression on 1e9 rows x 64 features over 8 GPUs (1.25e8 rows per GPU).

One step = the whole lazy pipeline, re-executed from the columnar source like every Spark action:

    price_ok = rangeRule(price)      (UDF, null or out of [0, 1e6] -> -1)
    guest_ok = notNullRule(guest)    (UDF, null -> -1)
    WHERE price_ok > 0 AND guest_ok > 0          -> fused DQ VM kernel (hipRTC, one pass, selection)
    VectorAssembler(f0..f63 -> features, bf16)   -> pack straight into MFMA-fragment tiles, dead
                                                    rows zeroed (no compaction)
    LinearRegression(normal, bf16 Gram)          -> MFMA Gram + RCCL all-reduce + f64 solve

Per-GPU work is fixed (weak scaling: --rows-per-gpu, default 1.25e8 so 8 GPUs = 1e9 rows).
Synthetic f32 feature columns, f64 price label with 1 % nulls, int32 guest with 0.5 % nulls.

    python benchmarks/bench_dq_pipeline.py [--rows-per-gpu 1.25e8] [--features 64] [--steps 5]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from harness import check_world, emit, self_launch, timed, world_info  # noqa: E402


def build(spark, n, d, seed, dev):
    import torch

    g = torch.Generator(device=dev).manual_seed(seed)
    data = {}
    beta = torch.linspace(0.5, 2.0, d, device=dev, dtype=torch.float64)
    acc = torch.full((n,), 100.0, dtype=torch.float64, device=dev)
    for j in range(d):
        x = torch.randn(n, generator=g, device=dev, dtype=torch.float32)
        acc += beta[j] * x.double()
        data[f"f{j}"] = x
    price = acc + 0.1 * torch.randn(n, generator=g, device=dev, dtype=torch.float64)
    pvalid = torch.rand(n, generator=g, device=dev) > 0.01
    guest = torch.randint(1, 36, (n,), generator=g, device=dev, dtype=torch.int32)
    gvalid = torch.rand(n, generator=g, device=dev) > 0.005
    data["price"] = (price, pvalid)
    data["guest"] = (guest, gvalid)
    return spark.createDataFrame(data), beta


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--rows-per-gpu", type=float, default=1.25e8)
    ap.add_argument("--features", type=int, default=64)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--sync", dest="use_async", action="store_false",
                    help="synchronous fits (host solve after a D2H every step); default: asynchronous "
                         "device solve, the host builds the next step's plan while the GPU runs")
    a = ap.parse_args(argv)
    rc = self_launch(a.gpus, __file__, argv)  # --gpus N: one process per GPU, before any GPU call
    if rc is not None:
        return rc
    import numpy as np

    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, SparkSession, VectorAssembler, callUDF, col
    from net.jgp.labs.sparkdq4ml_amd.dq.rules import NotNullRule, RangeRule
    import harness
    from net.jgp.labs.sparkdq4ml_amd.ops import dqvm, streamfuse
    from net.jgp.labs.sparkdq4ml_amd.parallel import comm
    from net.jgp.labs.sparkdq4ml_amd.sql.types import DataTypes

    comm.init()
    if not check_world(a.gpus):
        return 2
    rank, world = comm.rank(), comm.world_size()
    spark = SparkSession.builder().appName("bench-dq").master("local[*]") \
        .config("dq4ml.fit.async", "true" if a.use_async else "false").getOrCreate()
    dev = spark.device
    n = int(a.rows_per_gpu) if dev.type == "cuda" else min(int(a.rows_per_gpu), 200_000)
    d = a.features
    spark.udf().register("rangeRule", RangeRule(0.0, 1e6, name="rangeRule"), DataTypes.DoubleType)
    spark.udf().register("notNullRule", NotNullRule(name="notNullRule"), DataTypes.DoubleType)
    src, beta = build(spark, n, d, 777 + rank, dev)
    va = VectorAssembler(inputCols=[f"f{j}" for j in range(d)], outputCol="features",
                         outputDtype="bfloat16" if dev.type == "cuda" else "float64")
    lr = LinearRegression(solver="normal", gramDtype="bf16" if dev.type == "cuda" else "fp64",
                          labelCol="price_ok")

    def step():
        df = src.withColumn("price_ok", callUDF("rangeRule", col("price")))
        df = df.withColumn("guest_ok", callUDF("notNullRule", col("guest")))
        df = df.filter((col("price_ok") > 0) & (col("guest_ok") > 0))
        return lr.fit(va.transform(df))

    elapsed, model = timed(step, a.steps, a.warmup, dev)
    coef = np.asarray(model.coefficients.toArray())
    err = float(np.abs(coef - beta.cpu().numpy()).max())
    total = n * world
    kept = model.summary.numInstances
    info = world_info(dev)
    emit({"metric": "rows/sec DQ filters + VectorAssembler + LinearRegression.fit, 1e9x64 (BASELINE config 4)",
          "value": total * a.steps / elapsed, "unit": "rows/s", "n_gpus": world, "steps": a.steps,
          "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True,
          "scaling": "weak", "vs_baseline": None, "dtype": "bf16" if dev.type == "cuda" else "fp64",
          "data": "synthetic columns (f32 features, f64 label with 1% nulls, int guest with 0.5% nulls)",
          "config": {"model": f"DQ(range+notNull UDF filters) -> VectorAssembler -> LinearRegression d={d}",
                     "global_batch": total, "seq_len": d, "parallelism": f"dp{world}", "rows_per_gpu": n,
                     "rows_kept_global": int(kept), "coef_max_abs_err": err,
                     "dq_vm": dict(dqvm.STATS), "stream_dq_grams": dict(streamfuse.STATS),
                     "host_issue_ms_per_step": harness.LAST_ISSUE_S / a.steps * 1e3,
                     "fit_mode": "async" if (a.use_async and dev.type == "cuda") else "sync"}, **info}, a.json_out)
    comm.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
