#!/usr/bin/env python3
"""The lab application's fit path at scale: CSV -> DQ rules -> VectorAssembler -> LinearRegression.

DataQuality4MachineLearningApp.java:38-126 end to end on a synthetic ``guest,price`` CSV of the
reference datasets' format (headerless, CR-only row terminators, no terminator after the last
row, integer guests and 2-decimal prices), one action per step — exactly what one ``fit`` costs
in the app (Spark re-scans the file on every action):

    read.csv(inferSchema)            -> device scan K1/K2 (line ends, fused parse + type lattice),
                                        chunked through the pinned staging ring
    rename, minimumPriceRule + WHERE, cast, priceCorrelationRule + WHERE
                                     -> fused DQ whole-stage kernel (hipRTC), selection vector
    label, VectorAssembler(guest)    -> tiled bf16 pack of the kept rows
    LinearRegression(40, 1.0, 1.0)   -> MFMA Gram + all-reduce + OWLQN on the 2x2 system

Prints rows/s and input GB/s.  Multi-rank runs shard the file by byte range (each rank reads
only its rows; type masks merged with an all-reduce).

    python benchmarks/bench_csv_pipeline.py [--rows 1e8] [--steps 3] [--warmup 1]
"""
from __future__ import annotations

import argparse
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import harness  # noqa: E402
from harness import check_world, emit, self_launch, timed, world_info  # noqa: E402


def synth_csv(path: str, rows: int, seed: int = 7) -> int:
    """``guest,price`` rows like data/dataset-*.csv: guest in [1, 35], price ~ 5 * guest + 20 +
    noise with 1-2 decimals, ~5 % of rows violating each DQ rule.  Written in 16M-row blocks with
    vectorized (numpy) digit placement; returns the byte size."""
    import numpy as np

    rng = np.random.default_rng(seed)
    block = 1 << 24
    W = 10  # widest row: "35,999.99\r"
    with open(path, "wb") as f:
        for r0 in range(0, rows, block):
            m = min(block, rows - r0)
            g = rng.integers(1, 36, m)
            cents = np.round((5.0 * g + 20.0 + rng.normal(0.0, 3.0, m)) * 100).astype(np.int64)
            low = rng.random(m) < 0.05  # below the minimum price: rule 1 drops the row
            cents[low] = rng.integers(300, 1999, int(low.sum()))
            hi = (rng.random(m) < 0.05) & (g < 14)  # small party above 90: rule 2 drops the row
            cents[hi] = rng.integers(9100, 19900, int(hi.sum()))
            cents = np.clip(cents, 100, 99999)
            pi = cents // 100
            row = np.zeros((m, W), dtype=np.uint8)
            col = np.zeros(m, dtype=np.int64)
            every = np.ones(m, dtype=bool)

            def put(mask, vals):
                idx = np.nonzero(mask)[0]
                row[idx, col[idx]] = np.broadcast_to(vals, (m,))[idx]
                col[idx] += 1

            put(g >= 10, (g // 10 + 48).astype(np.uint8))
            put(every, (g % 10 + 48).astype(np.uint8))
            put(every, np.uint8(ord(",")))
            put(pi >= 100, (pi // 100 + 48).astype(np.uint8))
            put(pi >= 10, ((pi // 10) % 10 + 48).astype(np.uint8))
            put(every, (pi % 10 + 48).astype(np.uint8))
            put(every, np.uint8(ord(".")))
            put(every, ((cents // 10) % 10 + 48).astype(np.uint8))
            put(cents % 10 != 0, (cents % 10 + 48).astype(np.uint8))  # 1 or 2 decimals
            put(every, np.uint8(13))  # CR-only terminators, as in the reference data (R8)
            flat = row[np.arange(W)[None, :] < col[:, None]]
            if r0 + m >= rows:
                flat = flat[:-1]  # no terminator after the last row
            f.write(flat.tobytes())
    return os.path.getsize(path)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--rows", type=float, default=1e8, help="rows of the synthetic CSV (all ranks)")
    ap.add_argument("--path", default=None, help="CSV to use (default: synthesize under $TMPDIR)")
    ap.add_argument("--features", type=int, default=1,
                    help="1: the lab's guest,price CSV and DQ chain; d > 1: BASELINE-shape rows of d float "
                         "features + a label (range-rule DQ filter on the label, VectorAssembler of the d "
                         "columns, normal-equation fit)")
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args(argv)
    rc = self_launch(a.gpus, __file__, argv)  # --gpus N: one process per GPU, before any GPU call
    if rc is not None:
        return rc

    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, SparkSession, VectorAssembler, callUDF
    from net.jgp.labs.sparkdq4ml_amd.dq.rules import register_lab_rules
    from net.jgp.labs.sparkdq4ml_amd.ops import csvscan
    from net.jgp.labs.sparkdq4ml_amd.parallel import comm

    comm.init()
    if not check_world(a.gpus):
        return 2
    rank, world = comm.rank(), comm.world_size()
    spark = SparkSession.builder().appName("bench-csv").master("local[*]") \
        .config("dq4ml.fit.async", "true").getOrCreate()
    dev = spark.device
    rows = int(a.rows) if dev.type == "cuda" else min(int(a.rows), 200_000)
    d = a.features
    path = a.path
    if path is None:
        if d > 1:
            import csv_synth

            path = os.path.join(csv_synth.scratch_dir(int(rows * (9.6 * d + 9))), f"dq4ml_wide_{rows}x{d}.csv")
            if rank == 0 and not os.path.exists(path):
                csv_synth.write_wide_csv(path, rows, d, device=dev, y0=60.0)
        else:
            path = os.path.join(os.environ.get("TMPDIR", tempfile.gettempdir()), f"dq4ml_synth_{rows}.csv")
            if rank == 0 and not os.path.exists(path):
                synth_csv(path + ".tmp", rows)
                os.replace(path + ".tmp", path)
        comm.barrier()
    nbytes = os.path.getsize(path)
    register_lab_rules(spark)
    if d > 1:
        from net.jgp.labs.sparkdq4ml_amd import col
        from net.jgp.labs.sparkdq4ml_amd.dq.rules import RangeRule
        from net.jgp.labs.sparkdq4ml_amd.sql.types import DataTypes

        spark.udf().register("rangeRule", RangeRule(0.0, 150.0, name="rangeRule"), DataTypes.DoubleType)

    def step_wide():
        df = spark.read().format("csv").option("inferSchema", "true").option("header", "false").load(path)
        df = df.withColumn("y_ok", callUDF("rangeRule", col(f"_c{d}"))).filter(col("y_ok") > 0)
        df = df.withColumn("label", col("y_ok"))
        df = VectorAssembler().setInputCols([f"_c{i}" for i in range(d)]).setOutputCol("features").transform(df)
        return LinearRegression(solver="normal", regParam=1e-3).fit(df)

    def step():
        if d > 1:
            return step_wide()
        df = spark.read().format("csv").option("inferSchema", "true").option("header", "false").load(path)
        df = df.withColumnRenamed("_c0", "guest").withColumnRenamed("_c1", "price")
        df = df.withColumn("price_no_min", callUDF("minimumPriceRule", df.col("price")))
        df.createOrReplaceTempView("price")
        df = spark.sql("SELECT cast(guest as int) guest, price_no_min AS price FROM price WHERE price_no_min > 0")
        df = df.withColumn("price_correct_correl", callUDF("priceCorrelationRule", df.col("price"), df.col("guest")))
        df.createOrReplaceTempView("price")
        df = spark.sql("SELECT guest, price_correct_correl AS price FROM price WHERE price_correct_correl > 0")
        df = df.withColumn("label", df.col("price"))
        df = VectorAssembler().setInputCols(["guest"]).setOutputCol("features").transform(df)
        return LinearRegression().setMaxIter(40).setRegParam(1).setElasticNetParam(1).fit(df)

    # the first action also reads the file into the pinned host cache and HBM (runtime.filecache):
    # timed separately and reported, it is not part of the steady-state per-action number
    import time

    import torch

    if dev.type == "cuda":
        torch.cuda.synchronize()
    prof = None
    if os.environ.get("DQ4ML_BENCH_FIRST_PROFILE"):  # host-side profile of the first action only
        import cProfile

        prof = cProfile.Profile()
        prof.enable()
    t0 = time.perf_counter()
    step()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    first_ms = (time.perf_counter() - t0) * 1e3
    if prof is not None:
        prof.disable()
        prof.dump_stats(os.environ["DQ4ML_BENCH_FIRST_PROFILE"])
    elapsed, model = timed(step, a.steps, max(0, a.warmup - 1), dev)
    info = world_info(dev)
    from net.jgp.labs.sparkdq4ml_amd.ops import scancut

    emit({"metric": "rows/sec lab pipeline CSV -> DQ rules -> VectorAssembler -> LinearRegression.fit"
                    + ("" if d == 1 else f" ({d} float features per row)"),
          "value": rows * a.steps / elapsed, "unit": "rows/s", "n_gpus": world, "steps": a.steps,
          "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True,
          "scaling": "strong", "vs_baseline": None, "dtype": "fp64",
          "data": (f"synthetic CSV {nbytes / 1e9:.2f} GB (guest,price; CR terminators)" if d == 1 else
                   f"synthetic CSV {nbytes / 1e9:.2f} GB ({d} float features + label per row; CR terminators)"),
          "config": {"model": ("DataQuality4MachineLearningApp fit path (maxIter 40, regParam 1, elasticNet 1)"
                               if d == 1 else
                               f"RangeRule(label in (0, 150]) DQ filter -> VectorAssembler({d} columns) -> "
                               f"LinearRegression(solver=normal, regParam 1e-3)"),
                     "global_batch": rows, "csv_gbytes_per_s": nbytes * a.steps / elapsed / 1e9,
                     "rows_after_dq": int(model.summary.numInstances),
                     "coefficients": [float(v) for v in model.coefficients.toArray()],
                     "intercept": float(model.intercept), "parallelism": f"dp{world}",
                     "first_action_ms": first_ms, "host_issue_ms_per_step": harness.LAST_ISSUE_S / a.steps * 1e3,
                     "device_scans": csvscan.STATS["device_scans"], "scan_fallbacks": csvscan.STATS["fallbacks"],
                     "features": d, "csv_bytes": nbytes, "cut_grams": scancut.STATS["cut_grams"]},
          **info}, a.json_out)
    comm.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
