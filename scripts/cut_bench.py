#!/usr/bin/env python3
"""Time the CSV -> DQ -> Gram statistics action alone (``regression._fused_scan_stats``: the
byte-parallel cutter, or the per-line fused scan with DQ4ML_SCAN_CUT=0) on the lab CSV and the
BASELINE-shape wide CSV, for several environment variants in ONE process (the cutter's compile
cache is keyed by its knobs), e.g.

    DQ4ML_DIAG=1 VARIANTS="base;DQ4ML_SCAN_CUT=0;DQ4ML_CUT_ABLATE=1" python scripts/cut_bench.py --features 32 --rows 2e7

Prints one JSON line per variant: ms per action (median of --reps), CSV GB/s.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--features", type=int, default=1)
    ap.add_argument("--rows", type=float, default=1e8)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import torch

    import bench_csv_pipeline as B
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, SparkSession, VectorAssembler, callUDF, col
    from net.jgp.labs.sparkdq4ml_amd.dq.rules import RangeRule, register_lab_rules
    from net.jgp.labs.sparkdq4ml_amd.models import regression
    from net.jgp.labs.sparkdq4ml_amd.ops import scancut
    from net.jgp.labs.sparkdq4ml_amd.sql.types import DataTypes

    spark = SparkSession.builder().master("mi355x[*]").config("dq4ml.csv.deviceThresholdBytes", "0").getOrCreate()
    rows, d = int(a.rows), a.features
    tmp = os.environ.get("TMPDIR", "/tmp")
    if d > 1:
        import csv_synth

        path = os.path.join(csv_synth.scratch_dir(int(rows * (9.6 * d + 9))), f"cutb_{rows}x{d}.csv")
        if not os.path.exists(path):
            csv_synth.write_wide_csv(path, rows, d, device="cuda", y0=60.0)
        spark.udf().register("rangeRule", RangeRule(0.0, 150.0, name="rangeRule"), DataTypes.DoubleType)
    else:
        path = os.path.join(tmp, f"cutb_lab_{rows}.csv")
        if not os.path.exists(path):
            B.synth_csv(path, rows)
    register_lab_rules(spark)
    nbytes = os.path.getsize(path)
    spark.read().format("csv").option("inferSchema", "true").load(path).count()  # eager scan: facts

    def action():
        df = spark.read().format("csv").option("inferSchema", "true").load(path)
        if d > 1:
            df = df.withColumn("y_ok", callUDF("rangeRule", col(f"_c{d}"))).filter(col("y_ok") > 0)
            df = df.withColumn("label", col("y_ok"))
            df = VectorAssembler().setInputCols([f"_c{i}" for i in range(d)]).setOutputCol("features").transform(df)
            lr = LinearRegression(solver="normal", regParam=1e-3)
        else:
            df = df.withColumnRenamed("_c0", "guest").withColumnRenamed("_c1", "price")
            df = df.withColumn("price_no_min", callUDF("minimumPriceRule", df.col("price")))
            df.createOrReplaceTempView("price")
            df = spark.sql("SELECT cast(guest as int) guest, price_no_min AS price FROM price WHERE price_no_min > 0")
            df = df.withColumn("price_correct_correl", callUDF("priceCorrelationRule", df.col("price"),
                                                               df.col("guest")))
            df.createOrReplaceTempView("price")
            df = spark.sql("SELECT guest, price_correct_correl AS price FROM price WHERE price_correct_correl > 0")
            df = df.withColumn("label", df.col("price"))
            df = VectorAssembler().setInputCols(["guest"]).setOutputCol("features").transform(df)
            lr = LinearRegression().setMaxIter(40).setRegParam(1).setElasticNetParam(1)
        return regression._fused_scan_stats(lr, df)

    variants = os.environ.get("VARIANTS", "base").split(";")
    base_env = dict(os.environ)
    for v in variants:
        os.environ.clear()
        os.environ.update(base_env)
        for kv in v.split(","):
            if "=" in kv:
                k, val = kv.split("=", 1)
                os.environ[k] = val
        before = scancut.STATS["cut_grams"]
        fused = action()  # warm-up (compile)
        torch.cuda.synchronize()
        # back-to-back actions between two syncs: the host plans action k+1 while the GPU runs
        # action k, so the mean is the device time per action whenever it exceeds the host's
        times = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                fused = action()
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) / a.reps)
        times.sort()
        ms = times[1]
        rec = {"variant": v, "features": d, "rows": rows, "ms": round(ms, 4),
               "csv_gbytes_per_s": round(nbytes / ms / 1e6, 1),
               "cutter": scancut.STATS["cut_grams"] > before, "count": float(fused.flat[0]) if fused else None}
        if fused is not None:  # bit-identity of the statistics across variants
            import hashlib

            flat = fused.flat if torch.is_tensor(fused.flat) else torch.as_tensor(fused.flat)
            rec["digest"] = hashlib.sha1(flat.detach().cpu().double().numpy().tobytes()).hexdigest()[:16]
        if os.environ.get("DQ4ML_CUT_STAMPS") == "1" and "buf" in scancut.LAST_STAMPS:
            st = scancut.LAST_STAMPS["buf"].cpu().double()
            win = float(st[:, 6].sum())
            names = ["stage+masks+scan", "head seps", "scatter", "convert", "rows+chain", "gram+loop"]
            rec["cycles_per_window"] = {nm: round(float(st[:, k].sum()) / max(win, 1.0), 1)
                                        for k, nm in enumerate(names)}
            rec["windows"] = win
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
