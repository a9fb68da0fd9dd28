#!/usr/bin/env python3
"""BASELINE.json config #1: data/dataset-small.csv -> VectorAssembler -> LinearRegression on the
host engine (Spark ``local[1]`` analog; plumbing, no GPU).  One step = CSV read with schema
inference + DQ rules + SQL clean-ups + assemble + fit (maxIter 40, regParam 1, elasticNet 1) +
transform + summary — the lab pipeline end to end, nothing cached between steps.

    python benchmarks/bench_cpu_small.py [--data data/dataset-small.csv] [--steps 20]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from harness import ROOT, emit, timed  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--data", default=os.path.join(ROOT, "data", "dataset-small.csv"))
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args(argv)
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, SparkSession, VectorAssembler, callUDF
    from net.jgp.labs.sparkdq4ml_amd.dq.rules import register_lab_rules
    from net.jgp.labs.sparkdq4ml_amd.parallel import comm

    comm.init()
    spark = SparkSession.builder().appName("DQ4ML-small").master("local-cpu").getOrCreate()
    register_lab_rules(spark)

    def step():
        df = spark.read().format("csv").option("inferSchema", "true").option("header", "false").load(a.data)
        df = df.withColumnRenamed("_c0", "guest").withColumnRenamed("_c1", "price")
        df = df.withColumn("price_no_min", callUDF("minimumPriceRule", df.col("price")))
        df.createOrReplaceTempView("price")
        df = spark.sql("SELECT cast(guest as int) guest, price_no_min AS price FROM price WHERE price_no_min > 0")
        df = df.withColumn("price_correct_correl",
                           callUDF("priceCorrelationRule", df.col("price"), df.col("guest")))
        df.createOrReplaceTempView("price")
        df = spark.sql("SELECT guest, price_correct_correl AS price FROM price WHERE price_correct_correl > 0")
        df = df.withColumn("label", df.col("price"))
        df = VectorAssembler().setInputCols(["guest"]).setOutputCol("features").transform(df)
        lr = LinearRegression().setMaxIter(40).setRegParam(1).setElasticNetParam(1)
        model = lr.fit(df)
        model.transform(df).count()
        return model, df

    elapsed, (model, df) = timed(step, a.steps, a.warmup, spark.device)
    rows = df.count()
    emit({"metric": "pipelines/sec, dataset-small.csv DQ4ML pipeline on the host engine (BASELINE config 1)",
          "value": a.steps / elapsed, "unit": "pipelines/s", "n_gpus": 0, "steps": a.steps, "warmup": a.warmup,
          "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True, "scaling": "none", "vs_baseline": None,
          "dtype": "fp64", "data": os.path.relpath(a.data, ROOT),
          "config": {"model": "CSV -> DQ rules -> VectorAssembler -> LinearRegression(40, 1, 1)",
                     "rows_after_dq": rows, "coefficients": list(model.coefficients.toArray()),
                     "intercept": model.intercept, "parallelism": "local[1] host"}}, a.json_out)
    comm.shutdown()


if __name__ == "__main__":
    main()
