#!/usr/bin/env python3
"""Time the fused scan + DQ kernel alone (ops/scanfuse.py) on the lab chain over a synthetic CSV,
optionally as a diagnostic ablation build (``DQ4ML_SCAN_ABL=1``: line finding only, no per-line
work; ``=2``: parse + rules without the stores) — to see where the kernel's time goes.

    DQ4ML_DIAG=1 DQ4ML_SCAN_ABL=0|1|2 python scripts/scan_ablation.py [--rows 1e8] [--reps 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "benchmarks"))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1e8)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--gram", action="store_true", help="Gram mode (scanfuse.try_fused_gram) instead of table mode")
    a = ap.parse_args(argv)
    import torch

    from bench_csv_pipeline import synth_csv
    from net.jgp.labs.sparkdq4ml_amd import SparkSession, VectorAssembler, callUDF
    from net.jgp.labs.sparkdq4ml_amd.dq.rules import register_lab_rules
    from net.jgp.labs.sparkdq4ml_amd.ops import scanfuse
    from net.jgp.labs.sparkdq4ml_amd.sql.plan import CsvScanRelation, Filter, Project, prune_columns

    rows = int(a.rows)
    path = os.path.join(os.environ.get("TMPDIR", tempfile.gettempdir()), f"dq4ml_synth_{rows}.csv")
    if not os.path.exists(path):
        synth_csv(path + ".tmp", rows)
        os.replace(path + ".tmp", path)
    spark = SparkSession.builder().master("mi355x[*]").getOrCreate()
    register_lab_rules(spark)

    def chain():
        df = spark.read().format("csv").option("inferSchema", "true").load(path)
        raw = df
        df = df.withColumnRenamed("_c0", "guest").withColumnRenamed("_c1", "price")
        df = df.withColumn("price_no_min", callUDF("minimumPriceRule", df.col("price")))
        df.createOrReplaceTempView("price")
        df = spark.sql("SELECT cast(guest as int) guest, price_no_min AS price FROM price WHERE price_no_min > 0")
        df = df.withColumn("price_correct_correl", callUDF("priceCorrelationRule", df.col("price"), df.col("guest")))
        df.createOrReplaceTempView("price")
        df = spark.sql("SELECT guest, price_correct_correl AS price FROM price WHERE price_correct_correl > 0")
        df = df.withColumn("label", df.col("price"))
        return raw, VectorAssembler().setInputCols(["guest"]).setOutputCol("features").transform(df)

    chain()  # eager scan: records the file's facts
    raw, df = chain()
    assert isinstance(raw._plan, CsvScanRelation)
    plan = prune_columns(df._plan, {"features", "label"})
    if a.gram:
        def once():
            assert scanfuse.try_fused_gram(plan, "features", "label", spark) is not None
    else:
        plan = plan.child  # the chain below the assembler
        nodes, p = [], plan
        while isinstance(p, (Project, Filter)):
            nodes.append(p)
            p = p.child
        nodes.reverse()

        def once():
            scanfuse.try_fused_scan(nodes, p, plan, spark)
    for _ in range(3):
        once()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # Gram mode runs on the compute stream, table mode on the scan side stream
    side = torch.cuda.current_stream() if a.gram else scanfuse._scan_stream(torch.device("cuda", torch.cuda.current_device()))
    e0.record(side)
    for _ in range(a.reps):
        once()
    e1.record(side)
    torch.cuda.synchronize()
    print(json.dumps({"abl": int(os.environ.get("DQ4ML_SCAN_ABL", "0")), "gram": a.gram, "rows": rows,
                      "ms_per_scan": e0.elapsed_time(e1) / a.reps}), flush=True)


if __name__ == "__main__":
    main()
