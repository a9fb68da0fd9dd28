"""Fused DQ codegen kernels on the MI355X vs the host vectorized evaluator (same plans)."""
import math

import pytest
import torch

from net.jgp.labs.sparkdq4ml_amd import SparkSession, callUDF, col, lit, when
from net.jgp.labs.sparkdq4ml_amd.dq.rules import register_lab_rules
from net.jgp.labs.sparkdq4ml_amd.ops import dqvm
from net.jgp.labs.sparkdq4ml_amd.sql.expressions import SparkException

pytestmark = pytest.mark.gpu

ROWS = [(1, 23.1, 1.5), (2, None, 2.0), (None, 120.0, -1.0), (14, 95.0, None), (5, 3.0, 0.0), (30, 150.0, 7.25),
        (13, 91.0, 3.0), (0, 0.0, float("nan")), (-4, -20.5, 1e300)]


def _build(spark, body):
    df = spark.createDataFrame(ROWS, "guest int, price double, z double")
    register_lab_rules(spark)
    return body(spark, df)


def _q1(spark, df):
    df = df.withColumn("p2", callUDF("priceCorrelationRule", col("price"), col("guest")))
    df = df.withColumn("r", (col("price") * 2 + col("guest")) / col("z"))
    df = df.withColumn("c", col("price").cast("int")).withColumn("b", (col("price") > 50) | col("z").isNull())
    df = df.withColumn("w", when(col("guest") < 10, col("price")).otherwise(lit(-1.0)))
    return df.filter((col("p2") > 0) | col("guest").isNull())


def _q2(spark, df):
    df.createOrReplaceTempView("t")
    return spark.sql("SELECT guest % 4 AS g4, coalesce(price, z, 0.0) AS v, abs(z) AS az, sqrt(price) AS sp, "
                     "NOT (guest > 3 AND price < 100) AS nb FROM t WHERE guest IS NOT NULL OR price > 0")


def _collect(df):
    out = []
    for r in df.collect():
        out.append(tuple(None if v is None else (round(v, 9) if isinstance(v, float) and not math.isnan(v) else
                                                 ("nan" if isinstance(v, float) else v)) for v in r))
    return out


@pytest.mark.parametrize("q", [_q1, _q2])
def test_fused_matches_host(q):
    s = SparkSession.getActiveSession()
    if s is not None:
        s.stop()
    cpu = SparkSession.builder().master("cpu").getOrCreate()
    ref = _collect(_build(cpu, q))
    cpu.stop()
    gpu = SparkSession.builder().master("mi355x[*]").getOrCreate()
    before = dqvm.STATS["fused_launches"]
    got = _collect(_build(gpu, q))
    assert dqvm.STATS["fused_launches"] > before, "fused kernel not used"
    gpu.stop()
    assert got == ref


def test_rule1_null_raises_on_gpu():
    s = SparkSession.getActiveSession()
    if s is not None:
        s.stop()
    gpu = SparkSession.builder().master("mi355x[*]").getOrCreate()
    df = _build(gpu, lambda sp, d: d.withColumn("x", callUDF("minimumPriceRule", col("price"))))
    with pytest.raises(SparkException):
        df.count()
    # the same null filtered out first does not raise
    ok = _build(gpu, lambda sp, d: d.filter(col("price").isNotNull())
                .withColumn("x", callUDF("minimumPriceRule", col("price"))))
    assert ok.count() == 8
    gpu.stop()


def test_chain_cache_reuses_codegen_and_respects_structure(gpu_session):
    """The structural chain cache: a re-built identical chain over a new relation reuses the
    generated kernel; a different literal compiles anew; results match the plain computation."""
    spark = gpu_session
    rows = [(i % 7, float(i) * 0.5) for i in range(5000)]

    def run(thresh):
        df = spark.createDataFrame(rows, "g int, p double")
        df = df.withColumn("q", col("p") * 2.0).where(col("q") > thresh)
        got = df.collect()
        return len(got), sum(r.q for r in got)

    dqvm._CHAIN_CACHE.clear()
    before = dqvm.STATS["fused_launches"]
    a = run(10.0)
    n1 = len(dqvm._CHAIN_CACHE)
    b = run(10.0)
    assert a == b and len(dqvm._CHAIN_CACHE) == n1  # same structure: cache hit
    c = run(100.0)
    assert len(dqvm._CHAIN_CACHE) > n1  # a different literal is a different kernel
    assert dqvm.STATS["fused_launches"] - before >= 3
    ref = [r for r in rows if r[1] * 2.0 > 100.0]
    assert c[0] == len(ref) and abs(c[1] - sum(r[1] * 2.0 for r in ref)) < 1e-6
