"""The DQ chain in the stream Gram's stage prologue (ops/streamfuse.py) on the MI355X: config 4's
pipeline (range + not-null rule UDFs on price / guest with nulls, their filter, VectorAssembler of
f32 columns, bf16 / exact-f32 statistics) in ONE kernel equals the two-pass path (dqvm selection
kernel + stream Gram over the selection)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def spark():
    from net.jgp.labs.sparkdq4ml_amd import SparkSession

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    s = SparkSession.getActiveSession()
    if s is not None:
        s.stop()
    s = SparkSession.builder().master("mi355x[*]").getOrCreate()
    yield s
    s.stop()


def _df(spark, n, d, seed=3):
    from net.jgp.labs.sparkdq4ml_amd import VectorAssembler, callUDF, col
    from net.jgp.labs.sparkdq4ml_amd.dq.rules import NotNullRule, RangeRule
    from net.jgp.labs.sparkdq4ml_amd.sql.types import DataTypes

    spark.udf().register("rangeRule", RangeRule(0.0, 1e6, name="rangeRule"), DataTypes.DoubleType)
    spark.udf().register("notNullRule", NotNullRule(name="notNullRule"), DataTypes.DoubleType)
    g = torch.Generator(device="cuda").manual_seed(seed)
    data, acc = {}, torch.full((n,), 100.0, dtype=torch.float64, device="cuda")
    for j in range(d):
        x = torch.randn(n, generator=g, device="cuda")
        acc += (0.5 + j / d) * x.double()
        data[f"f{j}"] = x
    price = acc + 0.1 * torch.randn(n, generator=g, device="cuda", dtype=torch.float64)
    price[::997] = -5.0  # out of the rule's range: dropped
    data["price"] = (price, torch.rand(n, generator=g, device="cuda") > 0.01)
    data["guest"] = (torch.randint(1, 36, (n,), generator=g, device="cuda", dtype=torch.int32),
                     torch.rand(n, generator=g, device="cuda") > 0.005)
    df = spark.createDataFrame(data).withColumn("price_ok", callUDF("rangeRule", col("price")))
    df = df.withColumn("guest_ok", callUDF("notNullRule", col("guest")))
    df = df.filter((col("price_ok") > 0) & (col("guest_ok") > 0))
    return VectorAssembler(inputCols=[f"f{j}" for j in range(d)], outputCol="features").transform(df)


@pytest.mark.parametrize("d,n,gd", [(64, 300_007, "bf16"), (20, 200_000, "bf16"), (64, 150_000, "fp32"),
                                    (33, 100_050, "fp32"), (40, 120_000, "fp32split")])
def test_one_pass_equals_two_pass(spark, monkeypatch, d, n, gd):
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression
    from net.jgp.labs.sparkdq4ml_amd.models import regression
    from net.jgp.labs.sparkdq4ml_amd.ops import streamfuse

    lr = LinearRegression(solver="normal", gramDtype=gd, labelCol="price_ok")
    df = _df(spark, n, d)
    before = streamfuse.STATS["stream_grams"]
    fused = regression._fused_scan_stats(lr, df)
    assert fused is not None and streamfuse.STATS["stream_grams"] == before + 1
    one = fused.flat.cpu().numpy()
    monkeypatch.setenv("DQ4ML_STREAM_DQ", "0")
    assert regression._fused_scan_stats(lr, df) is None
    tbl, X, y = regression._features_label(lr, df)
    two = lr._wls_stats(df, tbl, X, y, d, False)[0].cpu().numpy()
    assert one[0] == two[0] and 0.9 * n < one[0] < n  # the same surviving rows
    np.testing.assert_allclose(one, two, rtol=2e-6, atol=1e-6 * np.abs(two).max())
    monkeypatch.delenv("DQ4ML_STREAM_DQ")
    m1, m2 = lr.fit(df), lr.fit(df)
    assert np.array_equal(m1.coefficients.toArray(), m2.coefficients.toArray())  # fixed-order folds
    assert np.abs(m1.coefficients.toArray() - (0.5 + np.arange(d) / d)).max() < 0.05


def test_rebuilt_chain_replays_the_analyzed_launch(spark):
    """An action that rebuilds the same chain over the same in-memory relation (config 4's loop)
    replays the analyzed stream launch (``streamfuse.replay``: no pruning, chain key or table
    walk); the statistics are bitwise the first action's.  A re-registered rule is a new
    structure: it is analyzed again and its own filter applies."""
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, VectorAssembler, callUDF, col
    from net.jgp.labs.sparkdq4ml_amd.dq.rules import RangeRule
    from net.jgp.labs.sparkdq4ml_amd.models import regression
    from net.jgp.labs.sparkdq4ml_amd.ops import streamfuse
    from net.jgp.labs.sparkdq4ml_amd.sql.types import DataTypes

    d, n = 24, 200_003
    base = _df(spark, n, d)
    src = base._plan
    while type(src).__name__ != "LocalRelation":
        src = src.child
    from net.jgp.labs.sparkdq4ml_amd.sql.dataframe import DataFrame

    raw = DataFrame(src, spark)

    def chain():
        df = raw.withColumn("price_ok", callUDF("rangeRule", col("price")))
        df = df.withColumn("guest_ok", callUDF("notNullRule", col("guest")))
        df = df.filter((col("price_ok") > 0) & (col("guest_ok") > 0))
        return VectorAssembler(inputCols=[f"f{j}" for j in range(d)], outputCol="features").transform(df)

    lr = LinearRegression(solver="normal", gramDtype="bf16", labelCol="price_ok")
    r0 = streamfuse.STATS["stream_replays"]
    one = regression._fused_scan_stats(lr, chain()).flat.cpu().numpy()
    two = regression._fused_scan_stats(lr, chain()).flat.cpu().numpy()
    assert streamfuse.STATS["stream_replays"] == r0 + 1
    assert np.array_equal(one, two)
    spark.udf().register("rangeRule", RangeRule(0.0, 100.0, name="rangeRule"), DataTypes.DoubleType)
    three = regression._fused_scan_stats(lr, chain()).flat.cpu().numpy()
    assert streamfuse.STATS["stream_replays"] == r0 + 1  # a new rule object: analyzed again
    assert three[0] < one[0]  # the narrower range keeps fewer rows
