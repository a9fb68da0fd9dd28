"""Spark SQL semantics beyond the lab transcript: NaN-aware float ordering (SQL comparisons vs the
Java UDF bodies), ``describe()``, and a null weight failing the fit."""
import numpy as np
import pytest
import torch

from conftest import data_path
from net.jgp.labs.sparkdq4ml_amd import LinearRegression, VectorAssembler, callUDF
from net.jgp.labs.sparkdq4ml_amd.dq.rules import register_lab_rules
from net.jgp.labs.sparkdq4ml_amd.sql.expressions import SparkException
from net.jgp.labs.sparkdq4ml_amd.utils.javafmt import java_str


def _nan_df(spark, tmp_path):
    p = tmp_path / "nan.csv"
    p.write_bytes(b"1,NaN\r2,30.0\r3,10.0\r4,120.0")
    df = spark.read().format("csv").option("inferSchema", "true").load(str(p))
    return df.withColumnRenamed("_c0", "guest").withColumnRenamed("_c1", "price")


def test_sql_nan_ordering(cpu_session, tmp_path):
    df = _nan_df(cpu_session, tmp_path)
    df.createOrReplaceTempView("t")
    q = lambda w: sorted(r[0] for r in cpu_session.sql(f"SELECT guest FROM t WHERE {w}").collect())  # noqa: E731
    assert q("price > 0") == [1, 2, 3, 4]          # NaN is above every double
    assert q("price = price") == [1, 2, 3, 4]      # NaN = NaN
    assert q("price < 1e300") == [2, 3, 4]
    assert q("price >= 120.0") == [1, 4]
    assert q("price <= 30.0") == [2, 3]
    assert q("price != price") == []


def test_lab_rules_keep_nan_like_spark(cpu_session, tmp_path):
    """Rule bodies compare like Java (NaN < 20 is false -> the price passes through), the SQL
    clean-up filter like Spark (NaN > 0 is true): the NaN row survives both DQ steps."""
    register_lab_rules(cpu_session)
    df = _nan_df(cpu_session, tmp_path)
    df = df.withColumn("price_no_min", callUDF("minimumPriceRule", df.col("price")))
    df.createOrReplaceTempView("price")
    df = cpu_session.sql("SELECT cast(guest as int) guest, price_no_min AS price FROM price WHERE price_no_min > 0")
    df = df.withColumn("price_correct_correl", callUDF("priceCorrelationRule", df.col("price"), df.col("guest")))
    df.createOrReplaceTempView("price")
    df = cpu_session.sql("SELECT guest, price_correct_correl AS price FROM price WHERE price_correct_correl > 0")
    rows = df.collect()
    assert [r[0] for r in rows] == [1, 2]  # (3, 10.0) fails rule 1, (4, 120.0) fails rule 2
    assert np.isnan(rows[0][1]) and rows[1][1] == 30.0


def test_describe_matches_spark_stats(cpu_session):
    df = cpu_session.read().format("csv").option("inferSchema", "true").load(data_path("dataset-abstract.csv"))
    out = df.describe()
    assert out.columns == ["summary", "_c0", "_c1"]
    rows = {r[0]: r[1:] for r in out.collect()}
    raw = np.array([[float(x) for x in ln.split(",")] for ln in
                    open(data_path("dataset-abstract.csv"), "rb").read().decode().split("\r")])
    assert rows["count"] == ("40", "40")
    assert rows["mean"][1] == java_str(float(raw[:, 1].mean()))
    assert float(rows["stddev"][0]) == pytest.approx(raw[:, 0].std(ddof=1), rel=1e-12)
    assert rows["min"] == (str(int(raw[:, 0].min())), java_str(raw[:, 1].min()))
    assert rows["max"] == (str(int(raw[:, 0].max())), java_str(raw[:, 1].max()))
    one = cpu_session.createDataFrame({"a": torch.tensor([2.5], dtype=torch.float64)}).describe("a").collect()
    assert one[2][1] == "NaN"  # stddev_samp of one value


def test_describe_drops_non_numeric_and_orders_nan_last(cpu_session):
    """StatFunctions.summary keeps numeric / string columns only (booleans and vectors
    vanish, even when named) and orders NaN above every double (min skips it, max returns it)."""
    df = cpu_session.createDataFrame({"x": torch.tensor([1.0, float("nan"), -2.0], dtype=torch.float64),
                                      "b": torch.tensor([True, False, True]),
                                      "v": torch.ones(2, 3, dtype=torch.float64)})
    from net.jgp.labs.sparkdq4ml_amd import VectorAssembler

    df = VectorAssembler().setInputCols(["x"]).setOutputCol("vec").transform(df.select("x", "b"))
    out = df.describe("x", "b", "vec")
    assert out.columns == ["summary", "x"]
    rows = {r[0]: r[1] for r in out.collect()}
    assert rows["min"] == "-2.0" and rows["max"] == "NaN" and rows["mean"] == "NaN"
    allnan = cpu_session.createDataFrame({"x": torch.tensor([float("nan")] * 2, dtype=torch.float64)}).describe()
    assert {r[0]: r[1] for r in allnan.collect()}["min"] == "NaN"


def test_null_weight_fails_fit(cpu_session):
    X = torch.arange(5, dtype=torch.float64).unsqueeze(0)
    y = 2 * X[0] + 1
    w = (torch.ones(5, dtype=torch.float64), torch.tensor([True, True, False, True, True]))
    df = cpu_session.createDataFrame({"features": X, "label": y, "w": w})
    with pytest.raises(SparkException, match="MatchError"):
        LinearRegression(weightCol="w").fit(df)
    ok = cpu_session.createDataFrame({"features": X, "label": y, "w": torch.ones(5, dtype=torch.float64)})
    m = LinearRegression(weightCol="w").fit(ok)
    assert m.coefficients[0] == pytest.approx(2.0) and m.summary.numInstances == 5


def test_assembler_null_error_surfaces_on_read(cpu_session):
    x = (torch.tensor([1.0, 2.0, 3.0], dtype=torch.float64), torch.tensor([True, False, True]))
    df = cpu_session.createDataFrame({"x": x, "label": torch.tensor([1.0, 2.0, 3.0], dtype=torch.float64)})
    with pytest.raises(SparkException, match="Values to assemble cannot be null"):
        VectorAssembler().setInputCols(["x"]).setOutputCol("features").transform(df).collect()
