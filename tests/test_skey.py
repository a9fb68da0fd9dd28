"""Structural sharing of analysis across actions (sql/skey.py): a chain rebuilt over
the same input reuses the analyzed nodes (fresh copies, never an execution result), and anything
that changes the computation -- another UDF registered under the same name, a replaced view, a
different literal -- changes the key."""
import pytest

from net.jgp.labs.sparkdq4ml_amd import SparkSession, VectorAssembler, callUDF, col
from net.jgp.labs.sparkdq4ml_amd.sql import dataframe as dfmod
from net.jgp.labs.sparkdq4ml_amd.sql.types import DataTypes


@pytest.fixture
def spark():
    s = SparkSession.builder().appName("skey").master("cpu").getOrCreate()
    yield s
    s.stop()


def _chain(spark, base, thresh=10.0):
    df = base.withColumnRenamed("a", "guest").withColumn("p2", callUDF("twice", col("b")))
    df.createOrReplaceTempView("t")
    df = spark.sql(f"SELECT guest, p2 AS price FROM t WHERE p2 > {thresh}")
    return VectorAssembler().setInputCols(["guest"]).setOutputCol("features").transform(df)


def test_rebuilt_chain_shares_analysis_not_results(spark):
    spark.udf().register("twice", lambda v: None if v is None else 2.0 * v, DataTypes.DoubleType)
    base = spark.createDataFrame([(1, 4.0), (2, 6.0), (3, 9.0)], ["a", "b"])
    d1 = _chain(spark, base)
    assert d1.count() == 2
    d2 = _chain(spark, base)
    assert d2._plan is not d1._plan and d2._plan.skey() == d1._plan.skey()
    assert d2._plan._memo is None  # nothing executed is handed to the next action
    assert d2.schema is d1.schema  # the analysis is
    assert sorted(r[0] for r in d2.collect()) == [2, 3]
    assert len(dfmod._DERIVED) > 0


def test_keys_follow_udfs_views_and_literals(spark):
    spark.udf().register("twice", lambda v: None if v is None else 2.0 * v, DataTypes.DoubleType)
    base = spark.createDataFrame([(1, 4.0), (2, 6.0), (3, 9.0)], ["a", "b"])
    k1 = _chain(spark, base)._plan.skey()
    assert _chain(spark, base, thresh=12.0)._plan.skey() != k1  # another literal
    spark.udf().register("twice", lambda v: None if v is None else 3.0 * v, DataTypes.DoubleType)
    d = _chain(spark, base)
    assert d._plan.skey() != k1  # the name now resolves to another UDF
    assert sorted(r[0] for r in d.collect()) == [1, 2, 3]  # 3 * b > 10 everywhere
    other = spark.createDataFrame([(7, 100.0)], ["a", "b"])
    assert _chain(spark, other)._plan.skey() != d._plan.skey()  # another input relation
    assert [r[0] for r in _chain(spark, other).collect()] == [7]
