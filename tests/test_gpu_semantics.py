"""GPU side of ``test_sql_semantics.py``: Spark NaN ordering through the fused hipRTC DQ chain,
and asynchronous fits on nullable data that never synchronise with the host (data errors ride
along as device flags, ``runtime/checks.py``)."""
import numpy as np
import pytest
import torch

from net.jgp.labs.sparkdq4ml_amd import LinearRegression, VectorAssembler, callUDF
from net.jgp.labs.sparkdq4ml_amd.dq.rules import register_lab_rules
from net.jgp.labs.sparkdq4ml_amd.sql.expressions import SparkException

pytestmark = pytest.mark.gpu


def test_fused_chain_nan_semantics(gpu_session, tmp_path):
    from net.jgp.labs.sparkdq4ml_amd.ops import dqvm

    p = tmp_path / "nan.csv"
    p.write_bytes(b"1,NaN\r2,30.0\r3,10.0\r4,120.0\r5,NaN")
    register_lab_rules(gpu_session)
    df = gpu_session.read().format("csv").option("inferSchema", "true").load(str(p))
    df = df.withColumnRenamed("_c0", "guest").withColumnRenamed("_c1", "price")
    df = df.withColumn("price_no_min", callUDF("minimumPriceRule", df.col("price")))
    df.createOrReplaceTempView("price")
    df = gpu_session.sql("SELECT cast(guest as int) guest, price_no_min AS price FROM price WHERE price_no_min > 0")
    df = df.withColumn("price_correct_correl", callUDF("priceCorrelationRule", df.col("price"), df.col("guest")))
    df.createOrReplaceTempView("price")
    df = gpu_session.sql("SELECT guest, price_correct_correl AS price FROM price WHERE price_correct_correl > 0")
    before = dqvm.STATS["fused_launches"]
    rows = df.collect()
    assert dqvm.STATS["fused_launches"] > before  # really the generated kernel
    assert [r[0] for r in rows] == [1, 2, 5] and np.isnan(rows[0][1]) and np.isnan(rows[2][1])
    df2 = gpu_session.read().format("csv").option("inferSchema", "true").load(str(p))
    df2.createOrReplaceTempView("t")
    got = sorted(r[0] for r in gpu_session.sql("SELECT _c0 FROM t WHERE _c1 = _c1 AND _c1 >= 120.0").collect())
    assert got == [1, 4, 5]


def test_async_fit_on_nullable_data_has_no_host_sync(gpu_session):
    gpu_session.conf.set("dq4ml.fit.async", "true")
    n = 200_000
    g = torch.Generator(device="cuda").manual_seed(3)
    x1 = torch.randn(n, generator=g, device="cuda", dtype=torch.float64)
    x2 = torch.randn(n, generator=g, device="cuda", dtype=torch.float64)
    valid = torch.ones(n, dtype=torch.bool, device="cuda")
    y = 3 * x1 - x2 + 1
    df = gpu_session.createDataFrame({"x1": (x1, valid), "x2": x2, "label": (y, valid)})
    df = VectorAssembler().setInputCols(["x1", "x2"]).setOutputCol("features").transform(df)
    lr = LinearRegression(solver="normal")
    lr.fit(df).coefficients  # warm-up: kernels, caches
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")  # any implicit device->host sync raises
    try:
        models = [lr.fit(df) for _ in range(3)]
    finally:
        torch.cuda.set_sync_debug_mode("default")
    for m in models:
        np.testing.assert_allclose(m.coefficients.toArray(), [3.0, -1.0], atol=1e-9)
    bad = valid.clone()
    bad[12345] = False
    df_bad = gpu_session.createDataFrame({"x1": (x1, bad), "x2": x2, "label": y})
    df_bad = VectorAssembler().setInputCols(["x1", "x2"]).setOutputCol("features").transform(df_bad)
    m = lr.fit(df_bad)  # no error yet: the null is a pending device flag
    with pytest.raises(SparkException, match="Values to assemble cannot be null"):
        m.coefficients
    gpu_session.conf.set("dq4ml.fit.async", "false")
