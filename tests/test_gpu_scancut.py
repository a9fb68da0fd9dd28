"""The byte-parallel CSV cutter (``ops/scancut.py``): CSV -> DQ chain -> VectorAssembler -> f64
normal-equation statistics in one kernel, checked against fp64 numpy sums of the values the CSV
holds (the generator returns them exactly) and against the per-line fused kernel."""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import ROOT, data_path

sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
pytestmark = pytest.mark.gpu


@pytest.fixture
def spark():
    from net.jgp.labs.sparkdq4ml_amd import SparkSession
    from net.jgp.labs.sparkdq4ml_amd.runtime import filecache

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    s = SparkSession.getActiveSession()
    if s is not None:
        s.stop()
    filecache.clear()
    s = SparkSession.builder().master("mi355x[*]").config("dq4ml.csv.deviceThresholdBytes", "0").getOrCreate()
    os.environ["DQ4ML_CUT_MIN_LINE"] = "0"  # the cutter on short rows too (routing is tested below)
    yield s
    os.environ.pop("DQ4ML_CUT_MIN_LINE", None)
    s.stop()


def _oracle(X, y, keep):
    """gram_stats layout over the kept rows: [n, n, n, Σy, Σy², Σx, Σxy, packed-upper Σxx]."""
    Xk, yk = X[:, keep].astype(np.float64), y[keep].astype(np.float64)
    d = Xk.shape[0]
    n = float(keep.sum())
    G = Xk @ Xk.T
    iu = [(i, j) for j in range(d) for i in range(j + 1)]
    return np.concatenate([[n, n, n, yk.sum(), (yk * yk).sum()], Xk.sum(1), Xk @ yk,
                           np.array([G[i, j] for i, j in iu])])


def _fit_stats(spark, path, d, lo=0.0, hi=150.0):
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, VectorAssembler, callUDF, col
    from net.jgp.labs.sparkdq4ml_amd.dq.rules import RangeRule
    from net.jgp.labs.sparkdq4ml_amd.models import regression
    from net.jgp.labs.sparkdq4ml_amd.sql.types import DataTypes

    spark.udf().register("rangeRule", RangeRule(lo, hi, name="rangeRule"), DataTypes.DoubleType)
    df = spark.read().format("csv").option("inferSchema", "true").load(path)
    df = df.withColumn("y_ok", callUDF("rangeRule", col(f"_c{d}"))).filter(col("y_ok") > 0)
    df = df.withColumn("label", col("y_ok"))
    df = VectorAssembler().setInputCols([f"_c{i}" for i in range(d)]).setOutputCol("features").transform(df)
    lr = LinearRegression(solver="normal", regParam=1e-3)
    return regression._fused_scan_stats(lr, df), lr, df


def _write(tmp_path, n, d, term=b"\r", seed=5):
    import csv_synth

    p = str(tmp_path / f"w{d}.csv")
    _, beta, X, y = csv_synth.write_wide_csv(p, n, d, seed=seed, device="cuda", keep=True, y0=60.0, chunk=1 << 16)
    if term != b"\r":
        data = open(p, "rb").read().replace(b"\r", term)
        open(p, "wb").write(data)
    return p, X.numpy(), y.numpy()


@pytest.mark.parametrize("d,n,term", [(32, 150_001, b"\r"), (8, 90_000, b"\n"), (9, 90_000, b"\r\n"),
                                      (64, 40_003, b"\r"), (3, 70_000, b"\r"), (40, 40_001, b"\n")])
def test_cutter_gram_matches_fp64_oracle(spark, tmp_path, d, n, term):
    from net.jgp.labs.sparkdq4ml_amd.ops import scancut

    path, X, y = _write(tmp_path, n, d, term)
    spark.read().format("csv").option("inferSchema", "true").load(path).count()  # eager scan: facts
    before = scancut.STATS["cut_grams"]
    fused, lr, df = _fit_stats(spark, path, d)
    assert fused is not None and scancut.STATS["cut_grams"] == before + 1
    got = fused.flat.cpu().numpy()
    from net.jgp.labs.sparkdq4ml_amd.runtime.checks import verify

    verify(fused.checks)
    keep = (y > 0) & (y <= 150.0)
    ref = _oracle(X, y, keep)
    # f64 sums in a different order: the error bound scales with the sum of |terms|
    absref = _oracle(np.abs(X), np.abs(y), keep)
    err = np.abs(got - ref)
    assert np.all(err <= 1e-13 * np.maximum(absref, 1.0)), (err / np.maximum(absref, 1.0)).max()
    # the fit itself through the fused path, and a repeat is bitwise identical (fixed-order folds)
    m1 = lr.fit(df)
    m2 = lr.fit(df)
    assert np.array_equal(m1.coefficients.toArray(), m2.coefficients.toArray())


def test_cutter_matches_per_line_kernel_on_lab_pipeline(spark, tmp_path, monkeypatch):
    """The lab's own chain (minimumPriceRule, SQL clean-up, priceCorrelationRule, cast, assembler
    of the int guest column, OWLQN fit) on a synthetic guest,price CSV: cutter == per-line kernel."""
    import bench_csv_pipeline as B

    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, VectorAssembler, callUDF
    from net.jgp.labs.sparkdq4ml_amd.dq.rules import register_lab_rules
    from net.jgp.labs.sparkdq4ml_amd.models import regression
    from net.jgp.labs.sparkdq4ml_amd.ops import scancut

    p = str(tmp_path / "lab.csv")
    B.synth_csv(p, 300_000)
    register_lab_rules(spark)
    spark.read().format("csv").option("inferSchema", "true").load(p).count()

    def stats():
        df = spark.read().format("csv").option("inferSchema", "true").load(p)
        df = df.withColumnRenamed("_c0", "guest").withColumnRenamed("_c1", "price")
        df = df.withColumn("price_no_min", callUDF("minimumPriceRule", df.col("price")))
        df.createOrReplaceTempView("price")
        df = spark.sql("SELECT cast(guest as int) guest, price_no_min AS price FROM price WHERE price_no_min > 0")
        df = df.withColumn("price_correct_correl", callUDF("priceCorrelationRule", df.col("price"), df.col("guest")))
        df.createOrReplaceTempView("price")
        df = spark.sql("SELECT guest, price_correct_correl AS price FROM price WHERE price_correct_correl > 0")
        df = df.withColumn("label", df.col("price"))
        df = VectorAssembler().setInputCols(["guest"]).setOutputCol("features").transform(df)
        lr = LinearRegression().setMaxIter(40).setRegParam(1).setElasticNetParam(1)
        return regression._fused_scan_stats(lr, df), lr, df

    before = scancut.STATS["cut_grams"]
    cut, lr, df = stats()
    assert scancut.STATS["cut_grams"] == before + 1
    monkeypatch.setenv("DQ4ML_SCAN_CUT", "0")
    line, _, _ = stats()
    a, b = cut.flat.cpu().numpy(), line.flat.cpu().numpy()
    assert a[0] == b[0] and 0 < a[0] < 300_000  # same surviving row count
    np.testing.assert_allclose(a, b, rtol=1e-13)
    monkeypatch.delenv("DQ4ML_SCAN_CUT")
    m = lr.fit(df)
    assert abs(m.coefficients[0] - 5.0) < 0.2


def test_cutter_on_reference_dataset_matches_golden(spark, tmp_path):
    """dataset-full.csv (CR-only, no final terminator, int + 1-2 decimal prices) through the
    cutter: the DQ survivors' statistics equal the host scanner's."""
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, VectorAssembler, callUDF, col
    from net.jgp.labs.sparkdq4ml_amd.dq.rules import register_lab_rules
    from net.jgp.labs.sparkdq4ml_amd.models import regression

    register_lab_rules(spark)
    path = data_path("dataset-full.csv")
    raw = np.array([[float(t) for t in r.split(",")] for r in open(path, "rb").read().decode().split("\r")])
    spark.read().format("csv").option("inferSchema", "true").load(path).count()
    df = spark.read().format("csv").option("inferSchema", "true").load(path)
    df = df.withColumn("p1", callUDF("minimumPriceRule", col("_c1"))).filter(col("p1") > 0)
    df = df.withColumn("label", col("p1"))
    df = VectorAssembler().setInputCols(["_c0"]).setOutputCol("features").transform(df)
    fused = regression._fused_scan_stats(LinearRegression(), df)
    if fused is None:
        pytest.skip("file below the device-scan threshold: host engine")
    keep = raw[:, 1] >= 20
    ref = _oracle(raw[:, :1].T, raw[:, 1], keep)
    np.testing.assert_allclose(fused.flat.cpu().numpy(), ref, rtol=1e-13)


def _lab_df(spark, path):
    from net.jgp.labs.sparkdq4ml_amd import VectorAssembler, callUDF

    df = spark.read().format("csv").option("inferSchema", "true").load(path)
    df = df.withColumnRenamed("_c0", "guest").withColumnRenamed("_c1", "price")
    df = df.withColumn("price_no_min", callUDF("minimumPriceRule", df.col("price")))
    df.createOrReplaceTempView("price")
    df = spark.sql("SELECT cast(guest as int) guest, price_no_min AS price FROM price WHERE price_no_min > 0")
    df = df.withColumn("price_correct_correl", callUDF("priceCorrelationRule", df.col("price"), df.col("guest")))
    df.createOrReplaceTempView("price")
    df = spark.sql("SELECT guest, price_correct_correl AS price FROM price WHERE price_correct_correl > 0")
    df = df.withColumn("label", df.col("price"))
    return VectorAssembler().setInputCols(["guest"]).setOutputCol("features").transform(df)


def test_lab_pipeline_on_csv_has_no_host_sync_and_defers_the_npe(spark, tmp_path):
    """the lab's CSV -> rules -> fit action issues no device->host sync (async fit,
    ``set_sync_debug_mode("error")``), and a null price still fails the job with the rule's NPE
    (``MinimumPriceDataQualityUdf.java:11-13``) — raised on the first host read of the model."""
    import bench_csv_pipeline as B

    from net.jgp.labs.sparkdq4ml_amd import LinearRegression
    from net.jgp.labs.sparkdq4ml_amd.dq.rules import register_lab_rules
    from net.jgp.labs.sparkdq4ml_amd.sql.expressions import SparkException

    spark.conf.set("dq4ml.fit.async", "true")
    register_lab_rules(spark)
    p = str(tmp_path / "lab.csv")
    B.synth_csv(p, 200_000)
    spark.read().format("csv").option("inferSchema", "true").load(p).count()  # the eager scan: facts
    lr = LinearRegression().setMaxIter(40).setRegParam(1).setElasticNetParam(1)
    ref = lr.fit(_lab_df(spark, p)).coefficients[0]  # warm-up: kernels compiled, plans cached
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        models = [lr.fit(_lab_df(spark, p)) for _ in range(2)]
    finally:
        torch.cuda.set_sync_debug_mode("default")
    assert all(m.coefficients[0] == ref for m in models)
    # a null price (an empty field) in the middle of the file
    data = bytearray(open(p, "rb").read())
    cut = data.index(b"\r", len(data) // 2) + 1
    comma = data.index(b",", cut)
    end = data.index(b"\r", comma)
    q = str(tmp_path / "lab_null.csv")
    open(q, "wb").write(bytes(data[:comma + 1] + data[end:]))
    spark.read().format("csv").option("inferSchema", "true").load(q).count()
    m = lr.fit(_lab_df(spark, q))
    with pytest.raises(SparkException, match="NullPointerException"):
        m.coefficients
    spark.conf.set("dq4ml.fit.async", "false")


def test_short_rows_route_to_the_per_line_kernel(spark, tmp_path, monkeypatch):
    """Below MIN_MEAN_LINE bytes per line (d <= 8) the per-line fused scan runs, not the cutter."""
    import bench_csv_pipeline as B

    from net.jgp.labs.sparkdq4ml_amd import LinearRegression
    from net.jgp.labs.sparkdq4ml_amd.dq.rules import register_lab_rules
    from net.jgp.labs.sparkdq4ml_amd.models import regression
    from net.jgp.labs.sparkdq4ml_amd.ops import scancut

    monkeypatch.delenv("DQ4ML_CUT_MIN_LINE")
    register_lab_rules(spark)
    p = str(tmp_path / "lab.csv")
    B.synth_csv(p, 100_000)
    spark.read().format("csv").option("inferSchema", "true").load(p).count()
    before = scancut.STATS["cut_grams"]
    fused = regression._fused_scan_stats(LinearRegression(), _lab_df(spark, p))
    assert fused is not None and scancut.STATS["cut_grams"] == before


def test_cutter_converts_quoted_numbers(spark, tmp_path):
    """a wide CSV whose numbers are partly written as ``"1.25"`` keeps the cutter.
    The eager scan records ``quoted_fast`` (every fast-path miss was a simple quoted number), the
    QUOTED build strips the quotes in the convert loop, and the Gram equals the unquoted file's."""
    from net.jgp.labs.sparkdq4ml_amd.ops import scancut

    d, n = 32, 60_001
    plain, X, y = _write(tmp_path, n, d)
    lines = open(plain, "rb").read().split(b"\r")
    out = []
    for i, ln in enumerate(lines):
        if not ln:
            out.append(ln)
            continue
        fs = ln.split(b",")
        out.append(b",".join(b'"' + f + b'"' if (i + j) % 2 == 0 else f for j, f in enumerate(fs)))
    quoted = str(tmp_path / "q.csv")
    open(quoted, "wb").write(b"\r".join(out))

    res = {}
    for name, p in (("plain", plain), ("quoted", quoted)):
        assert spark.read().format("csv").option("inferSchema", "true").load(p).count() == n  # eager: facts
        facts = spark.read().format("csv").option("inferSchema", "true").load(p)._plan.fused  # lazy re-read
        if name == "quoted":
            assert facts["fast_only"] is False and facts["quoted_fast"] is True
        before = scancut.STATS["cut_grams"]
        fused, lr, df = _fit_stats(spark, p, d)
        assert fused is not None and scancut.STATS["cut_grams"] == before + 1, name
        res[name] = (fused.flat.cpu().numpy(), lr.fit(df).coefficients.toArray())
    (g0, c0), (g1, c1) = res["plain"], res["quoted"]
    # same numbers, same fixed-order folds: the quoted file's Gram is the plain file's
    assert np.allclose(g1, g0, rtol=1e-12, atol=0)
    assert np.allclose(c1, c0, rtol=1e-10, atol=1e-12)
    keep = (y > 0) & (y <= 150.0)
    ref = _oracle(X, y, keep)
    absref = _oracle(np.abs(X), np.abs(y), keep)
    assert np.all(np.abs(g1 - ref) <= 1e-13 * np.maximum(absref, 1.0))
