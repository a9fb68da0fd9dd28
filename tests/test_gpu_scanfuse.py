"""Fused CSV scan + DQ chain (ops/scanfuse.py): the first read of a file is the eager device scan
(it records the file's schema / null / line facts), a re-read is a lazy relation whose DQ chain
runs fused into the scan.  Both must give the same rows, the same fit and the same errors; the
second read must actually take the fused kernel."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "benchmarks"))

from net.jgp.labs.sparkdq4ml_amd import LinearRegression, SparkSession, VectorAssembler, callUDF  # noqa: E402
from net.jgp.labs.sparkdq4ml_amd.dq.rules import register_lab_rules  # noqa: E402
from net.jgp.labs.sparkdq4ml_amd.ops import scanfuse  # noqa: E402
from net.jgp.labs.sparkdq4ml_amd.runtime import filecache  # noqa: E402
from net.jgp.labs.sparkdq4ml_amd.sql.plan import CsvScanRelation  # noqa: E402

pytestmark = pytest.mark.gpu


def _session():
    s = SparkSession.getActiveSession()
    if s is not None:
        s.stop()
    filecache.clear()
    spark = SparkSession.builder().master("mi355x[*]").config("dq4ml.csv.deviceThresholdBytes", "0").getOrCreate()
    register_lab_rules(spark)
    return spark


def _chain(spark, path, opts=None):
    r = spark.read().format("csv").option("inferSchema", "true")
    for k, v in (opts or {}).items():
        r = r.option(k, v)
    raw = r.load(path)
    df = raw.withColumnRenamed("_c0", "guest").withColumnRenamed("_c1", "price")
    df = df.withColumn("price_no_min", callUDF("minimumPriceRule", df.col("price")))
    df.createOrReplaceTempView("price")
    df = spark.sql("SELECT cast(guest as int) guest, price_no_min AS price FROM price WHERE price_no_min > 0")
    df = df.withColumn("price_correct_correl", callUDF("priceCorrelationRule", df.col("price"), df.col("guest")))
    df.createOrReplaceTempView("price")
    df = spark.sql("SELECT guest, price_correct_correl AS price FROM price WHERE price_correct_correl > 0")
    return raw, df.withColumn("label", df.col("price"))


def _rows(df):
    return [tuple(r) for r in df.collect()]


def _lab_csv(rng, n, term=b"\r", trailing=False, empty=0.0, long_comment=False, general=False):
    g = rng.integers(1, 36, n)
    price = np.round(5.0 * g + 20 + rng.normal(0, 3, n), 2)
    low = rng.random(n) < 0.05
    price[low] = rng.integers(3, 19, int(low.sum()))
    hi = (rng.random(n) < 0.05) & (g < 14)
    price[hi] = rng.integers(91, 199, int(hi.sum()))
    lines = []
    for i in range(n):
        if empty and rng.random() < empty:
            lines.append(b"")
        if long_comment and i % 997 == 5:
            lines.append(b"#" + b"x" * int(rng.integers(300, 5000)))
        p = repr(float(price[i])).encode()
        if general and i % 7 == 3:  # outside the numeric fast path: exponent / > 9 digits
            p = b"%.6e" % price[i] if i % 2 else b"%.9f" % price[i]
        lines.append(b"%d,%s" % (g[i], p))
    body = term.join(lines)
    return body + (term if trailing else b"")


@pytest.mark.parametrize("case", ["cr", "lf_trailing", "crlf_empty", "long_comment", "general"])
def test_fused_scan_matches_eager(tmp_path, case):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rng = np.random.default_rng(len(case))
    term = {"cr": b"\r", "lf_trailing": b"\n", "crlf_empty": b"\r\n", "long_comment": b"\n", "general": b"\r"}[case]
    data = _lab_csv(rng, 60000, term, trailing=case == "lf_trailing", empty=0.01 if case == "crlf_empty" else 0.0,
                    long_comment=case == "long_comment", general=case == "general")
    p = tmp_path / f"{case}.csv"
    p.write_bytes(data)
    opts = {"comment": "#"} if case == "long_comment" else None
    spark = _session()
    raw1, df1 = _chain(spark, str(p), opts)
    assert not isinstance(raw1._plan, CsvScanRelation)  # first read: eager scan, facts recorded
    eager = _rows(df1)
    before = scanfuse.STATS["fused_scans"]
    raw2, df2 = _chain(spark, str(p), opts)
    assert isinstance(raw2._plan, CsvScanRelation)
    assert raw2.schema == raw1.schema
    fused = _rows(df2)
    assert scanfuse.STATS["fused_scans"] == before + 1, "the re-read did not take the fused scan kernel"
    assert len(fused) == len(eager) > 40000
    assert fused == eager
    f = raw2._plan.fused
    assert f["fast_only"] == (case != "general")  # the general-parser build is exercised too
    # any other consumer of the lazy relation: the plain device scan, same rows
    raw3, _ = _chain(spark, str(p), opts)
    assert raw3.count() == raw1.count()
    spark.stop()


def test_fused_scan_fit_matches_eager(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from bench_csv_pipeline import synth_csv

    p = str(tmp_path / "lab.csv")
    synth_csv(p, 300000)
    spark = _session()

    def fit():
        _, df = _chain(spark, p)
        df = VectorAssembler().setInputCols(["guest"]).setOutputCol("features").transform(df)
        m = LinearRegression().setMaxIter(40).setRegParam(1).setElasticNetParam(1).fit(df)
        return m, df

    m1, _ = fit()
    # table mode: the fused scan stores guest / label / selection, the skinny Gram kernel reads them
    spark.conf.set("dq4ml.fit.fuseScan", "false")
    before, grams = scanfuse.STATS["fused_scans"], scanfuse.STATS["fused_grams"]
    m2, df2 = fit()
    assert scanfuse.STATS["fused_scans"] == before + 1 and scanfuse.STATS["fused_grams"] == grams
    assert m2.summary.numInstances == m1.summary.numInstances
    assert float(m2.intercept) == pytest.approx(float(m1.intercept), rel=1e-12, abs=1e-12)
    np.testing.assert_allclose(m2.coefficients.toArray(), m1.coefficients.toArray(), rtol=1e-12)
    # Gram mode: scan + DQ + assembler + statistics in one kernel, no row stored (other summation
    # order: per-window partials)
    spark.conf.set("dq4ml.fit.fuseScan", "true")
    m4, _ = fit()
    assert scanfuse.STATS["fused_grams"] == grams + 1
    assert m4.summary.numInstances == m1.summary.numInstances
    assert float(m4.intercept) == pytest.approx(float(m1.intercept), rel=1e-9, abs=1e-9)
    np.testing.assert_allclose(m4.coefficients.toArray(), m1.coefficients.toArray(), rtol=1e-9)
    assert m4.summary.rootMeanSquaredError == pytest.approx(m1.summary.rootMeanSquaredError, rel=1e-9)
    # async: the fused action issues no host sync before the fit result is read
    spark.conf.set("dq4ml.fit.async", "true")
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        _, df = _chain(spark, p)
        df = VectorAssembler().setInputCols(["guest"]).setOutputCol("features").transform(df)
        m3 = LinearRegression().setMaxIter(40).setRegParam(1).setElasticNetParam(1).fit(df)
    finally:
        torch.cuda.set_sync_debug_mode(0)
    np.testing.assert_allclose(m3.coefficients.toArray(), m1.coefficients.toArray(), rtol=1e-9)
    spark.stop()


def test_fused_scan_nulls_and_raise(tmp_path):
    """A null price: rule 1 raises (Java NPE) on the fused path exactly as on the eager one; null
    guests flow through rule 2 (-> -1, filtered)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rng = np.random.default_rng(3)
    lines = _lab_csv(rng, 30000, b"\n").split(b"\n")
    lines[100] = b"," + lines[100].split(b",")[1]  # null guest
    p = tmp_path / "nullguest.csv"
    p.write_bytes(b"\n".join(lines))
    spark = _session()
    _, d1 = _chain(spark, str(p))
    eager = _rows(d1)
    before = scanfuse.STATS["fused_scans"]
    _, d2 = _chain(spark, str(p))
    assert _rows(d2) == eager
    assert scanfuse.STATS["fused_scans"] == before + 1
    lines[200] = lines[200].split(b",")[0] + b","  # null price: minimumPriceRule throws
    p2 = tmp_path / "nullprice.csv"
    p2.write_bytes(b"\n".join(lines))
    from net.jgp.labs.sparkdq4ml_amd.sql.expressions import SparkException

    for _ in range(2):  # eager, then fused
        _, d = _chain(spark, str(p2))
        with pytest.raises(SparkException):
            _rows(d)
    spark.stop()


@pytest.mark.parametrize("case", ["header", "user_schema", "null_value", "whitespace", "nulls_fast"])
def test_fused_scan_reader_options(tmp_path, case):
    """Every reader option the device scanner takes also holds on the fused path: the eager read
    and the fused re-read of the same file give the same rows through a DQ chain (a cast, a
    filter over a nullable column, a computed column)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rng = np.random.default_rng(11)
    n = 40000
    a = rng.integers(-1000, 1000, n)
    b = np.round(rng.normal(0, 50, n), 3)
    rows = []
    for i in range(n):
        fa, fb = str(a[i]), repr(float(b[i]))
        if case in ("null_value", "nulls_fast") and i % 37 == 5:
            fb = "NA" if case == "null_value" else ""
        if case == "whitespace":
            fa, fb = " " + fa, fb + "\t"
        rows.append(f"{fa},{fb}")
    text = ("x,y\n" if case == "header" else "") + "\n".join(rows)
    p = tmp_path / f"{case}.csv"
    p.write_bytes(text.encode())
    opts = {"header": "true"} if case == "header" else {}
    if case == "null_value":
        opts["nullValue"] = "NA"
    if case == "whitespace":
        opts.update(ignoreLeadingWhiteSpace="true", ignoreTrailingWhiteSpace="true")
    spark = _session()

    def run():
        r = spark.read().format("csv").option("inferSchema", "true")
        for k, v in opts.items():
            r = r.option(k, v)
        if case == "user_schema":
            r = r.schema("x LONG, y DOUBLE")
        df = r.load(str(p))
        c0, c1 = df.columns
        df.createOrReplaceTempView("t")
        out = spark.sql(f"SELECT cast({c0} as double) * 2 AS a2, {c1} AS yy FROM t WHERE {c1} > -20 OR {c1} IS NULL")
        return df, [tuple(r) for r in out.collect()]

    d1, eager = run()
    before = scanfuse.STATS["fused_scans"]
    d2, fused = run()
    assert isinstance(d2._plan, CsvScanRelation)
    assert scanfuse.STATS["fused_scans"] == before + 1
    assert d2.schema == d1.schema
    assert len(fused) == len(eager) > 1000

    def same(x, y):
        return (x is None and y is None) or x == y

    assert all(same(u, v) for ra, rb in zip(fused, eager) for u, v in zip(ra, rb))
    fast = d2._plan.fused["fast_only"]
    assert fast == (case in ("header", "user_schema", "nulls_fast"))
    spark.stop()


def test_rebuilt_action_replays_the_lowered_fit(tmp_path, monkeypatch):
    """an action that rebuilds the lab chain over the same unchanged file reuses the
    first action's analysis and lowered kernel (sql/skey.py, scanfuse._Route) -- the kernel still
    runs every action, results bit-identical to the full path -- and a rewritten file is re-read."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from bench_csv_pipeline import synth_csv

    p = str(tmp_path / "lab.csv")
    synth_csv(p, 200000)
    spark = _session()

    def fit():
        _, df = _chain(spark, p)
        df = VectorAssembler().setInputCols(["guest"]).setOutputCol("features").transform(df)
        return LinearRegression().setMaxIter(40).setRegParam(1).setElasticNetParam(1).fit(df)

    fit()  # eager first read (facts)
    m_full = fit()  # lazy relation, lowered and remembered
    grams, replays = scanfuse.STATS["fused_grams"], scanfuse.STATS.get("route_replays", 0)
    ms = [fit() for _ in range(3)]
    assert scanfuse.STATS["fused_grams"] == grams + 3  # the fused kernel ran for every action
    assert scanfuse.STATS.get("route_replays", 0) == replays + 3
    for m in ms:
        assert np.array_equal(m.coefficients.toArray(), m_full.coefficients.toArray())
        assert float(m.intercept) == float(m_full.intercept)
    monkeypatch.setenv("DQ4ML_FUSE_ROUTES", "0")
    m_off = fit()
    assert np.array_equal(m_off.coefficients.toArray(), m_full.coefficients.toArray())
    monkeypatch.delenv("DQ4ML_FUSE_ROUTES")
    # the file changes: its identity changes, nothing stale is replayed
    import time

    time.sleep(0.01)
    synth_csv(p, 150000)
    fit()
    m_new = fit()
    assert m_new.summary.numInstances != m_full.summary.numInstances
    spark.stop()
