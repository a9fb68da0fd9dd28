"""SURVEY.md §5g / VERDICT r3 #4: the fused CSV -> DQ -> VectorAssembler -> Gram pass over an input
that is NOT resident in HBM.  The device cache is disabled (``DQ4ML_FILECACHE_DEVICE_BYTES=1``), so
``load()`` runs one streamed inference pass and the fit's action streams row-aligned chunks through
a two-slot device ring (``runtime.streams.ChunkSource``); the statistics must equal the resident
cutter / per-line path to f64 rounding, for a pinned (page-locked cache) and a mapped source."""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import ROOT

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
    s = (SparkSession.builder().master("mi355x[*]").config("dq4ml.csv.deviceThresholdBytes", "0")
         .config("dq4ml.csv.streamThresholdBytes", "0").config("dq4ml.csv.streamChunkBytes", str(3 << 20))
         .getOrCreate())
    yield s
    s.stop()
    filecache.clear()


def _stats(spark, path, d):
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, VectorAssembler, callUDF, col
    from net.jgp.labs.sparkdq4ml_amd.dq.rules import RangeRule
    from net.jgp.labs.sparkdq4ml_amd.models import regression
    from net.jgp.labs.sparkdq4ml_amd.runtime.checks import verify
    from net.jgp.labs.sparkdq4ml_amd.sql.types import DataTypes

    spark.udf().register("rangeRule", RangeRule(0.0, 150.0, name="rangeRule"), DataTypes.DoubleType)
    df = spark.read().format("csv").option("inferSchema", "true").load(path)
    df = df.withColumn("y_ok", callUDF("rangeRule", col(f"_c{d}"))).filter(col("y_ok") > 0)
    df = df.withColumn("label", col("y_ok"))
    df = VectorAssembler().setInputCols([f"_c{i}" for i in range(d)]).setOutputCol("features").transform(df)
    lr = LinearRegression(solver="normal", regParam=1e-3)
    fused = regression._fused_scan_stats(lr, df)
    assert fused is not None
    verify(fused.checks)
    return fused.flat.double().cpu().numpy(), lr.fit(df)


@pytest.mark.parametrize("d,n,mapped", [(32, 120_001, False), (32, 120_001, True), (3, 400_000, False)])
def test_streamed_fused_gram_equals_resident(spark, tmp_path, monkeypatch, d, n, mapped):
    import csv_synth

    from net.jgp.labs.sparkdq4ml_amd.ops import scanfuse
    from net.jgp.labs.sparkdq4ml_amd.runtime import filecache

    p = str(tmp_path / f"s{d}.csv")
    csv_synth.write_wide_csv(p, n, d, seed=d, device="cuda", keep=False, y0=60.0, chunk=1 << 16)
    size = os.path.getsize(p)
    # resident reference: the default device cache (a first load types the bytes)
    spark.read().format("csv").option("inferSchema", "true").load(p).count()
    ref, m_ref = _stats(spark, p, d)
    filecache.clear()
    monkeypatch.setenv("DQ4ML_FILECACHE_DEVICE_BYTES", "1")  # nothing may stay resident
    if mapped:
        monkeypatch.setattr(filecache, "MAX_BYTES", size // 2)  # beyond the pinned cache: read-only map
    before = scanfuse.STATS.get("streamed_grams", 0)
    got, m = _stats(spark, p, d)
    assert scanfuse.STATS.get("streamed_grams", 0) == before + 2  # the stats call and the fit
    assert size > 4 * (3 << 20)  # several chunks
    tol = 1e-12 * np.maximum(np.abs(ref), 1.0)
    assert np.all(np.abs(got - ref) <= tol), (np.abs(got - ref) / np.maximum(np.abs(ref), 1.0)).max()
    np.testing.assert_allclose(m.coefficients.toArray(), m_ref.coefficients.toArray(), rtol=1e-10, atol=1e-12)
    # a second action re-streams the same chunks: bitwise identical (fixed chunking, fixed order)
    again, _ = _stats(spark, p, d)
    assert np.array_equal(again, got)


def test_streamed_relation_other_actions_scan_eagerly(spark, tmp_path, monkeypatch):
    import csv_synth

    p = str(tmp_path / "e.csv")
    csv_synth.write_wide_csv(p, 60_000, 8, seed=3, device="cuda", keep=False, y0=60.0, chunk=1 << 16)
    monkeypatch.setenv("DQ4ML_FILECACHE_DEVICE_BYTES", "1")
    df = spark.read().format("csv").option("inferSchema", "true").load(p)
    assert df.count() == 60_000
    rows = df.take(3)
    assert len(rows) == 3 and len(rows[0]) == 9


@pytest.mark.parametrize("mapped,chunked", [(False, False), (True, False), (True, True)])
def test_first_upload_in_pieces_is_exact(spark, tmp_path, monkeypatch, mapped, chunked):
    """runtime.filecache first upload in many pieces (pinned: events on the side stream; mapped:
    the uploader thread's bounce buffers) consumed progressively by the first scan -- with
    ``chunked``, scan chunks (256 KiB) smaller than the pieces (1 MiB), so each chunk waits for the
    piece holding its last byte: the resident bytes equal the file and the scan equals a fresh
    host-staged one."""
    import csv_synth

    from net.jgp.labs.sparkdq4ml_amd.ops import csvscan
    from net.jgp.labs.sparkdq4ml_amd.runtime import filecache

    p = str(tmp_path / "u.csv")
    csv_synth.write_wide_csv(p, 50_000, 6, seed=5, device="cuda", keep=False, y0=60.0, chunk=1 << 16)
    size = os.path.getsize(p)
    monkeypatch.setattr(filecache, "_UPLOAD_PIECE", 1 << 20)  # ~ size / 1 MiB pieces
    if mapped:
        monkeypatch.setattr(filecache, "MAX_BYTES", size // 2)
    if chunked:
        monkeypatch.setattr(csvscan, "MIN_RESIDENT_CHUNK", 1 << 18)
        spark.conf.set("dq4ml.chunkBytes", str(1 << 18))
    try:
        df = spark.read().format("csv").option("inferSchema", "true").load(p)
        got = np.array([list(r) for r in df.collect()], dtype=np.float64)
    finally:
        spark.conf.set("dq4ml.chunkBytes", str(256 << 20))
    entries = list((filecache._mapped if mapped else filecache._cache).values())
    assert len(entries) == 1 and len(entries[0]._dev) == 1
    resident = next(iter(entries[0]._dev.values()))
    with open(p, "rb") as f:
        raw = np.frombuffer(f.read(), dtype=np.uint8)
    assert np.array_equal(resident.cpu().numpy(), raw)
    filecache.clear()
    monkeypatch.setenv("DQ4ML_FILECACHE_DEVICE_BYTES", "1")  # reference: nothing resident
    df2 = spark.read().format("csv").option("inferSchema", "true").load(p)
    ref = np.array([list(r) for r in df2.collect()], dtype=np.float64)
    assert got.shape == (50_000, 7) and np.array_equal(got, ref)


@pytest.mark.parametrize("hinted", [False, True])
def test_resident_multichunk_scan_writes_shared_planes(spark, tmp_path, monkeypatch, hinted):
    """A resident input scanned in many chunks: every chunk parses straight into one plane per
    column (csvscan._Planes, no per-chunk allocation, no concatenation); the table equals the
    one-chunk scan exactly, for the inferring scan and the hinted (typed) re-scan."""
    import csv_synth

    from net.jgp.labs.sparkdq4ml_amd.ops import csvscan
    from net.jgp.labs.sparkdq4ml_amd.runtime import filecache

    p = str(tmp_path / "m.csv")
    csv_synth.write_wide_csv(p, 40_000, 5, seed=9, device="cuda", keep=False, y0=60.0, chunk=1 << 16)

    def read():
        df = spark.read().format("csv").option("inferSchema", "true").load(p)
        if hinted:  # a second load of the same bytes: the typed (hinted) device scan
            df = spark.read().format("csv").option("inferSchema", "true").load(p)
        return np.array([list(r) for r in df.collect()], dtype=np.float64), df

    ref, _ = read()
    filecache.clear()
    monkeypatch.setattr(csvscan, "MIN_RESIDENT_CHUNK", 1 << 18)  # ~8 chunks
    spark.conf.set("dq4ml.chunkBytes", str(1 << 18))
    seen = []
    orig = csvscan._finish

    def spy(parts, *a, **k):
        seen.append(isinstance(parts, csvscan._Shared) and len(parts))
        return orig(parts, *a, **k)
    monkeypatch.setattr(csvscan, "_finish", spy)
    try:
        got, _ = read()
    finally:
        spark.conf.set("dq4ml.chunkBytes", str(256 << 20))
    assert seen and all(x and x > 2 for x in seen), seen  # every eager scan took the shared planes
    assert np.array_equal(got, ref)
