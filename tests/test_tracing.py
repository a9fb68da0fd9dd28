"""Per-stage tracing (utils/tracing.py): spans are recorded when enabled, free when disabled,
and dump to metrics.json."""
import json

import torch

from net.jgp.labs.sparkdq4ml_amd import LinearRegression
from net.jgp.labs.sparkdq4ml_amd.utils import tracing


def test_disabled_span_is_noop():
    with tracing.tracing(False):
        tracing.reset()
        with tracing.span("x"):
            pass
        assert "x" not in tracing.report()


def test_fit_records_stages(cpu_session, tmp_path):
    X = torch.randn(3, 500, dtype=torch.float64)
    y = torch.tensor([1.0, -2.0, 0.5], dtype=torch.float64) @ X + 0.25
    df = cpu_session.createDataFrame({"features": X, "label": y})
    with tracing.tracing(True):
        tracing.reset()
        m = LinearRegression(solver="normal").fit(df)
        m.summary.r2
        rep = tracing.report()
        doc = tracing.dump_json(str(tmp_path / "metrics.json"), {"run": "unit"})
    for stage in ("gram", "allreduce", "solve", "metrics"):
        assert rep[stage]["count"] >= 1 and rep[stage]["host_ms"] >= 0.0
    assert rep["gram"]["rows"] == 500 and rep["gram"]["rows_per_s"] > 0
    on_disk = json.loads((tmp_path / "metrics.json").read_text())
    assert on_disk["run"] == "unit" and set(on_disk["stages"]) == set(doc["stages"])


def test_session_config_enables_tracing():
    from net.jgp.labs.sparkdq4ml_amd import SparkSession

    prev = tracing.enabled()
    s = SparkSession.getActiveSession()
    if s is not None:
        s.stop()
    s = SparkSession.builder().master("cpu").config("dq4ml.trace", "true").config("dq4ml.bucketBytes", 1 << 20) \
        .getOrCreate()
    from net.jgp.labs.sparkdq4ml_amd.parallel import comm

    try:
        assert tracing.enabled()
        assert comm._bucket_bytes == 1 << 20
    finally:
        s.stop()
        tracing.enable(prev)
        comm.set_bucket_bytes(comm.DEFAULT_BUCKET_BYTES)


def test_session_gram_dtype_default():
    from net.jgp.labs.sparkdq4ml_amd import SparkSession
    from net.jgp.labs.sparkdq4ml_amd.models.regression import _gram_dtype

    s = SparkSession.getActiveSession()
    if s is not None:
        s.stop()
    s = SparkSession.builder().master("cpu").config("dq4ml.gramDtype", "bf16").getOrCreate()
    try:
        df = s.createDataFrame({"features": torch.randn(2, 10, dtype=torch.float64), "label": torch.randn(10)})
        assert _gram_dtype(LinearRegression(), df) == "bf16"
        assert _gram_dtype(LinearRegression(gramDtype="fp32"), df) == "fp32"
    finally:
        s.stop()


def test_logging_levels_and_log4j_pattern():
    """utils.logging mirrors log4j.properties (L4J:1-11): engine internals quiet, the app package
    at DEBUG, and the `%d -%5p --- [%15.15t] %-40.40l: %m` console pattern."""
    import logging
    import re

    from net.jgp.labs.sparkdq4ml_amd.utils import logging as dqlog

    dqlog.configure_logging()
    root = logging.getLogger(dqlog.ROOT)
    assert root.level >= logging.WARNING
    assert logging.getLogger(dqlog.ROOT + ".apps").level == logging.DEBUG
    rec = logging.LogRecord(dqlog.ROOT + ".apps.x", logging.WARNING, "/a/b/app.py", 42, "hello %s", ("world",),
                            None, func="start")
    line = dqlog._Fmt().format(rec)
    assert re.match(r"^\d{4}-\d\d-\d\d \d\d:\d\d:\d\d\.\d{3} - WARN --- \[.{15}\] .{40}: hello world$", line), line
