"""Pipelined asynchronous fits (``dq4ml.fit.pipeline``): consecutive fits' statistics passes run on
alternating compute streams so their Gram kernels overlap at the boundaries.  Every fit must still
produce exactly the statistics and model of an unpipelined fit."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_pipelined_fits_equal_serial_fits(gpu_session, dtype, monkeypatch):
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression

    gpu_session.conf.set("dq4ml.fit.async", "true")
    n, d = 400_000, 32
    g = torch.Generator(device="cuda").manual_seed(11)
    X = torch.randn(d, n, generator=g, device="cuda")
    y = torch.linspace(-1, 1, d, device="cuda") @ X + 0.5
    df = gpu_session.createDataFrame({"features": X.to(dtype), "label": y})
    lr = LinearRegression(solver="normal", gramDtype="bf16")
    try:
        monkeypatch.setenv("DQ4ML_FIT_PIPELINE", "1")
        serial = [lr.fit(df) for _ in range(3)]
        monkeypatch.setenv("DQ4ML_FIT_PIPELINE", "2")
        piped = [lr.fit(df) for _ in range(5)]
        torch.cuda.synchronize()
        ref = serial[0].coefficients.toArray()
        for m in serial + piped:
            np.testing.assert_array_equal(m.coefficients.toArray(), ref)
            assert m.intercept == serial[0].intercept
        assert piped[-1].summary.r2 == serial[0].summary.r2
    finally:
        gpu_session.conf.set("dq4ml.fit.async", "false")


def test_fit_replay_equals_full_path_and_invalidates(gpu_session, monkeypatch):
    # a repeated asynchronous fit of the same DataFrame replays the recorded Gram launch
    # (models/regression.py _FitReplay); every change of params / conf / data drops it
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression

    gpu_session.conf.set("dq4ml.fit.async", "true")
    n, d = 300_000, 24
    g = torch.Generator(device="cuda").manual_seed(12)
    X = torch.randn(d, n, generator=g, device="cuda")
    y = torch.linspace(-1, 1, d, device="cuda") @ X + 0.25
    df = gpu_session.createDataFrame({"features": X.to(torch.bfloat16), "label": y})
    df2 = gpu_session.createDataFrame({"features": (X * 2).to(torch.bfloat16), "label": y})
    try:
        monkeypatch.setenv("DQ4ML_FIT_REPLAY", "0")
        full = LinearRegression(solver="normal", gramDtype="bf16").fit(df)
        full_reg = LinearRegression(solver="normal", gramDtype="bf16", regParam=0.1).fit(df)
        full2 = LinearRegression(solver="normal", gramDtype="bf16").fit(df2)
        monkeypatch.delenv("DQ4ML_FIT_REPLAY")
        lr = LinearRegression(solver="normal", gramDtype="bf16")
        first = lr.fit(df)
        assert df._fit_replays.get(lr.uid) is not None
        again = [lr.fit(df) for _ in range(4)]
        for m in [first] + again:
            np.testing.assert_array_equal(m.coefficients.toArray(), full.coefficients.toArray())
            assert m.intercept == full.intercept
            assert m.summary.r2 == full.summary.r2
        lr.setRegParam(0.1)  # params changed: the full path
        np.testing.assert_array_equal(lr.fit(df).coefficients.toArray(), full_reg.coefficients.toArray())
        lr.setRegParam(0.0)
        m2 = lr.fit(df2)  # another DataFrame
        np.testing.assert_array_equal(m2.coefficients.toArray(), full2.coefficients.toArray())
        assert df2._fit_replays.get(lr.uid) is not None
        gpu_session.conf.set("dq4ml.fit.overlapTail", "false")  # conf changed
        m3 = lr.fit(df2)
        assert df2._fit_replays.get(lr.uid) is None
        np.testing.assert_array_equal(m3.coefficients.toArray(), full2.coefficients.toArray())
    finally:
        gpu_session.conf.set("dq4ml.fit.overlapTail", "true")
        gpu_session.conf.set("dq4ml.fit.async", "false")


def test_pipelined_first_fit_of_a_fresh_lazy_assembly(gpu_session, monkeypatch):
    """the first fit of a lazily assembled bf16 matrix materializes it on the CALLER's
    stream and the replays on the other pipeline stream wait for the recorded operands -- the
    pipelined fits of a fresh assembly equal the serial fit bit for bit."""
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, VectorAssembler

    n, d = 500_003, 24
    g = torch.Generator(device="cuda").manual_seed(21)
    cols = {f"f{i}": torch.randn(n, generator=g, device="cuda") for i in range(d)}
    cols["label"] = sum((0.1 * i - 1.0) * cols[f"f{i}"] for i in range(d)) + 0.5

    def frame():
        df = gpu_session.createDataFrame(dict(cols))
        return VectorAssembler(inputCols=[f"f{i}" for i in range(d)], outputCol="features",
                               outputDtype="bfloat16").transform(df)

    lr = LinearRegression(solver="normal", gramDtype="bf16")
    gpu_session.conf.set("dq4ml.fit.async", "true")
    try:
        monkeypatch.setenv("DQ4ML_FIT_PIPELINE", "1")
        ref = lr.fit(frame())
        ref_coef = ref.coefficients.toArray()
        monkeypatch.setenv("DQ4ML_FIT_PIPELINE", "2")
        df = frame()  # fresh: nothing materialized yet
        ms = [lr.fit(df) for _ in range(5)]
        for m in ms:
            np.testing.assert_array_equal(m.coefficients.toArray(), ref_coef)
            assert m.intercept == ref.intercept
    finally:
        gpu_session.conf.set("dq4ml.fit.async", "false")
