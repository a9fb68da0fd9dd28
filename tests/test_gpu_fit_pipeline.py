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
