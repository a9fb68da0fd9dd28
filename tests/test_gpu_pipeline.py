"""End-to-end lab pipeline on the MI355X: DQ + assemble + fit through the HIP kernels."""
import pytest
import torch

from conftest import data_path
from test_app_golden import ORACLE, run_pipeline

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", sorted(ORACLE))
def test_golden_gpu_fp64(gpu_session, name):
    counts, model, df = run_pipeline(gpu_session, name, "fp64")
    o = ORACLE[name]
    assert counts == o[:3]
    assert df._table().column("features").values.is_cuda
    assert model.coefficients[0] == pytest.approx(o[3], rel=1e-9)
    assert model.intercept == pytest.approx(o[4], rel=1e-9)
    assert model.summary.rootMeanSquaredError == pytest.approx(o[5], rel=1e-9)
    assert model.summary.r2 == pytest.approx(o[6], rel=1e-9)


@pytest.mark.parametrize("name", sorted(ORACLE))
def test_golden_gpu_bf16(gpu_session, name):
    # guest is a small integer (exact in bf16); the label keeps ~16 bits through the hi/lo split
    counts, model, _ = run_pipeline(gpu_session, name, "bf16")
    o = ORACLE[name]
    assert model.coefficients[0] == pytest.approx(o[3], rel=1e-4)
    assert model.intercept == pytest.approx(o[4], rel=1e-4)


def test_app_transcript_gpu(gpu_session, capsys):
    from net.jgp.labs.sparkdq4ml_amd.apps.dq4ml_app import DataQuality4MachineLearningApp

    gpu_session.stop()
    DataQuality4MachineLearningApp(data_path("dataset-abstract.csv"), "mi355x[*]").start()
    out = capsys.readouterr().out
    assert "Prediction for 40.0 guests is 218.00351106" in out
    assert "r2: 0.99653409533" in out
    assert torch.cuda.is_available()


def _synth_tensors(n=20_000, d=6, seed=0, outliers=False):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(d, n, generator=g, dtype=torch.float64) + 0.5
    y = torch.linspace(-1, 2, d, dtype=torch.float64) @ X + 0.7 + 0.3 * torch.randn(n, generator=g, dtype=torch.float64)
    if outliers:
        y[::50] += 40.0
    return X, y


@pytest.mark.parametrize("kw", [dict(solver="l-bfgs", regParam=0.05, elasticNetParam=0.5, tol=1e-10, maxIter=300),
                                dict(loss="huber", maxIter=100), dict(solver="normal", regParam=0.1,
                                                                       elasticNetParam=0.2)])
def test_gpu_matches_cpu_solvers(gpu_session, kw):
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, SparkSession

    X, y = _synth_tensors(outliers="loss" in kw)
    dfg = gpu_session.createDataFrame({"features": X.cuda(), "label": y.cuda()})
    mg = LinearRegression(**kw).fit(dfg)
    gpu_session.stop()
    cpu = SparkSession.builder().master("cpu").getOrCreate()
    mc = LinearRegression(**kw).fit(cpu.createDataFrame({"features": X, "label": y}))
    cpu.stop()
    import numpy as np

    np.testing.assert_allclose(mg.coefficients.toArray(), mc.coefficients.toArray(), rtol=1e-6, atol=1e-8)
    assert float(mg.intercept) == pytest.approx(float(mc.intercept), rel=1e-6, abs=1e-8)
