"""Asynchronous normal-equation fits (``dq4ml.fit.async``): device WLS Cholesky kernel
(``wls_small.hip``) resolved lazily must equal the synchronous native path, including the
edge cases the kernel hands back to the host driver."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def async_session():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from net.jgp.labs.sparkdq4ml_amd import SparkSession

    s = SparkSession.getActiveSession()
    if s is not None:
        s.stop()
    s = SparkSession.builder().master("mi355x[*]").config("dq4ml.fit.async", "true").getOrCreate()
    yield s
    s.stop()


def _fit_both(session, df, **kw):
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression

    m_async = LinearRegression(**kw).fit(df)
    assert m_async._pending is not None  # really deferred
    session.conf.set("dq4ml.fit.async", "false")
    m_sync = LinearRegression(**kw).fit(df)
    session.conf.set("dq4ml.fit.async", "true")
    return m_async, m_sync


@pytest.mark.parametrize("fit_intercept", [True, False])
@pytest.mark.parametrize("std", [True, False])
@pytest.mark.parametrize("reg", [0.0, 0.5])
def test_async_matches_sync(async_session, fit_intercept, std, reg):
    d, n = 17, 50_000
    g = torch.Generator(device="cuda").manual_seed(d)
    X = torch.randn(d, n, generator=g, device="cuda", dtype=torch.float64) * 2 + 1
    y = torch.linspace(-1, 1, d, device="cuda", dtype=torch.float64) @ X + 3 + 0.05 * torch.randn(
        n, generator=g, device="cuda", dtype=torch.float64)
    df = async_session.createDataFrame({"features": X, "label": y})
    a, s = _fit_both(async_session, df, solver="normal", regParam=reg, elasticNetParam=0.0,
                     fitIntercept=fit_intercept, standardization=std)
    np.testing.assert_allclose(a.coefficients.toArray(), s.coefficients.toArray(), rtol=1e-10, atol=1e-12)
    assert float(a.intercept) == pytest.approx(float(s.intercept), rel=1e-10, abs=1e-12)
    assert list(np.asarray(a.summary.objectiveHistory)) == list(np.asarray(s.summary.objectiveHistory))
    assert float(a.summary.r2) == pytest.approx(float(s.summary.r2), rel=1e-12)
    np.testing.assert_allclose(a.summary.coefficientStandardErrors, s.summary.coefficientStandardErrors, rtol=1e-8)


def test_async_constant_label_falls_back(async_session):
    X = torch.randn(3, 1000, device="cuda", dtype=torch.float64)
    y = torch.full((1000,), 4.25, device="cuda", dtype=torch.float64)
    df = async_session.createDataFrame({"features": X, "label": y})
    a, s = _fit_both(async_session, df, solver="normal")
    assert float(a.intercept) == pytest.approx(4.25) and np.all(a.coefficients.toArray() == 0)
    assert a.summary.solver == s.summary.solver


def test_async_singular_falls_back_to_lbfgs(async_session):
    x = torch.randn(2, 2000, device="cuda", dtype=torch.float64)
    X = torch.cat([x, torch.full((1, 2000), 3.0, device="cuda", dtype=torch.float64)])  # zero-variance feature
    y = 2 * x[0] - x[1] + 1  # standardized system has an exactly-zero pivot
    df = async_session.createDataFrame({"features": X, "label": y})
    a, s = _fit_both(async_session, df, solver="auto")
    assert a.summary.solver == s.summary.solver
    np.testing.assert_allclose(a.coefficients.toArray(), s.coefficients.toArray(), rtol=1e-9, atol=1e-12)


def test_async_bf16_tiled(async_session):
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression

    d, n = 32, 200_000
    g = torch.Generator(device="cuda").manual_seed(5)
    X = torch.randn(d, n, generator=g, device="cuda").to(torch.bfloat16)
    beta = torch.linspace(-2, 2, d, device="cuda")
    y = beta @ X.float() + 0.5
    df = async_session.createDataFrame({"features": X, "label": y})
    m = LinearRegression(solver="normal", gramDtype="bf16").fit(df)
    assert np.abs(m.coefficients.toArray() - beta.cpu().numpy()).max() < 1e-3
