"""Device OWLQN (L1 WLS): the one-wave HIP solver (``wls_qn_kernel``, k <= 128) and the
cooperative grid solver (``wls_qn_grid.hip``, larger k) against the native host driver; the lab's own L1 fit
(regParam 1, elasticNetParam 1) asynchronous and on the device end to end."""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import data_path

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def _host(flat, nf, icpt, reg, enet, stdf, max_iter=100):
    from net.jgp.labs.sparkdq4ml_amd.ops import native

    return native.host().wls_fit(flat, nf, icpt, reg, enet, stdf, True, 0, max_iter, 1e-6, False)


@pytest.mark.parametrize("nf,reg,enet,icpt,stdf", [(1, 1.0, 1.0, True, True), (5, 0.1, 1.0, True, True),
                                                  (30, 0.05, 0.5, True, False), (12, 0.3, 0.8, False, True),
                                                  (63, 0.02, 1.0, True, True), (100, 0.01, 1.0, True, True)])
def test_qn_kernel_matches_native(nf, reg, enet, icpt, stdf):
    from _qn_flat import _flat

    from net.jgp.labs.sparkdq4ml_amd.models.optim import owlqn_result
    from net.jgp.labs.sparkdq4ml_amd.ops import device

    flat = _flat(nf, 4000, nf, w=nf % 2 == 0)
    r = _host(flat, nf, icpt, reg, enet, stdf)
    out = device.wls_qn_small(torch.tensor(flat, device="cuda"), nf, icpt, reg, enet, stdf, True, 100, 1e-6)
    wls, _ = owlqn_result(out.cpu().numpy(), nf)
    np.testing.assert_allclose(wls.coefficients, r["coefficients"], rtol=1e-7, atol=1e-8)
    assert wls.intercept == pytest.approx(r["intercept"], rel=1e-7, abs=1e-9)
    hist, ref = wls.objectiveHistory, np.asarray(r["objective_history"])
    assert hist[0] == ref[0]
    m = min(len(hist), len(ref))
    assert abs(len(hist) - len(ref)) <= 3
    np.testing.assert_allclose(hist[:m], ref[:m], rtol=1e-8)
    assert hist[-1] == pytest.approx(ref[-1], rel=1e-9)


def test_qn_kernel_short_circuits_to_host():
    from net.jgp.labs.sparkdq4ml_amd.ops import device

    nf = 3
    flat = np.zeros(5 + 2 * nf + nf * (nf + 1) // 2)
    flat[:5] = [10, 10, 10, 20, 40]  # constant label 2.0: std 0
    out = device.wls_qn_small(torch.tensor(flat, device="cuda"), nf, True, 1.0, 1.0, True, True, 40, 1e-6).cpu()
    assert int(out[nf + 1]) == 3


def _lab_df(spark):
    from net.jgp.labs.sparkdq4ml_amd import VectorAssembler, callUDF
    from net.jgp.labs.sparkdq4ml_amd.dq.rules import register_lab_rules

    register_lab_rules(spark)
    df = spark.read().format("csv").option("inferSchema", "true").load(data_path("dataset-abstract.csv"))
    df = df.withColumnRenamed("_c0", "guest").withColumnRenamed("_c1", "price")
    df = df.withColumn("price_no_min", callUDF("minimumPriceRule", df.col("price")))
    df.createOrReplaceTempView("price")
    df = spark.sql("SELECT cast(guest as int) guest, price_no_min AS price FROM price WHERE price_no_min > 0")
    df = df.withColumn("price_correct_correl", callUDF("priceCorrelationRule", df.col("price"), df.col("guest")))
    df.createOrReplaceTempView("price")
    df = spark.sql("SELECT guest, price_correct_correl AS price FROM price WHERE price_correct_correl > 0")
    df = df.withColumn("label", df.col("price"))
    return VectorAssembler().setInputCols(["guest"]).setOutputCol("features").transform(df)


@pytest.mark.parametrize("fit_async", ["true", "false"])
def test_lab_l1_fit_on_device_matches_golden(gpu_session, fit_async):
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression

    gpu_session.conf.set("dq4ml.fit.async", fit_async)
    df = _lab_df(gpu_session)
    m = LinearRegression().setMaxIter(40).setRegParam(1).setElasticNetParam(1).fit(df)
    if fit_async == "true":
        assert m._pending is not None and m._pending._qn  # the OWLQN solve is enqueued, not run
    assert m.coefficients[0] == pytest.approx(4.9256080151, rel=1e-9)
    assert float(m.intercept) == pytest.approx(20.9791904606, rel=1e-9)
    s = m.summary
    assert s.rootMeanSquaredError == pytest.approx(2.8021924953, rel=1e-9)
    assert s.r2 == pytest.approx(0.9965340953, rel=1e-9)
    h = np.asarray(s.objectiveHistory)
    assert h[0] == 0.5 and np.all(np.diff(h) <= 0) and s.totalIterations <= 41
    assert h[-1] == pytest.approx(0.0222690086, rel=1e-8)
    assert m.predict(__import__("net.jgp.labs.sparkdq4ml_amd", fromlist=["Vectors"]).Vectors.dense(40.0)) == \
        pytest.approx(218.0035110637, rel=1e-9)
    gpu_session.conf.set("dq4ml.fit.async", "false")


def test_async_l1_fit_has_no_host_sync(gpu_session):
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression

    gpu_session.conf.set("dq4ml.fit.async", "true")
    n, d = 100_000, 20
    g = torch.Generator(device="cuda").manual_seed(1)
    X = torch.randn(d, n, generator=g, device="cuda", dtype=torch.float64)
    y = torch.linspace(-1, 1, d, device="cuda", dtype=torch.float64) @ X + 2.0
    df = gpu_session.createDataFrame({"features": X, "label": y})
    lr = LinearRegression(regParam=0.05, elasticNetParam=1.0)
    lr.fit(df).coefficients  # warm-up
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        ms = [lr.fit(df) for _ in range(3)]
    finally:
        torch.cuda.set_sync_debug_mode("default")
    gpu_session.conf.set("dq4ml.fit.async", "false")
    ref = lr.fit(df)
    for m in ms:
        np.testing.assert_allclose(m.coefficients.toArray(), ref.coefficients.toArray(), rtol=1e-10, atol=1e-13)


def _wide_flat(d, n, seed):
    from net.jgp.labs.sparkdq4ml_amd.ops import device

    g = torch.Generator(device="cuda").manual_seed(seed)
    X = torch.randn(d, n, generator=g, device="cuda", dtype=torch.float64)
    X = X * (0.5 + torch.rand(d, 1, generator=g, device="cuda", dtype=torch.float64) * 2)
    beta = torch.randn(d, generator=g, device="cuda", dtype=torch.float64) * \
        (torch.rand(d, generator=g, device="cuda") > 0.5)
    y = beta @ X + 1.0 + 0.1 * torch.randn(n, generator=g, device="cuda", dtype=torch.float64)
    return device.gram_stats(X, y, None, None, "fp64")


@pytest.mark.parametrize("d,reg,enet,icpt,stdf", [(128, 0.01, 1.0, True, True), (256, 0.02, 1.0, True, True),
                                                  (300, 0.05, 0.5, False, False), (1024, 0.01, 1.0, True, True)])
def test_qn_grid_kernel_matches_native(d, reg, enet, icpt, stdf):
    """k > 128: the cooperative grid OWLQN (wls_qn_grid.hip) vs the native host driver."""
    from net.jgp.labs.sparkdq4ml_amd.models.optim import owlqn_result
    from net.jgp.labs.sparkdq4ml_amd.ops import device

    flat = _wide_flat(d, max(4 * d, 20_000), d)
    out = device.wls_qn_small(flat, d, icpt, reg, enet, stdf, True, 100, 1e-6)
    out2 = device.wls_qn_small(flat, d, icpt, reg, enet, stdf, True, 100, 1e-6)
    used = d + 9 + int(out[d + 7])  # coefficients, status, scalars, H, reason, history (the rest is scratch)
    assert torch.equal(out[:used], out2[:used])  # fixed-order reductions: bitwise run to run
    wls, _ = owlqn_result(out.cpu().numpy(), d)
    r = _host(flat.cpu().numpy(), d, icpt, reg, enet, stdf)
    np.testing.assert_allclose(wls.coefficients, r["coefficients"], rtol=1e-6, atol=1e-8)
    assert wls.intercept == pytest.approx(r["intercept"], rel=1e-7, abs=1e-9)
    hist, ref = wls.objectiveHistory, np.asarray(r["objective_history"])
    assert hist[0] == pytest.approx(ref[0], rel=1e-12)
    assert abs(len(hist) - len(ref)) <= 3
    assert hist[-1] == pytest.approx(ref[-1], rel=1e-8)


def test_qn_grid_kernel_short_circuits_and_no_l1():
    from net.jgp.labs.sparkdq4ml_amd.ops import device

    nf = 200
    flat = np.zeros(5 + 2 * nf + nf * (nf + 1) // 2)
    flat[:5] = [10, 10, 10, 20, 40]  # constant label: std 0 -> the host owns it
    out = device.wls_qn_small(torch.tensor(flat, device="cuda"), nf, True, 1.0, 1.0, True, True, 40, 1e-6).cpu()
    assert int(out[nf + 1]) == 3
    flat = _wide_flat(nf, 5000, 3)
    out = device.wls_qn_small(flat, nf, True, 1.0, 0.0, True, True, 40, 1e-6).cpu()
    assert int(out[nf + 1]) == 9  # no L1 term


def test_wide_async_l1_fit_has_no_host_sync(gpu_session):
    """An L1 fit at d = 257 is enqueued (wide Gram -> grid OWLQN) with no host sync, and equals the
    synchronous fit."""
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression

    gpu_session.conf.set("dq4ml.fit.async", "true")
    n, d = 30_000, 257
    g = torch.Generator(device="cuda").manual_seed(5)
    X = torch.randn(d, n, generator=g, device="cuda", dtype=torch.float64)
    beta = torch.randn(d, generator=g, device="cuda", dtype=torch.float64) * (torch.rand(d, generator=g, device="cuda") > 0.6)
    y = beta @ X + 2.0 + 0.05 * torch.randn(n, generator=g, device="cuda", dtype=torch.float64)
    df = gpu_session.createDataFrame({"features": X, "label": y})
    lr = LinearRegression(regParam=0.01, elasticNetParam=1.0)
    lr.fit(df).coefficients  # warm-up
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        m = lr.fit(df)
        assert m._pending is not None and m._pending._qn
    finally:
        torch.cuda.set_sync_debug_mode("default")
    gpu_session.conf.set("dq4ml.fit.async", "false")
    ref = lr.fit(df)
    np.testing.assert_allclose(m.coefficients.toArray(), ref.coefficients.toArray(), rtol=1e-10, atol=1e-13)


def test_qn_grid_kernel_history_reset_terminates():
    """statistics whose standardized system is indefinite (correlations scaled past 1)
    make s.y < 0 -> the grid solver's history reset path (no line search, no grid barrier between
    block 0's write of the direction scalars and the other blocks' reads; double-buffered since).
    The solve must terminate, deterministically, on a k > 128 grid."""
    from net.jgp.labs.sparkdq4ml_amd.ops import device

    d = 200
    flat = _wide_flat(d, 20_000, 11).cpu().numpy().copy()
    W = flat[1]
    mean = flat[5:5 + d] / W
    i, j = np.triu_indices(d)
    order = np.argsort(i + j * (j + 1) // 2)
    ii, jj = i[order], j[order]
    aa = flat[5 + 2 * d:] / W
    cov = aa - mean[ii] * mean[jj]
    cov = np.where(ii == jj, cov, 3.0 * cov)  # |correlation| up to 3: indefinite
    flat[5 + 2 * d:] = (cov + mean[ii] * mean[jj]) * W
    t = torch.tensor(flat, device="cuda")
    outs = [device.wls_qn_small(t, d, True, 0.01, 1.0, True, True, 60, 1e-6) for _ in range(3)]
    torch.cuda.synchronize()
    used = d + 9 + int(outs[0][d + 7])
    for o in outs[1:]:
        assert torch.equal(o[:used], outs[0][:used])  # same decisions on every run
    H = int(outs[0][d + 7])
    assert 1 <= H <= 2 * 60 + 8
