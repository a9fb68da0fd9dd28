"""Squared-loss l-bfgs path with a data pass per cost evaluation:
Spark's ``LeastSquaresAggregator`` + Breeze L-BFGS / OWLQN (``models/lbfgs_path.py``
``_train_passes``, ``models/qn_device.py``), checked against the quadratic-form (Gram) route of
the same optimizer, sklearn, the single-process fit (gloo ranks) and its own checkpoints."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from net.jgp.labs.sparkdq4ml_amd import LinearRegression, col


def _synth(spark, n=3000, d=5, seed=0, weights=False, extra=False):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(d, n, generator=g, dtype=torch.float64) * torch.linspace(0.5, 3, d, dtype=torch.float64).unsqueeze(1) + 1.0
    beta = torch.linspace(-1, 2, d, dtype=torch.float64)
    y = beta @ X + 0.7 + 0.3 * torch.randn(n, generator=g, dtype=torch.float64)
    cols = {"features": X, "label": y}
    if weights:
        cols["w"] = 0.5 + torch.rand(n, generator=g, dtype=torch.float64)
    if extra:
        cols["z"] = torch.arange(n, dtype=torch.float64) % 7
    return spark.createDataFrame(cols)


def _fit(spark, df, mode, **kw):
    spark.conf.set("dq4ml.lbfgs.mode", mode)
    try:
        return LinearRegression(solver="l-bfgs", **kw).fit(df)
    finally:
        spark.conf.set("dq4ml.lbfgs.mode", "passes")


@pytest.mark.parametrize("kw", [
    dict(tol=1e-12, maxIter=200),                                           # L-BFGS, OLS
    dict(regParam=0.05, elasticNetParam=0.0, tol=1e-12, maxIter=200),        # L-BFGS + L2
    dict(regParam=0.05, elasticNetParam=0.7, tol=1e-12, maxIter=400),        # OWLQN
    dict(regParam=0.05, elasticNetParam=0.3, standardization=False, tol=1e-12, maxIter=400),
    dict(regParam=0.02, fitIntercept=False, tol=1e-12, maxIter=300),
])
def test_passes_match_gram_route(cpu_session, kw):
    df = _synth(cpu_session)
    a = _fit(cpu_session, df, "passes", **kw)
    b = _fit(cpu_session, df, "gram", **kw)
    np.testing.assert_allclose(a.coefficients.toArray(), b.coefficients.toArray(), rtol=1e-6, atol=1e-8)
    assert float(a.intercept) == pytest.approx(float(b.intercept), rel=1e-6, abs=1e-8)
    h = a.summary.objectiveHistory
    assert h[0] == pytest.approx(b.summary.objectiveHistory[0], rel=1e-9)
    assert np.all(np.diff(h) <= 1e-12) and a.summary.totalIterations == len(h)


def test_passes_weights_and_selection(cpu_session):
    """Instance weights and a DQ filter (selection vector) enter the passes as row weights."""
    df = _synth(cpu_session, weights=True, extra=True).filter(col("z") > 1)
    kw = dict(weightCol="w", regParam=0.03, elasticNetParam=0.5, tol=1e-12, maxIter=400)
    a = _fit(cpu_session, df, "passes", **kw)
    b = _fit(cpu_session, df, "gram", **kw)
    np.testing.assert_allclose(a.coefficients.toArray(), b.coefficients.toArray(), rtol=1e-6, atol=1e-8)
    assert float(a.intercept) == pytest.approx(float(b.intercept), rel=1e-6)


def test_auto_wide_routes_to_passes_without_gram(cpu_session, monkeypatch):
    """numFeatures > 4096 with solver=auto is Spark's l-bfgs switch: no d x d Gram is formed."""
    from net.jgp.labs.sparkdq4ml_amd.ops import kernels

    def no_gram(*a, **k):
        raise AssertionError("the l-bfgs data-pass route must not build the Gram")
    monkeypatch.setattr(kernels, "gram_stats", no_gram)
    n, d = 400, 4100
    g = torch.Generator().manual_seed(5)
    X = torch.randn(d, n, generator=g, dtype=torch.float64)
    y = X[:3].sum(0) + 0.1 * torch.randn(n, generator=g, dtype=torch.float64)
    df = cpu_session.createDataFrame({"features": X, "label": y})
    m = LinearRegression(regParam=0.1, elasticNetParam=1.0, maxIter=30).fit(df)
    assert m.summary.solver == "owlqn" and m.numFeatures == d
    c = m.coefficients.toArray()
    assert np.isfinite(c).all() and c[:3].min() > 0.3 and np.abs(c[3:]).max() < 0.2


def test_constant_label_short_circuit(cpu_session):
    X = torch.randn(3, 100, dtype=torch.float64)
    df = cpu_session.createDataFrame({"features": X, "label": torch.full((100,), 2.5, dtype=torch.float64)})
    m = LinearRegression(solver="l-bfgs").fit(df)
    assert np.all(m.coefficients.toArray() == 0) and float(m.intercept) == 2.5


def test_passes_checkpoint_resume_is_exact(cpu_session, tmp_path):
    """SURVEY.md §5d for the squared-loss l-bfgs path: a crash after a checkpointed iteration and a
    re-run resume from the saved Breeze state and end bit-identically to the uninterrupted fit."""
    from net.jgp.labs.sparkdq4ml_amd.models import lbfgs_path

    g = torch.Generator().manual_seed(2)
    d, n = 20, 3000
    Z = torch.randn(d, n, generator=g, dtype=torch.float64)
    X = (torch.eye(d, dtype=torch.float64) + 0.9 * torch.randn(d, d, generator=g, dtype=torch.float64)) @ Z  # correlated
    y = torch.linspace(-1, 2, d, dtype=torch.float64) @ X + 0.3 * torch.randn(n, generator=g, dtype=torch.float64)
    df = cpu_session.createDataFrame({"features": X, "label": y})
    kw = dict(regParam=0.05, elasticNetParam=0.4, tol=1e-14, maxIter=30)
    ref = _fit(cpu_session, df, "passes", **kw)
    assert ref.summary.totalIterations > 8
    cpu_session.conf.set("dq4ml.lbfgs.checkpointDir", str(tmp_path))
    cpu_session.conf.set("dq4ml.lbfgs.checkpointInterval", "3")
    try:
        lbfgs_path._QN_FAIL_AT_ITER = 7
        with pytest.raises(RuntimeError, match="injected failure"):
            _fit(cpu_session, df, "passes", **kw)
        assert len([f for f in os.listdir(tmp_path) if f.endswith(".npz")]) == 1  # the iteration-6 state
        lbfgs_path._QN_FAIL_AT_ITER = None
        got = _fit(cpu_session, df, "passes", **kw)
    finally:
        lbfgs_path._QN_FAIL_AT_ITER = None
        cpu_session.conf.set("dq4ml.lbfgs.checkpointDir", "")
    assert np.array_equal(got.coefficients.toArray(), ref.coefficients.toArray())
    assert got.intercept == ref.intercept
    assert np.array_equal(got.summary.objectiveHistory, ref.summary.objectiveHistory)
    assert not [f for f in os.listdir(tmp_path) if f.endswith(".npz")]


def test_host_lsq_oracle_matches_definition(cpu_session):
    """``kernels.lsq_passes`` (host) = Spark's LeastSquaresAggregator sums, written out."""
    from net.jgp.labs.sparkdq4ml_amd.ops import kernels

    g = torch.Generator().manual_seed(9)
    d, n = 6, 500
    X = torch.randn(d, n, generator=g, dtype=torch.float64)
    y = torch.randn(n, generator=g, dtype=torch.float64)
    w = torch.rand(n, generator=g, dtype=torch.float64)
    sel = torch.rand(n, generator=g) > 0.3
    X[:, ~sel] = float("nan")  # dead rows never contribute, whatever they hold
    P = kernels.lsq_passes(X, y, w, sel)
    cf = torch.randn(d, generator=g, dtype=torch.float64)
    out = P.evaluate(cf, torch.tensor(0.25, dtype=torch.float64), 0.5)
    Xs, ys, ws = X[:, sel], y[sel], w[sel]
    diff = cf @ Xs + 0.25 - 0.5 * ys
    assert float(out[0]) == pytest.approx(float((0.5 * ws * diff * diff).sum()), rel=1e-12)
    np.testing.assert_allclose(out[1:].numpy(), (Xs @ (ws * diff)).numpy(), rtol=1e-12)
    mo = P.moments()
    np.testing.assert_allclose(mo[:d].numpy(), (Xs @ ws).numpy(), rtol=1e-12)
    np.testing.assert_allclose(mo[d:].numpy(), ((Xs * Xs) @ ws).numpy(), rtol=1e-12)
    # line-search trials: u(cf) + a u(dcf) (wmargins) then the column pass (evaluate_u) = evaluate
    dcf = torch.randn(d, generator=g, dtype=torch.float64)
    u = P.wmargins(cf) + 0.6 * P.wmargins(dcf)
    lu = P.evaluate_u(u, cf + 0.6 * dcf, torch.tensor(0.25, dtype=torch.float64), 0.5)
    np.testing.assert_allclose(lu.numpy(), P.evaluate(cf + 0.6 * dcf, torch.tensor(0.25, dtype=torch.float64), 0.5).numpy(),
                               rtol=1e-10)


# ---- X4 across processes (gloo here; RCCL on the MI355X node) ---------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(n=4000, d=6):
    g = torch.Generator().manual_seed(11)
    X = torch.randn(d, n, generator=g, dtype=torch.float64) + 0.5
    y = torch.linspace(-1, 1, d, dtype=torch.float64) @ X + 0.3 + 0.05 * torch.randn(n, generator=g, dtype=torch.float64)
    return X, y


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), DQ4ML_DEVICE="cpu")
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, SparkSession
    from net.jgp.labs.sparkdq4ml_amd.parallel import comm

    comm.init(backend="gloo")
    X, y = _data()
    n = X.shape[1]
    lo, hi = rank * n // world, (rank + 1) * n // world
    spark = SparkSession.builder().master("cpu").getOrCreate()
    df = spark.createDataFrame({"features": X[:, lo:hi].contiguous(), "label": y[lo:hi].contiguous()})
    m = LinearRegression(solver="l-bfgs", regParam=0.05, elasticNetParam=0.5, tol=1e-12, maxIter=300).fit(df)
    q.put((rank, m.coefficients.toArray().tolist(), float(m.intercept), list(m.summary.objectiveHistory)))
    comm.barrier()
    comm.shutdown()


def test_dp_lbfgs_passes_match_single_process(cpu_session):
    X, y = _data()
    ref = LinearRegression(solver="l-bfgs", regParam=0.05, elasticNetParam=0.5, tol=1e-12, maxIter=300).fit(
        cpu_session.createDataFrame({"features": X, "label": y}))
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, coef, icpt, hist in res:
        np.testing.assert_allclose(coef, ref.coefficients.toArray(), rtol=1e-8, atol=1e-10)
        assert icpt == pytest.approx(float(ref.intercept), rel=1e-8)
        assert len(hist) == ref.summary.totalIterations
    # every rank runs the same optimizer on the same all-reduced evaluations
    assert res[0][1] == res[1][1] and res[0][3] == res[1][3]


@pytest.mark.parametrize("mode", ["passes", "gram"])
def test_constant_label_without_intercept(cpu_session, mode):
    """Spark 2.4 ``LinearRegression.train``: a constant nonzero label with fitIntercept=false cannot
    be regularized (``require(regParam == 0.0)``); unregularized it fits through the origin."""
    g = torch.Generator().manual_seed(3)
    X = torch.randn(3, 500, generator=g, dtype=torch.float64) + 2.0
    df = cpu_session.createDataFrame({"features": X, "label": torch.full((500,), 4.0, dtype=torch.float64)})
    with pytest.raises(ValueError, match="standard deviation of the label is zero. Model cannot be regularized"):
        _fit(cpu_session, df, mode, fitIntercept=False, regParam=0.1)
    m = _fit(cpu_session, df, mode, fitIntercept=False, regParam=0.0, tol=1e-12, maxIter=200)
    ls = np.linalg.lstsq(X.numpy().T, np.full(500, 4.0), rcond=None)[0]  # through the origin
    np.testing.assert_allclose(m.coefficients.toArray(), ls, rtol=1e-4, atol=1e-6)
