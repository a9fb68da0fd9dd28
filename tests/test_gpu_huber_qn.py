"""The Huber fit's device L-BFGS-B (``huber_qn.hip``): Breeze 0.13 ``LBFGSB`` semantics on the
device, checked against the host implementation of the same algorithm (``models/lbfgsb.py``, the
oracle: ``dq4ml.huber.device=false``) -- same objective history up to rounding, same optimum --
on dense f64 columns, bf16 wide tiles and fp8 wide tiles with shifted storage; then the
data-parallel form: two gloo ranks over row shards, and a forced one-rank RCCL fit that runs
under ``sync_debug_mode("error")`` (no host read anywhere in the fit); and an independent fp64
oracle (scipy L-BFGS-B on a numpy Huber objective)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from _gpu_huber_qn_worker import CASES, data, frame  # noqa: E402


def _fit(spark, df, kw, device):
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression

    spark.conf.set("dq4ml.huber.device", "true" if device else "false")
    try:
        return LinearRegression(loss="huber", tol=1e-9, **kw).fit(df)
    finally:
        spark.conf.set("dq4ml.huber.device", "true")


def _close(dev, host, hist_rtol=1e-7):
    a, b = dev.coefficients.toArray(), host.coefficients.toArray()
    scale = max(1.0, np.abs(b).max())
    assert np.abs(a - b).max() <= 1e-6 * scale, np.abs(a - b).max()
    assert float(dev.intercept) == pytest.approx(float(host.intercept), rel=1e-6, abs=1e-6)
    assert float(dev.scale) == pytest.approx(float(host.scale), rel=1e-6)
    hd, hh = np.asarray(dev.summary.objectiveHistory), np.asarray(host.summary.objectiveHistory)
    assert hd[0] == pytest.approx(hh[0], rel=1e-12)  # the same first evaluation at all ones
    assert abs(hd.size - hh.size) <= 2, (hd.size, hh.size)
    m = min(hd.size, hh.size)
    np.testing.assert_allclose(hd[:m], hh[:m], rtol=hist_rtol)


@pytest.mark.parametrize("case", ["dense", "bf16", "fp8"])
def test_device_huber_matches_host_lbfgsb(gpu_session, case):
    c = CASES[case]
    X, y = data(case, "cuda")
    df = frame(gpu_session, case, X, y, shift="auto" if case == "fp8" else None)
    dev = _fit(gpu_session, df, c["kw"], True)
    host = _fit(gpu_session, df, c["kw"], False)
    assert getattr(dev, "_huber_evaluations", None), "the device optimizer did not run"
    assert getattr(host, "_huber_evaluations", None) is None
    assert dev.summary.solver == host.summary.solver == "l-bfgs-b"
    _close(dev, host)
    if case == "dense":  # the robust fit ignores the outliers: near the generating model
        beta = np.linspace(-1.0, 2.0, c["d"])
        assert np.abs(dev.coefficients.toArray() - beta).max() < 0.02
        assert float(dev.intercept) == pytest.approx(0.7, abs=0.05)


def _oracle(X, y, reg, fit_icpt=True):
    """Independent fp64 optimum of Spark 2.4's Huber objective (HuberAggregator + L2 in the
    standardized space, epsilon 1.35): scipy's L-BFGS-B (Fortran, not Breeze's algorithm) driven
    to a tight tolerance on a numpy implementation that shares no code with either fit path.
    Returns (coefficients, intercept, scale)."""
    from scipy.optimize import minimize

    X, y = X.double().cpu().numpy(), y.double().cpu().numpy()
    d, n = X.shape
    sx = X.std(axis=1, ddof=1)
    Z = X / sx[:, None]
    eps = 1.35

    def fg(t):
        c, b, s = t[:d], (t[d] if fit_icpt else 0.0), t[-1]
        r = y - c @ Z - b
        inside = np.abs(r) <= s * eps
        loss = np.where(inside, 0.5 * (s + r * r / s), 0.5 * (s + 2 * eps * np.abs(r) - s * eps * eps))
        m = np.where(inside, -r / s, -eps * np.sign(r))
        gs = np.where(inside, 0.5 * (1 - (r / s) ** 2), 0.5 * (1 - eps * eps))
        f = loss.mean() + 0.5 * reg * c @ c
        g = np.concatenate([Z @ m / n + reg * c, [m.mean()] if fit_icpt else [], [gs.mean()]])
        return f, g

    t0 = np.ones(d + (2 if fit_icpt else 1))
    bounds = [(None, None)] * (t0.size - 1) + [(1e-12, None)]
    res = minimize(fg, t0, jac=True, method="L-BFGS-B", bounds=bounds,
                   options=dict(maxiter=5000, maxcor=20, ftol=1e-15, gtol=1e-12))
    t = res.x
    return t[:d] / sx, (t[d] if fit_icpt else 0.0), t[-1]


@pytest.mark.parametrize("reg", [0.0, 0.05])
def test_device_huber_matches_fp64_oracle(gpu_session, reg):
    X, y = data("dense", "cuda")
    m = _fit(gpu_session, frame(gpu_session, "dense", X, y), dict(maxIter=200, regParam=reg), True)
    assert getattr(m, "_huber_evaluations", None)
    c, b, s = _oracle(X, y, reg)
    coef = m.coefficients.toArray()
    assert np.abs(coef - c).max() <= 2e-5 * max(1.0, np.abs(c).max()), np.abs(coef - c).max()
    assert float(m.intercept) == pytest.approx(b, abs=2e-5)
    assert float(m.scale) == pytest.approx(s, rel=5e-5)


@pytest.mark.parametrize("kw", [dict(fitIntercept=False, maxIter=50), dict(standardization=False, regParam=0.1),
                                dict(maxIter=3)])
def test_device_huber_options(gpu_session, kw):
    """No intercept, unstandardized L2 weights, an iteration cap that stops mid-descent."""
    X, y = data("dense", "cuda")
    df = frame(gpu_session, "dense", X, y)
    dev = _fit(gpu_session, df, kw, True)
    host = _fit(gpu_session, df, kw, False)
    assert getattr(dev, "_huber_evaluations", None)
    _close(dev, host)
    if kw.get("maxIter") == 3:
        assert len(dev.summary.objectiveHistory) == len(host.summary.objectiveHistory) == 4


@pytest.mark.parametrize("layout", ["tiled_bf16", "wide_fp8", "wide_bf16_d40"])
def test_device_huber_fragment_layouts(gpu_session, layout):
    """The generic fused pass (fragment-tiled storage, d <= 16: ``huber_rows_kernel<16>``) and the
    chunked X^T m above it on narrow wide tiles, with shifted storage, against the host LBFGSB."""
    import torch

    from net.jgp.labs.sparkdq4ml_amd.ops import device

    d = 40 if layout.endswith("d40") else 12
    n = 30_011
    g = torch.Generator().manual_seed(d + 3)
    X = (torch.randn(d, n, generator=g) * (0.5 + torch.rand(d, 1, generator=g)) + 1.5).cuda()
    beta = torch.linspace(-1.0, 2.0, d).cuda()
    y = (beta @ X + 0.7 + 0.2 * torch.randn(n, generator=g).cuda()).double()
    y[::37] += 25.0
    if layout == "tiled_bf16":
        T = device.pack_tiled([X], None, shift="auto")
    else:
        T = device.pack_wide([X], 8 if layout == "wide_fp8" else 16, None, shift="auto")
    df = gpu_session.createDataFrame({"features": T, "label": y})
    kw = dict(maxIter=60, regParam=0.02)
    dev = _fit(gpu_session, df, kw, True)
    host = _fit(gpu_session, df, kw, False)
    assert getattr(dev, "_huber_evaluations", None)
    _close(dev, host, hist_rtol=1e-6)


def test_device_huber_weights_and_filter(gpu_session):
    """Instance weights (``weightCol``) and a DQ-style row filter (the selection vector the pass
    skips) on the device path, against the host-steered optimizer on the same frame."""
    import torch

    from net.jgp.labs.sparkdq4ml_amd.sql import functions as F

    X, y = data("dense", "cuda")
    n = X.shape[1]
    w = (0.5 + torch.rand(n, generator=torch.Generator().manual_seed(3), dtype=torch.float64)).cuda()
    df = gpu_session.createDataFrame({"features": X, "label": y, "w": w}).filter(F.col("label") > -3.0)
    kw = dict(weightCol="w", maxIter=80)
    dev = _fit(gpu_session, df, kw, True)
    host = _fit(gpu_session, df, kw, False)
    assert getattr(dev, "_huber_evaluations", None)
    _close(dev, host)


def _run_workers(args, world, timeout=180):
    here = os.path.dirname(os.path.abspath(__file__))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE=str(world),
                   LOCAL_RANK="0", DQ4ML_COMM_TIMEOUT="60")
        procs.append(subprocess.Popen([sys.executable, os.path.join(here, "_gpu_huber_qn_worker.py"), *args],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        try:
            so, se = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        assert p.returncode == 0, se[-3000:]
        outs.append(json.loads(so.strip().splitlines()[-1]))
    return outs


def test_device_huber_two_rank_gloo_matches_single_process(gpu_session):
    """Two processes on the one GPU, each holding half the rows: both end with the single-process
    device fit of all rows, bit for bit the same on both ranks."""
    c = CASES["dense"]
    X, y = data("dense", "cuda")
    ref = _fit(gpu_session, frame(gpu_session, "dense", X, y), c["kw"], True)
    outs = _run_workers(["gloo", "dense"], 2)
    b = ref.coefficients.toArray()
    for o in outs:
        assert o["evaluations"] is not None and o["evaluations"] > 0
        assert o["solver"] == "l-bfgs-b"
        assert np.abs(np.asarray(o["coef"]) - b).max() <= 1e-6 * max(1.0, np.abs(b).max())
        assert o["scale"] == pytest.approx(float(ref.scale), rel=1e-6)
        assert o["history"][0] == pytest.approx(float(ref.summary.objectiveHistory[0]), rel=1e-12)
    assert outs[0]["coef"] == outs[1]["coef"] and outs[0]["history"] == outs[1]["history"]


@pytest.mark.parametrize("case", ["dense", "fp8"])
def test_device_huber_forced_rccl_has_no_host_sync(case):
    """Every collective through a one-rank RCCL communicator: the asynchronous Huber fit enqueues
    passes, all-reduces and control kernels without one host read."""
    o = _run_workers(["rccl", case], 1)[0]
    assert o["evaluations"] is not None and o["evaluations"] > 0
    assert o["solver"] == "l-bfgs-b"
    assert len(o["history"]) >= 2 and o["history"][-1] < o["history"][0]
