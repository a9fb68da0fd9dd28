"""the squared-loss l-bfgs / OWLQN fit as ONE grid launch (``lsq_qn.hip``:
standardization from the device summarizer head, one fused data pass per cost evaluation, the
Breeze line searches on the device) against the host-steered path (``models/qn_device.py`` over
the two-pass ``lsq.hip`` evaluations, ``DQ4ML_LSQ_QN=0``) on the wide bf16 / fp8 tiles; an
asynchronous fit enqueues everything with no host sync."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _data(dev, d, n, seed, eb, y0=0.5, const=False):
    from net.jgp.labs.sparkdq4ml_amd.ops import device

    g = torch.Generator(device=dev).manual_seed(seed)
    X = torch.randn(d, n, generator=g, device=dev) * (0.5 + torch.rand(d, 1, generator=g, device=dev))
    beta = torch.zeros(d, device=dev)
    k = min(d, 40)
    beta[:k] = torch.linspace(-1.0, 2.0, k, device=dev)
    y = (beta @ X + y0 + 0.1 * torch.randn(n, generator=g, device=dev)).double()
    if const:
        y = torch.full((n,), 3.25, dtype=torch.float64, device=dev)
    return device.pack_wide([X], eb, None), y


def _fit(lr, df, monkeypatch, device_qn: bool):
    monkeypatch.setenv("DQ4ML_LSQ_QN", "1" if device_qn else "0")
    return lr.fit(df)


def _oracle(T, y, regParam, elasticNetParam, fitIntercept=True, standardization=True):
    """Independent fp64 optimum of Spark 2.4's standardized l-bfgs objective on the DEQUANTIZED
    tiles (``T.to_dense()``): sample-std standardization, ``effectiveRegParam = regParam / yStd``,
    0.5 c'Ac - b'c + L2 + L1 — a direct solve without L1, proximal gradient (ISTA, fp64) with it.
    Shares no code with either fit path."""
    X = T.to_dense().double()  # [d, n]
    y = y.double()
    n = X.shape[1]
    mx, my = X.mean(1), y.mean()
    sx = ((X - mx[:, None]) ** 2).sum(1).div(n - 1).sqrt()
    sy = float(((y - my) ** 2).sum().div(n - 1).sqrt())
    safe = torch.where(sx == 0, torch.ones_like(sx), sx)
    Xs = ((X - mx[:, None]) if fitIntercept else X) / safe[:, None]
    ys = ((y - my) if fitIntercept else y) / sy
    A = Xs @ Xs.T / n
    b = Xs @ ys / n
    eff = regParam / sy
    l1, l2 = elasticNetParam * eff, (1.0 - elasticNetParam) * eff
    w2 = torch.ones_like(sx) if standardization else 1.0 / (safe * safe)
    w1 = torch.full_like(sx, l1) if standardization else l1 / safe
    H = A + torch.diag(l2 * w2)
    if l1 == 0.0:
        c = torch.linalg.solve(H, b)
    else:
        L = float(torch.linalg.eigvalsh(H).max())
        c = torch.zeros_like(b)
        for _ in range(4000):
            z = c - (H @ c - b) / L
            c = torch.sign(z) * torch.clamp(z.abs() - w1 / L, min=0.0)
    coef = torch.where(sx == 0, torch.zeros_like(c), c * sy / safe)
    icpt = float(my - coef @ mx) if fitIntercept else 0.0
    return coef.cpu().numpy(), icpt


@pytest.mark.parametrize("eb,d,n,kw", [
    (16, 300, 60_001, dict(regParam=0.02, elasticNetParam=0.0)),                      # L-BFGS, strong Wolfe
    (16, 300, 60_001, dict(regParam=0.02, elasticNetParam=0.6)),                      # OWLQN, backtracking
    (8, 1100, 30_017, dict(regParam=0.01, elasticNetParam=1.0, fitIntercept=False)),
    (16, 5000, 8_003, dict(regParam=0.001, elasticNetParam=0.0, standardization=False)),
])
def test_device_qn_matches_host_steered(gpu_session, monkeypatch, eb, d, n, kw):
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression
    T, y = _data(gpu_session.device, d, n, d + eb, eb)
    df = gpu_session.createDataFrame({"features": T, "label": y})
    lr = LinearRegression(solver="l-bfgs", maxIter=60, tol=1e-9, **kw)
    m_dev = _fit(lr, df, monkeypatch, True)
    assert m_dev.summary.solver == ("owlqn" if kw["elasticNetParam"] else "l-bfgs")
    # the one-launch lsq_qn fit ran (set only by its pending result, lbfgs_path._PendingLsq)
    assert m_dev._qn_evaluations is not None and m_dev._qn_evaluations > 0
    m_host = _fit(lr, df, monkeypatch, False)
    assert getattr(m_host, "_qn_evaluations", None) is None  # the host-steered path really ran
    a, b = m_dev.coefficients.toArray(), m_host.coefficients.toArray()
    # the device pass sums the columns in a different f32 / f64 order than the two-pass kernels:
    # the iterates agree to the optimizer's own resolution, not bitwise
    assert np.abs(a - b).max() <= 2e-4 * max(1.0, np.abs(b).max()), np.abs(a - b).max()
    assert float(m_dev.intercept) == pytest.approx(float(m_host.intercept), rel=1e-4, abs=1e-5)
    hd, hh = np.asarray(m_dev.summary.objectiveHistory), np.asarray(m_host.summary.objectiveHistory)
    assert hd[0] == pytest.approx(hh[0], rel=1e-9)
    assert hd[-1] == pytest.approx(hh[-1], rel=1e-6)
    # near the optimum the two summation orders take different tails of FunctionValuesConverged
    assert abs(len(hd) - len(hh)) <= 3 + len(hh) // 5
    # the device fit is deterministic: fixed-order reductions everywhere
    m_again = _fit(lr, df, monkeypatch, True)
    assert np.array_equal(m_again.coefficients.toArray(), a)
    # independent fp64 oracle of the same dequantized problem (no code shared with either path)
    oc, oi = _oracle(T, y, **kw)
    scale = max(1.0, np.abs(oc).max())
    err = np.abs(a - oc).max()
    assert err <= 2e-3 * scale, (err, scale)
    assert float(m_dev.intercept) == pytest.approx(oi, rel=2e-3, abs=2e-3 * scale)


def test_device_qn_async_fit_has_no_host_sync(gpu_session, monkeypatch):
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression

    monkeypatch.setenv("DQ4ML_LSQ_QN", "1")
    T, y = _data(gpu_session.device, 4200, 20_000, 9, 16)
    df = gpu_session.createDataFrame({"features": T, "label": y})
    lr = LinearRegression(regParam=0.001, elasticNetParam=0.0, maxIter=40)  # numFeatures > 4096: auto -> l-bfgs
    gpu_session.conf.set("dq4ml.fit.async", "true")
    try:
        lr.fit(df).coefficients  # warm-up (allocator, launch plan)
        torch.cuda.synchronize()
        torch.cuda.set_sync_debug_mode("error")
        try:
            m = lr.fit(df)
            assert m._pending is not None
        finally:
            torch.cuda.set_sync_debug_mode("default")
    finally:
        gpu_session.conf.set("dq4ml.fit.async", "false")
    ref = lr.fit(df)
    np.testing.assert_array_equal(m.coefficients.toArray(), ref.coefficients.toArray())
    assert m.summary.solver == "l-bfgs"
    assert list(m.summary.objectiveHistory) == list(ref.summary.objectiveHistory)


def test_device_qn_constant_label_takes_the_host_semantics(gpu_session, monkeypatch):
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression

    monkeypatch.setenv("DQ4ML_LSQ_QN", "1")
    T, y = _data(gpu_session.device, 300, 5_000, 4, 16, const=True)
    df = gpu_session.createDataFrame({"features": T, "label": y})
    m = LinearRegression(solver="l-bfgs", regParam=0.1).fit(df)
    assert np.all(m.coefficients.toArray() == 0.0)
    assert float(m.intercept) == pytest.approx(3.25)


def test_device_qn_grid_barrier_is_bounded_when_the_grid_is_not_co_resident(monkeypatch):
    """``grid_barrier`` (common.h) relies on the launcher's one-block-per-CU grid being
    co-resident.  A grid five times the CU count (more blocks than a CU can ever hold at once)
    must not hang: the resident blocks give up on the first barrier after the poll bound, every
    later barrier passes, the launch drains and reports status 9 ("not finished", which re-runs
    the fit on the host-steered path).  A normal launch afterwards is unaffected."""
    from net.jgp.labs.sparkdq4ml_amd.ops import device, kernels, native

    d, n = 300, 20_000
    T, y = _data(torch.device("cuda"), d, n, 7, 16)
    P = kernels.lsq_passes(T, y, None, None)
    head = torch.cat([P.scalars(), P.moments()])
    args = (head, True, True, 0.02, 0.0, 20, 1e-9)
    cus = int(native.hip().device_info()["multiProcessorCount"])
    key = (P.device.index, P.layout, P.d)
    monkeypatch.setitem(device._lsq_qn_grid, key, 5 * cus)
    over = P.qn_fit(*args).cpu()
    assert int(over[d + 1]) == 9
    monkeypatch.delitem(device._lsq_qn_grid, key)
    ok = P.qn_fit(*args).cpu()
    assert int(ok[d + 1]) == 0 and int(ok[d + 5]) > 0


# ---- X4: the data-parallel form (pass, fold, all-reduce, one-block control kernel per evaluation)

@pytest.mark.parametrize("eb,d,n,kw", [
    (16, 300, 60_001, dict(regParam=0.02, elasticNetParam=0.0)),
    (16, 300, 60_001, dict(regParam=0.02, elasticNetParam=0.6)),
    (8, 1100, 30_017, dict(regParam=0.01, elasticNetParam=1.0, fitIntercept=False)),
])
def test_device_qn_dp_equals_one_launch(eb, d, n, kw):
    """At one rank the split form runs the same passes as the one-launch fit (fold order,
    deferred margin update, per-rank un-scaling before the identity reduce); only the four
    evaluation scalars are summed by one block instead of per-block partials, so the fits agree to
    rounding with the same evaluations -- enqueued with no host sync."""
    from net.jgp.labs.sparkdq4ml_amd.ops import kernels

    T, y = _data(torch.device("cuda"), d, n, d + eb, eb)
    P = kernels.lsq_passes(T, y, None, None)
    head = torch.cat([P.scalars(), P.moments()])
    fit_icpt = kw.get("fitIntercept", True)
    args = (head, fit_icpt, True, kw["regParam"], kw["elasticNetParam"], 60, 1e-9)
    one = P.qn_fit(*args).cpu()
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        dp = P.qn_fit_dp(*args, all_reduce=lambda t: t)
    finally:
        torch.cuda.set_sync_debug_mode("default")
    dp = dp.cpu()
    assert int(dp[d + 1]) == 0 and int(one[d + 1]) == 0
    assert int(dp[d + 5]) == int(one[d + 5]) > 0  # the same number of evaluations
    H = int(one[d + 3])
    assert int(dp[d + 3]) == H and int(dp[d + 2]) == int(one[d + 2])  # history length, stop reason
    torch.testing.assert_close(dp[:d + 1], one[:d + 1], rtol=1e-9, atol=1e-12)  # coefficients, intercept
    torch.testing.assert_close(dp[d + 11:d + 11 + H], one[d + 11:d + 11 + H], rtol=1e-12, atol=0.0)


def _run_workers(args, world, timeout=150):
    import json
    import os
    import socket
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE=str(world),
                   LOCAL_RANK="0", DQ4ML_COMM_TIMEOUT="60")
        procs.append(subprocess.Popen([sys.executable, os.path.join(here, "_gpu_qn_dp_worker.py"), *args], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
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


@pytest.mark.parametrize("case,shards", [("lbfgs", "split"), ("owlqn", "split"), ("lbfgs", "empty")])
def test_device_qn_two_rank_gloo_matches_single_process(gpu_session, monkeypatch, case, shards):
    """Two processes on the one GPU, each fitting its row shard (gloo: RCCL refuses two ranks on
    one device): every rank ends with the single-process device fit of all rows.  ``empty``: rank 1
    holds no row -- the ranks still agree on the device branch (an empty shard used to
    drop to the host path alone and deadlock its peer)."""
    import sys

    sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
    from _gpu_qn_dp_worker import CASES, data

    from net.jgp.labs.sparkdq4ml_amd import LinearRegression
    from net.jgp.labs.sparkdq4ml_amd.ops import device

    c = CASES[case]
    X, y = data(case, "cuda")
    T = device.pack_wide([X], c["eb"], None, shift=None)
    df = gpu_session.createDataFrame({"features": T, "label": y})
    ref = _fit(LinearRegression(solver="l-bfgs", maxIter=60, tol=1e-9, **c["kw"]), df, monkeypatch, True)
    assert ref._qn_evaluations is not None
    outs = _run_workers(["gloo", case] + (["empty"] if shards == "empty" else []), 2)
    b = ref.coefficients.toArray()
    for o in outs:
        assert o["evaluations"] is not None and o["evaluations"] > 0  # the device DP form ran
        assert o["solver"] == ref.summary.solver
        a = np.asarray(o["coef"])
        assert np.abs(a - b).max() <= 2e-4 * max(1.0, np.abs(b).max()), np.abs(a - b).max()
        assert o["intercept"] == pytest.approx(float(ref.intercept), rel=1e-4, abs=1e-5)
        assert o["history"][0] == pytest.approx(float(ref.summary.objectiveHistory[0]), rel=1e-9)
    assert outs[0]["coef"] == outs[1]["coef"]  # identical decisions on every rank


@pytest.mark.parametrize("case", ["lbfgs", "fp8"])
def test_device_qn_forced_rccl_has_no_host_sync(case):
    """Every collective forced through a one-rank RCCL communicator (DQ4ML_FORCE_COLLECTIVES): the
    l-bfgs fit takes the data-parallel device form and runs under sync_debug_mode("error")."""
    o = _run_workers(["rccl", case], 1)[0]
    assert o["evaluations"] is not None and o["evaluations"] > 0
