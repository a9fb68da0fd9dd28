"""K9 on the MI355X: the squared-loss l-bfgs evaluation passes (``ops/csrc/hip/lsq.hip``) against
the fp64 host oracle (``kernels._HostLsq``) on every feature layout, and the device l-bfgs / OWLQN
fits against the Gram route of the same optimizer."""
import numpy as np
import pytest
import torch

from net.jgp.labs.sparkdq4ml_amd.ops import device, kernels

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", torch.cuda.current_device())


def _layout(kind, X):
    if kind == "f64":
        return X
    if kind == "f32":
        return X.float()
    if kind == "bf16plain":
        return X.to(torch.bfloat16)
    if kind == "tall":
        return device.pack_tiled([X.float()], None)
    if kind == "widebf16":
        return device.pack_wide([X.float()], 16, None)
    if kind == "widefp8":
        return device.pack_wide([X.float()], 8, None)
    raise ValueError(kind)


def _dense64(Xl):
    return (Xl.to_dense() if hasattr(Xl, "to_dense") else Xl).to(torch.float64).cpu()


CASES = [("f64", 37, 100_003), ("f32", 37, 100_003), ("bf16plain", 37, 100_003), ("tall", 40, 100_003),
         ("widebf16", 300, 50_001), ("widefp8", 300, 50_001), ("widebf16", 2000, 20_003), ("widefp8", 2000, 20_003),
         ("widebf16", 33_000, 300)]  # the last: coefficients beyond the 128 KiB LDS copy (global reads)


@pytest.mark.parametrize("kind,d,n", CASES)
def test_lsq_passes_match_oracle(kind, d, n):
    dev = _dev()
    g = torch.Generator(device=dev).manual_seed(d + n)
    X = torch.randn(d, n, generator=g, device=dev, dtype=torch.float64) + 0.25
    y = torch.randn(n, generator=g, device=dev, dtype=torch.float64)
    w = 0.5 + torch.rand(n, generator=g, device=dev, dtype=torch.float64)
    sel = torch.rand(n, generator=g, device=dev) > 0.2
    Xl = _layout(kind, X)
    P = kernels.lsq_passes(Xl, y, w, sel)
    assert isinstance(P, device.LsqPasses)
    H = kernels._HostLsq(_dense64(Xl), y.cpu(), w.cpu(), sel.cpu())
    exact = kind in ("f64", "f32", "bf16plain")  # f64 arithmetic on the stored values
    rt = 1e-11 if exact else 2e-5
    cf = torch.randn(d, generator=g, device=dev, dtype=torch.float64) / np.sqrt(d)
    off = torch.tensor([0.3], dtype=torch.float64, device=dev)
    got = P.evaluate(cf, off, 0.7).cpu()
    ref = H.evaluate(cf.cpu(), off.cpu(), 0.7)
    # scale of each sum: sum |w diff x| bounds the f32 accumulation error
    Xd = H._Xz
    diff = cf.cpu() @ Xd + 0.3 - 0.7 * H.y
    v = H.w * diff
    gscale = (Xd.abs() @ v.abs()).numpy() + 1e-30
    assert abs(float(got[0]) - float(ref[0])) <= rt * float((0.5 * v.abs() * diff.abs()).sum())
    assert np.all(np.abs(got[1:].numpy() - ref[1:].numpy()) <= rt * gscale)
    again = P.evaluate(cf, off, 0.7).cpu()
    assert torch.equal(got, again)  # fixed-order reductions: bitwise repeatable
    mo = P.moments().cpu()
    mref = H.moments()
    s1 = (Xd.abs() @ H.w).numpy() + 1e-30
    assert np.all(np.abs(mo[:d].numpy() - mref[:d].numpy()) <= rt * s1)
    assert np.all(np.abs(mo[d:].numpy() - mref[d:].numpy()) <= rt * mref[d:].numpy() + 1e-30)
    sc = P.scalars().cpu()
    np.testing.assert_allclose(sc.numpy(), H.scalars().numpy(), rtol=1e-12)
    # a line-search trial cf + a dcf from u(cf) + a u(dcf) (wmargins) and the column pass alone
    dcf = torch.randn(d, generator=g, device=dev, dtype=torch.float64) / np.sqrt(d)
    a = 0.37
    u = P.wmargins(cf) + a * P.wmargins(dcf)
    got_u = P.evaluate_u(u, cf + a * dcf, off, 0.7).cpu()
    ref_u = H.evaluate(cf.cpu() + a * dcf.cpu(), off.cpu(), 0.7)
    diff_u = (cf.cpu() + a * dcf.cpu()) @ Xd + 0.3 - 0.7 * H.y
    v_u = H.w * diff_u
    assert abs(float(got_u[0]) - float(ref_u[0])) <= 2 * rt * float((0.5 * v_u.abs() * diff_u.abs()).sum()) + 1e-12
    assert np.all(np.abs(got_u[1:].numpy() - ref_u[1:].numpy()) <= 2 * rt * ((Xd.abs() @ v_u.abs()).numpy() + 1e-30))


@pytest.mark.parametrize("kw", [dict(regParam=0.02, elasticNetParam=0.0), dict(regParam=0.02, elasticNetParam=0.6)])
def test_gpu_lbfgs_passes_match_gram_route(gpu_session, kw):
    dev = gpu_session.device
    g = torch.Generator(device=dev).manual_seed(3)
    d, n = 24, 300_000
    X = torch.randn(d, n, generator=g, device=dev, dtype=torch.float64) * 2 + 1
    y = torch.linspace(-1, 1, d, device=dev, dtype=torch.float64) @ X + 0.5 + 0.1 * torch.randn(
        n, generator=g, device=dev, dtype=torch.float64)
    df = gpu_session.createDataFrame({"features": X, "label": y})
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression

    a = LinearRegression(solver="l-bfgs", tol=1e-12, maxIter=300, **kw).fit(df)
    gpu_session.conf.set("dq4ml.lbfgs.mode", "gram")
    try:
        b = LinearRegression(solver="l-bfgs", tol=1e-12, maxIter=300, **kw).fit(df)
    finally:
        gpu_session.conf.set("dq4ml.lbfgs.mode", "passes")
    np.testing.assert_allclose(a.coefficients.toArray(), b.coefficients.toArray(), rtol=1e-6, atol=1e-8)
    assert float(a.intercept) == pytest.approx(float(b.intercept), rel=1e-6)
    assert a.summary.solver == ("owlqn" if kw["elasticNetParam"] else "l-bfgs")


def test_gpu_lbfgs_wide_bf16_recovers_coefficients(gpu_session):
    """numFeatures > 4096, solver auto -> Spark's l-bfgs switch on the wide bf16 fragment layout."""
    dev = gpu_session.device
    g = torch.Generator(device=dev).manual_seed(8)
    d, n = 4200, 40_000
    X = torch.randn(d, n, generator=g, device=dev)
    beta = torch.zeros(d, device=dev)
    beta[:50] = torch.linspace(0.5, 2.0, 50, device=dev)
    y = beta @ X + 0.3 + 0.05 * torch.randn(n, generator=g, device=dev)
    T = device.pack_wide([X], 16, None)
    df = gpu_session.createDataFrame({"features": T, "label": y})
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression

    m = LinearRegression(regParam=0.001, elasticNetParam=0.0, maxIter=100).fit(df)
    assert m.summary.solver == "l-bfgs"
    err = np.abs(m.coefficients.toArray() - beta.double().cpu().numpy()).max()
    assert err < 0.05, err
