"""Large-k device WLS solve (``ops/csrc/hip/wls_large.hip``): the standardized dense system the
kernels assemble from the flat statistics against a NumPy fp64 assembly of the same algebra
(``csrc/host/wls.cpp``), the device Jacobi-PCG against a direct fp64 solve, and the fallbacks
(non-positive diagonal -> None -> Cholesky / quasi-newton)."""
import numpy as np
import pytest

from net.jgp.labs.sparkdq4ml_amd.models import optim

pytestmark = pytest.mark.gpu


def _stats(d, n, seed=0, zero_col=None):
    import torch

    from net.jgp.labs.sparkdq4ml_amd.ops import device

    g = torch.Generator(device="cuda").manual_seed(seed)
    X = torch.randn(d, n, generator=g, device="cuda", dtype=torch.float64) * 1.5 + 0.25
    if zero_col is not None:
        X[zero_col] = 3.0
    y = torch.linspace(-1, 1, d, device="cuda", dtype=torch.float64) @ X + 1.0 + 0.2 * torch.randn(
        n, generator=g, device="cuda", dtype=torch.float64)
    return device.gram_stats(X, y, None, None, "fp64")


def _ref_system(flat, nf, fit_intercept, eff_l2, std_f, std_l):
    wSum, bSum, bbSum = flat[1], flat[3], flat[4]
    aSum, abSum, aaP = flat[5:5 + nf], flat[5 + nf:5 + 2 * nf], flat[5 + 2 * nf:]
    rawBBar = bSum / wSum
    bStd = np.sqrt(max(bbSum / wSum - rawBBar * rawBBar, 0.0))
    I, J = optim.packed_upper_indices(nf)
    dj = np.arange(nf) + np.arange(nf) * (np.arange(nf) + 1) // 2
    m = aSum / wSum
    aStd = np.sqrt(np.maximum(aaP[dj] / wSum - m * m, 0.0))
    nz = aStd != 0
    safe = np.where(nz, aStd, 1.0)
    k = nf + 1 if fit_intercept else nf
    A = np.zeros((k, k))
    den = aStd[I] * aStd[J]
    with np.errstate(divide="ignore", invalid="ignore"):
        vals = np.where(den != 0, aaP / wSum / np.where(den != 0, den, 1.0), 0.0)
    A[I, J] = vals
    A[J, I] = vals
    lam = np.full(nf, eff_l2)
    if not std_f:
        lam = np.where(nz, lam / (safe * safe), 0.0)
    if not std_l:
        lam = lam * bStd
    A[np.arange(nf), np.arange(nf)] += lam
    b = np.where(nz, abSum / wSum / (safe * bStd), 0.0)
    if fit_intercept:
        A[:nf, nf] = A[nf, :nf] = np.where(nz, m / safe, 0.0)
        A[nf, nf] = 1.0
        b = np.concatenate([b, [rawBBar / bStd]])
    return A, b, aStd, bStd, rawBBar


@pytest.mark.parametrize("nf,fit_intercept,std_f,std_l,zero_col", [
    (1030, True, True, True, None), (1030, False, True, True, 7), (1100, True, False, True, 3),
    (1025, True, True, False, None), (1057, False, False, False, 40)])
def test_assemble_matches_numpy(nf, fit_intercept, std_f, std_l, zero_col):
    from net.jgp.labs.sparkdq4ml_amd.ops import device

    flat = _stats(nf, 4000, seed=nf, zero_col=zero_col)
    host = flat.cpu().numpy()
    eff_l2 = 0.05
    A_ref, b_ref, aStd_ref, bStd, _ = _ref_system(host, nf, fit_intercept, eff_l2, std_f, std_l)
    # (reg, enet) with (1 - enet) reg / bStd = eff_l2: the head scalars are the device's own
    s = device.wls_assemble(flat, nf, fit_intercept, eff_l2 * float(bStd), 0.0, std_f, std_l)
    o = s.o[:device.PCG_STATE_WORDS].cpu().numpy()
    assert o[device.PCG_STATUS] == 0.0 and o[device.PCG_BSTD] == pytest.approx(bStd, rel=1e-14)
    np.testing.assert_array_equal(o[device.PCG_HEAD:device.PCG_HEAD + 5], host[:5])
    A = s.A.cpu().numpy()
    np.testing.assert_allclose(A, A_ref, rtol=1e-13, atol=1e-15)
    assert np.array_equal(A, A.T)
    np.testing.assert_allclose(s.b.cpu().numpy(), b_ref, rtol=1e-13, atol=1e-15)
    np.testing.assert_allclose(s.aStd.cpu().numpy(), aStd_ref, rtol=1e-13, atol=1e-15)
    with np.errstate(divide="ignore"):
        np.testing.assert_allclose(s.minv.cpu().numpy(), 1.0 / np.diag(A_ref), rtol=1e-13)


@pytest.mark.parametrize("nf,fit_intercept", [(1030, True), (1101, False), (2048, True)])
def test_pcg_matches_direct_solve(nf, fit_intercept):
    import torch

    from net.jgp.labs.sparkdq4ml_amd.ops import device

    flat = _stats(nf, 3 * nf, seed=7)
    host = flat.cpu().numpy()
    A_ref, b_ref, aStd, bStd, _ = _ref_system(host, nf, fit_intercept, 0.02, True, True)
    s = device.wls_assemble(flat, nf, fit_intercept, 0.02 * float(bStd), 0.0, True, True)
    o = device.wls_pcg(s, nf, optim.PCG_RTOL)
    assert device.pcg_ok(o)
    k = s.k
    x = o[device.PCG_STATE_WORDS:device.PCG_STATE_WORDS + k]
    ref = torch.linalg.solve(torch.as_tensor(A_ref), torch.as_tensor(b_ref)).numpy()
    assert np.abs(x - ref).max() / np.abs(ref).max() < 1e-10
    coef = o[device.PCG_STATE_WORDS + k:]
    np.testing.assert_allclose(coef, x[:nf] * bStd / aStd, rtol=1e-12, atol=1e-14)
    # deterministic: the same control block bit for bit on a second solve
    s2 = device.wls_assemble(flat, nf, fit_intercept, 0.02 * float(bStd), 0.0, True, True)
    assert np.array_equal(device.wls_pcg(s2, nf, optim.PCG_RTOL), o)
    # enqueued whole (the asynchronous fit's form): the same iterates, converged ones are no-ops
    s3 = device.wls_assemble(flat, nf, fit_intercept, 0.02 * float(bStd), 0.0, True, True)
    device.wls_pcg_enqueue(s3, nf, optim.PCG_RTOL, 96)
    o3 = s3.o.cpu().numpy()
    w = device.PCG_STATE_WORDS
    assert device.pcg_ok(o3) and 0 < o3[device.PCG_ITERS] < 96
    assert np.array_equal(o3[w:], o[w:])


def test_pcg_declines_non_positive_diagonal_and_fit_falls_back():
    from net.jgp.labs.sparkdq4ml_amd.ops import device

    nf = 1040
    flat = _stats(nf, 3000, seed=11, zero_col=5)
    host = flat.cpu().numpy()
    # no intercept, no L2, unstandardized: the constant feature's diagonal is exactly 0
    s = device.wls_assemble(flat, nf, False, 0.0, 0.0, False, True)
    o = device.wls_pcg(s, nf, optim.PCG_RTOL)
    assert o[device.PCG_BAD] != 0.0 and not device.pcg_ok(o)
    # the fit itself still returns Spark's answer (Cholesky fails -> quasi-newton on the host)
    got, _ = optim.fit_wls_flat(flat, nf, False, 0.0, 0.0, False, True, "auto", 200, 1e-10)
    assert got.solver in ("l-bfgs", "quasi-newton") and np.isfinite(got.coefficients).all()


def test_device_fit_l2_matches_reference_no_intercept():
    nf = 1200
    flat = _stats(nf, 5000, seed=5)
    for std in (True, False):
        got, stats = optim.fit_wls_flat(flat, nf, False, 0.3, 0.0, std, True, "auto", 100, 1e-6)
        assert got.solver == "cholesky" and stats.aSum is None
        ref = optim.weighted_least_squares(optim.GramStats.from_flat(flat.cpu().numpy(), nf), False, 0.3, 0.0, std,
                                           True, "auto", 100, 1e-6)
        np.testing.assert_allclose(got.coefficients, ref.coefficients, rtol=1e-8, atol=1e-10)
        assert got.intercept == 0.0


def test_constant_label_short_circuits_to_host_driver():
    """A constant label: the device head sets STATUS, every solve kernel exits, and the fit takes the
    native driver's semantics (coefficients 0, intercept = the label)."""
    import torch

    from net.jgp.labs.sparkdq4ml_amd.ops import device

    nf = 1030
    g = torch.Generator(device="cuda").manual_seed(3)
    X = torch.randn(nf, 3000, generator=g, device="cuda", dtype=torch.float64)
    y = torch.full((3000,), 4.25, device="cuda", dtype=torch.float64)
    flat = device.gram_stats(X, y, None, None, "fp64")
    s = device.wls_assemble(flat, nf, True, 0.1, 0.0, True, False)
    o = device.wls_pcg(s, nf, optim.PCG_RTOL)
    assert o[device.PCG_STATUS] == 1.0
    got, _ = optim.fit_wls_flat(flat, nf, True, 0.1, 0.0, True, False, "auto", 100, 1e-6)
    assert np.all(got.coefficients == 0.0) and got.intercept == pytest.approx(4.25, rel=1e-12)
