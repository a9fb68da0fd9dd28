"""Native WLS driver (``csrc/host/wls.cpp``) against the NumPy reference implementation of Spark's
WeightedLeastSquares (``models/optim.weighted_least_squares``) on the same statistics."""
import itertools

import numpy as np
import pytest

from net.jgp.labs.sparkdq4ml_amd.models import optim
from net.jgp.labs.sparkdq4ml_amd.ops import kernels


def _flat(n=400, d=5, seed=0, const_label=None, zero_col=False):
    import torch

    rng = np.random.default_rng(seed)
    X = rng.normal(size=(d, n)) * np.linspace(0.5, 3, d)[:, None] + 1.0
    if zero_col:
        X[2] = 7.0  # constant feature -> aStd == 0
    y = np.linspace(-1, 1, d) @ X + 0.3 * rng.normal(size=n) + 2.0
    if const_label is not None:
        y = np.full(n, const_label)
    return kernels.gram_stats(torch.as_tensor(X), torch.as_tensor(y), None, None, "fp64").numpy(), d


CASES = list(itertools.product([True, False], [0.0, 0.3], [0.0, 0.5, 1.0], [True, False],
                               ["auto", "cholesky", "quasi-newton"]))


@pytest.mark.parametrize("fit_intercept,reg,enet,std,solver", CASES)
def test_native_matches_reference(fit_intercept, reg, enet, std, solver):
    flat, d = _flat(zero_col=(reg == 0.3 and enet == 0.5))
    stats = optim.GramStats.from_flat(flat, d)
    try:
        ref = optim.weighted_least_squares(stats, fit_intercept, reg, enet, std, True, solver, 100, 1e-9)
    except optim.SingularMatrixException:
        with pytest.raises(optim.SingularMatrixException):
            optim.fit_wls_flat(flat, d, fit_intercept, reg, enet, std, True, solver, 100, 1e-9)
        return
    got, _ = optim.fit_wls_flat(flat, d, fit_intercept, reg, enet, std, True, solver, 100, 1e-9)
    assert got.solver == ref.solver
    np.testing.assert_allclose(got.coefficients, ref.coefficients, rtol=1e-10, atol=1e-12)
    assert got.intercept == pytest.approx(ref.intercept, rel=1e-10, abs=1e-12)
    np.testing.assert_allclose(got.objectiveHistory, ref.objectiveHistory, rtol=1e-10, atol=1e-14)
    if got.solver == "cholesky":
        with np.errstate(divide="ignore", invalid="ignore"):
            np.testing.assert_allclose(got.diagInvAtWA, ref.diagInvAtWA, rtol=1e-9)


@pytest.mark.parametrize("fit_intercept", [True, False])
@pytest.mark.parametrize("label", [0.0, 3.5])
def test_native_constant_label(fit_intercept, label):
    flat, d = _flat(const_label=label)
    stats = optim.GramStats.from_flat(flat, d)
    args = (fit_intercept, 0.0, 0.0, True, True, "auto", 50, 1e-6)
    try:
        ref = optim.weighted_least_squares(stats, *args)
    except ValueError as e:
        with pytest.raises(ValueError, match=str(e)[:30]):
            optim.fit_wls_flat(flat, d, *args)
        return
    got, _ = optim.fit_wls_flat(flat, d, *args)
    np.testing.assert_allclose(got.coefficients, ref.coefficients, atol=1e-12)
    assert got.intercept == pytest.approx(ref.intercept, abs=1e-12)


def test_native_empty_and_zero_weight():
    d = 3
    flat = np.zeros(optim.GramStats.layout_size(d))
    with pytest.raises(ValueError, match="empty"):
        optim.fit_wls_flat(flat, d, True, 0.0, 0.0, True, True, "auto", 10, 1e-6)
    flat[0] = 5.0
    with pytest.raises(ValueError, match="Sum of weights"):
        optim.fit_wls_flat(flat, d, True, 0.0, 0.0, True, True, "auto", 10, 1e-6)


@pytest.mark.gpu
def test_device_large_k_matches_reference():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    d, n = 1100, 6000
    g = torch.Generator(device="cuda").manual_seed(3)
    X = torch.randn(d, n, generator=g, device="cuda", dtype=torch.float64) + 0.5
    y = torch.linspace(-1, 1, d, device="cuda", dtype=torch.float64) @ X + 1.0 + 0.1 * torch.randn(
        n, generator=g, device="cuda", dtype=torch.float64)
    from net.jgp.labs.sparkdq4ml_amd.ops import device

    flat = device.gram_stats(X, y, None, None, "fp64")
    got, stats = optim.fit_wls_flat(flat, d, True, 0.1, 0.0, True, True, "auto", 100, 1e-6)
    assert got.solver == "cholesky" and stats.aSum is None  # solved on the device
    ref = optim.weighted_least_squares(optim.GramStats.from_flat(flat.cpu().numpy(), d), True, 0.1, 0.0, True,
                                       True, "auto", 100, 1e-6)
    np.testing.assert_allclose(got.coefficients, ref.coefficients, rtol=1e-8, atol=1e-10)
    assert got.intercept == pytest.approx(ref.intercept, rel=1e-8)
    np.testing.assert_allclose(got.diagInvAtWA, ref.diagInvAtWA, rtol=1e-7)


def test_pcg_matches_direct_solve_and_declines_non_spd():
    """Large-k device solve: Jacobi-PCG (optim._pcg) reaches the direct solution; a non-positive
    diagonal or a non-converging (indefinite) system returns None -> Cholesky fallback path."""
    import torch

    from net.jgp.labs.sparkdq4ml_amd.models.optim import _pcg

    g = torch.Generator().manual_seed(3)
    X = torch.randn(3000, 300, generator=g, dtype=torch.float64)
    X[:, 1] = X[:, 0] + 1e-3 * torch.randn(3000, generator=g, dtype=torch.float64)  # collinear pair
    A = X.T @ X / 3000 + 1e-2 * torch.eye(300, dtype=torch.float64)
    b = torch.randn(300, generator=g, dtype=torch.float64)
    x = _pcg(A, b)
    ref = torch.linalg.solve(A, b)
    assert x is not None and float((x - ref).abs().max() / ref.abs().max()) < 1e-10
    B = A.clone()
    B[5, 5] = 0.0
    assert _pcg(B, b) is None
    C = torch.diag(torch.tensor([1.0, 2.0, 3.0], dtype=torch.float64))
    C[0, 1] = C[1, 0] = 5.0  # indefinite with a positive diagonal
    assert _pcg(C, torch.ones(3, dtype=torch.float64)) is None or torch.allclose(
        C @ _pcg(C, torch.ones(3, dtype=torch.float64)), torch.ones(3, dtype=torch.float64))
