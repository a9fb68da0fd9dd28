"""Simulated data parallelism on one GPU ("Distributed (simulated)"): split the rows
into uneven shards, run the device Gram (K4/K5) per shard, sum the partials the way the X1
all-reduce does, and require the result to equal the unsharded pass BIT FOR BIT.

Integer-valued features and labels keep every product and partial sum exact in bf16 inputs, f32
MFMA accumulators and the f64 fold, so any difference is a real indexing bug (a lost or doubled
row at a shard / slab / tile edge), not rounding.  The CPU f64 oracle (`ops/kernels.py`) pins the
absolute values."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _int_data(d, n, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    X = torch.randint(-4, 5, (d, n), generator=g, device="cuda").to(torch.float32)
    y = torch.randint(-8, 9, (n,), generator=g, device="cuda").to(torch.float32)
    sel = torch.rand(n, generator=g, device="cuda") > 0.25
    return X, y, sel


def _bounds(n, k):
    # deliberately uneven shards whose edges fall inside tiles / slabs
    cuts = [0] + [int(n * f) + 7 * i for i, f in enumerate([0.23, 0.61, 0.84][:k - 1], 1)] + [n]
    return list(zip(cuts[:-1], cuts[1:]))


@pytest.mark.parametrize("d,compute,k", [(32, "bf16", 3), (64, "bf16", 4), (1, "fp64", 3), (17, "fp64", 2)])
def test_sharded_gram_sum_equals_unsharded(d, compute, k):
    from net.jgp.labs.sparkdq4ml_amd.ops import device, kernels

    n = 1_000_003
    X, y, sel = _int_data(d, n, seed=d + k)

    def stats(lo, hi):
        Xs = X[:, lo:hi].contiguous()
        src = device.tile_bf16(Xs.to(torch.bfloat16)) if compute == "bf16" else Xs.to(torch.float64)
        return device.gram_stats(src, y[lo:hi].contiguous(), None, sel[lo:hi].contiguous(), compute)

    whole = stats(0, n)
    parts = [stats(lo, hi) for lo, hi in _bounds(n, k)]
    summed = torch.stack(parts).sum(0)
    assert torch.equal(summed, whole)

    oracle = kernels.gram_stats(X.cpu(), y.cpu(), None, sel.cpu(), "fp64")
    assert torch.equal(whole.cpu(), oracle)


def test_sharded_fit_matches_unsharded_fit(gpu_session):
    """Per-shard statistics summed (what every rank holds after X1) equal the single-pass
    statistics, and the fit over all rows recovers the exact integer model."""
    import numpy as np

    from net.jgp.labs.sparkdq4ml_amd import LinearRegression
    from net.jgp.labs.sparkdq4ml_amd.models.optim import GramStats
    from net.jgp.labs.sparkdq4ml_amd.ops import device

    d, n = 32, 2_000_011
    X, _, _ = _int_data(d, n, seed=5)
    g = torch.Generator(device="cuda").manual_seed(9)
    coef = torch.randint(-2, 3, (d,), generator=g, device="cuda").to(torch.float32)
    y = coef @ X + 2.0  # integers, |y| <= 258: exact everywhere
    df = gpu_session.createDataFrame({"features": X.to(torch.bfloat16), "label": y})
    ref = LinearRegression(solver="normal", gramDtype="bf16").fit(df)

    flat = sum(device.gram_stats(device.tile_bf16(X[:, lo:hi].contiguous().to(torch.bfloat16)),
                                 y[lo:hi].contiguous(), None, None, "bf16") for lo, hi in _bounds(n, 3))
    whole = device.gram_stats(device.tile_bf16(X.to(torch.bfloat16)), y, None, None, "bf16")
    assert torch.equal(flat, whole)
    assert GramStats.from_flat(flat.cpu().numpy(), d).count == n
    np.testing.assert_allclose(ref.coefficients.toArray(), coef.cpu().numpy(), atol=1e-6)
    assert float(ref.intercept) == pytest.approx(2.0, abs=1e-6)
