"""Race / determinism screens: the device reductions use fixed-order slab
reductions (no float atomics), so repeated launches must be bit-identical — a race in a kernel's
LDS pipeline or an unordered reduction shows up here as run-to-run differences."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("d,compute", [(32, "bf16"), (64, "bf16"), (17, "fp64")])
def test_tall_gram_bit_identical(d, compute):
    from net.jgp.labs.sparkdq4ml_amd.ops import device

    n = 3_000_017
    g = torch.Generator(device="cuda").manual_seed(d)
    X = torch.randn(d, n, generator=g, device="cuda", dtype=torch.float64 if compute == "fp64" else torch.float32)
    y = torch.randn(n, generator=g, device="cuda")
    sel = torch.rand(n, generator=g, device="cuda") > 0.2
    src = device.tile_bf16(X.to(torch.bfloat16)) if compute == "bf16" else X
    outs = [device.gram_stats(src, y, None, sel, compute) for _ in range(6)]
    for o in outs[1:]:
        assert torch.equal(o, outs[0])


@pytest.mark.parametrize("eb", [16, 8])
def test_wide_syrk_bit_identical(eb):
    from net.jgp.labs.sparkdq4ml_amd.ops import device

    d, n = 600, 150_000
    g = torch.Generator(device="cuda").manual_seed(eb)
    T = device.pack_wide([torch.randn(d, n, generator=g, device="cuda")], eb, None)
    y = torch.randn(n, generator=g, device="cuda")
    outs = [device.gram_stats(T, y, None, None, "fp8" if eb == 8 else "bf16", x_zero_dead=True) for _ in range(5)]
    for o in outs[1:]:
        assert torch.equal(o, outs[0])


def test_fit_and_metrics_bit_identical(gpu_session):
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression

    g = torch.Generator(device="cuda").manual_seed(1)
    X = torch.randn(32, 1_000_000, generator=g, device="cuda").to(torch.bfloat16)
    y = torch.linspace(-1, 1, 32, device="cuda") @ X.float() + 0.3
    df = gpu_session.createDataFrame({"features": X, "label": y})
    ms = [LinearRegression(solver="normal", gramDtype="bf16").fit(df) for _ in range(4)]
    ref = ms[0]
    for m in ms[1:]:
        assert (m.coefficients.toArray() == ref.coefficients.toArray()).all()
        assert float(m.intercept) == float(ref.intercept)
        assert float(m.summary.r2) == float(ref.summary.r2)
