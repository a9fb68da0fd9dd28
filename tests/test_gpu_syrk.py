"""Wide exact SYRK (``gram_syrk.hip``): f64 / exact-f32 MFMA statistics for d > 64 with weights
and DQ selection in-kernel, against a plain fp64 torch reference of the same sums; and the
in-place row mask of the wide fragment layouts (``wide_mask_rows_kernel``)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _oracle(X, y, w, sel):
    """Flat WLS layout in fp64: count, Σw, Σw², Σwy, Σwy², Σw·x, Σw·x·y, packed upper Σw·x·xᵀ."""
    Xd, yd = X.double(), y.double()
    n = Xd.shape[1]
    wv = torch.ones(n, dtype=torch.float64, device=X.device) if w is None else w.double()
    if sel is not None:
        wv = torch.where(sel, wv, torch.zeros_like(wv))
    live = wv != 0
    Xd = torch.where(live, Xd, torch.zeros_like(Xd))
    yd = torch.where(live, yd, torch.zeros_like(yd))
    d = Xd.shape[0]
    G = (Xd * wv) @ Xd.t()
    iu = torch.triu_indices(d, d, device=X.device)
    # packed upper, column-major over j: index i + j(j+1)/2
    order = torch.argsort(iu[0] + iu[1] * (iu[1] + 1) // 2)
    packed = G[iu[0], iu[1]][order]
    head = torch.stack([live.sum().double(), wv.sum(), (wv * wv).sum(), (wv * yd).sum(), (wv * yd * yd).sum()])
    return torch.cat([head, Xd @ wv, Xd @ (wv * yd), packed])


def _rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-300))


@pytest.mark.parametrize("d,n", [(65, 20_011), (257, 9_000), (1024, 3_001), (4096, 700)])
@pytest.mark.parametrize("xdt", [torch.float64, torch.float32])
@pytest.mark.parametrize("weighted", [False, True])
def test_syrk_f64_matches_oracle(d, n, xdt, weighted):
    from net.jgp.labs.sparkdq4ml_amd.ops import device

    g = torch.Generator(device="cuda").manual_seed(d + n)
    X = (torch.randn(d, n, generator=g, device="cuda", dtype=torch.float64) * 2 + 0.5).to(xdt)
    y = torch.randn(n, generator=g, device="cuda", dtype=torch.float64) * 3 - 1
    w = sel = None
    if weighted:
        w = torch.rand(n, generator=g, device="cuda", dtype=torch.float64) * 2
        w[::7] = 0.0  # zero weights skip the row entirely
        sel = torch.rand(n, generator=g, device="cuda") > 0.3
        X[:, 5] = float("nan")  # a dead row (w == 0 at index 0 mod 7... make row 5 dead explicitly)
        sel[5] = False
    out = device.gram_stats(X, y, w, sel, "fp64")
    ref = _oracle(X, y, w, sel)
    assert out.shape == ref.shape
    assert not torch.isnan(out).any()
    assert float(out[0]) == float(ref[0])
    assert _rel(out, ref) < 1e-12


@pytest.mark.parametrize("d,n", [(100, 50_000), (600, 4_000)])
def test_syrk_exact_f32_matches_oracle(d, n):
    from net.jgp.labs.sparkdq4ml_amd.ops import device

    g = torch.Generator(device="cuda").manual_seed(d)
    X = torch.randn(d, n, generator=g, device="cuda", dtype=torch.float32)
    y = torch.randn(n, generator=g, device="cuda", dtype=torch.float32)
    out = device.gram_stats(X, y, None, None, "fp32")
    ref = _oracle(X, y, None, None)
    assert _rel(out, ref) < 2e-5  # f32 products, f32 accumulation per split, f64 across splits


def test_syrk_weighted_bf16_request_uses_f32_kernel():
    from net.jgp.labs.sparkdq4ml_amd.ops import device

    d, n = 130, 30_000
    g = torch.Generator(device="cuda").manual_seed(11)
    X = torch.randn(d, n, generator=g, device="cuda").to(torch.bfloat16)
    y = torch.randn(n, generator=g, device="cuda")
    w = torch.rand(n, generator=g, device="cuda", dtype=torch.float64)
    out = device.gram_stats(X, y, w, None, "bf16")
    ref = _oracle(X.float(), y, w, None)
    assert _rel(out, ref) < 2e-5


def test_wide_linear_regression_fp64_weighted_matches_host(gpu_session):
    """The default-precision (fp64) wide fit on the device vs the same fit on the host engine."""
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, SparkSession

    d, n = 150, 20_000
    rng = np.random.default_rng(0)
    X = rng.standard_normal((d, n))
    beta = np.linspace(-1, 1, d)
    y = beta @ X + 0.3 + 0.01 * rng.standard_normal(n)
    w = rng.uniform(0.5, 2.0, n)
    dev = gpu_session.createDataFrame({"features": torch.tensor(X, device="cuda"),
                                       "label": torch.tensor(y, device="cuda"),
                                       "w": torch.tensor(w, device="cuda")})
    lr = LinearRegression(solver="normal", weightCol="w", regParam=0.01, elasticNetParam=0.0)
    m_dev = lr.fit(dev)
    gpu_session.stop()
    host = SparkSession.builder().master("cpu").getOrCreate()
    m_host = lr.fit(host.createDataFrame({"features": torch.tensor(X), "label": torch.tensor(y),
                                          "w": torch.tensor(w)}))
    host.stop()
    np.testing.assert_allclose(m_dev.coefficients.toArray(), m_host.coefficients.toArray(), rtol=1e-9, atol=1e-11)
    assert float(m_dev.intercept) == pytest.approx(float(m_host.intercept), rel=1e-9, abs=1e-11)


@pytest.mark.parametrize("eb", [8, 16])
def test_wide_mask_rows_equals_pack_with_selection(eb):
    from net.jgp.labs.sparkdq4ml_amd.ops import device

    d, n = 300, 10_007
    g = torch.Generator(device="cuda").manual_seed(eb)
    X = torch.randn(d, n, generator=g, device="cuda")
    sel = torch.rand(n, generator=g, device="cuda") > 0.4
    full = device.pack_wide([X], eb, None)
    masked = device.mask_wide_rows(full, sel)
    direct = device.pack_wide([X], eb, sel, inv_scale=None if eb == 16 else 1.0 / full.scales)
    assert torch.equal(masked.buf, direct.buf)  # same scales: bit-identical storage
    dense = masked.to_dense().float()
    ref = torch.where(sel, full.to_dense().float(), torch.zeros_like(dense))
    assert torch.equal(dense, ref)
