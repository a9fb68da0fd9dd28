"""Numerics of the gfx950 kernels against plain PyTorch fp64 references (run via gpurun)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from net.jgp.labs.sparkdq4ml_amd.ops import device, kernels, native  # noqa: E402


def _ref_stats(X, y, w, sel):
    return kernels.gram_stats(X.double().cpu(), y.double().cpu(), None if w is None else w.double().cpu(),
                              None if sel is None else sel.cpu(), "fp64")


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    scale = b.abs().max().clamp_min(1e-300)
    return float((a - b).abs().max() / scale)


@pytest.fixture(scope="module", autouse=True)
def _hip():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    native.hip()


@pytest.mark.parametrize("d", [1, 5, 32, 33, 64])
@pytest.mark.parametrize("n", [1, 63, 64, 1000, 100_003])
def test_gram_f64_matches_oracle(d, n):
    g = torch.Generator(device="cuda").manual_seed(d * 1000 + n)
    X = torch.randn(d, n, generator=g, device="cuda", dtype=torch.float64) + 0.5
    y = torch.randn(n, generator=g, device="cuda", dtype=torch.float64) * 3 + 1
    out = device.gram_stats(X, y, None, None, "fp64")
    ref = _ref_stats(X, y, None, None)
    assert _rel(out, ref) < 1e-12


@pytest.mark.parametrize("xdt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("d", [1, 7, 32, 48, 64])
@pytest.mark.parametrize("n", [5, 64, 4096 + 17, 250_000])
def test_gram_bf16_matches_oracle(xdt, d, n):
    g = torch.Generator(device="cuda").manual_seed(7 * d + n)
    X = (torch.randn(d, n, generator=g, device="cuda") + 0.25).to(xdt)
    y = torch.randn(n, generator=g, device="cuda") * 2 + 3
    out = device.gram_stats(X, y, None, None, "bf16")
    ref = _ref_stats(X.to(torch.bfloat16).float(), y, None, None)  # oracle on the bf16-rounded features
    # scalars exact-ish (f64), Gram blocks f32-accumulated
    assert _rel(out[:5], ref[:5]) < 1e-12
    if xdt == torch.float32:
        # f32 storage: the stream kernel's side sums Σw·x, Σw·x·y use the unrounded features
        exact = _ref_stats(X.double(), y, None, None)
        assert _rel(out[5:5 + 2 * d], exact[5:5 + 2 * d]) < 2e-6
        assert _rel(out[5 + 2 * d:], ref[5 + 2 * d:]) < 2e-5
    else:
        assert _rel(out[5:], ref[5:]) < 2e-5


@pytest.mark.parametrize("mode", ["fp64", "bf16"])
def test_gram_with_selection_and_weights(mode):
    g = torch.Generator(device="cuda").manual_seed(3)
    d, n = 32, 20_000
    X = torch.randn(d, n, generator=g, device="cuda", dtype=torch.float64)
    y = torch.randn(n, generator=g, device="cuda", dtype=torch.float64)
    sel = torch.rand(n, generator=g, device="cuda") > 0.3
    w = torch.rand(n, generator=g, device="cuda", dtype=torch.float64) + 0.5
    Xin = X if mode == "fp64" else X.to(torch.bfloat16)
    Xref = Xin.double()
    tol = 1e-12 if mode == "fp64" else 3e-3  # bf16 rounding of w*x in the weighted operand
    for ww, ss in ((None, sel), (w, None), (w, sel)):
        out = device.gram_stats(Xin, y, ww, ss, mode)
        ref = _ref_stats(Xref, y, ww, ss)
        assert _rel(out[:5], ref[:5]) < 1e-12
        assert _rel(out[5:], ref[5:]) < tol, (ww is None, ss is None)


@pytest.mark.parametrize("d", [1, 2, 3, 8])
@pytest.mark.parametrize("xdt", [torch.float64, torch.float32])
def test_gram_f64_skinny_selection_weights_and_dead_nans(d, xdt):
    """d <= 8 f64 statistics take the lane-per-row VALU kernel: selection, weights, f32 features,
    and NaN / inf garbage in dead rows (null labels) must not leak into the sums."""
    g = torch.Generator(device="cuda").manual_seed(40 + d)
    n = 123_457
    X = (torch.randn(d, n, generator=g, device="cuda", dtype=torch.float64) * 2 + 1).to(xdt)
    y = torch.randn(n, generator=g, device="cuda", dtype=torch.float64)
    sel = torch.rand(n, generator=g, device="cuda") > 0.25
    w = torch.rand(n, generator=g, device="cuda", dtype=torch.float64) + 0.5
    y_bad = y.clone()
    y_bad[~sel] = float("nan")
    Xb = X.clone()
    Xb[:, (~sel).nonzero()[:5, 0]] = float("inf")
    for ww in (None, w):
        out = device.gram_stats(Xb, y_bad, ww, sel, "fp64")
        ref = _ref_stats(X.double(), y, ww, sel)
        assert torch.isfinite(out).all()
        assert _rel(out, ref) < 1e-12
    out = device.gram_stats(X, y, None, None, "fp64")
    assert _rel(out, _ref_stats(X.double(), y, None, None)) < 1e-12


@pytest.mark.parametrize("d", [1, 4, 8])
def test_gram_skinny_cols_reads_mixed_source_columns(d):
    """Narrow f64 statistics straight from the assembler's source columns (int32 / f32 / f64 /
    bool / int64 mixed, one [2, n] vector part): equal to the stats of the packed f64 matrix."""
    g = torch.Generator(device="cuda").manual_seed(300 + d)
    n = 99_991
    pool = [
        lambda: torch.randint(1, 36, (n,), generator=g, device="cuda", dtype=torch.int32),
        lambda: torch.randn(n, generator=g, device="cuda") * 3,
        lambda: torch.randn(n, generator=g, device="cuda", dtype=torch.float64) + 1,
        lambda: torch.rand(n, generator=g, device="cuda") > 0.5,
        lambda: torch.randint(-9, 9, (n,), generator=g, device="cuda", dtype=torch.int64),
    ]
    parts = [pool[i % len(pool)]() for i in range(d)]
    if d >= 4:  # a vector-valued part: two feature rows of one [2, n] tensor
        parts = parts[:d - 2] + [torch.randn(2, n, generator=g, device="cuda", dtype=torch.float64)]
    X = torch.cat([p.reshape(-1, n).double() for p in parts])
    y = torch.randn(n, generator=g, device="cuda", dtype=torch.float64)
    sel = torch.rand(n, generator=g, device="cuda") > 0.3
    w = torch.rand(n, generator=g, device="cuda", dtype=torch.float64) + 0.5
    for ww, ss in ((None, None), (None, sel), (w, sel)):
        out = device.gram_skinny_cols(parts, y, ww, ss)
        assert _rel(out, _ref_stats(X, y, ww, ss)) < 1e-12


@pytest.mark.parametrize("mode", ["fp32", "fp32split"])
@pytest.mark.parametrize("d", [3, 20, 32, 33, 64])
@pytest.mark.parametrize("n", [1, 65, 77_777])
def test_gram_fp32_mode_exact_f32_kernel(d, n, mode):
    """gramDtype fp32 on f32 features: the exact-f32 MFMA stream kernel (gram_stream.hip) for
    d > 8 — f32 products and 1024-row f32 partial sums flushed to f64; d <= 8 keeps the f64
    skinny kernel.  Scalars (count, Σw, Σy...) stay f64.  fp32split: the same statistics from
    split-bf16 products (x = hi + mid + lo, six bf16 MFMAs per pair) at the same tolerance."""
    g = torch.Generator(device="cuda").manual_seed(90 + d + n)
    X = torch.randn(d, n, generator=g, device="cuda") + 0.3
    y = torch.randn(n, generator=g, device="cuda") * 2
    out = device.gram_stats(X, y, None, None, mode)
    ref = _ref_stats(X.double(), y.double(), None, None)
    assert _rel(out[:5], ref[:5]) < 1e-12
    assert _rel(out, ref) < (1e-12 if d <= 8 else 2e-6)


@pytest.mark.parametrize("mode", ["fp64", "fp32"])
@pytest.mark.parametrize("d", [17, 32, 40, 64])
def test_gram_stream_selection_weights_tails(mode, d):
    """Stream kernels with selection / weights (f32 and f64 labels and weights), ragged tails and
    unaligned label views; f32 features in both modes, f64 features in fp64 mode."""
    g = torch.Generator(device="cuda").manual_seed(500 + d)
    for n in (63, 64, 65, 4097, 33_333):
        for xdt in ((torch.float32, torch.float64) if mode == "fp64" else (torch.float32,)):
            X = (torch.randn(d, n, generator=g, device="cuda", dtype=torch.float64) + 0.2).to(xdt)
            ybig = torch.randn(n + 1, generator=g, device="cuda", dtype=torch.float64)
            y = ybig[1:]  # 8-byte offset view: re-based before the DMA path
            sel = torch.rand(n, generator=g, device="cuda") > 0.3
            w32 = torch.rand(n, generator=g, device="cuda") + 0.5
            tol = 1e-12 if mode == "fp64" else 5e-6
            for ww, ss in ((None, None), (None, sel), (w32, None), (w32.double(), sel)):
                out = device.gram_stats(X, y, ww, ss, mode)
                ref = _ref_stats(X.double(), y, ww, ss)
                assert _rel(out[:5], ref[:5]) < 1e-12, (n, xdt, ww is None, ss is None)
                assert _rel(out, ref) < tol, (n, xdt, ww is None, ss is None)


def test_gram_fp8_request_tall_uses_bf16_kernel():
    """gramDtype fp8 with d <= 64: served by the bf16 MFMA kernel (HBM-bound either way)."""
    g = torch.Generator(device="cuda").manual_seed(77)
    X = (torch.randn(16, 50_000, generator=g, device="cuda") + 0.2).to(torch.bfloat16)
    y = torch.randn(50_000, generator=g, device="cuda")
    out = device.gram_stats(X, y, None, None, "fp8")
    ref = device.gram_stats(X, y, None, None, "bf16")
    assert torch.equal(out, ref)


def test_gram_deterministic():
    g = torch.Generator(device="cuda").manual_seed(11)
    X = torch.randn(32, 300_000, generator=g, device="cuda").to(torch.bfloat16)
    y = torch.randn(300_000, generator=g, device="cuda")
    a = device.gram_stats(X, y, None, None, "bf16")
    b = device.gram_stats(X, y, None, None, "bf16")
    assert torch.equal(a, b)


@pytest.mark.parametrize("n", [0, 1, 4095, 4096, 100_001])
@pytest.mark.parametrize("limit", [None, 21])
def test_compact_indices(n, limit):
    g = torch.Generator(device="cuda").manual_seed(n + 1)
    sel = torch.rand(n, generator=g, device="cuda") > 0.5
    got = device.compact_indices(sel, limit)
    ref = torch.nonzero(sel.cpu()).flatten()
    if limit is not None:
        ref = ref[:limit]
    assert torch.equal(got.cpu(), ref)


def test_pack_columns():
    a = torch.arange(100, device="cuda", dtype=torch.int32)
    b = torch.randn(100, device="cuda", dtype=torch.float64)
    v = torch.randn(3, 100, device="cuda", dtype=torch.float32)
    for dt in (torch.float64, torch.float32, torch.bfloat16):
        out = device.pack_columns([a, b, v], dt)
        ref = torch.cat([a.unsqueeze(0).to(dt), b.unsqueeze(0).to(dt), v.to(dt)])
        assert out.shape == (5, 100)
        assert torch.equal(out.cpu(), ref.cpu())


def test_predict_and_metrics():
    g = torch.Generator(device="cuda").manual_seed(5)
    d, n = 7, 10_007
    X = torch.randn(d, n, generator=g, device="cuda", dtype=torch.float64)
    y = torch.randn(n, generator=g, device="cuda", dtype=torch.float64)
    sel = torch.rand(n, generator=g, device="cuda") > 0.2
    coef = np.linspace(-1, 1, d)
    p = device.predict(X, coef, 0.25)
    pref = kernels.predict(X.cpu(), coef, 0.25)
    assert _rel(p, pref) < 1e-13
    m = device.regression_metrics(X, y, coef, 0.25, sel, 0.1)
    mref = kernels.regression_metrics(X.cpu(), y.cpu(), coef, 0.25, sel.cpu(), 0.1)
    assert _rel(m, mref) < 1e-12


@pytest.mark.parametrize("d", [1, 7, 32, 33, 64])
@pytest.mark.parametrize("n", [1, 64, 1000, 100_003])
def test_tiled_layout_roundtrip_and_gram(d, n):
    from net.jgp.labs.sparkdq4ml_amd.ops.layout import TiledBF16

    g = torch.Generator(device="cuda").manual_seed(d + 17 * n)
    X = torch.randn(d, n, generator=g, device="cuda").to(torch.bfloat16)
    y = torch.randn(n, generator=g, device="cuda")
    T = device.tile_bf16(X)
    assert isinstance(T, TiledBF16)
    assert torch.equal(T.to_dense(), X)
    idx = torch.tensor([0, n // 2, n - 1], device="cuda")
    assert torch.equal(T.gather_rows(idx), X[:, idx])
    P = device.pack_tiled([X.float()])
    assert torch.equal(P.buf, T.buf)
    a = device.gram_stats(T, y, None, None, "bf16")
    b = device.gram_stats(X, y, None, None, "bf16")
    assert torch.equal(a, b)
    sel = torch.rand(n, generator=g, device="cuda") > 0.4
    c = device.gram_stats(T, y, None, sel, "bf16")
    Z = device.pack_tiled([X.float()], sel)
    e = device.gram_stats(Z, y, None, sel, "bf16", x_zero_dead=True)
    ref = _ref_stats(X.float(), y, None, sel)
    assert _rel(c[5:], ref[5:]) < 2e-5 and _rel(e[5:], ref[5:]) < 2e-5
    coef = np.linspace(-1, 1, d)
    assert _rel(device.predict(T, coef, 0.5), kernels.predict(X.float().cpu(), coef, 0.5)) < 1e-12
    m1 = device.regression_metrics(T, y, coef, 0.5, sel, 0.0)
    m2 = kernels.regression_metrics(X.float().cpu(), y.cpu(), coef, 0.5, sel.cpu(), 0.0)
    assert _rel(m1, m2) < 1e-10


@pytest.mark.parametrize("d", [1, 20, 32, 33, 64])
@pytest.mark.parametrize("n", [63, 4096 + 17, 300_001])
def test_gram_cols_fused_matches_pack_then_gram(d, n):
    # fused VectorAssembler + Gram over source columns == pack_tiled (dead rows zeroed) + tiled Gram
    g = torch.Generator(device="cuda").manual_seed(d * 7 + n)
    cols = [torch.randn(n, generator=g, device="cuda") * (1 + j % 3) for j in range(d)]
    if d > 2:
        cols[1] = cols[1].double()
        cols[2] = (cols[2] * 10).to(torch.int32)
    y = torch.randn(n, generator=g, device="cuda", dtype=torch.float64)
    sel = torch.rand(n, generator=g, device="cuda") > 0.3
    fused = device.gram_cols(cols, y, sel)
    T = device.pack_tiled(cols, sel)
    ref = device.gram_stats(T, y, None, sel, "bf16", x_zero_dead=True)
    assert _rel(fused[:5], ref[:5]) < 1e-12  # f64 scalars; summation order differs
    assert _rel(fused[5:], ref[5:]) < 1e-6
    fused_all = device.gram_cols(cols, y, None)
    ref_all = device.gram_stats(device.pack_tiled(cols, None), y, None, None, "bf16", x_zero_dead=True)
    assert _rel(fused_all, ref_all) < 1e-6


def test_assembler_fit_uses_fused_gram(gpu_session):
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, VectorAssembler, col
    from net.jgp.labs.sparkdq4ml_amd.sql.table import LazyVectorColumn

    n, d = 200_000, 12
    g = torch.Generator(device="cuda").manual_seed(3)
    data = {f"f{j}": torch.randn(n, generator=g, device="cuda") for j in range(d)}
    beta = torch.linspace(-1, 1, d, device="cuda", dtype=torch.float64)
    data["label"] = sum(beta[j] * data[f"f{j}"].double() for j in range(d)) + 2.0
    df = gpu_session.createDataFrame(data).filter(col("f0") > -1.0)
    out = VectorAssembler(inputCols=[f"f{j}" for j in range(d)], outputCol="features",
                          outputDtype="bfloat16").transform(df)
    m = LinearRegression(solver="normal", gramDtype="bf16").fit(out)
    feats = out._table().column("features")
    assert isinstance(feats, LazyVectorColumn) and not feats.materialized  # fit never packed the features
    ref = LinearRegression(solver="normal", gramDtype="bf16").fit(
        gpu_session.createDataFrame({"features": out._table().compact().column("features").dense(),
                                     "label": out._table().compact().column("label").values}))
    np.testing.assert_allclose(m.coefficients.toArray(), ref.coefficients.toArray(), rtol=1e-4, atol=1e-5)
    assert float(m.summary.r2) > 0.999  # summary materializes the features lazily
    assert feats.materialized


@pytest.mark.parametrize("d", [9, 20, 32, 33, 64])
@pytest.mark.parametrize("n", [63, 4096 + 17, 300_001])
def test_gram_cols_stream_all_f32_columns(d, n):
    """All-f32 aligned source columns take the LDS-DMA stream kernel (bf16 MFMA on tiles
    converted from the DMA'd f32, f32-VALU side sums from the unrounded features)."""
    g = torch.Generator(device="cuda").manual_seed(d * 11 + n)
    X = torch.randn(d, n, generator=g, device="cuda") + 0.5
    cols = [X[j].clone() for j in range(d)]  # separate (16-B aligned) allocations
    y = torch.randn(n, generator=g, device="cuda")
    for sel in (None, torch.rand(n, generator=g, device="cuda") > 0.3):
        out = device.gram_cols(cols, y, sel)
        exact = _ref_stats(X.double(), y, None, sel)
        rounded = _ref_stats(X.to(torch.bfloat16).double(), y, None, sel)
        assert _rel(out[:5], exact[:5]) < 1e-12
        assert _rel(out[5:5 + 2 * d], exact[5:5 + 2 * d]) < 2e-6
        assert _rel(out[5 + 2 * d:], rounded[5 + 2 * d:]) < 2e-5
    # the bf16 request on an assembled f32 matrix rides the same kernel
    out = device.gram_stats(X, y, None, None, "bf16")
    assert _rel(out[5 + 2 * d:], _ref_stats(X.to(torch.bfloat16).double(), y, None, None)[5 + 2 * d:]) < 2e-5


@pytest.mark.parametrize("d", [9, 33, 64])
@pytest.mark.parametrize("xdt", [torch.float64, torch.float32])
def test_gram_stream_cols_f64_and_f32_statistics(d, xdt):
    """fp64 / fp32 statistics straight from same-dtype source columns (weights, selection)."""
    g = torch.Generator(device="cuda").manual_seed(d + 700)
    n = 70_001
    X = (torch.randn(d, n, generator=g, device="cuda", dtype=torch.float64) + 0.1).to(xdt)
    cols = [X[j].clone() for j in range(d)]
    y = torch.randn(n, generator=g, device="cuda", dtype=torch.float64)
    sel = torch.rand(n, generator=g, device="cuda") > 0.2
    w = torch.rand(n, generator=g, device="cuda", dtype=torch.float64) + 0.5
    for ww, ss in ((None, None), (w, sel)):
        out = device.gram_stream_cols(cols, y, ww, ss, "fp64")
        assert _rel(out, _ref_stats(X.double(), y, ww, ss)) < 1e-12
        if xdt == torch.float32:
            out = device.gram_stream_cols(cols, y, ww, ss, "fp32")
            assert _rel(out, _ref_stats(X.double(), y, ww, ss)) < 5e-6
    mixed = cols[:-1] + [cols[-1].to(torch.float64 if xdt == torch.float32 else torch.float32)]
    assert device.gram_stream_cols(mixed, y, None, None, "fp64") is None


def test_assembled_f64_fit_reads_source_columns(gpu_session):
    """VectorAssembler (default float64 output) + fp64 / bf16 fit over 40 f32 columns: the
    statistics come from the source columns (no pack kernel), same model as the packed path."""
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, VectorAssembler
    from net.jgp.labs.sparkdq4ml_amd.sql.table import LazyVectorColumn

    g = torch.Generator(device="cuda").manual_seed(5)
    n, d = 50_000, 40
    X = torch.randn(d, n, generator=g, device="cuda")
    beta = torch.linspace(-1, 1, d, device="cuda")
    y = beta @ X + 0.25
    names = [f"c{i}" for i in range(d)]
    data = {nm: X[i].clone() for i, nm in enumerate(names)}
    data["label"] = y
    df = VectorAssembler().setInputCols(names).setOutputCol("features").transform(gpu_session.createDataFrame(data))
    for gd, tol in (("fp64", 1e-9), ("fp32", 1e-5), ("bf16", 3e-2)):
        m = LinearRegression(solver="normal", gramDtype=gd).fit(df)
        np.testing.assert_allclose(m.coefficients.toArray(), beta.double().cpu().numpy(), atol=tol)
    from net.jgp.labs.sparkdq4ml_amd.sql.plan import execute

    col = execute(df._plan, gpu_session).column("features")
    assert isinstance(col, LazyVectorColumn) and not col.materialized
