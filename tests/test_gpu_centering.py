"""Centred low-precision statistics: every bf16 / fp8 / exact-f32 /
split-f32 Gram path subtracts a per-column shift before it rounds (ops/shift.py) and un-shifts the
statistics in f64 (gram.h ``stats_unshift``).  Columns far off centre -- ``1000 + N(0, 1)`` and a
price-like ``U(20, 200)`` -- must give the covariances and the fitted coefficients of the fp64
oracle (Spark fits in f64, ``DataQuality4MachineLearningApp.java:126``), and the same data WITHOUT
the shift must be measurably worse (the test would fail on the round-3 code)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from net.jgp.labs.sparkdq4ml_amd.ops import device, kernels, native  # noqa: E402
from net.jgp.labs.sparkdq4ml_amd.ops import shift as shiftmod  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _hip():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    native.hip()


def _data(d, n, seed, sel_frac=0.0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    X = torch.randn(d, n, generator=g, device="cuda")
    X[0::3] += 1000.0                                                     # |mean| / std = 1000
    X[1::3] = torch.rand(len(range(1, d, 3)), n, generator=g, device="cuda") * 180.0 + 20.0  # price-like
    X[2::3] = X[2::3] * 0.5 + 10.0                                         # 10 +- 0.5
    beta = torch.linspace(-1.0, 1.0, d, device="cuda", dtype=torch.float64)
    y = (beta @ X.double()) + 3.0 + 0.1 * torch.randn(n, generator=g, device="cuda", dtype=torch.float64)
    sel = (torch.rand(n, generator=g, device="cuda") >= sel_frac) if sel_frac else None
    return X, y, sel, beta


def _cov(flat, d):
    f = flat.double().cpu()
    W = f[1]
    a, ab, aa = f[5:5 + d] / W, f[5 + d:5 + 2 * d] / W, f[5 + 2 * d:] / W
    ybar = f[3] / W
    i, j = torch.triu_indices(d, d)
    C = torch.empty(d, d, dtype=torch.float64)
    C[i, j] = aa[j * (j + 1) // 2 + i]
    C[j, i] = C[i, j]
    C -= torch.outer(a, a)
    cxy = ab - a * ybar
    vy = f[4] / W - ybar * ybar
    return C, cxy, vy


def _err(flat, ref, d):
    """Largest covariance error on the correlation scale: |ΔC_ij| / (σ_i σ_j), |ΔC_iy| / (σ_i σ_y)."""
    C, cxy, _ = _cov(flat, d)
    Cr, cr, vy = _cov(ref, d)
    s = torch.sqrt(torch.diagonal(Cr))
    ec = float(((C - Cr).abs() / torch.outer(s, s)).max())
    ey = float(((cxy - cr).abs() / (s * float(vy) ** 0.5)).max())
    return max(ec, ey)


def _oracle(X, y, sel):
    return kernels.gram_stats(X.double().cpu(), y.cpu(), None, None if sel is None else sel.cpu(), "fp64")


def test_column_shift_decisions():
    n = 100_000
    g = torch.Generator(device="cuda").manual_seed(1)
    centred = torch.randn(3, n, generator=g, device="cuda")
    assert shiftmod.column_shift([centred]) is None
    off = centred.clone()
    off[1] += 500.0
    s = shiftmod.column_shift([off])
    assert s is not None and s.host[0] == 0.0 and s.host[2] == 0.0 and abs(s.host[1] - 500.0) < 0.05
    assert shiftmod.column_shift([off]) is s  # memoized per live source tensor
    b = shiftmod.column_shift([off.to(torch.bfloat16)])
    assert float(torch.tensor(b.host[1]).to(torch.bfloat16).double()) == b.host[1]  # bf16-exact shift


@pytest.mark.parametrize("path", ["tile", "pack_sel", "cols", "stream_bf16", "dense_f32_bf16"])
def test_bf16_statistics_of_off_centre_columns(path, monkeypatch):
    d, n = 24, 300_017
    X, y, sel, _ = _data(d, n, 7, sel_frac=0.3 if path == "pack_sel" else 0.0)
    ref = _oracle(X, y, sel)

    def run():
        if path == "tile":
            return device.gram_stats(device.tile_bf16(X), y, None, None, "bf16")
        if path == "pack_sel":
            return device.gram_stats(device.pack_tiled([X], sel), y, None, sel, "bf16", x_zero_dead=True)
        cols = [X[i].clone() for i in range(d)]
        if path == "cols":
            cols[0] = cols[0].double()  # mixed dtypes: the fused assembler kernel (gram_cols_kernel)
            return device.gram_cols(cols, y, None)
        if path == "stream_bf16":
            return device.gram_stream_cols(cols, y, None, None, "bf16")
        return device.gram_stats(X, y, None, None, "bf16")

    e_shift = _err(run(), ref, d)
    assert e_shift < 1e-2, e_shift
    monkeypatch.setattr(device, "column_shift", lambda *a, **k: None)
    e_raw = _err(run(), ref, d)
    assert e_raw > 10 * e_shift, (e_raw, e_shift)  # what the round-3 code computed


@pytest.mark.parametrize("compute", ["fp32", "fp32split"])
def test_f32_statistics_of_off_centre_columns(compute, monkeypatch):
    d, n = 40, 400_001
    X, y, sel, _ = _data(d, n, 11, sel_frac=0.2)
    ref = _oracle(X, y, sel)
    cols = [X[i].clone() for i in range(d)]
    e_shift = _err(device.gram_stream_cols(cols, y, None, sel, compute), ref, d)
    assert e_shift < 1e-5, e_shift
    monkeypatch.setattr(device, "column_shift", lambda *a, **k: None)
    e_raw = _err(device.gram_stream_cols(cols, y, None, sel, compute), ref, d)
    assert e_raw > 10 * e_shift, (e_raw, e_shift)


@pytest.mark.parametrize("eb", [16, 8])
def test_wide_statistics_of_off_centre_columns(eb):
    d, n = 130, 120_001
    X, y, sel, _ = _data(d, n, 5, sel_frac=0.25)
    ref = _oracle(X, y, sel)
    T = device.pack_wide([X], eb, sel)
    assert T.shift is not None and T.shift.uniform
    e_shift = _err(device.gram_stats(T, y, None, sel, "bf16" if eb == 16 else "fp8", x_zero_dead=True), ref, d)
    T0 = device.pack_wide([X], eb, sel, shift=None)
    e_raw = _err(device.gram_stats(T0, y, None, sel, "bf16" if eb == 16 else "fp8", x_zero_dead=True), ref, d)
    assert e_shift < (1e-2 if eb == 16 else 6e-2), e_shift
    assert e_raw > 5 * e_shift, (e_raw, e_shift)


def test_shifted_tiles_round_trip_and_predict():
    d, n = 20, 50_003
    X, y, _, beta = _data(d, n, 3)
    T = device.tile_bf16(X)
    assert T.shift is not None
    dense = T.to_dense()
    assert dense.dtype == torch.float32
    s = T.shift.dev.unsqueeze(1)
    # bf16 keeps 2^-8 of |x - s| (not of |x|); + the f32 rounding of x' + s
    assert float(((dense - X).abs() - (X - s).abs() * 2.0 ** -8 - 1e-4).max()) <= 0.0
    coef = beta.cpu().numpy()
    p = device.predict(T, coef, 3.0)
    ref = (beta @ dense.double()) + 3.0
    # (the reference reads x' + s rounded to f32: 2^-24 of |x| ~ 1000 per term)
    assert float((p - ref).abs().max() / ref.abs().max()) < 1e-7


@pytest.mark.parametrize("dt,d", [("bfloat16", 24), ("float8", 96)])
def test_assembled_fit_of_off_centre_columns_matches_fp64(dt, d):
    # the DataFrame path: VectorAssembler(outputDtype) -> LinearRegression(gramDtype) on columns
    # 1000 + N(0,1), U(20, 200), 10 +- 0.5; coefficients vs the fp64 fit of the same table
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, SparkSession, VectorAssembler

    n = 200_003
    X, y, _, beta = _data(d, n, 21)
    spark = SparkSession.builder().appName("centering").master("mi355x[1]").getOrCreate()
    cols = {f"f{i}": X[i].clone() for i in range(d)}
    cols["label"] = y
    df = spark.createDataFrame(cols)
    names = [f"f{i}" for i in range(d)]
    fits = {}
    for odt, gd in (("float64", "fp64"), (dt, "bf16" if dt == "bfloat16" else "fp8")):
        va = VectorAssembler(inputCols=names, outputCol="features", outputDtype=odt)
        lr = LinearRegression(solver="normal", regParam=0.0, gramDtype=gd)
        m = lr.fit(va.transform(df))
        fits[gd] = (np.asarray(m.coefficients.toArray()), m.intercept)
    c64, c = fits["fp64"][0], fits["bf16" if dt == "bfloat16" else "fp8"][0]
    rel = np.abs(c - c64).max() / np.abs(c64).max()
    # fp8 bound: e4m3 keeps 3 mantissa bits; quantizing the centred columns of this table alone (CPU
    # simulation, torch.float8_e4m3fn, lstsq in f64) moves the worst coefficient by 4.4 % of max |coef|
    assert rel < (1e-2 if dt == "bfloat16" else 1e-1), rel
    assert np.abs(c64 - beta.cpu().numpy()).max() < 1e-2  # the fp64 fit itself recovers beta
