"""Wide (d > 64) path: fragment-ordered bf16 / fp8 storage + LDS-tiled MFMA SYRK (K5-wide,
csrc/hip/gram_wide.hip) against plain PyTorch fp64 references of the same (quantized) data."""
import numpy as np
import pytest
import torch

from net.jgp.labs.sparkdq4ml_amd.ops import layout


@pytest.mark.parametrize("eb", [16, 8])
def test_wide_offsets_is_a_bijection(eb):
    # host-only: every (feature, row) of a padded 2-panel, 3-superstep image maps to a distinct slot
    d, n = 300, 192
    nt = ((d + 255) // 256) * 8
    f = torch.arange(nt * 32).unsqueeze(1)
    r = torch.arange(n).unsqueeze(0)
    off = layout.wide_offsets(f, r, d, eb).reshape(-1)
    assert off.numel() == nt * 32 * n
    assert torch.unique(off).numel() == off.numel()
    assert int(off.min()) == 0 and int(off.max()) == nt * 32 * n - 1
    # one superstep (64 rows) of one 32-feature tile is one contiguous 2048-element chunk
    o = layout.wide_offsets(torch.arange(32).unsqueeze(1), torch.arange(64).unsqueeze(0), d, eb)
    assert sorted(o.reshape(-1).tolist()) == list(range(2048))
    if eb == 8:  # a lane's 32 bytes: rows {16 ki + 8 h + j} of one feature, halves 1 KiB apart
        rows = torch.tensor([r for r in range(64) if not (r >> 3) & 1]).unsqueeze(0)  # lane-half 0
        o = layout.wide_offsets(torch.tensor([[5]]), rows, d, eb).reshape(-1)
        lane0 = [int(x) for x in o if int(x) < 1024]
        assert sorted(lane0) == list(range(5 * 16, 5 * 16 + 16))


gpu = pytest.mark.gpu


def _hip():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from net.jgp.labs.sparkdq4ml_amd.ops import native

    return native.hip()


def _oracle(Xd, y, sel):
    from net.jgp.labs.sparkdq4ml_amd.ops import kernels

    return kernels.gram_stats(Xd.double().cpu(), y.double().cpu(), None, None if sel is None else sel.cpu(), "fp64")


def _parts(out, d):
    out = out.double().cpu()
    return out[:5], out[5:5 + d], out[5 + d:5 + 2 * d], out[5 + 2 * d:]


def _rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-300))


@gpu
@pytest.mark.parametrize("d", [65, 300, 600])
@pytest.mark.parametrize("n", [77, 5000, 70_001])
def test_wide_bf16_gram_matches_oracle(d, n):
    _hip()
    from net.jgp.labs.sparkdq4ml_amd.ops import device

    g = torch.Generator(device="cuda").manual_seed(d + n)
    X = (torch.randn(d, n, generator=g, device="cuda") + 0.3).to(torch.bfloat16)
    y = torch.randn(n, generator=g, device="cuda", dtype=torch.float64) * 2 + 1
    sel = torch.rand(n, generator=g, device="cuda") > 0.25
    T = device.pack_wide([X], 16, sel)
    assert torch.equal(T.to_dense().float(), torch.where(sel, X.float(), torch.zeros_like(X.float())))
    out = device.gram_stats(T, y, None, sel, "bf16", x_zero_dead=True)
    ref = _oracle(X.float(), y, sel)
    s, a, ab, aa = _parts(out, d)
    rs, ra, rab, raa = _parts(ref, d)
    assert s[0] == rs[0] and s[1] == rs[1]
    assert _rel(s[3:], rs[3:]) < 1e-4  # y = bf16 hi + bf16 lo
    assert _rel(a, ra) < 1e-5
    assert _rel(ab, rab) < 1e-4
    assert _rel(aa, raa) < 1e-5


@gpu
@pytest.mark.parametrize("d", [100, 513])
def test_wide_fp8_gram_matches_dequantized_oracle(d):
    _hip()
    from net.jgp.labs.sparkdq4ml_amd.ops import device

    n = 40_000
    g = torch.Generator(device="cuda").manual_seed(d)
    X = torch.randn(d, n, generator=g, device="cuda") * torch.linspace(0.1, 5.0, d, device="cuda").unsqueeze(1)
    y = torch.randn(n, generator=g, device="cuda", dtype=torch.float64) * 4 - 2
    T = device.pack_wide([X], 8, None)
    assert T.eb == 8 and T.scales.shape == (d,)
    Xq = T.to_dense()  # dequantized fp8
    assert _rel(Xq.double().cpu(), X.double().cpu()) < 0.07
    out = device.gram_stats(T, y, None, None, "fp8", x_zero_dead=True)
    ref = _oracle(Xq, y, None)
    s, a, ab, aa = _parts(out, d)
    rs, ra, rab, raa = _parts(ref, d)
    assert s[0] == n
    assert _rel(s[3:], rs[3:]) < 1e-2  # y = fp8 hi + fp8 lo (~2^-8 relative)
    assert _rel(a, ra) < 1e-5
    assert _rel(ab, rab) < 1e-2
    assert _rel(aa, raa) < 1e-5  # fp8 x fp8 products exact, f32 accumulation


@gpu
@pytest.mark.parametrize("eb", [16, 8])
def test_wide_predict_and_metrics(eb):
    _hip()
    from net.jgp.labs.sparkdq4ml_amd.ops import device

    d, n = 130, 9999
    g = torch.Generator(device="cuda").manual_seed(eb)
    X = torch.randn(d, n, generator=g, device="cuda")
    T = device.pack_wide([X], eb, None)
    Xd = T.to_dense().double()
    coef = np.random.default_rng(eb).normal(size=d)
    p = device.predict(T, coef, 0.5)
    ref = torch.as_tensor(coef, device="cuda") @ Xd + 0.5
    assert _rel(p, ref) < 1e-5
    y = ref + 0.1
    m = device.regression_metrics(T, y, coef, 0.5, None, 0.0)
    assert float(m[0]) == n
    assert abs(float(m[3]) - 0.1 * n) < 1e-3 * n


@gpu
def test_wide_linear_regression_end_to_end(gpu_session):
    _hip()
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression

    d, n = 200, 60_000
    g = torch.Generator(device="cuda").manual_seed(11)
    X = torch.randn(d, n, generator=g, device="cuda").to(torch.bfloat16)
    beta = torch.linspace(-1, 1, d, device="cuda", dtype=torch.float64)
    y = beta @ X.double() + 3.0 + 0.01 * torch.randn(n, generator=g, device="cuda", dtype=torch.float64)
    df = gpu_session.createDataFrame({"features": X, "label": y})
    lr = LinearRegression(maxIter=1, regParam=0.0, solver="normal", gramDtype="bf16")
    m = lr.fit(df)
    coef = np.asarray(m.coefficients.toArray())
    assert np.abs(coef - beta.cpu().numpy()).max() < 5e-3
    assert abs(m.intercept - 3.0) < 5e-3
    assert m.summary.r2 > 0.999


@gpu
def test_assembler_fp8_wide_fit(gpu_session):
    _hip()
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, VectorAssembler

    d, n = 80, 30_000
    g = torch.Generator(device="cuda").manual_seed(5)
    cols = {f"f{i}": torch.rand(n, generator=g, device="cuda", dtype=torch.float64) * 4 - 2 for i in range(d)}
    beta = np.linspace(0.5, 1.5, d)
    y = sum(float(beta[i]) * cols[f"f{i}"] for i in range(d)) + 1.0
    cols["label"] = y
    df = gpu_session.createDataFrame(cols)
    va = VectorAssembler(inputCols=[f"f{i}" for i in range(d)], outputCol="features", outputDtype="float8")
    m = LinearRegression(maxIter=1, regParam=0.0, solver="normal", gramDtype="fp8").fit(va.transform(df))
    # fp8 features: coefficients within a few % (quantization noise acts like errors-in-variables)
    assert np.abs(np.asarray(m.coefficients.toArray()) - beta).max() < 0.15
    assert m.summary.r2 > 0.95


@gpu
@pytest.mark.parametrize("wide", [False, True])
def test_pack_mixed_dtypes_and_misaligned_columns(wide):
    # f64 / f32 / bf16 / int32 columns, some starting at a non-16-byte-aligned offset (scalar path)
    _hip()
    from net.jgp.labs.sparkdq4ml_amd.ops import device

    n = 10_007
    g = torch.Generator(device="cuda").manual_seed(9)
    base = torch.randn(4, n + 3, generator=g, device="cuda", dtype=torch.float64)
    cols = [base[0, :n], base[1, 3:].float(), base[2, 1:n + 1].to(torch.bfloat16)[0:],
            (base[3, :n] * 10).to(torch.int32), base[1, 1:n + 1]]  # last: f64 view at +8 bytes
    cols = cols * (20 if wide else 4)  # d = 100 (wide) / 20 (tall)
    sel = torch.rand(n, generator=g, device="cuda") > 0.3
    dense = torch.stack([c.float() for c in cols]) * sel
    T = device.pack_wide(cols, 16, sel) if wide else device.pack_tiled(cols, sel)
    assert torch.equal(T.to_dense().float(), dense.to(torch.bfloat16).float())


@gpu
@pytest.mark.parametrize("eb", [16, 8])
@pytest.mark.parametrize("sched", ["gang", "gang3", "gangc", "gangc3", "queue", "grid"])
@pytest.mark.parametrize("d", [300, 1100])
def test_wide_schedules_match_oracle(eb, sched, d, monkeypatch):
    # every SYRK schedule (the gang's merged diagonal + augmentation units included) gives the
    # same statistics as the fp64 oracle of the stored (quantized) values.  gang3 at d = 1100: 15
    # units x 3 row ranges = 45 units over 32 blocks per group -- a partial last round, which the
    # round barrier must skip (its blocks would wait for arrivals that never come).  gangc: the
    # classic unit list (what long row ranges run), forced at this size
    _hip()
    from net.jgp.labs.sparkdq4ml_amd.ops import device

    monkeypatch.setenv("DQ4ML_WIDE_SCHED", sched[:4] if sched.startswith("gang") else sched)
    monkeypatch.setenv("DQ4ML_WIDE_GANG_S", "3" if sched.endswith("3") else "2")
    if sched.startswith("gangc"):
        monkeypatch.setattr(device, "_LONG_UNIT_MAX_SUP", -1)
    monkeypatch.setenv("DQ4ML_WIDE_H", "1")
    n = 70_001
    g = torch.Generator(device="cuda").manual_seed(d + eb)
    X = torch.randn(d, n, generator=g, device="cuda") + 0.2
    y = torch.randn(n, generator=g, device="cuda", dtype=torch.float64) * 3 + 1
    sel = torch.rand(n, generator=g, device="cuda") > 0.2
    T = device.pack_wide([X.to(torch.bfloat16) if eb == 16 else X], eb, sel)
    out = device.gram_stats(T, y, None, sel, "bf16" if eb == 16 else "fp8", x_zero_dead=True)
    Xq = T.to_dense().double()
    live = sel.double()
    s, a, ab, aa = _parts(out, d)
    assert s[0] == float(sel.sum())
    ref_a = (Xq * live).sum(1).cpu()
    assert _rel(a, ref_a) < 1e-5
    assert _rel(ab, (Xq * (y * live)).sum(1).cpu()) < (1e-4 if eb == 16 else 1e-2)
    G = (Xq * live) @ Xq.T
    ii, jj = torch.triu_indices(d, d, device="cuda")  # packed upper: (i, j), i <= j at j(j+1)/2 + i
    ref = torch.empty(d * (d + 1) // 2, dtype=torch.float64, device="cuda")
    ref[jj * (jj + 1) // 2 + ii] = G[ii, jj]
    assert _rel(aa, ref.cpu()) < 1e-5


@gpu
@pytest.mark.parametrize("eb", [16, 8])
def test_wide_gang_long_units_match_oracle(eb, monkeypatch):
    # d = 2100: 36 off-diagonal panel pairs >= the 32 blocks of a group, so 32 of them run as LONG
    # units (all S row ranges in one K loop, one partial tile per group) beside short ones
    _hip()
    from net.jgp.labs.sparkdq4ml_amd.ops import device

    monkeypatch.setenv("DQ4ML_WIDE_GANG_S", "3")
    d, n = 2100, 50_003
    rows, units, base, tiles = device._gang_table((d + 255) // 256, 3, device._wide_grid(device.native.hip()) // 8)
    assert any((r[2] >> 16) == 3 for r in rows) and any((r[2] >> 16) == 1 for r in rows)
    g = torch.Generator(device="cuda").manual_seed(eb)
    X = torch.randn(d, n, generator=g, device="cuda") - 0.1
    y = torch.randn(n, generator=g, device="cuda", dtype=torch.float64) + 2
    T = device.pack_wide([X.to(torch.bfloat16) if eb == 16 else X], eb, None)
    out = device.gram_stats(T, y, None, None, "bf16" if eb == 16 else "fp8", x_zero_dead=True)
    Xq = T.to_dense().double()
    s, a, ab, aa = _parts(out, d)
    assert s[0] == n
    assert _rel(a, Xq.sum(1).cpu()) < 1e-5
    G = Xq @ Xq.T
    ii, jj = torch.triu_indices(d, d, device="cuda")
    ref = torch.empty(d * (d + 1) // 2, dtype=torch.float64, device="cuda")
    ref[jj * (jj + 1) // 2 + ii] = G[ii, jj]
    # a long unit's f32 MFMA accumulators sum all S ranges of its group (3 x 2 084 rows here):
    # f32 rounding of the longer chains, ~1e-5 relative (the fp8 inputs' own quantization is ~1e-2)
    assert _rel(aa, ref.cpu()) < 5e-5


@gpu
def test_wide_gang_full_width_matches_queue():
    # BASELINE config-5 width (P = 16 panels: S = 4, 17 equal units per block of the gang)
    _hip()
    import os

    from net.jgp.labs.sparkdq4ml_amd.ops import device

    d, n = 4096, 40_000
    g = torch.Generator(device="cuda").manual_seed(5)
    X = torch.randn(d, n, generator=g, device="cuda")
    y = torch.randn(n, generator=g, device="cuda", dtype=torch.float64)
    T = device.pack_wide([X], 8, None)
    outs = {}
    for sched in ("gang", "queue"):
        os.environ["DQ4ML_WIDE_SCHED"] = sched
        try:
            outs[sched] = device.gram_stats(T, y, None, None, "fp8", x_zero_dead=True)
        finally:
            os.environ.pop("DQ4ML_WIDE_SCHED", None)
    assert _rel(outs["gang"], outs["queue"]) < 1e-6
    Xq = T.to_dense().double()
    G = Xq @ Xq.T
    dg = outs["gang"][5 + 2 * d:]
    j = torch.arange(d, device="cuda")
    assert _rel(dg[j * (j + 1) // 2 + j].cpu(), G.diagonal().cpu()) < 5e-5  # f32 sums of 1250-row splits
    assert _rel(dg[j * (j + 1) // 2].cpu(), G[0].cpu()) < 5e-5
