"""In-kernel slab fold of the tall bf16 Gram and the fused assembler Gram (``slab_fold_tail`` in
ops/csrc/hip/gram.hip): the last block of each XCD group folds its group, the last group writes the
packed statistics.  Checked against the separate ``gram_reduce`` kernel (same slabs, different
fixed summation order: 1e-13) and for run-to-run bitwise equality, across grid sizes that leave
groups of unequal size and fewer blocks than groups, on two streams."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from net.jgp.labs.sparkdq4ml_amd.ops import device, native  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _hip():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    native.hip()


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-300))


def _with_fold(mode, fn, monkeypatch):
    monkeypatch.setenv("DQ4ML_GRAM_FOLD", mode)
    out = fn()
    torch.cuda.synchronize()
    return out.clone()


@pytest.mark.parametrize("d", [3, 32, 64])
@pytest.mark.parametrize("blocks", [1, 5, 8, 13, 256])
@pytest.mark.parametrize("sel", [False, True])
def test_tiled_gram_in_kernel_fold(d, blocks, sel, monkeypatch):
    n = 200_003
    g = torch.Generator(device="cuda").manual_seed(d * 31 + blocks)
    X = torch.randn(d, n, generator=g, device="cuda") + 0.3
    y = torch.randn(n, generator=g, device="cuda") * 2 + 1
    s = (torch.rand(n, generator=g, device="cuda") > 0.3) if sel else None
    T = device.tile_bf16(X)

    def run():
        return device.gram_stats(T, y, None, s, "bf16", blocks=blocks)

    sep = _with_fold("separate", run, monkeypatch)
    k1 = _with_fold("kernel", run, monkeypatch)
    k2 = _with_fold("kernel", run, monkeypatch)
    assert torch.equal(k1, k2)  # fixed fold order: bitwise run to run
    assert _rel(k1, sep) < 1e-13
    assert float(k1[0]) == float(s.sum() if sel else n)  # row count exact


def test_fold_counters_reset_across_streams_and_launches(monkeypatch):
    monkeypatch.setenv("DQ4ML_GRAM_FOLD", "kernel")
    d, n = 32, 100_000
    X = torch.randn(d, n, device="cuda")
    y = torch.randn(n, device="cuda")
    T = device.tile_bf16(X)
    ref = device.gram_stats(T, y, None, None, "bf16", blocks=19)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    outs = []
    with torch.cuda.stream(side):
        for _ in range(5):
            outs.append(device.gram_stats(T, y, None, None, "bf16", blocks=19))
    for _ in range(5):
        outs.append(device.gram_stats(T, y, None, None, "bf16", blocks=19))
    torch.cuda.synchronize()
    for o in outs:
        assert torch.equal(o, ref)
    for t in device._tickets.values():
        assert int(t.abs().sum()) == 0  # every launch leaves its stream's counters zeroed


@pytest.mark.parametrize("d", [9, 40])
def test_gram_cols_in_kernel_fold(d, monkeypatch):
    n = 150_001
    g = torch.Generator(device="cuda").manual_seed(d)
    cols = [torch.randn(n, generator=g, device="cuda") for _ in range(d)]
    cols[1] = cols[1].double()  # mixed source dtypes: the fused assembler Gram kernel, not the stream path
    y = torch.randn(n, generator=g, device="cuda", dtype=torch.float64)
    sel = torch.rand(n, generator=g, device="cuda") > 0.5

    def run():
        return device.gram_cols(cols, y, sel)

    sep = _with_fold("separate", run, monkeypatch)
    k1 = _with_fold("kernel", run, monkeypatch)
    k2 = _with_fold("kernel", run, monkeypatch)
    assert torch.equal(k1, k2)
    assert _rel(k1, sep) < 1e-13
    assert np.isclose(float(k1[0]), float(sel.sum()))
