"""The per-column shift of the low-precision Gram paths (ops/shift.py) on the host:
off-centre columns are shifted by their mean, centred ones are not, and an integral column (the
lab's guest count) gets an integer shift so that x - s stays exactly representable."""
import numpy as np
import torch

from net.jgp.labs.sparkdq4ml_amd.ops import shift as shiftmod


def test_shift_decisions_and_integral_columns():
    g = torch.Generator().manual_seed(3)
    n = 20_000
    x = torch.randn(4, n, generator=g, dtype=torch.float64)
    x[1] += 1000.0                                              # off centre, fractional
    x[2] = torch.randint(1, 36, (n,), generator=g).double()      # integral, |mean| > std
    x[3] = x[3] * 0.1                                            # centred
    s = shiftmod.column_shift([x])
    assert s is not None
    h = s.host
    assert h[0] == 0.0 and h[3] == 0.0
    assert abs(h[1] - 1000.0) < 0.05 and h[1] != round(h[1])
    assert h[2] == round(h[2]) and abs(h[2] - float(x[2].mean())) <= 0.5
    ints = torch.randint(1, 36, (n,), generator=g, dtype=torch.int32)
    si = shiftmod.column_shift([ints])
    assert si is not None and si.host[0] == round(si.host[0])
    # x - s of an integral column is exact in bf16 while |x - s| <= 256
    xs = (ints.double() - si.host[0]).to(torch.bfloat16).double()
    assert torch.equal(xs, ints.double() - si.host[0])


def test_small_inputs_are_not_shifted():
    assert shiftmod.column_shift([torch.full((100,), 500.0)]) is None
    assert np.isfinite(shiftmod.CENTER_RATIO)
