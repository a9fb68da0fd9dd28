"""The device Huber path's feature moments (``models/huber.py _device_moments``: torch ops on the
all-reduced statistics, so the fit reads nothing back) equal the host path's ``_sample_moments``
bit for bit, and its L2 weights follow Spark's standardization rule (CPU tensors: the same
elementwise expressions run on the GPU)."""
import numpy as np
import pytest
import torch

from net.jgp.labs.sparkdq4ml_amd.models.huber import _device_moments
from net.jgp.labs.sparkdq4ml_amd.models.lbfgs_path import _sample_moments
from net.jgp.labs.sparkdq4ml_amd.models.optim import GramStats
from net.jgp.labs.sparkdq4ml_amd.ops import kernels


@pytest.mark.parametrize("std", [True, False])
@pytest.mark.parametrize("weighted", [False, True])
def test_device_moments_match_host(std, weighted):
    g = torch.Generator().manual_seed(5)
    d, n = 7, 501
    X = torch.randn(d, n, generator=g, dtype=torch.float64) * torch.linspace(0.5, 3.0, d, dtype=torch.float64)[:, None]
    X[3] = 0.0  # a constant (all-zero) feature: std exactly 0, no L2 weight when unstandardized
    y = torch.randn(n, generator=g, dtype=torch.float64)
    w = (0.2 + torch.rand(n, generator=g, dtype=torch.float64)) if weighted else None
    flat = kernels.gram_stats(X, y, w, None, "fp64")
    sx_h = _sample_moments(GramStats.from_flat(flat.numpy(), d))[1]
    reg = 0.3
    sx, lam = _device_moments(flat, d, reg, std)
    assert np.array_equal(sx.numpy(), sx_h)
    safe = np.where(sx_h == 0.0, 1.0, sx_h)
    lam_h = np.full(d, reg) if std else np.where(sx_h != 0.0, reg / (safe * safe), 0.0)
    assert np.array_equal(lam.numpy(), lam_h)
    assert sx_h[3] == 0.0 and (lam.numpy()[3] == (reg if std else 0.0))
