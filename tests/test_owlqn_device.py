"""The device-resident OWLQN (``models/owlqn_device.py``) against the native host driver
(``csrc/host/solvers.cpp``): same Breeze algorithm, so the same solution and the same
objectiveHistory up to floating-point summation order.  Runs on CPU tensors here; the HIP
one-workgroup version is checked against both in ``test_gpu_owlqn.py``."""
import numpy as np
import pytest
import torch

from net.jgp.labs.sparkdq4ml_amd.models.owlqn_device import solve_owlqn_device
from net.jgp.labs.sparkdq4ml_amd.ops import native


def _flat(nf, n, seed, w=False):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, nf)) * rng.uniform(0.5, 3.0, nf) + rng.uniform(-2, 2, nf)
    beta = rng.standard_normal(nf) * (rng.random(nf) > 0.4)
    y = X @ beta + 1.5 + 0.3 * rng.standard_normal(n)
    wv = rng.uniform(0.2, 2.0, n) if w else np.ones(n)
    iu = np.triu_indices(nf)
    order = np.argsort(iu[0] + iu[1] * (iu[1] + 1) // 2)
    G = (X * wv[:, None]).T @ X
    packed = G[iu[0], iu[1]][order]
    head = [n, wv.sum(), (wv * wv).sum(), (wv * y).sum(), (wv * y * y).sum()]
    return np.concatenate([head, X.T @ wv, X.T @ (wv * y), packed])


@pytest.mark.parametrize("nf,reg,enet,icpt,stdf", [(1, 1.0, 1.0, True, True), (5, 0.1, 1.0, True, True),
                                                  (30, 0.05, 0.5, True, False), (12, 0.3, 0.8, False, True),
                                                  (80, 0.02, 1.0, True, True)])
def test_torch_owlqn_matches_native(nf, reg, enet, icpt, stdf):
    flat = _flat(nf, 4000, nf, w=nf % 2 == 0)
    h = native.host()
    r = h.wls_fit(flat, nf, icpt, reg, enet, stdf, True, 0, 100, 1e-6, False)
    assert r["solver"] == "owlqn"
    out = solve_owlqn_device(torch.tensor(flat), nf, icpt, reg, enet, stdf, True, 100, 1e-6)
    coef, b0, hist, reason = out
    np.testing.assert_allclose(coef, r["coefficients"], rtol=1e-7, atol=1e-9)
    assert b0 == pytest.approx(r["intercept"], rel=1e-7, abs=1e-9)
    ref_hist = np.asarray(r["objective_history"])
    assert hist[0] == ref_hist[0]
    # the last iterations sit at the convergence tolerance, where summation order can move the
    # stopping point by an iteration or two: compare the common prefix and the end
    m = min(len(hist), len(ref_hist))
    assert abs(len(hist) - len(ref_hist)) <= 3
    np.testing.assert_allclose(hist[:m], ref_hist[:m], rtol=1e-8)
    assert hist[-1] == pytest.approx(ref_hist[-1], rel=1e-9)
    assert np.all(np.diff(hist) <= 1e-12 * abs(hist[0]))
