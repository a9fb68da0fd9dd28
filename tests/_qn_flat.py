"""Synthetic WLS statistics for the OWLQN solver tests (``test_gpu_owlqn.py``)."""
import numpy as np


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
