"""Huber regression (``LinearRegression(loss="huber")``), Spark 2.4 ``HuberAggregator`` objective:

    L(c, b, σ) = 1/W Σ_i w_i [ σ + H_ε(y_i - x_i·c/σ_x - b)/σ ... ] / 2 + L2(c)

optimized over (coefficients in the std-scaled space, intercept, σ) with σ > 0 — Spark uses
Breeze ``LBFGSB``; here a projected L-BFGS (two-loop direction, projection of σ onto its lower
bound, backtracking Armijo search).  The optimum is the same (the problem is convex in that
parametrization); iteration counts / objectiveHistory lengths are not pinned to Breeze's.
Each evaluation is one fused device pass (``kernels.huber_pass``: margin -> loss/multipliers,
then Xᵀm) plus one all-reduce of d+4 f64.
"""
from __future__ import annotations

import numpy as np

from ..ops import kernels
from ..parallel import comm
from ..utils.logging import get_logger
from .linalg import DenseVector
from .optim import GramStats

log = get_logger("huber")
MIN_SIGMA = np.finfo(np.float64).tiny


def train_huber(est, df, tbl, X, y, w, sel, d):
    from .lbfgs_path import _sample_moments
    from .regression import LinearRegressionModel, LinearRegressionTrainingSummary

    flat = comm.all_reduce_sum(kernels.gram_stats(X.values, y.values, w, sel, "fp64"))
    stats = GramStats.from_flat(flat.cpu().numpy(), d)
    _, sx, _, _, _, _, _ = _sample_moments(stats)
    fit_icpt = bool(est.getOrDefault("fitIntercept"))
    eps = float(est.getOrDefault("epsilon"))
    reg, enet = float(est.getOrDefault("regParam")), float(est.getOrDefault("elasticNetParam"))
    if enet != 0.0 and reg != 0.0:
        raise ValueError("requirement failed: LinearRegression with huber loss only supports L2 regularization, "
                         "but got elasticNetParam = " + str(enet) + ".")
    std_flag = bool(est.getOrDefault("standardization"))
    l2 = reg
    safe = np.where(sx == 0.0, 1.0, sx)
    lam = np.full(d, l2) if std_flag else np.where(sx != 0.0, l2 / (safe * safe), 0.0)
    dim = d + (2 if fit_icpt else 1)

    def fg(theta):
        c = theta[:d]
        icpt = theta[d] if fit_icpt else 0.0
        sigma = theta[-1]
        ceff = np.where(sx != 0.0, c / safe, 0.0)
        out = comm.all_reduce_sum(kernels.huber_pass(X.values, y.values, w, sel, ceff, icpt, sigma, eps))
        out = out.cpu().numpy()
        loss_sum, wsum, g_icpt, g_sigma = out[:4]
        gx = np.where(sx != 0.0, out[4:4 + d] / safe, 0.0)
        f = loss_sum / wsum + 0.5 * float(np.sum(lam * c * c))
        g = np.zeros(dim)
        g[:d] = gx / wsum + lam * c
        if fit_icpt:
            g[d] = g_icpt / wsum
        g[-1] = g_sigma / wsum
        return f, g

    lo = np.full(dim, -np.inf)
    lo[-1] = MIN_SIGMA
    max_iter, tol = int(est.getOrDefault("maxIter")), float(est.getOrDefault("tol"))
    ck = _Checkpoint.of(df, flat, (d, dim, fit_icpt, eps, reg, std_flag, max_iter, tol))
    state = ck.load() if ck is not None else None
    if state is not None:  # resume: the exact optimizer state of the last checkpoint
        start, theta, f, g, S, Y, hist, f_hist = state
        log.info("resuming huber l-bfgs at iteration %d from %s", start, ck.path)
    else:
        start = 0
        theta = np.ones(dim)
        f, g = fg(theta)
        hist = [f]
        S, Y = [], []
        f_hist = [np.inf]
    for it in range(start, max_iter):
        if ck is not None and it > start and it % ck.every == 0:
            ck.save(it, theta, f, g, S, Y, hist, f_hist)
        if _FAIL_AT_ITER is not None and it == _FAIL_AT_ITER:  # fault injection (tests)
            raise RuntimeError(f"injected failure at huber iteration {it}")
        # projected gradient convergence
        pg = np.where((theta <= lo) & (g > 0), 0.0, g)
        if np.linalg.norm(pg) <= max(tol * abs(f), 1e-8):
            break
        q = g.copy()
        alphas = []
        for s, yv in zip(reversed(S), reversed(Y)):
            rho = 1.0 / np.dot(yv, s)
            a = rho * np.dot(s, q)
            alphas.append((a, rho, s, yv))
            q -= a * yv
        if S:
            q *= np.dot(S[-1], Y[-1]) / np.dot(Y[-1], Y[-1])
        for a, rho, s, yv in reversed(alphas):
            b = rho * np.dot(yv, q)
            q += (a - b) * s
        direction = -q
        direction = np.where((theta <= lo) & (direction < 0), 0.0, direction)
        if np.dot(direction, g) >= 0:
            direction = -pg
            S, Y = [], []
        step = 1.0 if it > 0 else min(1.0, 1.0 / max(np.linalg.norm(g), 1e-12))
        while True:
            cand = np.maximum(theta + step * direction, lo)
            fc, gc = fg(cand)
            if fc <= f + 1e-4 * np.dot(g, cand - theta) or step < 1e-12:
                break
            step *= 0.5
        s, yv = cand - theta, gc - g
        if np.dot(s, yv) > 1e-12:
            S.append(s)
            Y.append(yv)
            if len(S) > 10:
                S.pop(0)
                Y.pop(0)
        theta, f, g = cand, fc, gc
        hist.append(f)
        f_hist.append(f)
        f_hist = f_hist[-20:]
        if len(f_hist) >= 2 and abs(f - max(f_hist)) <= tol * abs(hist[0]):
            break
    if ck is not None:
        ck.clear()
    coef = np.where(sx != 0.0, theta[:d] / safe, 0.0)
    icpt = float(theta[d]) if fit_icpt else 0.0
    model = LinearRegressionModel(est.uid, DenseVector(coef), icpt, float(theta[-1]))
    est.copyValues(model)
    model._set_summary(LinearRegressionTrainingSummary(model, df, None, np.array(hist), stats=stats, solver="l-bfgs-b"))
    return model


_FAIL_AT_ITER = None  # tests: raise at this iteration (simulated crash between checkpoints)


class _Checkpoint:
    """Optimizer-state checkpoints of the iterative (data-pass per evaluation) Huber fit
    (SURVEY.md §5d): with ``dq4ml.lbfgs.checkpointDir`` set, the complete L-BFGS state (iterate,
    value, gradient, the s/y memory, objective histories, next iteration) is written every
    ``dq4ml.lbfgs.checkpointInterval`` iterations (atomic rename; rank 0 writes, every rank
    reads).  A re-run of the same fit — same parameters and the same data, fingerprinted by its
    all-reduced Gram statistics — resumes from it and finishes exactly as the uninterrupted run
    would have.  The file is removed when the fit completes."""

    def __init__(self, path: str, every: int):
        self.path, self.every = path, max(1, int(every))

    @classmethod
    def of(cls, df, flat, params):
        import hashlib
        import os

        sess = getattr(df, "sparkSession", None)
        root = sess.conf.get("dq4ml.lbfgs.checkpointDir", "") if sess is not None else ""
        if not root:
            return None
        h = hashlib.sha1(repr(params).encode())
        h.update(np.ascontiguousarray(flat.cpu().numpy()).tobytes())
        os.makedirs(root, exist_ok=True)
        return cls(os.path.join(root, f"huber-{h.hexdigest()[:20]}.npz"),
                   int(sess.conf.get("dq4ml.lbfgs.checkpointInterval", "10")))

    def save(self, it, theta, f, g, S, Y, hist, f_hist):
        import os

        if comm.rank() != 0:
            return
        dim = theta.shape[0]
        tmp = self.path + ".tmp.npz"
        np.savez(tmp, it=np.array(it), theta=theta, f=np.array(f), g=g,
                 S=np.array(S).reshape(-1, dim), Y=np.array(Y).reshape(-1, dim),
                 hist=np.array(hist), f_hist=np.array(f_hist))
        os.replace(tmp, self.path)

    def load(self):
        import os

        comm.barrier()  # a rank-0 write of an earlier attempt is complete before anyone reads
        if not os.path.exists(self.path):
            return None
        z = np.load(self.path)  # allow_pickle=False: plain arrays only
        return (int(z["it"]), z["theta"], float(z["f"]), z["g"], list(z["S"]), list(z["Y"]),
                list(z["hist"]), list(z["f_hist"]))

    def clear(self):
        import os

        comm.barrier()
        if comm.rank() == 0 and os.path.exists(self.path):
            os.remove(self.path)
