"""Huber regression (``LinearRegression(loss="huber")``), Spark 2.4 ``HuberAggregator`` objective:

    L(c, b, σ) = 1/W Σ_i w_i [ σ + H_ε(y_i - x_i·c/σ_x - b)/σ ... ] / 2 + L2(c)

optimized over (coefficients in the std-scaled space, intercept, σ) from all ones, with the bounds
Spark passes to Breeze's ``LBFGSB`` (every coordinate in [Double.MinValue, Double.MaxValue], σ >=
Double.MinPositiveValue) and memory 10: :class:`.lbfgsb.LBFGSB` reproduces that optimizer's
algorithm -- generalized Cauchy point, direct primal subspace minimization, strong-Wolfe search
on the unprojected ray, Breeze's convergence checks -- so iteration counts and
``objectiveHistory`` follow it.  Each evaluation is one fused device pass
(``kernels.huber_pass``: margin -> loss/multipliers, then Xᵀm) plus one all-reduce of d+4 f64;
the optimizer's O(k m) bookkeeping runs on the host between passes.
"""
from __future__ import annotations

import numpy as np

from ..ops import kernels
from ..parallel import comm
from ..utils.logging import get_logger
from .lbfgsb import LBFGSB, LBFGSBState
from .linalg import DenseVector
from .optim import GramStats

log = get_logger("huber")
MIN_SIGMA = 5e-324  # Double.MinPositiveValue: Spark's lower bound of σ
_DMAX = float(np.finfo(np.float64).max)


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

    lower = np.full(dim, -_DMAX)
    lower[-1] = MIN_SIGMA
    upper = np.full(dim, _DMAX)
    max_iter, tol = int(est.getOrDefault("maxIter")), float(est.getOrDefault("tol"))
    opt = LBFGSB(lower, upper, max_iter, 10, tol)
    ck = _Checkpoint.of(df, flat, (d, dim, fit_icpt, eps, reg, std_flag, max_iter, tol))
    resumed = ck.load() if ck is not None else None
    state, hist0 = (resumed if resumed is not None else (None, []))
    if state is not None:  # resume: the exact optimizer state of the last checkpoint
        log.info("resuming huber l-bfgs-b at iteration %d from %s", state.iter, ck.path)

    def on_state(st, hist):
        if ck is not None and st.iter % ck.every == 0:
            ck.save(st, hist0[:-1] + hist if hist0 else hist)
        if _FAIL_AT_ITER is not None and st.iter == _FAIL_AT_ITER:  # fault injection (tests)
            raise RuntimeError(f"injected failure at huber iteration {st.iter}")
    st, hist, why = opt.minimize(fg, np.ones(dim), state=state, on_state=on_state)
    hist = hist0[:-1] + hist if hist0 else hist
    log.info("l-bfgs-b (huber) converged: %s after %d iterations", why, st.iter)
    if ck is not None:
        ck.clear()
    theta = st.x
    coef = np.where(sx != 0.0, theta[:d] / safe, 0.0)
    icpt = float(theta[d]) if fit_icpt else 0.0
    model = LinearRegressionModel(est.uid, DenseVector(coef), icpt, float(theta[-1]))
    est.copyValues(model)
    model._set_summary(LinearRegressionTrainingSummary(model, df, None, np.array(hist), stats=stats, solver="l-bfgs-b"))
    return model


_FAIL_AT_ITER = None  # tests: raise at this iteration (simulated crash between checkpoints)


class _Checkpoint:
    """Optimizer-state checkpoints of the iterative (data-pass per evaluation) Huber fit
    (SURVEY.md §5d): with ``dq4ml.lbfgs.checkpointDir`` set, the complete L-BFGS-B state (iterate,
    value, gradient, θ and the s/y memory, the function-value window, failure flags, objective
    history, iteration) is written every
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

    def save(self, st: LBFGSBState, hist):
        import os

        if comm.rank() != 0:
            return
        dim = st.x.shape[0]
        tmp = self.path + ".tmp.npz"
        np.savez(tmp, it=np.array(st.iter), x=st.x, f=np.array(st.value), g=st.grad, f0=np.array(st.initial_value),
                 theta=np.array(st.theta), S=np.array(st.S).reshape(-1, dim), Y=np.array(st.Y).reshape(-1, dim),
                 fvals=np.array(st.fvals), flags=np.array([st.failed_once, st.search_failed]), hist=np.array(hist))
        os.replace(tmp, self.path)

    def load(self):
        """(state, objective history up to and including it) of the last checkpoint, or None."""
        import os

        comm.barrier()  # a rank-0 write of an earlier attempt is complete before anyone reads
        if not os.path.exists(self.path):
            return None
        z = np.load(self.path)  # allow_pickle=False: plain arrays only
        st = LBFGSBState(z["x"], float(z["f"]), z["g"], int(z["it"]), float(z["f0"]), float(z["theta"]), list(z["S"]),
                         list(z["Y"]), [float(v) for v in z["fvals"]], bool(z["flags"][0]), bool(z["flags"][1]))
        return st, [float(v) for v in z["hist"]]

    def clear(self):
        import os

        comm.barrier()
        if comm.rank() == 0 and os.path.exists(self.path):
            os.remove(self.path)
