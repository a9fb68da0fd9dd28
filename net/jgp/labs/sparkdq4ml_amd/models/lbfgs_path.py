"""Iterative path of ``LinearRegression.fit`` (``solver="l-bfgs"``, ``numFeatures > 4096`` with
``solver="auto"``, or ``loss="huber"``) — Spark 2.4.4 ``LinearRegression.train`` semantics:

* features/label standardized with the **sample** (n-1) std of ``MultivariateOnlineSummarizer``;
* ``effectiveRegParam = regParam / yStd`` (squared error) or ``regParam`` (huber);
* squared error: Breeze L-BFGS (L2 only) or OWLQN (L1 > 0) over the standardized least-squares
  loss ``1/2W Σ w (Σ_j c_j (x_j-μ_j)/σ_j - (y-ȳ)/σ_y)^2 + L2``; the intercept is closed form
  afterwards (GLMNET style);
* huber: L-BFGS-B over (coefficients, intercept, σ) with σ > 0 (see :func:`_train_huber`).

MI355X design: Spark re-scans the data every iteration (``LeastSquaresAggregator`` inside a
``treeAggregate``).  For squared error that loss is a quadratic form in the
sufficient statistics, so ONE fused MFMA Gram pass (the same kernel as the normal-equation path)
plus an O(d^2) f64 iteration replaces maxIter data passes — identical objective, identical
optimizer, no per-iteration all-reduce; with 288 GB of HBM the d x d Gram fits for any d this path
targets.  Huber is not quadratic and keeps per-iteration device passes (``kernels.huber_loss_grad``)
with one all-reduce of (d+3) f64 per evaluation.
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import kernels, native
from ..parallel import comm
from ..utils.logging import get_logger
from .linalg import DenseVector
from .optim import GramStats, packed_upper_indices

log = get_logger("lbfgs")


def _sample_moments(stats: GramStats):
    """(mean_x, std_x sample, mean_y, std_y sample, cov_xx packed, cov_xy) with Spark's weighted
    unbiased variance: var = M2 / (W - W2/W)."""
    W, W2 = stats.wSum, stats.wwSum
    denom = W - W2 / W
    mx = stats.aSum / W
    my = stats.bSum / W
    I, J = packed_upper_indices(stats.k)
    m2_xx = stats.aaSum - W * mx[I] * mx[J]  # Σ w (x_i-μ_i)(x_j-μ_j)
    m2_xy = stats.abSum - W * mx * my
    m2_yy = stats.bbSum - W * my * my
    diag = np.array([j + j * (j + 1) // 2 for j in range(stats.k)], dtype=np.int64)
    var_x = np.maximum(m2_xx[diag], 0.0) / denom if denom > 0 else np.zeros(stats.k)
    var_y = max(m2_yy, 0.0) / denom if denom > 0 else 0.0
    return mx, np.sqrt(var_x), my, float(np.sqrt(var_y)), m2_xx, m2_xy, m2_yy


def train_lbfgs(est, df, tbl, X, y, d):
    from ..runtime.checks import verify
    from .regression import (LinearRegressionModel, LinearRegressionTrainingSummary, _fit_checks, _weight_of)

    loss = est.getOrDefault("loss")
    verify(_fit_checks(est, tbl, X))  # the iterative path reads host statistics at once anyway
    w = _weight_of(est, tbl)
    sel = tbl.sel
    if y.valid is not None:
        sel = y.valid if sel is None else (sel & y.valid)
    if loss == "huber":
        return _train_huber(est, df, tbl, X, y, w, sel, d)
    flat = kernels.gram_stats(X.values, y.values, w, sel, est.getOrDefault("gramDtype"))
    flat = comm.all_reduce_sum(flat)
    stats = GramStats.from_flat(flat.cpu().numpy(), d)
    fit_icpt = bool(est.getOrDefault("fitIntercept"))
    std_flag = bool(est.getOrDefault("standardization"))
    reg, enet = float(est.getOrDefault("regParam")), float(est.getOrDefault("elasticNetParam"))
    max_iter, tol = int(est.getOrDefault("maxIter")), float(est.getOrDefault("tol"))
    mx, sx, my, raw_ys, m2_xx, m2_xy, m2_yy = _sample_moments(stats)

    def finish(coef, icpt, hist, solver):
        model = LinearRegressionModel(est.uid, DenseVector(coef), float(icpt))
        est.copyValues(model)
        model._set_summary(LinearRegressionTrainingSummary(model, df, None, hist, stats=stats, solver=solver))
        return model

    if raw_ys == 0.0 and (fit_icpt or my == 0.0):
        log.warning("The standard deviation of the label is zero, so the coefficients will be zeros and the "
                    "intercept will be the mean of the label; as a result, training is not needed.")
        return finish(np.zeros(d), my if fit_icpt else 0.0, np.zeros(1), "none")
    ys = raw_ys if raw_ys > 0 else abs(my)
    eff_reg = reg / ys
    l1, l2 = enet * eff_reg, (1.0 - enet) * eff_reg
    W = stats.wSum
    I, J = packed_upper_indices(d)
    safe = np.where(sx == 0.0, 1.0, sx)
    if fit_icpt:
        A = m2_xx / (W * safe[I] * safe[J])
        b = m2_xy / (W * safe * ys)
        s = m2_yy / (W * ys * ys)
    else:  # no centering: raw second moments
        A = stats.aaSum / (W * safe[I] * safe[J])
        b = stats.abSum / (W * safe * ys)
        s = stats.bbSum / (W * ys * ys)
    zero = (sx == 0.0)
    A = np.where(zero[I] | zero[J], 0.0, A)
    b = np.where(zero, 0.0, b)
    diag = np.array([j + j * (j + 1) // 2 for j in range(d)], dtype=np.int64)
    if l2 != 0.0:
        lam = np.full(d, l2) if std_flag else np.where(sx != 0.0, l2 / (safe * safe), 0.0)
        A[diag] += lam
    l1vec = None
    if enet != 0.0 and eff_reg != 0.0:
        l1vec = np.full(d, l1) if std_flag else np.where(sx != 0.0, l1 / safe, 0.0)
    x, hist, reason = native.host().quasi_newton(0.0, s, b, A, np.zeros(d), False, max_iter, tol, l1vec)
    log.info("l-bfgs path: %s after %d states", reason, len(hist))
    coef = np.where(zero, 0.0, np.asarray(x) * ys / safe)
    icpt = my - float(np.dot(coef, mx)) if fit_icpt else 0.0
    return finish(coef, icpt, hist, "owlqn" if l1vec is not None else "l-bfgs")


def _train_huber(est, df, tbl, X, y, w, sel, d):
    from .huber import train_huber

    return train_huber(est, df, tbl, X, y, w, sel, d)


_ = torch
