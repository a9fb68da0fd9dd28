"""Iterative path of ``LinearRegression.fit`` (``solver="l-bfgs"``, ``numFeatures > 4096`` with
``solver="auto"``, or ``loss="huber"``) — Spark 2.4.4 ``LinearRegression.train`` semantics:

* features/label standardized with the **sample** (n-1) std of ``MultivariateOnlineSummarizer``;
* ``effectiveRegParam = regParam / yStd`` (squared error) or ``regParam`` (huber);
* squared error: Breeze L-BFGS (L2 only) or OWLQN (L1 > 0) over the standardized least-squares
  loss ``1/2W Σ w (Σ_j c_j (x_j-μ_j)/σ_j - (y-ȳ)/σ_y)^2 + L2``; the intercept is closed form
  afterwards (GLMNET style);
* huber: L-BFGS-B over (coefficients, intercept, σ) with σ > 0 (see :func:`_train_huber`).

MI355X design: Spark re-scans the data for every cost evaluation
(``LeastSquaresAggregator`` inside a ``treeAggregate``).  Here too, by default
(``dq4ml.lbfgs.mode = passes``): one summarizer pass for the feature moments, then per evaluation
two streaming HIP passes over the HBM-resident shard (``ops/csrc/hip/lsq.hip``: margins, then
Σ w·diff·x) and ONE RCCL all-reduce of (d + 1) f64 — O(n·d) device work per evaluation, never the
d x d Gram.  The Breeze optimizer state lives on the device (``models/qn_device.py``).

``dq4ml.lbfgs.mode = gram``: squared error is a quadratic form in the sufficient statistics, so ONE
fused MFMA Gram pass plus an O(d^2) host iteration gives the same optimum (the same optimizer on the
same objective) — cheaper when n·d^2 of MFMA work beats maxIter data passes.  Huber is not quadratic
and keeps per-iteration device passes (``kernels.huber_pass``).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..ops import kernels, native
from ..parallel import comm
from ..utils import tracing
from ..runtime.checks import verify
from ..utils.logging import get_logger
from .linalg import DenseVector
from .optim import GramStats, packed_upper_indices
from .qn_device import REASONS

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
    from .regression import (LinearRegressionModel, LinearRegressionTrainingSummary, _fit_checks, _weight_of)

    loss = est.getOrDefault("loss")
    checks = _fit_checks(est, tbl, X)
    w = _weight_of(est, tbl)
    sel = tbl.sel
    if y.valid is not None:
        sel = y.valid if sel is None else (sel & y.valid)
    sess = getattr(df, "sparkSession", None)
    mode = str(sess.conf.get("dq4ml.lbfgs.mode", "passes")).lower() if sess is not None else "passes"
    if loss != "huber" and mode != "gram":
        return _train_passes(est, df, X, y, w, sel, d, checks)
    if loss == "huber":  # (verifies the checks itself: its device path reads nothing at once)
        return _train_huber(est, df, tbl, X, y, w, sel, d, checks)
    verify(checks)  # the host-steered paths read statistics at once anyway
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
    _check_constant_label(raw_ys, reg)
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


def _check_constant_label(raw_ys: float, reg: float) -> None:
    """Spark 2.4 ``LinearRegression.train`` for a constant nonzero label without an intercept:
    ``require(regParam == 0.0, ...)``, else a warning (the caller has already returned for the
    fitIntercept / zero-mean cases)."""
    if raw_ys != 0.0:
        return
    if reg != 0.0:
        raise ValueError("requirement failed: The standard deviation of the label is zero. "
                         "Model cannot be regularized.")
    log.warning("The standard deviation of the label is zero. Consider setting fitIntercept=true.")


def _device_qn_ok(df, P) -> bool:
    """The whole fit on the device: wide tiles on a GPU, no optimizer checkpoints (those read the
    state on the host every few iterations).  One rank: ONE grid launch
    (``LsqPasses.qn_fit``); with collectives active: the data-parallel form
    (``LsqPasses.qn_fit_dp``: pass, fold, all-reduce, control kernel per evaluation)."""
    sess = getattr(df, "sparkSession", None)
    return (P.device.type == "cuda" and P.layout in (2, 3)
            and not (sess is not None and sess.conf.get("dq4ml.lbfgs.checkpointDir", ""))
            and os.environ.get("DQ4ML_LSQ_QN", "1") != "0")


class _PendingLsq:
    """A device l-bfgs / OWLQN fit (``lsq_qn.hip``) enqueued on the current stream; ``resolve()``
    reads its result once.  Cases the kernel hands back (empty data, constant label, history
    capacity) re-run on the host-steered path, which owns Spark's warnings and exceptions."""

    pending_fit = True

    def __init__(self, out, d, solver, checks, fallback):
        self.out, self.d, self.solver, self._checks, self._fallback = out, d, solver, list(checks), fallback
        self._res = None
        # the fit's stream: resolve() may run under another stream context, so its read waits on
        # this event instead of on whatever stream is current then
        self._done = torch.cuda.Event()
        self._done.record()

    def resolve(self):
        if self._res is None:
            from .optim import WLSModel

            torch.cuda.current_stream(self.out.device).wait_event(self._done)
            host = self.out.cpu().numpy()
            verify(self._checks)
            d = self.d
            if int(host[d + 1]) != 0:
                if int(host[d + 1]) == 9:  # evaluation bound, or a grid barrier gave up (grid_barrier)
                    log.warning("device l-bfgs fit did not finish (status 9); re-running it host-steered")
                model = self._fallback()
                self._res = (model._wls_result, model._stats_result)
                return self._res
            H = int(host[d + 3])
            reason = REASONS[int(host[d + 2])]
            self.evaluations = int(host[d + 5])
            log.info("l-bfgs path (device, one pass per evaluation): %s after %d states, %d evaluations", reason, H,
                     self.evaluations)
            wls = WLSModel(host[:d].copy(), float(host[d]), np.zeros(1), host[d + 11:d + 11 + H].copy(), self.solver)
            self._res = (wls, GramStats.scalars_only(host[d + 6:d + 11], d))
        return self._res


def _train_passes(est, df, X, y, w, sel, d, checks=(), device_qn=True):
    """Spark 2.4 ``LinearRegression.train`` l-bfgs branch with squared error, data pass per
    evaluation: summarizer moments -> standardization / regularization constants -> Breeze
    L-BFGS (L2) or OWLQN (L1 > 0) over ``LeastSquaresCostFun`` -> un-standardize.

    On one GPU with wide tiles the whole sequence is ONE grid launch (``lsq_qn.hip``: one
    fused data pass per evaluation, the line search on the device), enqueued with the summarizer
    pass; with ``dq4ml.fit.async`` the fit returns at once.  Otherwise the Breeze state stays on
    the device and the host steers (``models/qn_device.py``)."""
    from .qn_device import minimize
    from .regression import LinearRegressionModel, LinearRegressionTrainingSummary, _async_conf, _async_model

    P = kernels.lsq_passes(X.values, y.values, w, sel)
    dev = P.device
    with tracing.span("gram"):  # the summarizer pass (feature moments), one all-reduce with the scalars
        head = comm.all_reduce_sum(torch.cat([P.scalars(), P.moments()]))
    fit_icpt = bool(est.getOrDefault("fitIntercept"))
    std_flag = bool(est.getOrDefault("standardization"))
    reg, enet = float(est.getOrDefault("regParam")), float(est.getOrDefault("elasticNetParam"))
    max_iter, tol = int(est.getOrDefault("maxIter")), float(est.getOrDefault("tol"))
    use_dev = device_qn and _device_qn_ok(df, P) and P.qn_eligible()
    if comm.collectives_active():
        # the device fit and the host-steered one issue different collectives: every rank must
        # take the same branch (a rank whose shard is empty, or holds another layout, would
        # otherwise deadlock its peers) -- a host-side vote, no device sync
        use_dev = comm.all_agree(use_dev)
    if use_dev:
        with tracing.span("solve"):
            # X4: one (d + 2)-f64 all-reduce per evaluation, no host read.  DQ4ML_QN_SPLIT=1 runs
            # the same split form on one rank without a group (plain launches: counter runs)
            if comm.collectives_active() or os.environ.get("DQ4ML_QN_SPLIT") == "1":
                out = P.qn_fit_dp(head, fit_icpt, std_flag, reg, enet, max_iter, tol, comm.all_reduce_sum)
            else:
                out = P.qn_fit(head, fit_icpt, std_flag, reg, enet, max_iter, tol)
        if out is not None:
            solver = "owlqn" if enet != 0.0 and reg != 0.0 else "l-bfgs"

            def fallback():
                return _train_passes(est, df, X, y, w, sel, d, (), device_qn=False)

            pending = _PendingLsq(out, d, solver, checks, fallback)
            pending._keep = P
            if _async_conf(df):
                return _async_model(est, df, pending)
            wls, stats = pending.resolve()
            model = LinearRegressionModel(est.uid, DenseVector(wls.coefficients), float(wls.intercept))
            est.copyValues(model)
            model._set_summary(LinearRegressionTrainingSummary(model, df, None, wls.objectiveHistory, stats=stats,
                                                               solver=solver))
            model._qn_evaluations = getattr(pending, "evaluations", None)
            return model
    verify(checks)
    host = head.cpu().numpy()
    count, W, W2, bsum, bbsum = (float(v) for v in host[:5])
    sx_sum, sxx_sum = host[5:5 + d], host[5 + d:5 + 2 * d]
    stats = GramStats.scalars_only(host[:5], d)
    if W <= 0.0:
        raise ValueError("requirement failed: The training dataset is empty (weight sum is 0).")
    denom = W - W2 / W
    mx = sx_sum / W
    my = bsum / W
    var_x = np.maximum(sxx_sum - W * mx * mx, 0.0) / denom if denom > 0 else np.zeros(d)
    var_y = max(bbsum - W * my * my, 0.0) / denom if denom > 0 else 0.0
    sx, raw_ys = np.sqrt(var_x), float(np.sqrt(var_y))

    def finish(coef, icpt, hist, solver):
        from .optim import WLSModel

        model = LinearRegressionModel(est.uid, DenseVector(coef), float(icpt))
        est.copyValues(model)
        model._set_summary(LinearRegressionTrainingSummary(model, df, None, hist, stats=stats, solver=solver))
        # (a device fit's fallback hands these back to its pending result)
        model._wls_result = WLSModel(np.asarray(coef, dtype=np.float64), float(icpt), np.zeros(1),
                                     np.asarray(hist, dtype=np.float64), solver)
        model._stats_result = stats
        return model

    if raw_ys == 0.0 and (fit_icpt or my == 0.0):
        log.warning("The standard deviation of the label is zero, so the coefficients will be zeros and the "
                    "intercept will be the mean of the label; as a result, training is not needed.")
        return finish(np.zeros(d), my if fit_icpt else 0.0, np.zeros(1), "none")
    _check_constant_label(raw_ys, reg)
    ys = raw_ys if raw_ys > 0 else abs(my)
    eff_reg = reg / ys
    l1, l2 = enet * eff_reg, (1.0 - enet) * eff_reg
    nz = sx != 0.0
    safe = np.where(nz, sx, 1.0)
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64), device=dev)  # noqa: E731
    inv_sx, mx_t = t(np.where(nz, 1.0 / safe, 0.0)), t(mx)
    reg_w = None  # L2 weights per coordinate (standardization=false: 1 / sigma^2)
    if l2 != 0.0:
        reg_w = torch.ones(d, dtype=torch.float64, device=dev) if std_flag else t(np.where(nz, 1.0 / (safe * safe), 0.0))
    icpt0 = torch.tensor(my / ys if fit_icpt else 0.0, dtype=torch.float64, device=dev)
    inv_ys, inv_w = 1.0 / ys, 1.0 / W

    # L-BFGS line searches (not OWLQN: its projected trial is not affine in alpha): a trial x + a d
    # has u = w (x' . cf) = u(x) + a u(d), so only a search's first trial forms u(d) (a margin
    # pass); every trial then runs the column pass alone, and the loss along the search is an
    # exact quadratic in a (no per-trial rounding noise: the searches accept at once)
    ucache = {}   # id(x) -> (x, u(x)) of the current base point and its trials
    udir = [None]  # (d, base x, u(d)) of the current search

    def fg(x, line=None):
        cf = x * inv_sx
        offset = icpt0 - torch.dot(cf, mx_t) if fit_icpt else icpt0
        if line is not None and l1vec is None:
            bx, dvec, a = line
            ent = ucache.get(id(bx))
            if ent is None or ent[0] is not bx:
                with tracing.span("lsq_pass"):
                    ent = (bx, P.wmargins(bx * inv_sx))
                ucache.clear()
                ucache[id(bx)] = ent
            cur = udir[0]
            if cur is None or cur[0] is not dvec or cur[1] is not bx:
                with tracing.span("lsq_pass"):
                    cur = udir[0] = (dvec, bx, P.wmargins(dvec * inv_sx))
                for k in [k for k, e in ucache.items() if e[0] is not bx]:  # a new search: old trials go
                    del ucache[k]
            u = ent[1] + a * cur[2]
            # keep the base point and THIS trial only (a search accepts its last trial, which is
            # the next search's base): an n-f64 margin vector per earlier trial would pile up
            for k in [k for k, e in ucache.items() if e[0] is not bx]:
                del ucache[k]
            ucache[id(x)] = (x, u)
            with tracing.span("lsq_pass"):
                out = P.evaluate_u(u, cf, offset, inv_ys)
        else:
            with tracing.span("lsq_pass"):
                out = P.evaluate(cf, offset, inv_ys)
        with tracing.span("allreduce"):
            out = comm.all_reduce_sum(out)  # X4: (d + 1) f64 per evaluation
        tracing.add_rows("lsq_pass", P.n)
        loss = out[0] * inv_w
        g = out[1:] * inv_sx * inv_w
        if reg_w is not None:
            rx = reg_w * x
            loss = loss + 0.5 * l2 * torch.dot(x, rx)
            g = g + l2 * rx
        return loss, g

    l1vec = None
    if enet != 0.0 and eff_reg != 0.0:
        l1vec = torch.full((d,), l1, dtype=torch.float64, device=dev) if std_flag else t(np.where(nz, l1 / safe, 0.0))
    ck = _QNCheckpoint.of(df, head, (d, fit_icpt, reg, enet, std_flag, max_iter, tol))
    resume = ck.load() if ck is not None else None
    if resume is not None:
        log.info("resuming l-bfgs at iteration %d from %s", int(resume["iter"]), ck.path)
    fg.line_aware = True
    x0 = torch.zeros(d, dtype=torch.float64, device=dev)
    ucache[id(x0)] = (x0, torch.zeros(P.n, dtype=torch.float64, device=dev))  # u(0) = 0
    x, hist, reason = minimize(fg, x0, max_iter, tol, l1vec,
                               resume=resume, on_iteration=ck.maybe_save if ck is not None else None)
    if ck is not None:
        ck.clear()
    log.info("l-bfgs path (data passes): %s after %d states", reason, len(hist))
    coef = np.where(nz, x.cpu().numpy() * ys / safe, 0.0)
    icpt = my - float(np.dot(coef, mx)) if fit_icpt else 0.0
    return finish(coef, icpt, np.asarray(hist, dtype=np.float64), "owlqn" if l1vec is not None else "l-bfgs")


_QN_FAIL_AT_ITER = None  # tests: raise after this iteration's checkpoint (simulated crash)


class _QNCheckpoint:
    """Optimizer-state checkpoints of the squared-loss l-bfgs path, the counterpart
    of the Huber fit's ``_Checkpoint``: with ``dq4ml.lbfgs.checkpointDir`` set, the complete Breeze
    state (iterate, gradients, s/y history, function-value window, objective history, failure
    flags) is written every ``dq4ml.lbfgs.checkpointInterval`` iterations; a re-run of the same fit
    on the same data (fingerprinted by its all-reduced moments) resumes from it and ends exactly as
    the uninterrupted run."""

    def __init__(self, path: str, every: int):
        self.path, self.every = path, max(1, int(every))

    @classmethod
    def of(cls, df, head, params):
        import hashlib
        import os

        sess = getattr(df, "sparkSession", None)
        root = sess.conf.get("dq4ml.lbfgs.checkpointDir", "") if sess is not None else ""
        if not root:
            return None
        h = hashlib.sha1(repr(params).encode())
        h.update(np.ascontiguousarray(head.cpu().numpy()).tobytes())
        os.makedirs(root, exist_ok=True)
        return cls(os.path.join(root, f"lsq-{h.hexdigest()[:20]}.npz"),
                   int(sess.conf.get("dq4ml.lbfgs.checkpointInterval", "10")))

    def maybe_save(self, state):
        import os

        it = int(state["iter"])
        if it % self.every == 0 and comm.rank() == 0:
            host = {k: (v.cpu().numpy() if torch.is_tensor(v) else v) for k, v in state.items() if k not in ("S", "Y")}
            S = np.stack([s.cpu().numpy() for s in state["S"]]) if state["S"] else np.zeros((0, 0))
            Y = np.stack([y.cpu().numpy() for y in state["Y"]]) if state["Y"] else np.zeros((0, 0))
            tmp = self.path + ".tmp.npz"
            np.savez(tmp, S=S, Y=Y, **{k: np.asarray(v) for k, v in host.items()})
            os.replace(tmp, self.path)
        if _QN_FAIL_AT_ITER is not None and it == _QN_FAIL_AT_ITER:
            raise RuntimeError(f"injected failure after l-bfgs iteration {it}")

    def load(self):
        import os

        comm.barrier()
        if not os.path.exists(self.path):
            return None
        z = np.load(self.path)  # allow_pickle=False: plain arrays only
        st = {k: z[k] for k in z.files}
        st["S"] = list(st["S"]) if st["S"].size else []
        st["Y"] = list(st["Y"]) if st["Y"].size else []
        st["fvals"] = [float(v) for v in st["fvals"]]
        st["history"] = [float(v) for v in st["history"]]
        return st

    def clear(self):
        import os

        comm.barrier()
        if comm.rank() == 0 and os.path.exists(self.path):
            os.remove(self.path)


def _train_huber(est, df, tbl, X, y, w, sel, d, checks=()):
    from .huber import train_huber

    return train_huber(est, df, tbl, X, y, w, sel, d, checks)


_ = torch
