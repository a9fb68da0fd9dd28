"""Huber regression (``LinearRegression(loss="huber")``), Spark 2.4 ``HuberAggregator`` objective:

    L(c, b, σ) = 1/W Σ_i w_i [ σ + H_ε(y_i - x_i·c/σ_x - b)/σ ... ] / 2 + L2(c)

optimized over (coefficients in the std-scaled space, intercept, σ) from all ones, with the bounds
Spark passes to Breeze's ``LBFGSB`` (every coordinate in [Double.MinValue, Double.MaxValue], σ >=
Double.MinPositiveValue) and memory 10: :class:`.lbfgsb.LBFGSB` reproduces that optimizer's
algorithm -- generalized Cauchy point, direct primal subspace minimization, strong-Wolfe search
on the unprojected ray, Breeze's convergence checks -- so iteration counts and
``objectiveHistory`` follow it.  Each evaluation is one fused device pass
(``kernels.huber_pass``: margin -> loss/multipliers, then Xᵀm) plus one all-reduce of d+4 f64.

On GPU data the optimizer runs on the device too (``ops/csrc/hip/huber_qn.hip``, the same
algorithm as :class:`.lbfgsb.LBFGSB`): the row pass reads its trial point from HBM, a one-block
control kernel consumes the all-reduced evaluation and writes the next trial, and the host only
enqueues -- no read per evaluation, so with ``dq4ml.fit.async`` the fit returns before the device
has run it and the model resolves on first read.  The host-steered optimizer below stays the path
for CPU data, checkpointed fits (``dq4ml.lbfgs.checkpointDir``) and the cases the device hands
back (empty data, history capacity).
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import kernels, native
from ..parallel import comm
from ..runtime.checks import verify
from ..utils import tracing
from ..utils.logging import get_logger
from .lbfgsb import LBFGSB, LBFGSBState
from .linalg import DenseVector
from .optim import GramStats, WLSModel

log = get_logger("huber")
MIN_SIGMA = 5e-324  # Double.MinPositiveValue: Spark's lower bound of σ
_DMAX = float(np.finfo(np.float64).max)


def train_huber(est, df, tbl, X, y, w, sel, d, checks=(), device=True):
    from .lbfgs_path import _sample_moments
    from .regression import LinearRegressionModel, LinearRegressionTrainingSummary, _async_conf, _async_model

    fit_icpt = bool(est.getOrDefault("fitIntercept"))
    eps = float(est.getOrDefault("epsilon"))
    reg, enet = float(est.getOrDefault("regParam")), float(est.getOrDefault("elasticNetParam"))
    if enet != 0.0 and reg != 0.0:
        raise ValueError("requirement failed: LinearRegression with huber loss only supports L2 regularization, "
                         "but got elasticNetParam = " + str(enet) + ".")
    std_flag = bool(est.getOrDefault("standardization"))
    max_iter, tol = int(est.getOrDefault("maxIter")), float(est.getOrDefault("tol"))
    flat = comm.all_reduce_sum(kernels.gram_stats(X.values, y.values, w, sel, "fp64"))
    use_dev = device and _device_ok(df, X.values, d)
    if comm.collectives_active():  # the two paths issue different collectives: one branch for all
        use_dev = comm.all_agree(use_dev)
    if use_dev:
        from ..ops import device as dv

        with tracing.span("solve"):
            sxd, lamd = _device_moments(flat, d, reg, std_flag)
            all_reduce = comm.all_reduce_sum if comm.collectives_active() else None
            out, keep = dv.huber_fit_dp(X.values, y.values, w, sel, sxd, lamd, fit_icpt, eps, max_iter, tol, all_reduce)

        def fallback():
            return train_huber(est, df, tbl, X, y, w, sel, d, (), device=False)

        pending = _PendingHuber(out, flat, d, checks, fallback)
        pending._keep = keep
        if _async_conf(df):
            return _async_model(est, df, pending)
        wls, stats = pending.resolve()
        model = LinearRegressionModel(est.uid, DenseVector(wls.coefficients), float(wls.intercept), wls.scale)
        est.copyValues(model)
        model._set_summary(LinearRegressionTrainingSummary(model, df, None, wls.objectiveHistory, stats=stats,
                                                           solver="l-bfgs-b"))
        model._huber_evaluations = pending.evaluations
        return model
    verify(checks)
    stats = GramStats.from_flat(flat.cpu().numpy(), d)
    _, sx, _, _, _, _, _ = _sample_moments(stats)
    l2 = reg
    safe = np.where(sx == 0.0, 1.0, sx)
    lam = np.full(d, l2) if std_flag else np.where(sx != 0.0, l2 / (safe * safe), 0.0)
    dim = d + (2 if fit_icpt else 1)

    cache = [None, None]  # Breeze CachedDiffFunction: the last point and its (f, g)

    def fg(theta):
        if cache[0] is not None and np.array_equal(cache[0], theta):
            return cache[1]
        cache[0], cache[1] = np.array(theta, dtype=np.float64), _fg(theta)
        return cache[1]

    def _fg(theta):
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
    # (a device fit's fallback hands these back to its pending result)
    res = WLSModel(np.asarray(coef, dtype=np.float64), icpt, np.zeros(1), np.asarray(hist, dtype=np.float64),
                   "l-bfgs-b")
    res.scale = float(theta[-1])
    model._wls_result, model._stats_result = res, stats
    return model


def _ck_root(df) -> str:
    sess = getattr(df, "sparkSession", None)
    return sess.conf.get("dq4ml.lbfgs.checkpointDir", "") if sess is not None else ""


def _device_ok(df, Xv, d) -> bool:
    """The device optimizer runs GPU data without checkpoints or fault injection (the
    host-steered loop owns both); ``dq4ml.huber.device=false`` turns it off."""
    sess = getattr(df, "sparkSession", None)
    if sess is not None and str(sess.conf.get("dq4ml.huber.device", "true")).lower() in ("0", "false", "no"):
        return False
    if _FAIL_AT_ITER is not None or _ck_root(df) or d < 1 or not kernels._on_gpu(Xv if torch.is_tensor(Xv) else Xv.buf):
        return False
    return native.hip_available()


def _device_moments(flat: torch.Tensor, d: int, reg: float, std_flag: bool):
    """Feature std (Spark's weighted unbiased variance) and the L2 weights, on the device, from
    the all-reduced statistics -- the same elementwise expressions as ``_sample_moments``."""
    W, W2 = flat[1], flat[2]
    mx = flat[5:5 + d] / W
    j = torch.arange(d, device=flat.device)
    diag = flat[5 + 2 * d + j + j * (j + 1) // 2]
    denom = W - W2 / W
    var = torch.where(denom > 0, torch.clamp(diag - W * mx * mx, min=0.0) / denom, torch.zeros_like(mx))
    sx = torch.sqrt(var)
    safe = torch.where(sx == 0.0, torch.ones_like(sx), sx)
    full = torch.full_like(sx, reg)  # (tensor / tensor: the host's numpy division, bit for bit)
    lam = full if std_flag else torch.where(sx != 0.0, full / (safe * safe), torch.zeros_like(sx))
    return sx.contiguous(), lam.contiguous()


_WHY = {0: "projected step converged", 1: "max iterations", 2: "function values converged", 3: "gradient converged",
        4: "search failed", -1: "history capacity"}


class _PendingHuber:
    """A device Huber fit (``huber_qn.hip``) enqueued on the current stream; ``resolve()`` reads
    its output once.  Cases the device hands back (status != 0, empty data) re-run on the host-
    steered optimizer, which owns Spark's behavior there."""

    pending_fit = True

    def __init__(self, out, flat, d, checks, fallback):
        self.out, self.flat, self.d, self._checks, self._fallback = out, flat, d, list(checks), fallback
        self._res = None
        self.evaluations = None
        self._done = torch.cuda.Event()
        self._done.record()

    def resolve(self):
        if self._res is None:
            torch.cuda.current_stream(self.out.device).wait_event(self._done)
            host = self.out.cpu().numpy()
            flat = self.flat.cpu().numpy()
            self._keep = None
            verify(self._checks)
            d = self.d
            stats = GramStats.from_flat(flat, d)
            if int(host[d + 2]) != 0 or not stats.wSum > 0.0:
                model = self._fallback()
                self._res = (model._wls_result, model._stats_result)
                return self._res
            H, iters, self.evaluations = int(host[d + 4]), int(host[d + 5]), int(host[d + 6])
            log.info("l-bfgs-b (huber, device) converged: %s after %d iterations, %d evaluations",
                     _WHY.get(int(host[d + 3]), "?"), iters, self.evaluations)
            res = WLSModel(host[:d].copy(), float(host[d]), np.zeros(1), host[d + 8:d + 8 + H].copy(), "l-bfgs-b")
            res.scale = float(host[d + 1])
            self._res = (res, stats)
        return self._res


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
