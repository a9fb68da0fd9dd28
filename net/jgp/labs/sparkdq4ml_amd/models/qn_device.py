"""Breeze 0.13 L-BFGS / OWLQN (the optimizers Spark 2.4.4 ``LinearRegression`` runs, POM:14) over a
cost function whose every evaluation is device work — the squared-loss l-bfgs path's
``LeastSquaresAggregator`` passes (``ops/csrc/hip/lsq.hip``) plus the X4 all-reduce.

The iterate, the gradients and the s/y history stay in HBM as f64 torch tensors; only the
scalars that steer the algorithm cross to the host, ONE read per cost evaluation (value and
directional derivative together) and one per iteration (history sanity + convergence norms).
The control flow is the native host driver's (``ops/csrc/host/solvers.cpp``) line for line:

* L-BFGS: two-loop recursion (memory 10, diagonal ``s.y / y.y``), strong-Wolfe cubic-interpolation
  line search (c1 1e-4, c2 0.9, first step ``1 / |dir|``), ``StepSizeUnderflow`` below 1e-10;
* OWLQN: the same recursion on the pseudo-gradient, orthant projection of every trial point,
  backtracking search (shrink 0.1 then 0.5, grow 2.1, first step ``0.5 / |g|``);
* convergence: max iterations | FunctionValuesConverged over the last 20 values (tol relative to
  the first adjusted value) | ``|adjusted gradient| <= max(tol |f|, 1e-8)`` | a second failed
  line search (the first one resets the history);
* Breeze's ``CachedDiffFunction``: re-evaluating the last point (``phi(0)``, the accepted step)
  costs no data pass.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import numpy as np
import torch

__all__ = ["minimize", "REASONS"]

REASONS = ("max iterations", "function values converged", "gradient converged", "search failed")
_FVAL_MEMORY = 20


class _FirstOrderError(Exception):
    pass


class _State:
    __slots__ = ("x", "value", "grad", "adj_value", "adj_grad", "value_h", "adj_h", "gnorm", "iter")


def minimize(fg: Callable[[torch.Tensor], Tuple[torch.Tensor, torch.Tensor]], x0: torch.Tensor, max_iter: int,
             tol: float, l1: Optional[torch.Tensor] = None, memory: int = 10, resume: Optional[dict] = None,
             on_iteration: Optional[Callable[[dict], None]] = None):
    """Minimize ``fg`` (x -> (value 0-d tensor, gradient)) from ``x0``; with ``l1`` (per-coordinate
    L1 weights) Breeze OWLQN, else Breeze L-BFGS.  Returns ``(x, objectiveHistory, reason)``.

    ``on_iteration(state)`` sees the complete optimizer state after every finished loop pass
    (checkpointing); ``resume`` restores such a state instead of starting at ``x0``."""
    owlqn = l1 is not None
    lz = (l1 == 0) if owlqn else None
    hist_s, hist_y = [], []
    last = {}  # CachedDiffFunction: the last evaluated trial point

    def adjust(x, g, v):
        if not owlqn:
            return v, g
        av = v + torch.sum(torch.abs(l1 * x))
        dp, dm = g + l1, g - l1
        at0 = torch.where(dm > 0, dm, torch.where(dp < 0, dp, torch.zeros_like(g)))
        ag = torch.where(x == 0, at0, g + torch.sign(x) * l1)
        return av, torch.where(lz, g, ag)

    line_aware = getattr(fg, "line_aware", False)

    def evaluate(x, line=None):
        # line = (x, d, a) of a trial x + a d: a line-aware fg may combine its passes along the line
        v, g = fg(x, line) if (line_aware and line is not None) else fg(x)
        av, ag = adjust(x, g, v)
        return v, g, av, ag

    def apply(st, grad):
        d = grad.clone()
        diag = sy0 = None
        if hist_s:
            sy0 = torch.dot(hist_s[0], hist_y[0])
            diag = sy0 / torch.dot(hist_y[0], hist_y[0])
        rho, alphas = [], []
        for s, y in zip(hist_s, hist_y):
            r = torch.dot(s, y)
            a = torch.dot(s, d) / r
            d = d - a * y
            rho.append(r)
            alphas.append(a)
        if diag is not None:
            d = d * diag
        for i in range(len(hist_s) - 1, -1, -1):
            beta = torch.dot(hist_y[i], d) / rho[i]
            d = d + (alphas[i] - beta) * hist_s[i]
        if sy0 is not None:  # one host read for the NaN / negative-curvature exceptions
            chk = torch.stack([sy0] + alphas).tolist()
            if chk[0] < 0 or np.isnan(chk[0]) or any(np.isnan(v) for v in chk[1:]):
                raise _FirstOrderError("NaNHistory")
        return -d

    def take_step(st, d, a):
        nx = st.x + d * a
        if owlqn:
            orth = torch.where(st.x != 0, torch.sign(st.x), torch.sign(-st.adj_grad))
            nx = torch.where(torch.sign(nx) != orth, torch.zeros_like(nx), nx)
        return nx

    def phi(st, d, a):
        """(value, directional derivative) at step a as host floats; a = 0 is the cached state."""
        if a == 0.0:
            dd = torch.dot(st.adj_grad if owlqn else st.grad, d)
            return (st.adj_h if owlqn else st.value_h), float(dd)
        nx = take_step(st, d, a)
        v, g, av, ag = evaluate(nx, None if owlqn else (st.x, d, a))
        f, dd = torch.stack([av if owlqn else v, torch.dot(ag if owlqn else g, d)]).tolist()
        last.clear()
        last.update(a=a, x=nx, v=v, g=g, av=av, ag=ag)
        return f, dd

    def backtracking(st, d):
        initfval = st.adj_h
        shrink, grow, c1, c2 = (0.1 if st.iter < 1 else 0.5), 2.1, 1e-4, 0.9
        _, initd = phi(st, d, 0.0)
        alpha = 0.5 / float(torch.linalg.vector_norm(st.grad)) if st.iter < 1 else 1.0
        fv, fd = phi(st, d, alpha)
        it = 0
        while True:
            if fv > initfval + alpha * initd * c1:
                mult = shrink
            elif fd < c2 * initd:
                mult = grow
            elif fd > -c2 * initd:
                mult = shrink
            else:
                mult = 1.0
            if mult == 1.0:
                return alpha
            na = alpha * mult
            if it >= 20:
                raise _FirstOrderError("LineSearchFailed")
            if na < 1e-10:
                raise _FirstOrderError("StepSizeUnderflow")
            if na > 1e10:
                raise _FirstOrderError("StepSizeOverflow")
            alpha = na
            fv, fd = phi(st, d, alpha)
            if it + 1 >= 20:
                return alpha  # takeWhile(iter < maxIterations) keeps the last state
            it += 1

    def strong_wolfe(st, d):
        c1, c2 = 1e-4, 0.9
        f0, d0 = phi(st, d, 0.0)
        t = 1.0 / float(torch.linalg.vector_norm(d)) if st.iter == 0 else 1.0
        if d0 > 0:
            raise _FirstOrderError("Line search invoked with non-descent direction")
        low = (0.0, d0, f0)  # (t, dd, f)

        def ev(tt):
            f, dd = phi(st, d, tt)
            return (tt, dd, f)

        def interp(lo, hi):
            d1 = lo[1] + hi[1] - 3 * (lo[2] - hi[2]) / (lo[0] - hi[0])
            d2 = np.sqrt(d1 * d1 - lo[1] * hi[1])
            mul = hi[0] - lo[0]
            tt = hi[0] - mul * (hi[1] + d2 - d1) / (hi[1] - lo[1] + 2 * d2)
            lb, ub = lo[0] + 0.1 * mul, lo[0] + 0.9 * mul
            return lb if tt < lb else (ub if tt > ub else tt)

        def zoom(lo, hi):
            for _ in range(10):
                tt = interp(hi, lo) if lo[0] > hi[0] else interp(lo, hi)
                c = ev(tt)
                if c[2] > f0 + c1 * c[0] * d0 or c[2] >= lo[2]:
                    hi = c
                else:
                    if abs(c[1]) <= c2 * abs(d0):
                        return c[0]
                    if c[1] * (hi[0] - lo[0]) >= 0:
                        hi = lo
                    lo = c
            raise _FirstOrderError("Line search zoom failed")

        for i in range(10):
            c = ev(t)
            if not np.isfinite(c[2]):
                t /= 2.0
                continue
            if c[2] > f0 + c1 * t * d0 or (c[2] >= low[2] and i > 0):
                return zoom(low, c)
            if abs(c[1]) <= c2 * abs(d0):
                return c[0]
            if c[1] >= 0:
                return zoom(c, low)
            low = c
            t *= 1.5
        raise _FirstOrderError("Line search failed")

    st = _State()
    if resume is not None:
        dev = x0.device
        st.x = torch.as_tensor(resume["x"], device=dev)
        st.value, st.grad, st.adj_value, st.adj_grad = (torch.as_tensor(resume[k], device=dev)
                                                        for k in ("value", "grad", "adj_value", "adj_grad"))
        st.value_h, st.adj_h, st.gnorm = (float(resume[k]) for k in ("value_h", "adj_h", "gnorm"))
        st.iter = int(resume["iter"])
        hist_s[:] = [torch.as_tensor(v, device=dev) for v in resume["S"]]
        hist_y[:] = [torch.as_tensor(v, device=dev) for v in resume["Y"]]
        fvals = list(resume["fvals"])
        history = list(resume["history"])
        initial_adj = float(resume["initial_adj"])
        search_failed, failed_once = bool(resume["search_failed"]), bool(resume["failed_once"])
    else:
        st.x = x0  # never modified in place (every step builds a new tensor): a line-aware fg may key on it
        st.value, st.grad, st.adj_value, st.adj_grad = evaluate(st.x)
        st.value_h, st.adj_h, st.gnorm = torch.stack([st.value, st.adj_value,
                                                      torch.linalg.vector_norm(st.adj_grad)]).tolist()
        st.iter = 0
        initial_adj = st.adj_h
        fvals = [float("inf")]
        history = [st.adj_h]
        search_failed, failed_once = False, False

    def converged():
        if max_iter >= 0 and st.iter >= max_iter:
            return 0
        if len(fvals) >= 2 and abs(st.adj_h - max(fvals)) <= tol * abs(initial_adj):
            return 1
        if st.gnorm <= max(tol * abs(st.value_h), 1e-8):
            return 2
        if search_failed:
            return 3
        return -1

    why = converged()
    while why < 0:
        try:
            d = apply(st, st.adj_grad if owlqn else st.grad)
            if owlqn:
                d = torch.where(d * st.adj_grad < 0, d, torch.zeros_like(d))
                step = backtracking(st, d)
            else:
                step = strong_wolfe(st, d)
                if step * float(torch.linalg.vector_norm(st.grad)) < 1e-10:
                    raise _FirstOrderError("StepSizeUnderflow")
            if last.get("a") == step:
                nx, v, g, av, ag = last["x"], last["v"], last["g"], last["av"], last["ag"]
            else:
                nx = take_step(st, d, step)
                v, g, av, ag = evaluate(nx, None if owlqn else (st.x, d, step))
            hist_s.insert(0, nx - st.x)
            hist_y.insert(0, g - st.grad)
            del hist_s[memory:], hist_y[memory:]
            v_h, av_h, gn = torch.stack([v, av, torch.linalg.vector_norm(ag)]).tolist()
            fvals.append(v_h)
            del fvals[:-_FVAL_MEMORY]
            st.x, st.value, st.grad, st.adj_value, st.adj_grad = nx, v, g, av, ag
            st.value_h, st.adj_h, st.gnorm = v_h, av_h, gn
            st.iter += 1
            failed_once = False
        except _FirstOrderError:
            if not failed_once:
                failed_once = True
                hist_s.clear()
                hist_y.clear()
            else:
                search_failed = True
        last.clear()
        history.append(st.adj_h)
        why = converged()
        if on_iteration is not None and why < 0:
            on_iteration({"x": st.x, "value": st.value, "grad": st.grad, "adj_value": st.adj_value,
                          "adj_grad": st.adj_grad, "value_h": st.value_h, "adj_h": st.adj_h, "gnorm": st.gnorm,
                          "iter": st.iter, "S": list(hist_s), "Y": list(hist_y), "fvals": list(fvals),
                          "history": list(history), "initial_adj": initial_adj, "search_failed": search_failed,
                          "failed_once": failed_once})
    return st.x, history, REASONS[why]
