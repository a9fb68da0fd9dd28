"""Bound-constrained L-BFGS (L-BFGS-B) with the semantics of Breeze 0.13's ``LBFGSB`` -- the
optimizer Spark 2.4.4 runs for ``LinearRegression(loss="huber")`` (``new BreezeLBFGSB(lower,
upper, maxIter, 10, tol)``; the estimator surface the reference configures at
``DataQuality4MachineLearningApp.java:120-123``).

The algorithm is Byrd, Lu, Nocedal & Zhu (1995) in the compact limited-memory representation
B = θI - W M Wᵀ (W = [Y, θS], M = [[-D, Lᵀ], [L, θSᵀS]]⁻¹), as Breeze implements it:

* direction: the generalized Cauchy point along the projected steepest-descent path (breakpoints
  sorted, piecewise quadratic minimized segment by segment); on the first iteration the step to
  the Cauchy point itself, afterwards the direct primal subspace minimization over the variables
  the Cauchy point leaves free (Breeze's ``findAlpha`` always returns 1 -- its max(a, min(b, a))
  -- so the subspace step is taken whole and then projected onto the box);
* step: Breeze's ``StrongWolfeLineSearch(maxZoomIter = 64, maxLineSearchIter = 64)`` from t = 1
  on the UNPROJECTED ray x + t d (``LineSearch.functionFromSearchDirection``); the accepted point
  is projected (``adjustWithinBound``);
* memory: a pair is kept when |sᵀy| > ε yᵀy; θ = yᵀy / sᵀy;
* convergence: ``||P(x - g) - x||_inf <= 1e-5`` (ProjectedStepConverged) || max iterations ||
  |f - max(last 20 f)| <= tol |f0| || ||g|| <= max(tol |f|, 1e-8) || a search failed twice (the
  first ``FirstOrderException`` resets the memory, as ``FirstOrderMinimizer`` does);
* ``objectiveHistory``: the value of every state of the iterator, the initial one included.

Only the optimizer's O(k m) bookkeeping lives here; every cost evaluation is the caller's (for
Huber: one fused device pass + one (d + 4)-f64 all-reduce, ``models/huber.py``).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, List, Optional, Tuple

import numpy as np

__all__ = ["LBFGSB", "LBFGSBState", "FirstOrderException"]

_EPS = 2.2e-16
PROJ_GRADIENT_EPS = 1e-5


class FirstOrderException(RuntimeError):
    """A line-search failure (Breeze ``FirstOrderException``): the first resets the memory."""


@dataclass
class LBFGSBState:
    x: np.ndarray
    value: float
    grad: np.ndarray
    iter: int
    initial_value: float
    theta: float = 1.0
    S: List[np.ndarray] = field(default_factory=list)  # oldest first
    Y: List[np.ndarray] = field(default_factory=list)
    fvals: List[float] = field(default_factory=lambda: [np.inf])  # FunctionValuesConverged info
    failed_once: bool = False
    search_failed: bool = False


class LBFGSB:
    def __init__(self, lower: np.ndarray, upper: np.ndarray, max_iter: int = 100, m: int = 5,
                 tolerance: float = 1e-8, max_zoom_iter: int = 64, max_line_search_iter: int = 64):
        self.lower = np.asarray(lower, dtype=np.float64)
        self.upper = np.asarray(upper, dtype=np.float64)
        self.max_iter, self.m, self.tol = int(max_iter), int(m), float(tolerance)
        self.max_zoom_iter, self.max_ls_iter = int(max_zoom_iter), int(max_line_search_iter)

    # ---- compact representation -----------------------------------------------------------
    def _WM(self, st: LBFGSBState) -> Tuple[np.ndarray, np.ndarray]:
        n = st.x.size
        if not st.S:
            return np.zeros((n, 0)), np.zeros((0, 0))
        S = np.stack(st.S, axis=1)
        Y = np.stack(st.Y, axis=1)
        W = np.concatenate([Y, S * st.theta], axis=1)
        A = S.T @ Y
        L = np.tril(A, -1)
        D = -np.diag(np.diag(A))
        MM = np.block([[D, L.T], [L, (S.T @ S) * st.theta]])
        return W, np.linalg.inv(MM)

    def _clamp(self, p: np.ndarray) -> np.ndarray:
        return np.minimum(np.maximum(p, self.lower), self.upper)

    def _cauchy_point(self, st: LBFGSBState, W: np.ndarray, M: np.ndarray):
        x, g, theta = st.x, st.grad, st.theta
        n = x.size
        with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
            # breakpoint of every coordinate along -g (Double.MaxValue where g_i = 0)
            t = np.where(g < 0, (x - self.upper) / g, (x - self.lower) / g)
            t = np.where(g == 0.0, np.finfo(np.float64).max, t)
        d = np.where((g != 0.0) & (t != 0.0), -g, 0.0)
        p = W.T @ d
        c = np.zeros(M.shape[0])
        f1 = np.float64(g @ d)
        f2 = np.float64(-theta * f1 - float(p @ (M @ p)))
        with np.errstate(divide="ignore", invalid="ignore"):
            dt_min = -(f1 / f2)
        old_t = 0.0
        order = np.argsort(t, kind="stable")  # (a stable sort, as Scala's sortWith)
        nz = np.nonzero(t[order] != 0.0)[0]
        i = int(nz[0])  # (Breeze: indexWhere(t != 0))
        b = order[i]
        min_t = t[b]
        delta_t = min_t - old_t
        xc = x.copy()
        while delta_t <= dt_min and i < n:
            xc[b] = self.upper[b] if d[b] > 0 else self.lower[b]
            zb = xc[b] - x[b]
            c = c + p * delta_t
            gb = g[b]
            wb = W[b, :]
            f1 += delta_t * f2 + gb * gb + theta * gb * zb - gb * float(wb @ (M @ c))
            f2 += -theta * gb * gb - 2.0 * (gb * float(wb @ (M @ p))) - gb * gb * float(wb @ (M @ wb))
            p = p + wb * gb
            d[b] = 0.0
            with np.errstate(divide="ignore", invalid="ignore"):
                dt_min = -np.float64(f1) / np.float64(f2)
            old_t = min_t
            i += 1
            if i < n:
                b = order[i]
                min_t = t[b]
                delta_t = min_t - old_t
        dt_min = max(dt_min, 0.0)
        old_t += dt_min
        rest = order[i:]
        xc[rest] = x[rest] + old_t * d[rest]
        c = c + p * dt_min
        return xc, c

    def _subspace_min(self, st: LBFGSBState, W, M, xc: np.ndarray, c: np.ndarray) -> np.ndarray:
        inv_theta = 1.0 / st.theta
        free = np.nonzero((xc != self.upper) & (xc != self.lower))[0]
        WZ = W[free, :].T
        r = st.grad + (xc - st.x) * st.theta - W @ (M @ c)
        rc = r[free]
        v = M @ (WZ @ rc)
        N = np.eye(M.shape[0]) - M @ ((WZ @ WZ.T) * inv_theta)
        if v.size:
            v = np.linalg.solve(N, v)
        du = -(rc * inv_theta + (WZ.T @ v) * (inv_theta * inv_theta))
        out = xc.copy()
        out[free] = xc[free] + du  # findAlpha: 1.0
        return out

    def _direction(self, st: LBFGSBState) -> np.ndarray:
        W, M = self._WM(st)
        xc, c = self._cauchy_point(st, W, M)
        xc = self._clamp(xc)
        if st.iter == 0:
            return xc - st.x
        return self._clamp(self._subspace_min(st, W, M, xc, c)) - st.x

    # ---- Breeze StrongWolfeLineSearch -------------------------------------------------------
    def _line_search(self, fg, x: np.ndarray, direction: np.ndarray) -> float:
        c1, c2 = 1e-4, 0.9

        def phi(t):
            f, g = fg(x + direction * t)
            return t, float(g @ direction), float(f)

        t = 1.0
        low = phi(0.0)
        f0, d0 = low[2], low[1]
        if d0 > 0:
            raise FirstOrderException(f"Line search invoked with non-descent direction: {d0}")

        def interp(l, r):
            d1 = l[1] + r[1] - 3 * (l[2] - r[2]) / (l[0] - r[0])
            d2 = np.sqrt(d1 * d1 - l[1] * r[1])
            mul = r[0] - l[0]
            tt = r[0] - mul * (r[1] + d2 - d1) / (r[1] - l[1] + 2 * d2)
            lb, ub = l[0] + 0.1 * mul, l[0] + 0.9 * mul
            return lb if tt < lb else (ub if tt > ub else tt)

        def zoom(lo, hi):
            for _ in range(self.max_zoom_iter):
                tt = interp(hi, lo) if lo[0] > hi[0] else interp(lo, hi)
                cc = phi(tt)
                if cc[2] > f0 + c1 * cc[0] * d0 or cc[2] >= lo[2]:
                    hi = cc
                else:
                    if abs(cc[1]) <= c2 * abs(d0):
                        return cc[0]
                    if cc[1] * (hi[0] - lo[0]) >= 0:
                        hi = lo
                    lo = cc
            raise FirstOrderException("Line search zoom failed")

        for i in range(self.max_ls_iter):
            cc = phi(t)
            if not np.isfinite(cc[2]):
                t /= 2.0
                continue
            if cc[2] > f0 + c1 * t * d0 or (cc[2] >= low[2] and i > 0):
                return zoom(low, cc)
            if abs(cc[1]) <= c2 * abs(d0):
                return cc[0]
            if cc[1] >= 0:
                return zoom(cc, low)
            low = cc
            t *= 1.5
        raise FirstOrderException("Line search failed")

    # ---- FirstOrderMinimizer ------------------------------------------------------------------
    def converged(self, st: LBFGSBState) -> Optional[str]:
        pmx = self._clamp(st.x - st.grad) - st.x
        if np.max(np.abs(pmx), initial=0.0) <= PROJ_GRADIENT_EPS:
            return "projected step converged"
        if self.max_iter >= 0 and st.iter >= self.max_iter:
            return "max iterations"
        if len(st.fvals) >= 2 and abs(st.value - max(st.fvals)) <= self.tol * abs(st.initial_value):
            return "function values converged"
        if np.linalg.norm(st.grad) <= max(self.tol * abs(st.value), 1e-8):
            return "gradient converged"
        if st.search_failed:
            return "search failed"
        return None

    def initial_state(self, fg, x0: np.ndarray) -> LBFGSBState:
        x0 = np.asarray(x0, dtype=np.float64).copy()
        f, g = fg(x0)
        return LBFGSBState(x0, float(f), np.asarray(g, dtype=np.float64), 0, float(f))

    def step(self, fg, st: LBFGSBState) -> LBFGSBState:
        """One iteration of ``FirstOrderMinimizer.infiniteIterations``."""
        try:
            direction = self._direction(st)
            t = self._line_search(fg, st.x, direction)
            x = self._clamp(st.x + direction * t)
            f, g = fg(x)
            g = np.asarray(g, dtype=np.float64)
            s, y = x - st.x, g - st.grad
            S, Y, theta = list(st.S), list(st.Y), st.theta
            if _EPS * float(y @ y) < abs(float(s @ y)):
                S.append(s)
                Y.append(y)
                if len(S) > self.m:
                    S.pop(0)
                    Y.pop(0)
                theta = float(y @ y) / float(s @ y)
            fvals = (st.fvals + [float(f)])[-20:]
            return LBFGSBState(x, float(f), g, st.iter + 1, st.initial_value, theta, S, Y, fvals, False, False)
        except FirstOrderException:
            if not st.failed_once:  # reset the memory (initialHistory) and try again
                return LBFGSBState(st.x, st.value, st.grad, st.iter, st.initial_value, 1.0, [], [], st.fvals, True,
                                   False)
            return LBFGSBState(st.x, st.value, st.grad, st.iter, st.initial_value, st.theta, st.S, st.Y, st.fvals,
                               st.failed_once, True)

    def minimize(self, fg: Callable, x0: np.ndarray, state: Optional[LBFGSBState] = None,
                 on_state: Optional[Callable] = None):
        """Iterate from ``x0`` (or a resumed ``state``) until converged.  Returns ``(state,
        objective_history, reason)`` (the history from the start state on); ``on_state(state,
        history)`` sees every new state before its convergence check (checkpoints)."""
        st = state if state is not None else self.initial_state(fg, x0)
        hist = [st.value]
        why = self.converged(st)
        while why is None:
            st = self.step(fg, st)
            hist.append(st.value)
            if on_state is not None:
                on_state(st, hist)
            why = self.converged(st)
        return st, hist, why
