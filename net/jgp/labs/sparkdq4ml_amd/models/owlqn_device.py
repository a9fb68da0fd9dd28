"""OWLQN (L1 / elastic-net WLS, the lab's own ``setRegParam(1).setElasticNetParam(1)`` at
``DataQuality4MachineLearningApp.java:120-126``) with the standardized normal equations kept on
the device.

Two engines, one algorithm -- the Breeze 0.13 OWLQN of Spark 2.4.4 exactly as the native host
driver implements it (``ops/csrc/host/solvers.cpp``: L-BFGS two-loop on the pseudo-gradient,
orthant projection, backtracking line search seeded with 0.5/|g| on the first iteration,
FunctionValuesConverged over the last 20 values, one history reset on a failed search):

* ``k <= 128``: ONE wave runs the whole solve (``ops/csrc/hip/wls_small.hip``,
  ``wls_qn_kernel``) -- no host round trip, so an L1 fit can be asynchronous;
* ``128 < k <= QN_DEVICE_MAX_K`` (4608): ONE cooperative grid launch, one block per CU
  (``ops/csrc/hip/wls_qn_grid.hip``): the dense standardized system in HBM, row panels per block,
  one grid barrier per cost evaluation with every block taking the same line-search decisions --
  no host round trip either, so these fits are asynchronous too;
* this module's torch version (``DQ4ML_QN_ENGINE=torch``, kept for A/B): vectors and the dense
  k x k system stay in HBM, every cost evaluation is one f64 GEMV there, and the scalars that
  steer the line search cross to the host on every evaluation.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch

__all__ = ["standardized_system", "owlqn_torch", "solve_owlqn_device", "QN_SMALL_MAX_K", "QN_DEVICE_MAX_K",
           "QN_TORCH_MIN_K", "qn_engine"]

QN_SMALL_MAX_K = 128
QN_DEVICE_MAX_K = 4608  # kWlsQnGridMaxK (wls_small.h)


def qn_engine() -> str:
    """``hip`` (default: the one-wave / grid HIP solvers) or ``torch`` (host-steered, A/B)."""
    import os

    return "torch" if os.environ.get("DQ4ML_QN_ENGINE", "hip") == "torch" else "hip"
# device-resident torch engine from this k on (scripts/owlqn_bench.py, 1x MI355X, L1 = 0.01:
# k = 1025 device 12.1 ms vs host 6.3 ms; k = 4097 device 22.4 ms vs host 267 ms)
QN_TORCH_MIN_K = 2048
_FVAL_MEMORY = 20
_REASONS = ("max iterations", "function values converged", "gradient converged", "search failed")


class _FirstOrderError(Exception):
    pass


def standardized_system(flat: torch.Tensor, nf: int, fit_intercept: bool, reg: float, enet: float,
                        std_f: bool, std_l: bool):
    """WLS standardization on the device (same algebra as ``wls.cpp``).  Returns None for the
    label short-circuits (the native driver owns their semantics), else a dict with the dense
    standardized ``A`` (k x k), ``atb``, ``l1`` (k,), ``aBar``/``aStd`` (nf,) and the scalars."""
    from .optim import _packed_diag_index, packed_upper_indices

    dev = flat.device
    head = flat[:5].double().cpu().tolist()
    count, wSum, _, bSum, bbSum = head
    if wSum <= 0.0:
        return None
    rawBBar = bSum / wSum
    rawBStd = float(np.sqrt(max(bbSum / wSum - rawBBar * rawBBar, 0.0)))
    if rawBStd == 0.0:
        return None
    bStd = rawBStd
    I, J = (torch.as_tensor(v, device=dev) for v in packed_upper_indices(nf))
    dj = torch.as_tensor(_packed_diag_index(nf), device=dev)
    aSum, abSum, aaP = flat[5:5 + nf], flat[5 + nf:5 + 2 * nf], flat[5 + 2 * nf:]
    m = aSum / wSum
    aStd = torch.sqrt(torch.clamp(aaP[dj] / wSum - m * m, min=0.0))
    nz = aStd != 0.0
    safe = torch.where(nz, aStd, torch.ones_like(aStd))
    aBar = torch.where(nz, m / safe, torch.zeros_like(m))
    abBar = torch.where(nz, abSum / wSum / (safe * bStd), torch.zeros_like(m))
    den = aStd[I] * aStd[J]
    vals = torch.where(den != 0.0, aaP / wSum / torch.where(den != 0.0, den, torch.ones_like(den)),
                       torch.zeros_like(den))
    k = nf + 1 if fit_intercept else nf
    A = torch.zeros(k, k, dtype=torch.float64, device=dev)
    A[I, J] = vals
    A[J, I] = vals
    eff_reg = reg / bStd
    eff_l1, eff_l2 = enet * eff_reg, (1.0 - enet) * eff_reg
    lam = torch.full((nf,), eff_l2, dtype=torch.float64, device=dev)
    if not std_f:
        lam = torch.where(nz, lam / (safe * safe), torch.zeros_like(lam))
    if not std_l:
        lam = lam * bStd
    ar = torch.arange(nf, device=dev)
    A[ar, ar] += lam
    bBar = rawBBar / bStd
    atb = abBar
    if fit_intercept:
        A[:nf, nf] = aBar
        A[nf, :nf] = aBar
        A[nf, nf] = 1.0
        atb = torch.cat([abBar, torch.tensor([bBar], dtype=torch.float64, device=dev)])
    l1 = torch.full((k,), eff_l1, dtype=torch.float64, device=dev)
    if not std_f:
        l1[:nf] = torch.where(nz, eff_l1 / safe, torch.zeros_like(safe))
    if fit_intercept:
        l1[nf] = 0.0
    return {"A": A, "atb": atb, "l1": l1, "aBar": aBar, "aStd": aStd, "bStd": bStd, "bBar": bBar,
            "bbBar": bbSum / wSum / (bStd * bStd), "eff_l1": eff_l1, "k": k, "nf": nf}


def owlqn_torch(bBar: float, bbBar: float, ab: torch.Tensor, A: torch.Tensor, aBar: torch.Tensor,
                fit_intercept: bool, max_iter: int, tol: float, l1: torch.Tensor,
                memory: int = 10) -> Tuple[torch.Tensor, list, str]:
    """Breeze OWLQN on ``f(x) = 1/2 bbBar - x.ab + 1/2 x^T A x`` (intercept re-set to
    ``bBar - coef . aBar`` on every evaluation).  Returns (x, objectiveHistory, reason)."""
    k = ab.numel()
    nf = aBar.numel()
    lz = l1 == 0

    def cost(x):
        x = x.clone()
        if fit_intercept:
            x[nf] = bBar - torch.dot(x[:nf], aBar)
        aax = torch.mv(A, x)
        loss = 0.5 * bbBar - torch.dot(ab, x) + 0.5 * torch.dot(x, aax)
        return x, loss, aax - ab

    def adjust(x, g, v):
        av = v + torch.sum(torch.abs(l1 * x))
        dp, dm = g + l1, g - l1
        at0 = torch.where(dm > 0, dm, torch.where(dp < 0, dp, torch.zeros_like(g)))
        ag = torch.where(x == 0, at0, g + torch.sign(x) * l1)
        return av, torch.where(lz, g, ag)

    hist_s, hist_y = [], []

    def apply(grad):
        d = grad.clone()
        if hist_s:
            sy, yy = torch.dot(hist_s[0], hist_y[0]), torch.dot(hist_y[0], hist_y[0])
            diag = sy / yy
        else:
            sy = diag = None
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
        if sy is not None:  # one host read for the NaN/negative-curvature exceptions
            chk = torch.stack([sy] + alphas).tolist()
            if chk[0] < 0 or np.isnan(chk[0]) or any(np.isnan(v) for v in chk[1:]):
                raise _FirstOrderError("NaNHistory")
        return -d

    def take_step(x, adj_grad, d, a):
        nx = x + d * a
        orth = torch.where(x != 0, torch.sign(x), torch.sign(-adj_grad))
        return torch.where(torch.sign(nx) != orth, torch.zeros_like(nx), nx)

    def phi(x, adj_grad, d, a):
        nx = take_step(x, adj_grad, d, a)
        _, v, g = cost(nx)
        av, ag = adjust(nx, g, v)
        return av, torch.dot(ag, d)

    x = torch.zeros(k, dtype=torch.float64, device=A.device)
    if fit_intercept:
        x[k - 1] = bBar
    x, value, grad = cost(x)
    adj_value, adj_grad = adjust(x, grad, value)
    sc = torch.stack([value, adj_value]).tolist()
    value_h, adj_h = sc
    initial_adj = adj_h
    fvals = [float("inf")]
    it, search_failed, failed_once = 0, False, False
    history = [adj_h]

    def converged():
        if max_iter >= 0 and it >= max_iter:
            return 0
        if len(fvals) >= 2 and abs(adj_h - max(fvals)) <= tol * abs(initial_adj):
            return 1
        if gnorm <= max(tol * abs(value_h), 1e-8):
            return 2
        if search_failed:
            return 3
        return -1

    gnorm = float(torch.linalg.vector_norm(adj_grad))
    why = converged()
    while why < 0:
        try:
            d = apply(adj_grad)
            d = torch.where(d * adj_grad < 0, d, torch.zeros_like(d))
            # backtracking line search (OWLQN)
            initfval = adj_h
            shrink, grow, c1, c2 = (0.1 if it < 1 else 0.5), 2.1, 1e-4, 0.9
            _, initd_t = phi(x, adj_grad, d, 0.0)
            if it < 1:
                alpha = 0.5 / float(torch.linalg.vector_norm(grad))
            else:
                alpha = 1.0
            fv_t, fd_t = phi(x, adj_grad, d, alpha)
            initd, fv, fd = torch.stack([initd_t, fv_t, fd_t]).tolist()
            ls_it = 0
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
                    break
                na = alpha * mult
                if ls_it >= 20:
                    raise _FirstOrderError("LineSearchFailed")
                if na < 1e-10:
                    raise _FirstOrderError("StepSizeUnderflow")
                if na > 1e10:
                    raise _FirstOrderError("StepSizeOverflow")
                alpha = na
                fv_t, fd_t = phi(x, adj_grad, d, alpha)
                fv, fd = torch.stack([fv_t, fd_t]).tolist()
                if ls_it + 1 >= 20:
                    break
                ls_it += 1
            nx = take_step(x, adj_grad, d, alpha)
            nx, v, g = cost(nx)
            av, ag = adjust(nx, g, v)
            hist_s.insert(0, nx - x)
            hist_y.insert(0, g - grad)
            del hist_s[memory:], hist_y[memory:]
            v_h, av_h, gn = torch.stack([v, av, torch.linalg.vector_norm(ag)]).tolist()
            fvals.append(v_h)
            del fvals[:-_FVAL_MEMORY]
            x, value, grad, adj_value, adj_grad = nx, v, g, av, ag
            value_h, adj_h, gnorm = v_h, av_h, gn
            it += 1
            failed_once = False
        except _FirstOrderError:
            if not failed_once:
                failed_once = True
                hist_s.clear()
                hist_y.clear()
            else:
                search_failed = True
        history.append(adj_h)
        why = converged()
    return x, history, _REASONS[why]


def solve_owlqn_device(flat: torch.Tensor, nf: int, fit_intercept: bool, reg: float, enet: float, std_f: bool,
                       std_l: bool, max_iter: int, tol: float) -> Optional[tuple]:
    """(coefficients ndarray, intercept, objectiveHistory ndarray, reason) of the OWLQN branch,
    or None when the native driver must handle the case (label short-circuits, no L1 term)."""
    sysd = standardized_system(flat, nf, fit_intercept, reg, enet, std_f, std_l)
    if sysd is None or sysd["eff_l1"] == 0.0:
        return None
    x, hist, reason = owlqn_torch(sysd["bBar"], sysd["bbBar"], sysd["atb"], sysd["A"], sysd["aBar"], fit_intercept,
                                  max_iter, tol, sysd["l1"])
    aStd, bStd = sysd["aStd"], sysd["bStd"]
    nz = aStd != 0
    coef = torch.where(nz, x[:nf] * bStd / torch.where(nz, aStd, torch.ones_like(aStd)), torch.zeros_like(aStd))
    icpt = float(x[nf]) * bStd if fit_intercept else 0.0
    return coef.cpu().numpy(), icpt, np.asarray(hist, dtype=np.float64), reason
