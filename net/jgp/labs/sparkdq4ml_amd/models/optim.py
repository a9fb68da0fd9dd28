"""WeightedLeastSquares: aggregated sufficient statistics -> standardized normal equations ->
Cholesky / OWLQN / L-BFGS -> coefficients in the original space.

Mirrors the behaviour of Spark 2.4.4 ``WeightedLeastSquares.fit`` as used by
``LinearRegression.fit`` at ``DataQuality4MachineLearningApp.java:126``: population
std, ``effectiveRegParam = regParam / bStd``, L2 on the standardized diagonal, L1 via OWLQN with an
unpenalized intercept, Cholesky fallback to quasi-Newton on a singular system, constant-label
short-circuit.  The statistics come from the device Gram kernels (``ops.kernels.gram_stats``) and
are already all-reduced across ranks; the solve itself is the native f64 host library
(``_dq4ml_host``) for k <= ``DEVICE_SOLVE_MIN_K`` and torch-on-device f64 above.
"""
from __future__ import annotations

import functools
from dataclasses import dataclass
from typing import Optional

import numpy as np

from ..ops import native
from ..utils.logging import get_logger

__all__ = ["GramStats", "WLSModel", "weighted_least_squares", "SingularMatrixException"]

log = get_logger("optim")
MAX_NUM_FEATURES = 4096
DEVICE_SOLVE_MIN_K = 1025


class SingularMatrixException(RuntimeError):
    pass


@dataclass
class GramStats:
    """Sufficient statistics of the (weighted) normal equations (Spark's WLS ``Aggregator``)."""

    k: int
    count: float
    wSum: float
    wwSum: float
    bSum: float
    bbSum: float
    aSum: np.ndarray
    abSum: np.ndarray
    aaSum: np.ndarray  # packed upper, column-major, length k(k+1)/2

    @staticmethod
    def layout_size(k: int) -> int:
        return 5 + 2 * k + k * (k + 1) // 2

    @classmethod
    def from_flat(cls, flat: np.ndarray, k: int) -> "GramStats":
        flat = np.asarray(flat, dtype=np.float64)
        assert flat.shape[0] == cls.layout_size(k), (flat.shape, k)
        return cls(k, flat[0], flat[1], flat[2], flat[3], flat[4], flat[5:5 + k].copy(),
                   flat[5 + k:5 + 2 * k].copy(), flat[5 + 2 * k:].copy())

    # derived (Aggregator accessors)
    @property
    def aBar(self):
        return self.aSum / self.wSum

    @property
    def bBar(self):
        return self.bSum / self.wSum

    @property
    def bbBar(self):
        return self.bbSum / self.wSum

    @property
    def bStd(self):
        return float(np.sqrt(max(self.bbSum / self.wSum - self.bBar ** 2, 0.0)))

    @property
    def abBar(self):
        return self.abSum / self.wSum

    @property
    def aaBar(self):
        return self.aaSum / self.wSum

    def diag_aa(self):
        return self.aaSum[_packed_diag_index(self.k)]

    @property
    def aStd(self):
        aw = self.aSum / self.wSum
        return np.sqrt(np.maximum(self.diag_aa() / self.wSum - aw * aw, 0.0))

    @property
    def aVar(self):
        aw = self.aSum / self.wSum
        return np.maximum(self.diag_aa() / self.wSum - aw * aw, 0.0)


class WLSModel:
    """Solution of the normal equations.  ``diagInvAtWA`` (needed only for the summary's standard
    errors) is computed lazily from the retained system: the fit itself never pays for the
    O(k^3) inverse."""

    def __init__(self, coefficients, intercept, diag_inv, objective_history, solver):
        self.coefficients = coefficients
        self.intercept = intercept
        self._diag_inv = diag_inv
        self.objectiveHistory = objective_history
        self.solver = solver

    @property
    def diagInvAtWA(self) -> np.ndarray:
        if callable(self._diag_inv):
            self._diag_inv = self._diag_inv()
        return self._diag_inv


@functools.lru_cache(maxsize=64)
def _packed_diag_index(k):
    return np.array([j + j * (j + 1) // 2 for j in range(k)], dtype=np.int64)


def _solve_cholesky(k, aa, ab):
    """-> (x, callable returning the packed inverse)."""
    h = native.host()
    if k >= DEVICE_SOLVE_MIN_K:
        return _device_cholesky(k, aa, ab)
    try:
        x = h.cholesky_solve(k, aa, ab)
    except h.SingularMatrixError as e:
        raise SingularMatrixException(str(e)) from None
    return x, (lambda: h.cholesky_inverse(k, aa))


@functools.lru_cache(maxsize=64)
def packed_upper_indices(k):
    """(row, col) of every entry of a packed upper column-major matrix, in storage order."""
    J = np.repeat(np.arange(k), np.arange(1, k + 1))
    I = np.concatenate([np.arange(j + 1) for j in range(k)]) if k else np.zeros(0, np.int64)
    return I, J


def _device_cholesky(k, aa, ab):
    """Large-k path: f64 Cholesky on the GPU (rocSOLVER via torch.linalg)."""
    import torch

    dev = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
    I, J = (torch.as_tensor(v, device=dev) for v in packed_upper_indices(k))
    ap = torch.as_tensor(aa, dtype=torch.float64, device=dev)
    m = torch.zeros(k, k, dtype=torch.float64, device=dev)
    m[I, J] = ap
    m[J, I] = ap
    L, info = torch.linalg.cholesky_ex(m)
    if int(info.item()) != 0:
        raise SingularMatrixException("LAPACK.dppsv returned a non-positive pivot: A is not positive definite.")
    x = torch.cholesky_solve(torch.as_tensor(ab, dtype=torch.float64, device=dev).unsqueeze(1), L).squeeze(1)
    # (AᵀA)⁻¹ only when the summary asks for standard errors (lazy diagInvAtWA)
    return x.cpu().numpy(), (lambda: torch.cholesky_inverse(L)[I, J].cpu().numpy())


def weighted_least_squares(stats: GramStats, fit_intercept: bool, reg_param: float, elastic_net: float,
                           standardize_features: bool, standardize_label: bool, solver_type: str,
                           max_iter: int, tol: float) -> WLSModel:
    """``WeightedLeastSquares.fit`` on pre-aggregated statistics (solver_type: auto|cholesky|quasi-newton)."""
    if reg_param == 0.0:
        log.warning("regParam is zero, which might cause numerical instability and overfitting.")
    if stats.wSum <= 0.0:
        raise ValueError("Sum of weights cannot be zero." if stats.count > 0 else "Training dataset is empty.")
    nf = stats.k
    k = nf + 1 if fit_intercept else nf
    rawBStd, rawBBar = stats.bStd, stats.bBar
    bStd = abs(rawBBar) if rawBStd == 0.0 else rawBStd
    if rawBStd == 0.0:
        if fit_intercept or rawBBar == 0.0:
            if rawBBar == 0.0:
                log.warning("Mean and standard deviation of the label are zero, so the coefficients and the "
                            "intercept will all be zero; as a result, training is not needed.")
            else:
                log.warning("The standard deviation of the label is zero, so the coefficients will be zeros and "
                            "the intercept will be the mean of the label; as a result, training is not needed.")
            return WLSModel(np.zeros(nf), rawBBar, np.zeros(1), np.zeros(1), "none")
        if reg_param > 0.0 and standardize_label:
            raise ValueError("The standard deviation of the label is zero. Model cannot be regularized with "
                             "standardization=true")
        log.warning("The standard deviation of the label is zero. Consider setting fitIntercept=true.")

    bBar = rawBBar / bStd
    bbBar = stats.bbBar / (bStd * bStd)
    aStd = stats.aStd
    safe = np.where(aStd == 0.0, 1.0, aStd)
    aBar = np.where(aStd == 0.0, 0.0, stats.aBar / safe)
    abBar = np.where(aStd == 0.0, 0.0, stats.abBar / (safe * bStd))
    aaBar = stats.aaBar.copy()
    ii, jj = packed_upper_indices(nf)
    denom = aStd[ii] * aStd[jj]
    aaBar = np.where(denom == 0.0, 0.0, aaBar / np.where(denom == 0.0, 1.0, denom))

    eff_reg = reg_param / bStd
    eff_l1 = elastic_net * eff_reg
    eff_l2 = (1.0 - elastic_net) * eff_reg
    diag = _packed_diag_index(nf)
    lam = np.full(nf, eff_l2)
    if not standardize_features:
        lam = np.where(aStd != 0.0, lam / np.where(aStd == 0, 1.0, aStd * aStd), 0.0)
    if not standardize_label:
        lam = lam * bStd
    aaBar[diag] += lam

    def get_ata():
        return np.concatenate([aaBar, aBar, [1.0]]) if fit_intercept else aaBar.copy()

    def get_atb():
        return np.concatenate([abBar, [bBar]]) if fit_intercept else abBar.copy()

    use_qn = (solver_type == "auto" and elastic_net != 0.0 and reg_param != 0.0) or solver_type == "quasi-newton"
    h = native.host()
    aa_inv = None
    history = np.zeros(1)
    if use_qn:
        l1 = None
        if eff_l1 != 0.0:
            if standardize_features:
                l1 = np.full(k, eff_l1)
            else:
                l1 = np.concatenate([np.where(aStd != 0.0, eff_l1 / np.where(aStd == 0, 1.0, aStd), 0.0),
                                     [0.0] if fit_intercept else []])
            if fit_intercept:
                l1[nf] = 0.0
        x, history, reason = h.quasi_newton(bBar, bbBar, get_atb(), get_ata(), aBar, fit_intercept, max_iter, tol, l1)
        used = "owlqn" if l1 is not None else "l-bfgs"
        log.info("quasi-newton converged: %s after %d states", reason, len(history))
    else:
        try:
            x, aa_inv = _solve_cholesky(k, get_ata(), get_atb())
            used = "cholesky"
        except SingularMatrixException:
            if solver_type != "auto":
                raise
            log.warning("Cholesky solver failed due to singular covariance matrix. Retrying with Quasi-Newton solver.")
            x, history, reason = h.quasi_newton(bBar, bbBar, get_atb(), get_ata(), aBar, fit_intercept, max_iter,
                                                tol, None)
            used = "l-bfgs"
    x = np.asarray(x, dtype=np.float64)
    if fit_intercept:
        coef, intercept = x[:nf].copy(), float(x[nf] * bStd)
    else:
        coef, intercept = x.copy(), 0.0
    coef = coef * np.where(aStd != 0.0, bStd / np.where(aStd == 0, 1.0, aStd), 0.0)
    if aa_inv is not None:
        inv_fn, wsum = aa_inv, stats.wSum

        def diag_inv():
            inv = inv_fn()
            d = []
            for i in range(1, k + 1):
                mult = 1.0 if (i == k and fit_intercept) else aStd[i - 1] * aStd[i - 1]
                d.append(inv[i + (i - 1) * i // 2 - 1] / (wsum * mult))
            return np.array(d)
    else:
        diag_inv = np.zeros(1)
    return WLSModel(coef, intercept, diag_inv, np.asarray(history, dtype=np.float64), used)


_ = Optional
