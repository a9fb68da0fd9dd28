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
        # views, not copies: at k = 4096 the packed block alone is 67 MB
        return cls(k, float(flat[0]), float(flat[1]), float(flat[2]), float(flat[3]), float(flat[4]),
                   flat[5:5 + k], flat[5 + k:5 + 2 * k], flat[5 + 2 * k:])

    @classmethod
    def scalars_only(cls, head, k: int) -> "GramStats":
        """Statistics whose vector parts stayed on the device (large-k device solve)."""
        h = [float(v) for v in head[:5]]
        return cls(k, h[0], h[1], h[2], h[3], h[4], None, None, None)

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


_SOLVER_CODES = {"auto": 0, "cholesky": 1, "quasi-newton": 2}


def fit_wls_flat(flat, nf: int, fit_intercept: bool, reg_param: float, elastic_net: float,
                 standardize_features: bool, standardize_label: bool, solver_type: str, max_iter: int,
                 tol: float, host_only: bool = False):
    """``WeightedLeastSquares.fit`` straight from the (all-reduced) flat statistics.

    Returns ``(WLSModel, GramStats)``.  k <= 1024 (or host statistics): one D2H of the flat vector
    and the native driver ``_dq4ml_host.wls_fit`` (standardize -> Cholesky / OWLQN / L-BFGS ->
    un-standardize in C++).  Larger k with the statistics on the device and no L1 term: the
    standardized system is assembled and Cholesky-solved on the device (f64), only the
    coefficients come back.  ``host_only``: straight to the native driver (the cases a device
    solver handed back: running the device solve again would only repeat its answer)."""
    import torch

    k = nf + 1 if fit_intercept else nf
    if host_only:
        host = flat.detach().cpu().numpy() if torch.is_tensor(flat) else np.asarray(flat, dtype=np.float64)
        stats = GramStats.from_flat(host, nf)
        return _wls_native(host, stats, fit_intercept, reg_param, elastic_net, standardize_features,
                           standardize_label, solver_type, max_iter, tol), stats
    use_qn = (solver_type == "auto" and elastic_net != 0.0 and reg_param != 0.0) or solver_type == "quasi-newton"
    if torch.is_tensor(flat) and flat.is_cuda and use_qn and elastic_net != 0.0 and reg_param != 0.0:
        res = wls_owlqn_device(flat, nf, fit_intercept, reg_param, elastic_net, standardize_features,
                               standardize_label, max_iter, tol)
        if res is not None:
            return res
    if torch.is_tensor(flat) and flat.is_cuda and k >= DEVICE_SOLVE_MIN_K and not use_qn:
        return _wls_device(flat, nf, fit_intercept, reg_param, elastic_net, standardize_features,
                           standardize_label, solver_type, max_iter, tol)
    host = flat.detach().cpu().numpy() if torch.is_tensor(flat) else np.asarray(flat, dtype=np.float64)
    stats = GramStats.from_flat(host, nf)
    return _wls_native(host, stats, fit_intercept, reg_param, elastic_net, standardize_features,
                       standardize_label, solver_type, max_iter, tol), stats


def owlqn_result(host: np.ndarray, nf: int):
    """(WLSModel, GramStats) from the host copy of a ``wls_qn_small`` output, or None when the
    kernel handed the case back (status != 0: label / weight short-circuits, no L1 term)."""
    if int(host[nf + 1]) != 0:
        return None
    H = int(host[nf + 7])
    reason = ("max iterations", "function values converged", "gradient converged", "search failed")[int(host[nf + 8])]
    log.info("quasi-newton converged: %s after %d states", reason, H)
    wls = WLSModel(host[:nf].copy(), float(host[nf]), np.zeros(1), host[nf + 9:nf + 9 + H].copy(), "owlqn")
    return wls, GramStats.scalars_only(host[nf + 2:nf + 7], nf)


QN_DEVICE_MAX_K = 4608  # kWlsQnGridMaxK (wls_small.h): the device OWLQN's largest k


def wls_owlqn_device(flat, nf, fit_intercept, reg_param, elastic_net, standardize_features, standardize_label,
                     max_iter, tol):
    """The OWLQN branch with the statistics on the device: one wave for k <= 128
    (``wls_qn_kernel``), one co-resident grid launch up to ``QN_DEVICE_MAX_K`` (``wls_qn_grid.hip``);
    one D2H of the result.  None = the native host driver owns the case (k beyond the grid
    solver, or a short-circuit the kernel hands back).  (The round-2/3 host-steered torch OWLQN,
    kept for A/B, lost at every k: profiles/r3_owlqn_grid.md; removed in round 4.)"""
    from ..ops import device

    k = nf + 1 if fit_intercept else nf
    if k > QN_DEVICE_MAX_K:
        return None
    out = device.wls_qn_small(flat, nf, fit_intercept, reg_param, elastic_net, standardize_features,
                              standardize_label, max_iter, tol)
    return owlqn_result(out.cpu().numpy(), nf)


def _check_status(status: int, singular_fallback: bool = False):
    if status == 1:
        raise ValueError("Sum of weights cannot be zero.")
    if status == 2:
        raise ValueError("Training dataset is empty.")
    if status == 3:
        log.warning("The standard deviation of the label is zero, so the coefficients will be zeros and the "
                    "intercept will be the mean of the label; as a result, training is not needed.")
    elif status == 4:
        log.warning("Mean and standard deviation of the label are zero, so the coefficients and the intercept "
                    "will all be zero; as a result, training is not needed.")
    elif status == 5:
        raise ValueError("The standard deviation of the label is zero. Model cannot be regularized with "
                         "standardization=true")
    elif status == 6:
        log.warning("The standard deviation of the label is zero. Consider setting fitIntercept=true.")
    if singular_fallback:
        log.warning("Cholesky solver failed due to singular covariance matrix. Retrying with Quasi-Newton solver.")


def _wls_native(flat_np, stats, fit_intercept, reg_param, elastic_net, standardize_features, standardize_label,
                solver_type, max_iter, tol) -> WLSModel:
    if reg_param == 0.0:
        log.warning("regParam is zero, which might cause numerical instability and overfitting.")
    nf = stats.k
    h = native.host()
    try:
        r = h.wls_fit(flat_np, nf, fit_intercept, float(reg_param), float(elastic_net), bool(standardize_features),
                      bool(standardize_label), _SOLVER_CODES[solver_type], int(max_iter), float(tol), True)
    except h.SingularMatrixError as e:
        raise SingularMatrixException(str(e)) from None
    _check_status(r["status"], r["singular_fallback"])
    if r["status"] in (3, 4):
        return WLSModel(np.zeros(nf), float(r["intercept"]), np.zeros(1), np.zeros(1), "none")
    if r["converged_reason"]:
        log.info("quasi-newton converged: %s after %d states", r["converged_reason"], len(r["objective_history"]))
    diag_inv = np.zeros(1)
    if r["solver"] == "cholesky":
        ata, a_std, wsum = r["ata"], r["a_std"], float(r["w_sum"])
        k = nf + 1 if fit_intercept else nf

        def diag_inv():
            inv = h.cholesky_inverse(k, ata)
            mult = np.ones(k)
            mult[:nf] = a_std * a_std
            idx = np.arange(1, k + 1)
            return inv[idx + (idx - 1) * idx // 2 - 1] / (wsum * mult)
    return WLSModel(np.asarray(r["coefficients"]), float(r["intercept"]), diag_inv,
                    np.asarray(r["objective_history"], dtype=np.float64), r["solver"])


def _wls_device(flat, nf, fit_intercept, reg_param, elastic_net, standardize_features, standardize_label,
                solver_type, max_iter, tol):
    """Large-k Cholesky branch of WLS on the device (f64; same algebra as ``wls.cpp``).

    The standardized dense system is assembled by ``wls_large.hip`` (head scalars, one prep and one
    tiled kernel, no index scatter, no host read) and solved by the device Jacobi-PCG (two kernels
    per iteration, one host read of the control block per chunk); rocSOLVER Cholesky is the
    fallback with dppsv's exact non-SPD semantics."""
    from ..ops import device

    sysm = device.wls_assemble(flat, nf, fit_intercept, reg_param, elastic_net, standardize_features,
                               standardize_label)
    if solver_type == "auto":
        o = device.wls_pcg(sysm, nf, PCG_RTOL)
    else:
        o = sysm.o[:device.PCG_STATE_WORDS].cpu().numpy()
    return wls_large_result(flat, sysm, o, nf, fit_intercept, reg_param, elastic_net, standardize_features,
                            standardize_label, solver_type, max_iter, tol)


def wls_large_result(flat, sysm, o, nf, fit_intercept, reg_param, elastic_net, standardize_features,
                     standardize_label, solver_type, max_iter, tol):
    """``(WLSModel, GramStats)`` of a large-k device solve from its host control block ``o``: the
    PCG solution when it converged and passed its residual check, else the rocSOLVER Cholesky of
    the assembled system; a short-circuit head (no weight, constant label) and a Cholesky failure
    go to the native host driver, which owns those cases' warnings and errors."""
    import torch

    from ..ops import device

    head = np.asarray(o[device.PCG_HEAD:device.PCG_HEAD + 5], dtype=np.float64)
    stats = GramStats.scalars_only(head, nf)
    if o[device.PCG_STATUS] != 0.0:  # rare short-circuits: the native driver owns their semantics
        host = flat.cpu().numpy()
        full = GramStats.from_flat(host, nf)
        return _wls_native(host, full, fit_intercept, reg_param, elastic_net, standardize_features,
                           standardize_label, solver_type, max_iter, tol), full
    if reg_param == 0.0:
        log.warning("regParam is zero, which might cause numerical instability and overfitting.")
    wSum, bStd = float(o[device.PCG_WSUM]), float(o[device.PCG_BSTD])
    k = sysm.k
    A, b, aStd = sysm.A, sysm.b, sysm.aStd
    L = None
    if solver_type == "auto" and device.pcg_ok(o):
        w = device.PCG_STATE_WORDS
        x = o[w:w + k]
        coef = np.array(o[w + k:w + k + nf], dtype=np.float64)
        intercept = float(x[nf] * bStd) if fit_intercept else 0.0
    else:
        L, info = torch.linalg.cholesky_ex(A)
        if int(info.item()) != 0:
            if solver_type != "auto":
                raise SingularMatrixException("LAPACK.dppsv returned a non-positive pivot: A is not positive definite.")
            host = flat.cpu().numpy()
            full = GramStats.from_flat(host, nf)
            return _wls_native(host, full, fit_intercept, reg_param, elastic_net, standardize_features,
                               standardize_label, "quasi-newton", max_iter, tol), full
        xt = torch.cholesky_solve(b.unsqueeze(1), L).squeeze(1)
        nz = aStd != 0.0
        safe = torch.where(nz, aStd, torch.ones_like(aStd))
        coef = torch.where(nz, xt[:nf] * bStd / safe, torch.zeros_like(aStd)).cpu().numpy()
        intercept = float(xt[nf].item() * bStd) if fit_intercept else 0.0

    def diag_inv():
        Lf = L if L is not None else torch.linalg.cholesky(A)
        inv = torch.cholesky_inverse(Lf).diagonal()
        mult = torch.ones(k, dtype=torch.float64, device=A.device)
        mult[:nf] = aStd * aStd
        return (inv / (wSum * mult)).cpu().numpy()
    return WLSModel(coef, intercept, diag_inv, np.zeros(1), "cholesky"), stats


PCG_RTOL = 1e-13


def _pcg(A, b, rtol: float = PCG_RTOL, chunk: int = 8, max_iter: int = 96):
    """Jacobi-preconditioned conjugate gradients on the standardized SPD system, on the device.

    The large-k solve (k = 4097 in BASELINE config 5) through rocSOLVER potrf + potrs took ~15 ms,
    latency bound (33 small diagonal-block kernels + sequential triangular solves); a standardized
    Gram with a ridge term is usually well conditioned, where CG reaches a relative residual of
    1e-13 in a dozen memory-bound GEMVs (134 MB each).  The recursion is checked once per
    ``chunk`` iterations (one host sync), converged iterations are frozen by masks (no NaN from a
    vanishing ``pAp``), and the final TRUE residual must pass too.  Returns None — the caller
    falls back to the Cholesky factorization, with its exact non-SPD semantics — when a diagonal
    entry is <= 0 or CG has not converged within ``max_iter``."""
    import torch

    dg = A.diagonal()
    if bool((dg <= 0).any()):
        return None
    minv = 1.0 / dg
    x = torch.zeros_like(b)
    r = b.clone()
    z = minv * r
    p = z.clone()
    rz = torch.dot(r, z)
    thr = (rtol * rtol) * torch.dot(b, b)
    zero = torch.zeros((), dtype=b.dtype, device=b.device)
    done = False
    for _ in range(0, max_iter, chunk):
        for _ in range(chunk):
            act = torch.dot(r, r) > thr
            Ap = torch.mv(A, p)
            alpha = torch.where(act, rz / torch.dot(p, Ap), zero)
            x.add_(alpha * p)
            r.sub_(alpha * Ap)
            z = minv * r
            rz_new = torch.dot(r, z)
            beta = torch.where(act, rz_new / rz, zero)
            p = z + beta * p
            rz = torch.where(act, rz_new, rz)
        if bool(torch.dot(r, r) <= thr):
            done = True
            break
    if not done:
        return None
    res = b - torch.mv(A, x)
    if not bool(torch.dot(res, res) <= 100.0 * thr):
        return None
    return x


def weighted_least_squares(stats: GramStats, fit_intercept: bool, reg_param: float, elastic_net: float,
                           standardize_features: bool, standardize_label: bool, solver_type: str,
                           max_iter: int, tol: float) -> WLSModel:
    """``WeightedLeastSquares.fit`` on pre-aggregated statistics (solver_type: auto|cholesky|quasi-newton)
    — the NumPy reference implementation of the native driver (``csrc/host/wls.cpp``), kept as the
    test oracle for it."""
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
