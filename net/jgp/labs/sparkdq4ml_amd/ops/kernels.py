"""Device-op facade.

Every op takes/returns torch tensors.  CUDA (ROCm) tensors go to the gfx950 kernels of
``_dq4ml_hip`` — a missing extension is a hard error on a GPU box, never a silent torch
fallback.  CPU tensors (``local-cpu`` sessions, unit tests) run the host implementations, which
are also the fp64 oracles of the kernel tests.

Ops:
  K3  ``selected_indices``   stream compaction of a selection vector
  K4  ``pack_columns``       columns -> feature-major [d, n] matrix (cast)
  K5  ``gram_stats``         WLS sufficient statistics (MFMA Gram) of [X | 1 | y] with weights/mask
  K7+K8 ``predict`` / ``regression_metrics``  fused GEMV + metric reductions
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np
import torch

from . import native

__all__ = ["selected_indices", "pack_columns", "gram_stats", "predict", "regression_metrics",
           "gram_layout_size"]


def _on_gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


# ------------------------------------------------------------------------------------------
# K3 — compaction
# ------------------------------------------------------------------------------------------
def selected_indices(sel: torch.Tensor, limit: Optional[int] = None) -> torch.Tensor:
    """Indices (int64) of the true entries of ``sel``, in order; at most ``limit`` of them."""
    if _on_gpu(sel):
        from . import device

        return device.compact_indices(sel, limit)
    idx = torch.nonzero(sel, as_tuple=False).flatten()
    return idx if limit is None else idx[:limit]


# ------------------------------------------------------------------------------------------
# K4 — pack
# ------------------------------------------------------------------------------------------
def pack_columns(parts: Sequence[torch.Tensor], dtype: torch.dtype) -> torch.Tensor:
    """Stack 1-row/k-row pieces (each ``[k_i, n]``) into one feature-major ``[d, n]`` matrix."""
    if parts and _on_gpu(parts[0]):
        from . import device

        return device.pack_columns(list(parts), dtype)
    return torch.cat([p.to(dtype) for p in parts], dim=0)


def pack_tiled(parts: Sequence[torch.Tensor], sel: Optional[torch.Tensor] = None):
    """GPU only: columns -> MFMA-fragment-ordered bf16 (``ops.layout.TiledBF16``); rows outside
    ``sel`` are written as zeros."""
    from . import device

    return device.pack_tiled(list(parts), sel)


def gram_cols(parts: Sequence[torch.Tensor], y: torch.Tensor, sel: Optional[torch.Tensor] = None):
    """GPU only: fused VectorAssembler + bf16 Gram over the source columns (d <= 64)."""
    from . import device

    return device.gram_cols(list(parts), y, sel)


def gram_stream_cols(parts: Sequence[torch.Tensor], y: torch.Tensor, w: Optional[torch.Tensor] = None,
                     sel: Optional[torch.Tensor] = None, compute: str = "fp64"):
    """GPU only: WLS statistics of 9..64 same-dtype source columns through the LDS-DMA stream
    kernels (``gram_stream.hip``); None when the sources do not qualify."""
    from . import device

    return device.gram_stream_cols(list(parts), y, w, sel, compute)


def gram_skinny_cols(parts: Sequence[torch.Tensor], y: torch.Tensor, w: Optional[torch.Tensor] = None,
                     sel: Optional[torch.Tensor] = None):
    """GPU only: f64 statistics of a narrow (d <= 8) assembly read from its source columns."""
    from . import device

    return device.gram_skinny_cols(list(parts), y, w, sel)


def pack_wide(parts: Sequence[torch.Tensor], eb: int, sel: Optional[torch.Tensor] = None):
    """GPU only: columns -> wide (d > 64) fragment layout, bf16 (eb 16) or fp8 e4m3 with
    per-feature scales (eb 8) (``ops.layout.TiledWide``); rows outside ``sel`` become zeros."""
    from . import device

    return device.pack_wide(list(parts), eb, sel)


# ------------------------------------------------------------------------------------------
# K5 — Gram / WLS statistics
# ------------------------------------------------------------------------------------------
def gram_layout_size(d: int) -> int:
    return 5 + 2 * d + d * (d + 1) // 2


_upper_idx = {}


def packed_upper(aa: torch.Tensor) -> torch.Tensor:
    """Packed upper (column-major) entries of a square matrix; index vectors cached per (d, device)."""
    d = aa.shape[0]
    key = (d, aa.device)
    idx = _upper_idx.get(key)
    if idx is None:
        J = torch.repeat_interleave(torch.arange(d, device=aa.device), torch.arange(1, d + 1, device=aa.device))
        I = torch.cat([torch.arange(j + 1, device=aa.device) for j in range(d)]) if d else J
        if len(_upper_idx) > 32:
            _upper_idx.clear()
        idx = _upper_idx[key] = (I, J)
    return aa[idx[0], idx[1]]


def gram_stats(X: torch.Tensor, y: torch.Tensor, w: Optional[torch.Tensor], sel: Optional[torch.Tensor],
               compute: str = "fp64", x_zero_dead: bool = False, defer: bool = False) -> torch.Tensor:
    """Flat f64 ``[count, wSum, wwSum, bSum, bbSum, aSum[d], abSum[d], aaSum packed-upper]`` over
    live rows (``sel``), with instance weights ``w`` (default 1) — Spark WLS ``Aggregator.add`` over
    every row, in one pass.  ``X`` is feature-major ``[d, n]``."""
    d, n = X.shape
    if int(y.shape[0]) != n or (w is not None and w.shape[0] != n) or (sel is not None and sel.shape[0] != n):
        raise ValueError("gram_stats: row-count mismatch between features, label, weight and selection")
    if _on_gpu(X):
        from . import device

        return device.gram_stats(X, y, w, sel, compute, x_zero_dead=x_zero_dead, defer=defer)
    Xd = (X.to_dense() if hasattr(X, "to_dense") else X).to(torch.float64)
    yd = y.to(torch.float64)
    wv = torch.ones(n, dtype=torch.float64) if w is None else w.to(torch.float64)
    live = torch.ones(n, dtype=torch.bool) if sel is None else sel
    wv = torch.where(live, wv, torch.zeros_like(wv))
    count = float(live.sum())
    Xw = Xd * wv
    aa = Xw @ Xd.t()
    out = torch.empty(gram_layout_size(d), dtype=torch.float64)
    out[0] = count
    out[1] = wv.sum()
    out[2] = (wv * wv).sum()
    out[3] = (wv * yd).sum()
    out[4] = (wv * yd * yd).sum()
    out[5:5 + d] = Xw.sum(1)
    out[5 + d:5 + 2 * d] = Xw @ yd
    out[5 + 2 * d:] = packed_upper(aa)
    return out


# ------------------------------------------------------------------------------------------
# K7 / K8 — predict and regression metrics
# ------------------------------------------------------------------------------------------
def predict(X: torch.Tensor, coef: np.ndarray, intercept: float) -> torch.Tensor:
    if _on_gpu(X):
        from . import device

        return device.predict(X, coef, intercept)
    c = torch.as_tensor(np.asarray(coef), dtype=torch.float64)
    return c @ X.to(torch.float64) + intercept


def regression_metrics(X: torch.Tensor, y: torch.Tensor, coef: np.ndarray, intercept: float,
                       sel: Optional[torch.Tensor], shift: float) -> torch.Tensor:
    """f64 sums over live rows: [n, Σ(y-s), Σ(y-s)², Σr, Σr², Σ|r|, Σ(p-s), Σ(p-s)²], r = y - p."""
    if _on_gpu(X):
        from . import device

        return device.regression_metrics(X, y, coef, intercept, sel, shift)
    p = predict(X, coef, intercept)
    yd = y.to(torch.float64)
    live = torch.ones_like(yd, dtype=torch.bool) if sel is None else sel
    yd, p = yd[live], p[live]
    r = yd - p
    ys, ps = yd - shift, p - shift
    return torch.stack([torch.tensor(float(yd.numel()), dtype=torch.float64), ys.sum(), (ys * ys).sum(), r.sum(),
                        (r * r).sum(), r.abs().sum(), ps.sum(), (ps * ps).sum()])


# ------------------------------------------------------------------------------------------
# K9 — huber loss/gradient pass
# ------------------------------------------------------------------------------------------
def huber_pass(X, y, w, sel, ceff: np.ndarray, icpt: float, sigma: float, eps: float) -> torch.Tensor:
    """f64 ``[lossSum, weightSum, g_intercept, g_sigma, Σ_r m_r x_r (d)]`` (Spark HuberAggregator
    sums before division by the weight sum); ``ceff`` = coefficients / feature std."""
    if _on_gpu(X if torch.is_tensor(X) else X.buf):
        from . import device

        return device.huber_pass(X, y, w, sel, ceff, icpt, sigma, eps)
    Xd = (X.to_dense() if hasattr(X, "to_dense") else X).to(torch.float64)
    yd = y.to(torch.float64)
    n = yd.shape[0]
    wt = torch.ones(n, dtype=torch.float64) if w is None else w.to(torch.float64)
    if sel is not None:
        wt = torch.where(sel, wt, torch.zeros_like(wt))
    margin = torch.as_tensor(ceff, dtype=torch.float64) @ Xd + icpt
    lin = yd - margin
    inside = lin.abs() <= sigma * eps
    q = lin / sigma
    loss = torch.where(inside, 0.5 * wt * (sigma + lin * lin / sigma),
                       0.5 * wt * (sigma + 2.0 * eps * lin.abs() - sigma * eps * eps))
    sgn = torch.where(lin >= 0, -1.0, 1.0).to(torch.float64)
    m = torch.where(inside, -wt * q, wt * sgn * eps)
    gs = torch.where(inside, 0.5 * wt * (1.0 - q * q), 0.5 * wt * (1.0 - eps * eps) * torch.ones_like(q))
    live = wt != 0
    out = torch.empty(4 + Xd.shape[0], dtype=torch.float64)
    out[0] = loss[live].sum()
    out[1] = wt.sum()
    out[2] = m[live].sum()
    out[3] = gs[live].sum()
    out[4:] = Xd @ torch.where(live, m, torch.zeros_like(m))
    return out


# ------------------------------------------------------------------------------------------
# K9 — squared-loss l-bfgs evaluation passes
# ------------------------------------------------------------------------------------------
class _HostLsq:
    """fp64 host implementation of :class:`ops.device.LsqPasses` (CPU engine; the kernel tests'
    oracle)."""

    def __init__(self, X, y, w, sel):
        self.X = (X.to_dense() if hasattr(X, "to_dense") else X).to(torch.float64)
        self.d, self.n = int(self.X.shape[0]), int(self.X.shape[1])
        wt = torch.ones(self.n, dtype=torch.float64) if w is None else w.to(torch.float64)
        if sel is not None:
            wt = torch.where(sel.to(torch.bool), wt, torch.zeros_like(wt))
        self.w = wt
        self.y = torch.where(wt != 0, y.to(torch.float64), torch.zeros_like(wt))
        self.device = self.X.device
        self._Xz = torch.where(wt.unsqueeze(0) != 0, self.X, torch.zeros_like(self.X))  # dead rows: no NaN

    def scalars(self):
        w, y = self.w, self.y
        return torch.stack([(w != 0).sum().to(torch.float64), w.sum(), (w * w).sum(), (w * y).sum(),
                            (w * y * y).sum()])

    def moments(self):
        return torch.cat([self._Xz @ self.w, (self._Xz * self._Xz) @ self.w])

    def evaluate(self, cf, offset, inv_ystd):
        cf = cf.to(torch.float64)
        diff = cf @ self._Xz + torch.as_tensor(offset, dtype=torch.float64).reshape(()) - self.y * inv_ystd
        v = torch.where(self.w != 0, self.w * diff, torch.zeros_like(diff))
        out = torch.empty(1 + self.d, dtype=torch.float64)
        out[0] = (0.5 * v * diff).sum()
        out[1:] = self._Xz @ v
        return out

    def wmargins(self, cf):
        return self.w * (cf.to(torch.float64) @ self._Xz)

    def evaluate_u(self, u, cf, offset, inv_ystd):
        live = self.w != 0
        v = torch.where(live, u + self.w * (torch.as_tensor(offset, dtype=torch.float64).reshape(()) - self.y * inv_ystd),
                        torch.zeros_like(u))
        out = torch.empty(1 + self.d, dtype=torch.float64)
        out[0] = torch.where(live, 0.5 * v * v / torch.where(live, self.w, torch.ones_like(self.w)),
                             torch.zeros_like(v)).sum()
        out[1:] = self._Xz @ v
        return out


def lsq_passes(X, y: torch.Tensor, w: Optional[torch.Tensor], sel: Optional[torch.Tensor]):
    """Per-fit state of the squared-loss l-bfgs path: ``.scalars()``,
    ``.moments()`` (summarizer pass) and ``.evaluate(cf, offset, inv_ystd)`` (one
    ``LeastSquaresAggregator`` pass) — device kernels for device data, fp64 torch on the host."""
    if _on_gpu(X if torch.is_tensor(X) else X.buf):
        from . import device

        return device.LsqPasses(X, y, w, sel)
    return _HostLsq(X, y, w, sel)


_ = (List, native)
