"""Per-column shifts for the low-precision Gram paths.

Spark's WLS aggregator sums raw ``x`` and forms the population variance as ``E[x²] - E[x]²``
(``DataQuality4MachineLearningApp.java:126``) in f64.  The bf16 / fp8 / exact-f32
Gram kernels round every feature before the MFMA and accumulate in f32, so a column whose mean
is large next to its spread (a price in [128, 256) has a bf16 step of 1.0; a feature at 10 ± 1
has an fp8 e4m3 step of 1.0) loses its variance to the rounding and to the f32 sums.

The fix is the classic shifted-data algorithm: every kernel that rounds subtracts a per-column
shift ``s`` first (``GramArgs::xshift`` in-kernel, or at tiling time for the stored bf16 / fp8
layouts) and accumulates the statistics of ``x' = x - s``; ``stats_unshift`` then restores those
of ``x`` exactly in f64 (Σw·x = Σw·x' + s·Σw, Σw·xᵢ·xⱼ = Σw·x'ᵢ·x'ⱼ + sᵢ·Σw·x'ⱼ + sⱼ·Σw·x'ᵢ +
sᵢ·sⱼ·Σw).  The algebra holds for ANY fixed shift, so the DQ selection and the weights need no
special handling; how close ``s`` is to the true mean only decides how many digits survive.

``s`` is the mean of a strided sample of the column (at most 65 536 rows, every row's position
equally likely to be sampled), rounded to f32 -- or to bf16 for a bf16 source, so that ``x - s``
of two bf16 values of similar magnitude is exact.  A column that the sample shows already
centred (``|mean| <= std``) gets ``s = 0``; when every column is centred (or there are fewer than
256 rows) there is no shift at all and the kernels run exactly as before.  The sample costs one small host read per source
matrix, memoized per source tensor.
"""
from __future__ import annotations

import weakref
from typing import List, Optional, Sequence

import numpy as np
import torch

__all__ = ["Shift", "column_shift", "SAMPLE_ROWS", "CENTER_RATIO"]

SAMPLE_ROWS = 65536
CENTER_RATIO = 1.0  # |mean| <= CENTER_RATIO * std: already centred, s = 0 (bf16 keeps 2^-8 of 2 std)
MIN_ROWS = 256      # fewer rows: no shift (f32 sums of a handful of rows stay exact enough)


class Shift:
    """One shift vector: ``dev`` f32 [d] on the data's device (what the kernels subtract) and
    ``host`` f64 [d] (the same f32 values: intercept / offset corrections on the host)."""

    __slots__ = ("dev", "host", "uniform", "_dev64", "__weakref__")

    def __init__(self, host: np.ndarray, device, uniform: bool = False):
        h32 = np.ascontiguousarray(host, dtype=np.float32)
        self.host = h32.astype(np.float64)
        self.dev = torch.from_numpy(h32).to(device)
        # the same on every data-parallel rank (agreed by an all-reduce, or fixed by the caller):
        # shifted statistics may then be summed over ranks before the un-shift
        self.uniform = bool(uniform)
        self._dev64 = None

    @property
    def d(self) -> int:
        return int(self.host.shape[0])

    @property
    def dev64(self) -> torch.Tensor:
        if self._dev64 is None:
            self._dev64 = self.dev.to(torch.float64)
        return self._dev64

    def dot(self, coef) -> float:
        """Σ s_j·c_j on the host (the intercept correction of x·c = x'·c + s·c)."""
        return float(np.dot(self.host, np.asarray(coef, dtype=np.float64)))

    def __repr__(self):
        nz = int(np.count_nonzero(self.host))
        return f"Shift(d={self.d}, shifted_columns={nz})"


def _rows_of(parts: Sequence[torch.Tensor]) -> List[torch.Tensor]:
    rows = []
    for p in parts:
        if p.dim() == 1:
            rows.append(p)
        else:
            rows.extend(p[i] for i in range(p.shape[0]))
    return rows


_memo: dict = {}


def _root(t: torch.Tensor) -> torch.Tensor:
    """The tensor that owns a view's storage (views made per call -- ``p[i]``, ``unsqueeze`` --
    are new objects every time; their base is not)."""
    while t._base is not None:
        t = t._base
    return t


def _key(t: torch.Tensor):
    return (t.data_ptr(), tuple(t.shape), tuple(t.stride()), t.dtype, t._version)


def _sample_stats(rows: List[torch.Tensor]):
    """[d] sample sums, sums of squares and counts (f64, on the rows' device) over the finite
    values of a strided sample of every row."""
    n = int(rows[0].numel())
    step = max(1, n // SAMPLE_ROWS)
    samp = torch.stack([r[::step][:SAMPLE_ROWS].to(torch.float64) for r in rows])
    fin = torch.isfinite(samp)
    z = torch.where(fin, samp, torch.zeros_like(samp))
    frac = (z != torch.round(z)).sum(1).to(torch.float64)  # sampled values off the integer grid
    return torch.stack([z.sum(1), (z * z).sum(1), fin.sum(1).to(torch.float64), frac])


def column_shift(parts: Sequence[torch.Tensor], uniform: bool = False) -> Optional[Shift]:
    """The shift of a list of source columns (1-D ``[n]`` or 2-D ``[k, n]`` pieces, any dtype):
    None when every column is already centered (or n == 0).  ``uniform``: the sample statistics
    are summed over the data-parallel ranks first, so every rank gets the same shift (needed
    where shifted statistics are all-reduced before they are un-shifted: the wide Gram's f32
    wire).  Reads one small sample back to the host (memoized per source tensor)."""
    rows = _rows_of(parts)
    if not rows or rows[0].numel() < MIN_ROWS:
        return None
    from ..parallel import comm

    coll = uniform and comm.collectives_active()
    key = (tuple(_key(r) for r in rows), coll)
    bases = [_root(r) for r in rows]
    # a rank-uniform shift never comes from the memo: whether a lookup hits depends on this
    # process's tensor lifetimes (and the memo's clearing), so ranks could disagree on whether to
    # issue the all-reduce below and hang; the collective is one small sample per pack_wide
    hit = None if coll else _memo.get(key)
    if hit is not None:
        refs, val = hit
        if all(ref() is b for ref, b in zip(refs, bases)):  # same live tensors, not a reused address
            return val
    st = _sample_stats(rows)
    if coll:
        st = comm.all_reduce_sum(st)
    s, ss, cnt, frac = st.cpu().numpy()
    cnt = np.maximum(cnt, 1.0)
    mean = s / cnt
    var = np.maximum(ss / cnt - mean * mean, 0.0)
    need = np.isfinite(mean) & (np.abs(mean) > CENTER_RATIO * np.sqrt(var))
    val = None
    if need.any():
        shift = np.where(need, mean, 0.0)
        # an integral column (the lab's guest count) keeps exact values: x - s must stay on the
        # integer grid, or the bf16 cast of x - s rounds what x alone kept exactly
        shift = np.where(frac == 0.0, np.rint(shift), shift)
        bf16 = np.array([r.dtype == torch.bfloat16 for r in rows])
        if bf16.any():
            sb = torch.from_numpy(shift).to(torch.bfloat16).to(torch.float64).numpy()
            shift = np.where(bf16, sb, shift)
        val = Shift(shift, rows[0].device, uniform=coll or not comm.collectives_active())
    if not coll:
        if len(_memo) >= 256:
            _memo.clear()
        _memo[key] = ([weakref.ref(b) for b in bases], val)
    return val


def shift_of(X) -> Optional[Shift]:
    """The shift a stored layout (``TiledBF16`` / ``TiledWide``) was built with, else None."""
    return getattr(X, "shift", None)
