"""Physical layouts of assembled feature matrices.

``TiledBF16`` is the MI355X-native storage of a bf16 ``vector`` column: the MFMA-fragment order
of ``v_mfma_f32_32x32x16_bf16`` (csrc/hip/gram.h).  For superstep ``s`` (64 rows), 32-feature tile
``t`` and k-step ``i``, the 64 lanes' 16-byte fragments are contiguous, so the Gram kernel's
every wave load is one contiguous KiB and the pass runs at HBM speed (measured 6.25 TB/s vs
3.06 TB/s for the same kernel on plain feature-major storage, scripts/gram_ab.py).  Rows are
zero padded to whole supersteps, features to whole tiles.

Everything that needs individual rows (show/collect/compaction) gathers them with
:meth:`gather_rows`; the hot consumers (Gram, predict, metrics) read the tiles directly.

Both layouts may store the features SHIFTED: ``shift`` (an ``ops.shift.Shift`` or None) holds a
per-feature value ``s`` that was subtracted before the low-precision cast (``x' = x - s`` is
what the tiles hold; dead and padding rows are exactly 0).  Consumers correct for it: the Gram
un-shifts its statistics in f64, predictions add ``s . coef`` to the intercept, and
:meth:`gather_rows` returns ``x' + s`` (f32).
"""
from __future__ import annotations

import torch

__all__ = ["TiledBF16", "tiled_offsets"]


def tiled_offsets(feats: torch.Tensor, rows: torch.Tensor, d: int) -> torch.Tensor:
    """Element offsets of (feature, row) pairs (broadcast) in the tiled layout."""
    NT = (d + 31) // 32
    s = rows >> 6
    h = (rows >> 5) & 1
    i = (rows >> 3) & 3
    j = rows & 7
    t = feats >> 5
    lane = 32 * h + (feats & 31)
    return ((((s * NT + t) * 4 + i) * 64 + lane) << 3) + j


def _unshift_rows(vals: torch.Tensor, shift) -> torch.Tensor:
    if shift is None:
        return vals
    return vals.to(torch.float32) + shift.dev.to(vals.device).unsqueeze(1)


class TiledBF16:
    def __init__(self, buf: torch.Tensor, d: int, n: int, shift=None):
        assert buf.dtype == torch.bfloat16 and buf.dim() == 1
        self.buf, self.d, self.n = buf, int(d), int(n)
        self.shift = shift

    @property
    def shape(self):
        return (self.d, self.n)

    @property
    def device(self):
        return self.buf.device

    @property
    def dtype(self):
        return torch.bfloat16

    @property
    def is_cuda(self):
        return self.buf.is_cuda

    def dim(self):
        return 2

    def gather_rows(self, rows: torch.Tensor) -> torch.Tensor:
        """Dense ``[d, k]`` of the given rows: bf16, or f32 ``x' + s`` for shifted storage."""
        rows = rows.to(self.buf.device, torch.int64)
        f = torch.arange(self.d, device=self.buf.device, dtype=torch.int64).unsqueeze(1)
        return _unshift_rows(self.buf[tiled_offsets(f, rows.unsqueeze(0), self.d)], self.shift)

    def to_dense(self) -> torch.Tensor:
        return self.gather_rows(torch.arange(self.n, device=self.buf.device))

    def slice_rows(self, start: int, stop: int) -> torch.Tensor:
        return self.gather_rows(torch.arange(start, stop, device=self.buf.device))

    def __repr__(self):
        return f"TiledBF16(d={self.d}, n={self.n}, device={self.buf.device})"


def wide_offsets(feats: torch.Tensor, rows: torch.Tensor, d: int, eb: int = 16) -> torch.Tensor:
    """Element offsets in the wide (d > 64) fragment layout, tiles padded to whole 256-feature
    panels (csrc/hip/gram_wide.hip).  Per (superstep s = 64 rows, 32-feature tile t) one chunk of
    512 elements: bf16 ``[k-step][64 lanes][8]``; fp8 ``[half][64 lanes][16]`` where a lane's 32
    bytes are its 4 k-steps (half = k-step >> 1) — one K=64 block-scaled MFMA operand."""
    NT = ((d + 255) // 256) * 8
    s = rows >> 6
    ki = (rows >> 4) & 3
    h = (rows >> 3) & 1
    j = rows & 7
    t = feats >> 5
    lane = 32 * h + (feats & 31)
    if eb == 8:
        return (s * NT + t) * 2048 + (((ki >> 1) * 64 + lane) << 4) + ((ki & 1) << 3) + j
    return ((((s * NT + t) * 4 + ki) * 64 + lane) << 3) + j


class TiledWide:
    """Wide MFMA-fragment storage: bf16 (eb=16) or fp8 e4m3 OCP with per-feature scales (eb=8)."""

    def __init__(self, buf: torch.Tensor, d: int, n: int, eb: int, scales=None, shift=None):
        self.buf, self.d, self.n, self.eb = buf, int(d), int(n), int(eb)
        self.scales = scales  # f32 [d] (fp8 only): x = q * scale (+ shift)
        self.shift = shift

    @property
    def nt(self):
        return ((self.d + 255) // 256) * 8

    @property
    def shape(self):
        return (self.d, self.n)

    @property
    def device(self):
        return self.buf.device

    @property
    def dtype(self):
        return torch.bfloat16 if self.eb == 16 else torch.float8_e4m3fn

    @property
    def is_cuda(self):
        return self.buf.is_cuda

    def dim(self):
        return 2

    def gather_rows(self, rows: torch.Tensor) -> torch.Tensor:
        rows = rows.to(self.buf.device, torch.int64)
        f = torch.arange(self.d, device=self.buf.device, dtype=torch.int64).unsqueeze(1)
        off = wide_offsets(f, rows.unsqueeze(0), self.d, self.eb)
        if self.eb == 16:
            return _unshift_rows(self.buf.view(torch.bfloat16)[off], self.shift)
        q = self.buf.view(torch.float8_e4m3fn)[off].to(torch.float32)
        return _unshift_rows(q * self.scales.unsqueeze(1), self.shift)

    def to_dense(self) -> torch.Tensor:
        return self.gather_rows(torch.arange(self.n, device=self.buf.device))

    def slice_rows(self, start: int, stop: int) -> torch.Tensor:
        return self.gather_rows(torch.arange(start, stop, device=self.buf.device))

    def __repr__(self):
        return f"TiledWide(d={self.d}, n={self.n}, eb={self.eb}, device={self.buf.device})"
