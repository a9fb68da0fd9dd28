"""Python launchers of the gfx950 kernels (``_dq4ml_hip``).

Allocation policy: every output/workspace comes from torch's caching allocator on the current
device and every kernel runs on ``torch.cuda.current_stream()`` — no hipMalloc/hipMemcpy in any
launch path, so these ops compose with torch work and HIP-graph capture.  Shapes and dtypes are
validated HERE, on the host, before any launch (a kernel's indexing assumes them)."""
from __future__ import annotations

import functools
from dataclasses import dataclass
import os
from typing import List, Optional

import numpy as np
import torch

from ..parallel import comm
from ..runtime import faststream
from . import native

__all__ = ["dtype_code", "gram_stats", "compact_indices", "pack_columns", "predict", "regression_metrics",
           "GRAM_MODES"]

_DT = {torch.float64: 0, torch.float32: 1, torch.bfloat16: 2, torch.int32: 3, torch.int64: 4, torch.uint8: 5,
       torch.bool: 5, torch.float16: 6}
GRAM_MODES = {"fp64": 0, "fp32": 1, "bf16": 2, "fp8": 3, "fp32split": 4}
_plan_cache = {}


# CUs a full-chip Gram pass leaves to the fit tail (``dq4ml.gram.reserveCUs`` /
# DQ4ML_GRAM_RESERVE_CUS, default 0).  The pipelined tail of fit k (fold, RCCL all-reduce,
# one-block solve; models/regression.py _PendingWLS) runs beside fit k+1's pass; with a reserve
# the Gram grid is `reserve` CUs' worth of blocks short (and, opt-in, the streams CU-masked).
# Measured, a tail kernel starts within ~6 us beside a running pass without any reserve, and the
# HBM-bound pass streams at the same rate on 248 of 256 CUs (profiles/r5_tail_reserve.md).
_gram_reserve = int(os.environ.get("DQ4ML_GRAM_RESERVE_CUS", "-1"))
_cus_cache = {}


def set_gram_reserve(n: int) -> None:
    """CUs the full-chip Gram grids leave free for the fit tail (-1: the default, 0)."""
    global _gram_reserve
    _gram_reserve = int(n)
    _plan_cache.clear()


def gram_reserve() -> int:
    return max(0, _gram_reserve)


def _cus(h) -> int:
    dev = torch.cuda.current_device()
    c = _cus_cache.get(dev)
    if c is None:
        c = _cus_cache[dev] = int(h.device_info()["multiProcessorCount"])
    return c


def _plan_blocks(h, mode, d, n, xdt, xmode):
    reserve = gram_reserve()
    key = (torch.cuda.current_device(), mode, d, n, xdt, xmode, reserve)
    nb = _plan_cache.get(key)
    if nb is None:
        nb = int(h.gram_plan_blocks(mode, int(d), int(n), xdt, xmode))
        cus = _cus(h)
        if reserve > 0 and nb >= cus:  # a full residency wave of blocks: give `reserve` CUs back
            per = nb // cus
            nb = max(1, nb - reserve * per)
        _plan_cache[key] = nb
    return nb


def _h2d(arr: np.ndarray, dev) -> torch.Tensor:
    """Upload a small host table (kernel descriptors: source pointers + dtype codes, pair lists,
    scales) WITHOUT a host-device sync: staged through torch's caching pinned-host allocator and
    copied with ``non_blocking`` (a pageable H2D copy blocks the host until the stream drains,
    which serialized the host's plan building with the GPU's previous step)."""
    t = torch.from_numpy(np.ascontiguousarray(arr))
    if torch.device(dev).type != "cuda":
        return t.to(dev)
    return t.pin_memory().to(dev, non_blocking=True)


def dtype_code(t: torch.Tensor) -> int:
    try:
        return _DT[t.dtype]
    except KeyError:
        raise TypeError(f"unsupported dtype {t.dtype}") from None


def _stream() -> int:
    """The current device's current stream (raw handle; the torch C entry points directly, see
    ``runtime/faststream.py``)."""
    return torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())


def _ptr(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else t.data_ptr()


def _check_dev(*ts):
    dev = None
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise ValueError("device op given a host tensor")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise ValueError(f"tensors on different devices: {dev} vs {t.device}")


def _feature_view(X: torch.Tensor, align_elems: int):
    """(base tensor, ld): a feature-major view whose rows are ``align_elems``-aligned."""
    if X.dim() != 2:
        raise ValueError("feature matrix must be 2-D [d, n]")
    d, n = X.shape
    if X.stride(1) != 1 or (d > 1 and X.stride(0) % align_elems) or X.data_ptr() % 16:
        ld = (n + 63) // 64 * 64
        buf = torch.zeros(d, ld, dtype=X.dtype, device=X.device)
        buf[:, :n] = X
        return buf, ld
    return X, (X.stride(0) if d > 1 else max(n, 1))


# ------------------------------------------------------------------------------------------
from .layout import TiledBF16, TiledWide  # noqa: E402
from .shift import column_shift  # noqa: E402

FP8_MAX = 448.0


def _auto_shift(parts, shift, uniform=False):
    """``shift`` = "auto": the sampled per-column shift of the sources (ops/shift.py), else as given."""
    if isinstance(shift, str):
        if shift != "auto":
            raise ValueError(f"shift: 'auto', None or an ops.shift.Shift, not {shift!r}")
        return column_shift(parts, uniform=uniform)
    return shift


def _sptr(shift) -> int:
    return 0 if shift is None else shift.dev.data_ptr()


def _unshift(h, out: torch.Tensor, shift, d: int) -> torch.Tensor:
    """Statistics of x' = x - s -> those of x, in place on the current stream (gram.h
    ``stats_unshift``); a no-op without a shift."""
    if shift is not None:
        h.stats_unshift(out.data_ptr(), shift.dev.data_ptr(), int(d), _stream())
    return out


def tile_bf16(X: torch.Tensor, shift="auto") -> TiledBF16:
    """[d, n] features -> MFMA-fragment-ordered bf16 tiles of x - s (``shift``: "auto" = the
    sampled per-column shift, None = unshifted, or an ``ops.shift.Shift``)."""
    h = native.hip()
    _check_dev(X)
    d, n = X.shape
    if X.stride(1) != 1:
        X = X.contiguous()
    shift = _auto_shift([X], shift)
    ld = X.stride(0) if d > 1 else max(n, 1)
    buf = torch.empty(int(h.tiled_elems(d, n)), dtype=torch.bfloat16, device=X.device)
    h.tile_bf16(X.data_ptr(), dtype_code(X), int(ld), int(d), int(n), buf.data_ptr(), _stream(), _sptr(shift))
    return TiledBF16(buf, d, n, shift)


class DeferredGram:
    """Gram partial slabs whose final fold (``gram_reduce``) has not been enqueued yet: the
    asynchronous fit runs it on its side stream with the all-reduce and the solve, so the compute
    stream moves on to the next launch right after the Gram kernel."""

    is_cuda = True

    def __init__(self, h, mode, partials, nb, d, out, shift=None):
        self._h, self.mode, self.partials, self.nb, self.d, self.out = h, mode, partials, nb, d, out
        self.shift = shift
        self.device = out.device

    def finish(self) -> torch.Tensor:
        """Enqueue the fold (and the un-shift) on the CURRENT stream (the caller orders it after
        the Gram kernel)."""
        st = faststream.current(faststream.dev_index(self.device))
        self.partials.record_stream(st)
        self.out.record_stream(st)
        self._h.gram_reduce(self.mode, self.partials.data_ptr(), int(self.nb), int(self.d), self.out.data_ptr(),
                            st.cuda_stream)
        if self.shift is not None:
            self.shift.dev.record_stream(st)
            self._h.stats_unshift(self.out.data_ptr(), self.shift.dev.data_ptr(), int(self.d), st.cuda_stream)
        return self.out


def gram_stats(X, y, w, sel, compute: str = "fp64", x_zero_dead: bool = False, blocks: Optional[int] = None,
               defer: bool = False):
    """WLS statistics.  ``defer``: the tiled bf16 path may return a :class:`DeferredGram`, the wide
    fragment path a :class:`DeferredWide` (call ``finish()``); every other path returns the final
    tensor."""
    h = native.hip()
    if isinstance(X, TiledWide):
        return _gram_wide(h, X, y, w, sel, x_zero_dead, defer)
    if isinstance(X, TiledBF16):
        return _gram_tiled(h, X, y, w, sel, x_zero_dead, blocks, defer)
    _check_dev(X, y, w, sel)
    d, n = X.shape
    mode = GRAM_MODES[compute]
    out = torch.empty(5 + 2 * d + d * (d + 1) // 2, dtype=torch.float64, device=X.device)
    if n == 0:
        out.zero_()
        return out
    if d > 64 and mode in (2, 3) and w is None:
        # ingest into the wide fragment layout once, then the LDS-tiled MFMA SYRK
        return _gram_wide(h, tile_wide(X, 16 if mode == 2 else 8, sel), y, None, sel, True)
    if mode == 3 and d <= 64:
        mode = 2  # tall fp8 request: the bf16 MFMA kernel is HBM-bound already and more precise
    if d > 64:
        # fp64: f64 MFMA SYRK; fp32 and weighted bf16/fp8 requests: exact-f32 MFMA SYRK (at least
        # the requested precision; the fragment kernels carry no per-row weights)
        return _gram_syrk(h, X, y, w, sel, compute_f64=mode == 0)
    if mode in (1, 4):
        # "fp32" statistics: f32 features -> exact-f32 MFMA stream kernel (gram_stream.hip);
        # "fp32split": the same statistics from split-bf16 products on the bf16 MFMA; anything
        # else (f64 storage, unaligned views) -> the f64 kernel, at least as precise
        if X.dtype not in (torch.float32, torch.float64):
            X = X.to(torch.float32)
        if X.dtype != torch.float32 or d <= 8:
            mode = 0  # d <= 8: the f64 lane-per-row skinny kernel (exact, and HBM-bound already)
    if mode == 2 and X.dtype not in (torch.bfloat16, torch.float32, torch.float64):
        X = X.to(torch.float32)
    if mode == 0 and X.dtype not in (torch.float64, torch.float32):
        X = X.to(torch.float64)
    shift = None
    if mode in (1, 2, 4):
        # rounded features (bf16 / exact-f32 / split-f32 MFMA, f32 accumulators): centre the
        # off-centre columns first (ops/shift.py); the stream kernels subtract in-kernel, other
        # storage is tiled shifted once
        shift = column_shift([X])
        if shift is not None and X.dtype != torch.float32:
            if mode == 2 and w is None:
                return _gram_tiled(h, tile_bf16(X, shift), y, None, sel, False, blocks, defer)
            X = X.to(torch.float32).contiguous()
    align = 16 // X.element_size()
    Xv, ld = _feature_view(X, align)
    y = y.contiguous()
    if y.dtype not in (torch.float64, torch.float32):
        y = y.to(torch.float64)
    if w is not None:
        w = w.contiguous()
        if w.dtype not in (torch.float64, torch.float32):
            w = w.to(torch.float64)
    if sel is not None:
        sel = sel.contiguous()
        if sel.dtype != torch.bool:
            sel = sel.to(torch.bool)
    if y.numel() != n or (w is not None and w.numel() != n) or (sel is not None and sel.numel() != n):
        raise ValueError("gram_stats: row-count mismatch")
    if mode in (0, 1, 4) or X.dtype == torch.float32:
        # the LDS-DMA stream kernels (gram_stream.hip) read labels / weights as 16-B chunks and the
        # selection as 4-B words: re-base unaligned views (an n-element copy, far below the pass)
        y = y if y.data_ptr() % 16 == 0 else y.clone()
        w = w if w is None or w.data_ptr() % 16 == 0 else w.clone()
        sel = sel if sel is None or sel.data_ptr() % 4 == 0 else sel.clone()
    if w is not None:
        xmode = 2
    elif sel is not None and not x_zero_dead:
        xmode = 1
    else:
        xmode = 0
    if shift is not None:
        xmode = max(xmode, 1)  # dead / padding rows must weigh 0: their stored zeros are -s after the shift
    nb = int(blocks or _plan_blocks(h, mode, d, n, dtype_code(Xv), xmode))
    P = int(h.gram_partial_stride(mode, d))
    partials = torch.empty(nb * P, dtype=torch.float64, device=X.device)
    h.gram_tall(mode, Xv.data_ptr(), int(ld), int(d), int(n), dtype_code(Xv), y.data_ptr(), dtype_code(y),
                _ptr(w), dtype_code(w) if w is not None else 0, _ptr(sel), xmode, partials.data_ptr(), nb,
                out.data_ptr(), _stream(), 0, True, _sptr(shift))
    return _unshift(h, out, shift, d)


def gram_skinny_cols(parts: List[torch.Tensor], y, w, sel, blocks: Optional[int] = None):
    """f64 WLS statistics of a narrow (d <= 8) VectorAssembler output straight from its SOURCE
    columns (any of f64/f32/bf16/int32/int64/bool, mixed): the assembled [d, n] f64 matrix is
    never written — for the lab's ``features = [guest]`` that is an int32 column read in place of
    a 0.8 GB f64 pack (``gram.hip: gram_skinny_f64_kernel<.., COLS>``)."""
    h = native.hip()
    rows = _rows_of(parts)
    d, n = len(rows), rows[0].numel()
    if not 1 <= d <= 8:
        raise ValueError("gram_skinny_cols: 1 <= d <= 8")
    for r in rows:
        _check_dev(r)
        if r.numel() != n:
            raise ValueError("gram_skinny_cols: columns of different lengths")
    dev = rows[0].device
    y, w, sel = _prep_rows(y, w, sel, n)
    out = torch.empty(5 + 2 * d + d * (d + 1) // 2, dtype=torch.float64, device=dev)
    if n == 0:
        out.zero_()
        return out
    xmode = 2 if w is not None else (1 if sel is not None else 0)
    nb = int(blocks or _plan_blocks(h, 0, d, n, 0, xmode))
    P = int(h.gram_partial_stride(0, d))
    partials = torch.empty(nb * P, dtype=torch.float64, device=dev)
    h.gram_skinny_cols([r.data_ptr() for r in rows], [dtype_code(r) for r in rows], int(n), y.data_ptr(),
                       dtype_code(y), _ptr(w), dtype_code(w) if w is not None else 0, _ptr(sel),
                       partials.data_ptr(), nb, out.data_ptr(), _stream())
    return out


def gram_cols(parts: List[torch.Tensor], y, sel, blocks: Optional[int] = None):
    """Fused VectorAssembler + bf16 Gram over the SOURCE columns (d <= 64, unit weights): the
    assembled matrix is never written (``gram.hip: gram_cols_kernel``)."""
    h = native.hip()
    rows = _rows_of(parts)
    d, n = len(rows), rows[0].numel()
    if not 1 <= d <= 64:
        raise ValueError("gram_cols: 1 <= d <= 64")
    for r in rows:
        _check_dev(r)
        if r.numel() != n:
            raise ValueError("gram_cols: columns of different lengths")
        dtype_code(r)
    dev = rows[0].device
    y, _, sel = _prep_rows(y, None, sel, n)
    out = gram_stream_cols(rows, y, None, sel, "bf16")
    if out is not None:
        return out
    if sel is None:  # the kernel's loads are branch-free: an all-ones selection
        sel = _ones_sel(n, dev)
    shift = column_shift(rows)
    desc = _srcw_desc(h, rows, dev)
    nb = int(blocks or _cols_blocks(h, d, n))
    P = int(h.gram_partial_stride(2, d))
    partials = torch.empty(nb * P, dtype=torch.float64, device=dev)
    out = torch.empty(5 + 2 * d + d * (d + 1) // 2, dtype=torch.float64, device=dev)
    codes = {dtype_code(r) for r in rows}
    sdt = codes.pop() if len(codes) == 1 else -1
    if sdt not in (0, 1, 2) or any(r.data_ptr() % 16 for r in rows):
        sdt = -1  # mixed / unaligned columns: per-element typed loads
    h.gram_cols(desc.data_ptr(), int(sdt), d, n, y.data_ptr(), dtype_code(y), _ptr(sel), partials.data_ptr(), nb,
                out.data_ptr(), _stream(), _sptr(shift))
    return _unshift(h, out, shift, d)


_cols_plan = {}
_ones = {}


def gram_stream_cols(parts, y, w, sel, compute: str):
    """WLS statistics straight from the assembler's SOURCE columns through the LDS-DMA stream
    kernels (gram_stream.hip): every column is DMA'd into the swizzled LDS tiles, the assembled
    matrix is never written.  ``compute``: fp64 (f64 MFMA; all-f64 or all-f32 sources), fp32
    (exact-f32 MFMA; f32 sources), bf16 (bf16 MFMA on converted tiles; f32 sources, unit weights).
    Returns None when the sources do not qualify (mixed / unaligned / d outside 9..64): the caller
    takes the packing or the typed-load kernels instead."""
    rows = _rows_of(parts)
    d = len(rows)
    if not 9 <= d <= 64 or not rows[0].is_cuda:
        return None
    n = rows[0].numel()
    dts = {r.dtype for r in rows}
    if len(dts) != 1 or any(r.numel() != n or r.data_ptr() % 16 for r in rows):
        return None
    xdt = dts.pop()
    mode = GRAM_MODES[compute]
    if xdt not in (torch.float32, torch.float64) or (mode in (1, 2, 4) and xdt != torch.float32):
        return None
    if mode == 3 or (mode == 2 and w is not None):
        return None
    h = native.hip()
    dev = rows[0].device
    y, w, sel = _prep_rows(y, w, sel, n)
    y = y if y.data_ptr() % 16 == 0 else y.clone()
    w = w if w is None or w.data_ptr() % 16 == 0 else w.clone()
    sel = sel if sel is None or sel.data_ptr() % 4 == 0 else sel.clone()
    out = torch.empty(5 + 2 * d + d * (d + 1) // 2, dtype=torch.float64, device=dev)
    if n == 0:
        return out.zero_()
    desc = _srcw_desc(h, rows, dev)
    xc = dtype_code(rows[0])
    key = ("stream", torch.cuda.current_device(), mode, d, n, xc)
    nb = _cols_plan.get(key)
    if nb is None:
        nb = _cols_plan[key] = int(h.gram_stream_blocks(mode, d, n, xc))
    P = int(h.gram_partial_stride(mode, d))
    partials = torch.empty(nb * P, dtype=torch.float64, device=dev)
    shift = column_shift(rows) if mode in (1, 2, 4) else None  # rounded / f32-accumulated modes
    h.gram_stream_cols(mode, desc.data_ptr(), d, n, xc, y.data_ptr(), dtype_code(y), _ptr(w),
                       dtype_code(w) if w is not None else 0, _ptr(sel), partials.data_ptr(), nb, out.data_ptr(),
                       _stream(), _sptr(shift))
    return _unshift(h, out, shift, d)


def _ones_sel(n, dev):
    t = _ones.get(dev)
    if t is None or t.numel() < n:
        t = _ones[dev] = torch.ones(max(n, 1 << 20) + 64, dtype=torch.bool, device=dev)
    return t[:n]


def _cols_blocks(h, d, n):
    key = (torch.cuda.current_device(), d, n)
    nb = _cols_plan.get(key)
    if nb is None:
        nb = _cols_plan[key] = int(h.gram_cols_blocks(int(d), int(n)))
    return nb


def _prep_rows(y, w, sel, n):
    y = y.contiguous()
    if y.dtype not in (torch.float64, torch.float32):
        y = y.to(torch.float64)
    if w is not None:
        w = w.contiguous()
        if w.dtype not in (torch.float64, torch.float32):
            w = w.to(torch.float64)
    if sel is not None:
        sel = sel.contiguous().to(torch.bool)
    if y.numel() != n or (w is not None and w.numel() != n) or (sel is not None and sel.numel() != n):
        raise ValueError("gram_stats: row-count mismatch")
    return y, w, sel


class TiledGramPlan:
    """The resolved launch of one tiled bf16 Gram pass (``gram_tall`` mode 2 with the fold left to
    the fit's side stream): row operands prepared, block count planned and argument tuple built
    once, so a repeated fit of the same table only allocates its outputs and launches
    (``models/regression.py`` fit replay, ~0.14 ms of device work per fit at the 8-GPU shard)."""

    __slots__ = ("h", "T", "y", "w", "sel", "d", "nb", "flat_len", "part_len", "dev", "pre", "post")

    def __init__(self, h, T: "TiledBF16", y, w, sel, x_zero_dead):
        d, n = T.d, T.n
        if d > 64:
            raise ValueError("tiled Gram supports d <= 64")
        _check_dev(T.buf, y, w, sel)
        y, w, sel = _prep_rows(y, w, sel, n)
        xmode = 2 if w is not None else (1 if (sel is not None and not x_zero_dead) else 0)
        self.h, self.T, self.y, self.w, self.sel, self.d, self.dev = h, T, y, w, sel, d, T.device
        self.nb = int(_plan_blocks(h, 2, d, n, 2, xmode))
        self.flat_len = 5 + 2 * d + d * (d + 1) // 2
        self.part_len = self.nb * int(h.gram_partial_stride(2, d))
        self.pre = (2, T.buf.data_ptr(), 0, int(d), int(n), 2, y.data_ptr(), dtype_code(y), _ptr(w),
                    dtype_code(w) if w is not None else 0, _ptr(sel), xmode)

    def launch(self, stream: int, defer: bool):
        """Enqueue the pass on ``stream``: a :class:`DeferredGram` (``defer``, the fold and the
        un-shift left to the caller) or the folded, un-shifted statistics."""
        out = torch.empty(self.flat_len, dtype=torch.float64, device=self.dev)
        partials = torch.empty(self.part_len, dtype=torch.float64, device=self.dev)
        self.h.gram_tall(*self.pre, partials.data_ptr(), self.nb, out.data_ptr(), stream, 1, not defer, 0)
        sh = self.T.shift
        if defer:
            return DeferredGram(self.h, 2, partials, self.nb, self.d, out, sh)
        if sh is not None:
            self.h.stats_unshift(out.data_ptr(), sh.dev.data_ptr(), self.d, stream)
        return out


def _gram_tiled(h, T: "TiledBF16", y, w, sel, x_zero_dead, blocks, defer=False):
    d, n = T.d, T.n
    if d > 64:
        raise ValueError("tiled Gram supports d <= 64")
    _check_dev(T.buf, y, w, sel)
    y, w, sel = _prep_rows(y, w, sel, n)
    out = torch.empty(5 + 2 * d + d * (d + 1) // 2, dtype=torch.float64, device=T.device)
    xmode = 2 if w is not None else (1 if (sel is not None and not x_zero_dead) else 0)
    nb = int(blocks or _plan_blocks(h, 2, d, n, 2, xmode))
    P = int(h.gram_partial_stride(2, d))
    partials = torch.empty(nb * P, dtype=torch.float64, device=T.device)
    # (the tiles hold x - s already: the kernel takes no shift, the statistics are un-shifted after the fold)
    h.gram_tall(2, T.buf.data_ptr(), 0, int(d), int(n), 2, y.data_ptr(), dtype_code(y), _ptr(w),
                dtype_code(w) if w is not None else 0, _ptr(sel), xmode, partials.data_ptr(), nb, out.data_ptr(),
                _stream(), 1, not defer, 0)
    if defer:
        return DeferredGram(h, 2, partials, nb, d, out, T.shift)
    return _unshift(h, out, T.shift, d)


_syrk_pairs = {}


def _syrk_pair_table(P: int, dev) -> torch.Tensor:
    """Upper 128-panel pairs of the augmented matrix in Z-order (the blocks an XCD runs together
    are consecutive in this list and share few panels), uploaded once per (P, device)."""
    key = (P, str(dev))
    t = _syrk_pairs.get(key)
    if t is None:
        pairs = sorted(((i, j) for i in range(P) for j in range(i, P)), key=lambda p: _morton(*p))
        t = _syrk_pairs[key] = _h2d(np.asarray(pairs, dtype=np.int32).reshape(-1), dev)
    return t


def _gram_syrk(h, X, y, w, sel, compute_f64: bool):
    """d > 64 at fp64 / exact-f32 precision, and weighted low-precision requests: the LDS-tiled
    MFMA SYRK of ``gram_syrk.hip`` over the augmented [X | 1 | y] with the weight x selection
    row factor applied in-kernel -- one pass, no library GEMM, no dense copies of X."""
    d, n = X.shape
    dev = X.device
    out = torch.empty(5 + 2 * d + d * (d + 1) // 2, dtype=torch.float64, device=dev)
    if n == 0:
        return out.zero_()
    if X.dtype not in (torch.float64, torch.float32, torch.bfloat16):
        X = X.to(torch.float64 if compute_f64 else torch.float32)
    Xv, ld = _feature_view(X, 16 // X.element_size())
    y, w, sel = _prep_rows(y, w, sel, n)
    yd = y.to(torch.float64).contiguous()
    weff = None
    if w is not None:
        weff = w.to(torch.float64)
        if sel is not None:
            weff = torch.where(sel, weff, torch.zeros_like(weff))
    elif sel is not None:
        weff = sel.to(torch.float64)
    weff = None if weff is None else weff.contiguous()
    P = int(h.syrk_panels(d))
    npair = P * (P + 1) // 2
    nst = int(h.syrk_stages(n))
    target = 4 * _wide_grid(h)  # >= 4 blocks per CU slot wave (2 resident per CU at f64)
    splitk = max(1, min(-(-target // npair), max(1, nst // 8)))
    splitk = max(1, min(splitk, nst))
    part = torch.empty(int(h.syrk_partials(d, splitk)), dtype=torch.float64, device=dev)
    h.gram_syrk(1 if compute_f64 else 0, Xv.data_ptr(), int(ld), int(d), int(n), dtype_code(Xv), yd.data_ptr(),
                _ptr(weff), _syrk_pair_table(P, dev).data_ptr(), npair, splitk, part.data_ptr(), out.data_ptr(),
                _stream())
    # the two non-Gram scalars (Spark's aggregator skips zero-weight rows: count = rows with w != 0)
    if weff is None:
        out[0:1].fill_(float(n))
        out[2:3].fill_(float(n))
    else:
        out[0:1].copy_((weff != 0).sum().to(torch.float64).reshape(1))
        out[2:3].copy_((weff * weff).sum().reshape(1))
    return out


# ------------------------------------------------------------------------------------------
def compact_indices(sel: torch.Tensor, limit: Optional[int] = None) -> torch.Tensor:
    h = native.hip()
    _check_dev(sel)
    sel = sel.contiguous()
    if sel.dtype != torch.bool:
        sel = sel.to(torch.bool)
    n = sel.numel()
    nb = int(h.compact_blocks(n))
    counts = torch.empty(nb + 1, dtype=torch.int64, device=sel.device)
    s = _stream()
    h.compact_count_scan(sel.data_ptr(), n, counts.data_ptr(), s)
    total = int(counts[nb].item())
    k = total if limit is None else min(total, int(limit))
    out = torch.empty(k, dtype=torch.int64, device=sel.device)
    if k > 0:
        h.compact_write(sel.data_ptr(), n, counts.data_ptr(), k, out.data_ptr(), s)
    return out


def _pack_desc(h, parts, dev):
    rows = []
    for p in parts:
        _check_dev(p)
        if p.dim() == 1:
            p = p.unsqueeze(0)
        for i in range(p.shape[0]):
            r = p[i]
            if not r.is_contiguous():
                r = r.contiguous()
            if r.dtype == torch.bool:
                r = r.to(torch.uint8)
            rows.append(r)
    n = rows[0].numel() if rows else 0
    for r in rows:
        if r.numel() != n:
            raise ValueError("pack: columns of different lengths")
    desc = np.zeros((len(rows), 2), dtype=np.int64)  # PackSrcW {ptr, dt, pad}
    for i, r in enumerate(rows):
        desc[i, 0] = r.data_ptr()
        desc[i, 1] = dtype_code(r)
    desc_dev = _h2d(desc.reshape(-1).view(np.uint8), dev)
    return rows, n, desc_dev


def pack_tiled(parts: List[torch.Tensor], sel: Optional[torch.Tensor] = None, shift="auto") -> TiledBF16:
    """Columns -> tiled bf16 of x - s, dead rows (``sel``) exactly 0 (``shift``: see tile_bf16)."""
    h = native.hip()
    dev = parts[0].device
    shift = _auto_shift(parts, shift)
    rows, n, desc_dev = _pack_desc(h, parts, dev)
    d = len(rows)
    if d > 64:
        raise ValueError("tiled bf16 storage supports d <= 64")
    buf = torch.empty(int(h.tiled_elems(d, n)), dtype=torch.bfloat16, device=dev)
    if sel is not None:
        _check_dev(sel)
        sel = sel.contiguous().to(torch.bool)
        if sel.numel() != n:
            raise ValueError("pack_tiled: selection length mismatch")
    h.pack_tiled(desc_dev.data_ptr(), d, n, _ptr(sel), buf.data_ptr(), _stream(), _sptr(shift))
    del rows
    return TiledBF16(buf, d, n, shift)


# ------------------------------------------------------------------------------------------
def pack_columns(parts: List[torch.Tensor], dtype: torch.dtype, sel: Optional[torch.Tensor] = None) -> torch.Tensor:
    h = native.hip()
    rows = []
    for p in parts:
        _check_dev(p)
        if p.dim() == 1:
            p = p.unsqueeze(0)
        for i in range(p.shape[0]):
            r = p[i]
            if not r.is_contiguous():
                r = r.contiguous()
            if r.dtype == torch.bool:
                r = r.to(torch.uint8)
            rows.append(r)
    d = len(rows)
    n = rows[0].numel() if rows else 0
    for r in rows:
        if r.numel() != n:
            raise ValueError("pack_columns: columns of different lengths")
    ld = (n + 63) // 64 * 64
    dev = rows[0].device if rows else torch.device("cuda")
    out = torch.empty(d, max(ld, 1), dtype=dtype, device=dev)
    srcb = int(h.pack_src_bytes())
    desc = np.zeros((d, srcb // 8), dtype=np.int64)
    for i, r in enumerate(rows):
        desc[i, 0] = r.data_ptr()
        desc[i, 1] = dtype_code(r)
    desc_dev = _h2d(desc.reshape(-1).view(np.uint8), dev)
    keep = rows  # keep sources alive until the kernel is enqueued
    if sel is not None:
        sel = sel.contiguous().to(torch.bool)
    h.pack_columns(desc_dev.data_ptr(), d, n, out.data_ptr(), dtype_code(out), ld, _ptr(sel), _stream())
    del keep
    return out[:, :n]


# ------------------------------------------------------------------------------------------
def _coef_dev(coef, device):
    return torch.as_tensor(np.ascontiguousarray(coef, dtype=np.float64), device=device)


def _x_args(X):
    """(ptr, dtype code, ld, tiled flag) of a feature matrix (fp8 wide: the caller pre-scales the
    coefficients by ``X.scales``)."""
    if isinstance(X, TiledWide):
        return X.buf, 2, 0, 2 if X.eb == 16 else 3
    if isinstance(X, TiledBF16):
        return X.buf, 2, 0, 1
    if X.stride(1) != 1:
        X = X.contiguous()
    d, n = X.shape
    return X, dtype_code(X), (X.stride(0) if d > 1 else max(n, 1)), 0


def _icpt(X, coef, intercept: float) -> float:
    """Intercept for shifted storage: x . c + b = x' . c + (b + s . c)."""
    sh = getattr(X, "shift", None)
    return float(intercept) if sh is None else float(intercept) + sh.dot(coef)


def predict(X, coef, intercept: float) -> torch.Tensor:
    h = native.hip()
    d, n = X.shape
    intercept = _icpt(X, coef, intercept)
    Xb, xdt, ld, tiled = _x_args(X)
    _check_dev(Xb)
    c = _coef_dev(coef, X.device)
    if c.numel() != d:
        raise ValueError("predict: coefficient length != number of features")
    if isinstance(X, TiledWide) and X.eb == 8:
        c = c * X.scales.to(torch.float64)
    out = torch.empty(n, dtype=torch.float64, device=X.device)
    h.predict(Xb.data_ptr(), xdt, int(ld), int(d), int(n), c.data_ptr(), float(intercept), out.data_ptr(),
              _stream(), tiled)
    return out


def regression_metrics(X, y, coef, intercept, sel, shift):
    h = native.hip()
    d, n = X.shape
    intercept = _icpt(X, coef, intercept)
    Xb, xdt, ld, tiled = _x_args(X)
    _check_dev(Xb, y, sel)
    y = y.contiguous()
    if sel is not None:
        sel = sel.contiguous().to(torch.bool)
    c = _coef_dev(coef, X.device)
    if isinstance(X, TiledWide) and X.eb == 8:
        c = c * X.scales.to(torch.float64)
    nb = int(h.metrics_blocks(n))
    partials = torch.empty(nb * 8, dtype=torch.float64, device=X.device)
    out = torch.empty(8, dtype=torch.float64, device=X.device)
    h.regression_metrics(Xb.data_ptr(), xdt, int(ld), int(d), int(n), y.data_ptr(), dtype_code(y), _ptr(sel),
                         c.data_ptr(), float(intercept), float(shift), partials.data_ptr(), out.data_ptr(), _stream(),
                         tiled)
    return out


def huber_pass(X, y, w, sel, ceff, icpt, sigma, eps):
    h = native.hip()
    d, n = X.shape
    icpt = _icpt(X, ceff, icpt)
    Xb, xdt, ld, tiled = _x_args(X)
    _check_dev(Xb, y, w, sel)
    y, w, sel = _prep_rows(y, w, sel, n)
    c = _coef_dev(ceff, Xb.device)
    fp8 = isinstance(X, TiledWide) and X.eb == 8
    if fp8:
        c = c * X.scales.to(torch.float64)
    mult = torch.empty(max(n, 1) if d > 16 else 1, dtype=torch.float64, device=Xb.device)
    partials = torch.empty(int(h.huber_partials(n, d)), dtype=torch.float64, device=Xb.device)
    out = torch.empty(4 + d, dtype=torch.float64, device=Xb.device)
    h.huber_pass(Xb.data_ptr(), xdt, int(ld), int(d), int(n), tiled, y.data_ptr(), dtype_code(y), _ptr(w),
                 dtype_code(w) if w is not None else 0, _ptr(sel), c.data_ptr(), float(icpt), float(sigma), float(eps),
                 mult.data_ptr(), partials.data_ptr(), out.data_ptr(), _stream())
    if fp8:  # the row pass saw q = x / scale
        out[4:] *= X.scales.to(torch.float64)
    sh = getattr(X, "shift", None)
    if sh is not None:  # Σ m x = Σ m x' + s Σ m  (out[2] = Σ m over the live rows)
        out[4:] += sh.dev64 * out[2]
    return out


def huber_fit_dp(X, y, w, sel, sx: torch.Tensor, lam: torch.Tensor, fit_icpt: bool, eps: float, max_iter: int,
                 tol: float, all_reduce=None, batch: int = 4):
    """The Huber fit with the L-BFGS-B state on the device (``huber_qn.hip``): per evaluation the
    row pass over THIS rank's rows at the trial the control kernel wrote (``huber_pass_dev``), the
    all-reduce of its (d + 4) f64 (``all_reduce``: in place on the current stream, or None on one
    rank), then the control kernel.  ``sx`` / ``lam``: f64 device vectors (feature std, L2
    weights).  Nothing is read back per evaluation: evaluations are enqueued ``batch`` at a time,
    at most two batches ahead of the device, until a pinned copy of the control word reads done.
    Returns the output block ``[coef (d) | intercept | scale | status | why | states | iterations |
    evaluations | - | history]`` (status 9: evaluation bound reached, 2: history capacity) and
    the workspaces the enqueued kernels use (keep them alive until the output is read)."""
    import time

    h = native.hip()
    d, n = X.shape
    d, n = int(d), int(n)
    Xb, xdt, ld, tiled = _x_args(X)
    _check_dev(Xb, y, w, sel)
    y, w, sel = _prep_rows(y, w, sel, n)
    dev = Xb.device
    if sx.numel() != d or lam.numel() != d:
        raise ValueError("huber_fit_dp: sx / lam must hold d values")
    sx = sx.to(device=dev, dtype=torch.float64).contiguous()
    lam = lam.to(device=dev, dtype=torch.float64).contiguous()
    scale = X.scales.to(torch.float64).contiguous() if isinstance(X, TiledWide) and X.eb == 8 else None
    sh = getattr(X, "shift", None)
    shift = None if sh is None else sh.dev64.to(dev).contiguous()
    cap = wls_qn_cap(max_iter)
    work = torch.zeros(int(h.huber_qn_work(d, bool(fit_icpt))), dtype=torch.float64, device=dev)
    act = work[:1].view(torch.int32)[:1]  # HCtl.act: the struct's first word
    trial = torch.zeros(d + 2, dtype=torch.float64, device=dev)
    red = torch.zeros(4 + d, dtype=torch.float64, device=dev)
    mult = torch.empty(max(n, 1) if d > 16 else 1, dtype=torch.float64, device=dev)  # (d > 16: the Xᵀm pass)
    partials = torch.empty(int(h.huber_partials(n, d)), dtype=torch.float64, device=dev)
    out = torch.zeros(int(h.huber_qn_out(d, cap)), dtype=torch.float64, device=dev)
    out[d + 2:d + 3].fill_(9.0)
    st = _stream()
    qn = (d, bool(fit_icpt), int(max_iter), float(tol), cap, sx.data_ptr(), lam.data_ptr(), _ptr(scale), _ptr(shift),
          work.data_ptr(), trial.data_ptr())
    rows = (Xb.data_ptr(), xdt, int(ld), d, n, tiled, y.data_ptr(), dtype_code(y), _ptr(w),
            dtype_code(w) if w is not None else 0, _ptr(sel), trial.data_ptr(), act.data_ptr(), float(eps),
            _ptr(scale), _ptr(shift), mult.data_ptr(), partials.data_ptr(), red.data_ptr(), st)
    h.huber_qn_init(*qn, out.data_ptr(), st)
    # a loop pass costs at most 1 + 64 + 64 + 1 evaluations (bracket, zoom, projected point)
    bound = cap * 130 + 2
    flags = torch.empty(2, dtype=torch.int32, pin_memory=True)
    inflight = []
    done, k, slot = False, 0, 0
    while not done and k < bound:
        for _ in range(min(batch, bound - k)):
            h.huber_pass_dev(*rows)
            if all_reduce is not None:
                r = all_reduce(red)
                if r.data_ptr() != red.data_ptr():  # (gloo reduces a host copy)
                    red.copy_(r)
            h.huber_qn_ctl(*qn, red.data_ptr(), out.data_ptr(), st)
            k += 1
        flags[slot].copy_(act[0], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        inflight.append((ev, slot))
        slot ^= 1
        if len(inflight) == 2:
            ev0, s0 = inflight.pop(0)
            while not ev0.query():
                time.sleep(20e-6)
            done = int(flags[s0]) == int(h.HUBER_DONE)
    return out, (work, trial, red, mult, partials, sx, lam, scale, shift, flags, y, w, sel)


# ------------------------------------------------------------------------------------------
# K9 -- squared-loss l-bfgs evaluation passes (lsq.hip)
class LsqPasses:
    """Device state of one squared-loss l-bfgs / OWLQN fit (Spark ``LeastSquaresAggregator``): the
    feature matrix as the kernels read it, the label and the effective row weights (selection and
    label nulls folded in: w = 0) as f64 rows, and the per-evaluation workspaces.  Every method
    enqueues on the current stream and returns device tensors (no host sync)."""

    def __init__(self, X, y, w, sel):
        h = self._h = native.hip()
        d, n = X.shape
        self.d, self.n = int(d), int(n)
        self.scales = None
        self.shift = getattr(X, "shift", None)  # shifted storage: x = x' + s
        if isinstance(X, TiledWide):
            self._xb, self.layout, self.xdt, self.ld = X.buf, (2 if X.eb == 16 else 3), 2, 0
            if X.eb == 8:
                self.scales = X.scales.to(torch.float64)
        elif isinstance(X, TiledBF16):
            self._xb, self.layout, self.xdt, self.ld = X.buf, 1, 2, 0
        else:
            if X.dtype not in (torch.float64, torch.float32, torch.bfloat16):
                X = X.to(torch.float64)
            Xv, ld = _feature_view(X, 4)
            self._xb, self.layout, self.xdt, self.ld = Xv, 0, dtype_code(Xv), int(ld)
        _check_dev(self._xb, y, w, sel)
        dev = self.device = self._xb.device
        if y.numel() != n or (w is not None and w.numel() != n) or (sel is not None and sel.numel() != n):
            raise ValueError("lsq: row-count mismatch between features, label, weight and selection")
        wt = torch.ones(n, dtype=torch.float64, device=dev) if w is None else w.to(torch.float64)
        if sel is not None:
            wt = torch.where(sel.to(torch.bool), wt, torch.zeros_like(wt))
        self.w = wt.contiguous()
        self.y = torch.where(self.w != 0, y.to(torch.float64), torch.zeros_like(self.w)).contiguous()
        self._desc = (self._xb.data_ptr(), self.layout, self.xdt, self.ld, self.d, self.n)
        self.nl = int(h.lsq_margin_blocks(*self._desc))
        self._v = torch.empty(max(self.n, 1), dtype=torch.float64, device=dev)
        self._lpart = torch.empty(self.nl, dtype=torch.float64, device=dev)
        self._part = {m: torch.empty(max(int(h.lsq_part_doubles(*self._desc, m)), 1), dtype=torch.float64,
                                     device=dev) for m in (0, 1)}

    def scalars(self) -> torch.Tensor:
        """[count, wSum, wwSum, Σ w y, Σ w y²] over the live rows."""
        w, y = self.w, self.y
        return torch.stack([(w != 0).sum().to(torch.float64), w.sum(), (w * w).sum(), (w * y).sum(),
                            (w * y * y).sum()])

    def moments(self) -> torch.Tensor:
        """[Σ w x_j (d), Σ w x_j² (d)] (f64; the summarizer pass of the l-bfgs path)."""
        out = torch.empty(2 * self.d, dtype=torch.float64, device=self.device)
        self._h.lsq_columns(*self._desc, 1, self.w.data_ptr(), 0, 0, self._part[1].data_ptr(), out.data_ptr(),
                            _stream())
        if self.scales is not None:  # the pass saw q = x / scale
            out[:self.d] *= self.scales
            out[self.d:] *= self.scales * self.scales
        if self.shift is not None:  # Σw x = Σw x' + sΣw,  Σw x² = Σw x'² + 2sΣw x' + s²Σw
            s, W = self.shift.dev64, self.w.sum()
            m1 = out[:self.d].clone()
            out[self.d:] += (2.0 * s) * m1 + (s * s) * W
            out[:self.d] += s * W
        return out

    def evaluate(self, cf: torch.Tensor, offset: torch.Tensor, inv_ystd: float) -> torch.Tensor:
        """[Σ ½ w diff², Σ w diff x_j (d)] with diff = x . cf + offset - y * inv_ystd (f64; ``offset``
        a one-element device tensor, read by the kernel: launching a pass needs no host sync)."""
        c = cf.to(torch.float64)
        off = offset.to(torch.float64).reshape(1)
        if self.shift is not None:  # x . c + off = x' . c + (off + s . c)
            off = off + (self.shift.dev64 * c).sum().reshape(1)
        off = off.contiguous()
        if self.scales is not None:
            c = c * self.scales
        c = c.contiguous() if self.layout == 0 else c.to(torch.float32).contiguous()
        out = torch.empty(1 + self.d, dtype=torch.float64, device=self.device)
        st = _stream()
        self._h.lsq_margin(*self._desc, c.data_ptr(), off.data_ptr(), float(inv_ystd), self.y.data_ptr(),
                           self.w.data_ptr(), self._v.data_ptr(), self._lpart.data_ptr(), st)
        self._h.lsq_columns(*self._desc, 0, self._v.data_ptr(), self._lpart.data_ptr(), self.nl,
                            self._part[0].data_ptr(), out.data_ptr(), st)
        if self.scales is not None:
            out[1:] *= self.scales
        if self.shift is not None:  # Σ v x = Σ v x' + s Σ v  (v = w diff per row)
            out[1:] += self.shift.dev64 * self._v[:self.n].sum()
        return out

    def wmargins(self, cf: torch.Tensor) -> torch.Tensor:
        """u = w (x' . cf) per row (f64 [n], a fresh tensor): the coefficient-linear part of a
        trial's v = w diff, so a line search's trials are u(x) + alpha u(dir) (``evaluate_u``)."""
        c = cf.to(torch.float64)
        if self.scales is not None:
            c = c * self.scales
        c = c.contiguous() if self.layout == 0 else c.to(torch.float32).contiguous()
        zero = torch.zeros(1, dtype=torch.float64, device=self.device)
        self._h.lsq_margin(*self._desc, c.data_ptr(), zero.data_ptr(), 0.0, self.y.data_ptr(), self.w.data_ptr(),
                           self._v.data_ptr(), self._lpart.data_ptr(), _stream())
        return self._v[:self.n].clone()

    def evaluate_u(self, u: torch.Tensor, cf: torch.Tensor, offset: torch.Tensor, inv_ystd: float) -> torch.Tensor:
        """``evaluate`` from the trial's u = w (x' . cf) (``wmargins``, combined along the line): v =
        u + w (offset - y inv_ystd), the loss Σ ½ v² / w, then the column pass alone (one read of X)."""
        c = cf.to(torch.float64)
        off = offset.to(torch.float64).reshape(())
        if self.shift is not None:
            off = off + (self.shift.dev64 * c).sum()
        v = u + self.w * (off - self.y * inv_ystd)
        live = self.w != 0
        loss = torch.where(live, 0.5 * v * v / torch.where(live, self.w, torch.ones_like(self.w)), torch.zeros_like(v)).sum()
        self._v[:self.n].copy_(v)
        self._lpart.zero_()
        self._lpart[:1].copy_(loss.reshape(1))
        out = torch.empty(1 + self.d, dtype=torch.float64, device=self.device)
        self._h.lsq_columns(*self._desc, 0, self._v.data_ptr(), self._lpart.data_ptr(), self.nl,
                            self._part[0].data_ptr(), out.data_ptr(), _stream())
        if self.scales is not None:
            out[1:] *= self.scales
        if self.shift is not None:
            out[1:] += self.shift.dev64 * v.sum()
        return out


    def qn_eligible(self) -> bool:
        """The device l-bfgs / OWLQN forms apply: wide tile layout, 1 <= d <= LSQ_QN_MAX_D (an empty
        row shard is eligible: its passes contribute zero partials)."""
        return self.layout in (2, 3) and 1 <= self.d <= int(self._h.LSQ_QN_MAX_D)

    def qn_fit(self, head: torch.Tensor, fit_icpt: bool, std_f: bool, reg: float, enet: float, max_iter: int,
               tol: float) -> Optional[torch.Tensor]:
        """The whole squared-loss l-bfgs / OWLQN fit as ONE grid launch (``lsq_qn.hip``):
        standardization from the summarizer ``head`` ([scalars(5), moments(2d)], on the device),
        one fused data pass per cost evaluation, the Breeze control flow on the device.  Enqueued
        on the current stream, no host sync.  Returns ``[coef(d), intercept, status, reason, H,
        iterations, spare, head(5), history(cap)]`` or None (not a wide tile layout / d too large)."""
        h = self._h
        if self.layout not in (2, 3) or not 1 <= self.d <= int(h.LSQ_QN_MAX_D) or self.n < 1:
            return None
        key = (self.device.index, self.layout, self.d)
        nb = _lsq_qn_grid.get(key)
        if nb is None:
            nb = _lsq_qn_grid[key] = int(h.lsq_qn_blocks(self.layout, self.d))
        cap = wls_qn_cap(max_iter)
        work = torch.empty(int(h.lsq_qn_work(self.d, nb, self.n)), dtype=torch.float64, device=self.device)
        out = torch.empty(self.d + 11 + cap, dtype=torch.float64, device=self.device)
        head = head.to(torch.float64).contiguous()
        if head.numel() != 5 + 2 * self.d:
            raise ValueError("lsq_qn: the summarizer head must hold 5 + 2d values")
        shift = None if self.shift is None else self.shift.dev64.to(self.device).contiguous()
        h.lsq_qn(self._xb.data_ptr(), self.layout, self.d, self.n, self.y.data_ptr(), self.w.data_ptr(),
                 _ptr(self.scales), _ptr(shift), head.data_ptr(), bool(fit_icpt), bool(std_f), float(reg), float(enet),
                 int(max_iter), float(tol), cap, work.data_ptr(), nb, out.data_ptr(), _stream())
        self._qn_keep = (work, head, shift)  # alive until the launch has run (caching allocator reuse)
        return out


    def qn_fit_dp(self, head: torch.Tensor, fit_icpt: bool, std_f: bool, reg: float, enet: float, max_iter: int,
                  tol: float, all_reduce, batch: int = 4) -> Optional[torch.Tensor]:
        """Data-parallel form of :meth:`qn_fit` (X4, ``lsq_qn.hip`` ``lsq_qn_dp_*``): per cost
        evaluation the pass + fold kernels over THIS rank's rows, ``all_reduce`` (in place, on the
        current stream) of the (d + 2) f64 partials, then a one-block control kernel holding the
        Breeze state machine in HBM.  ``head`` must already be summed over the ranks.  Nothing is
        read back per evaluation: evaluations are enqueued ``batch`` at a time, at most two batches
        ahead of the device, and enqueueing stops once a pinned copy of the state's action reads
        "done" (the kernels of a batch enqueued past the end return at once).  Same output layout
        as :meth:`qn_fit`.

        Host-synchronous in time, not in API: no call here blocks on the device (events are
        polled, copies are pinned and non-blocking, so ``sync_debug_mode("error")`` stays quiet),
        but the host keeps enqueueing until the optimizer is done -- under collectives an
        ``dq4ml.fit.async`` l-bfgs fit therefore returns only after the device fit has run.  (The
        one-launch single-rank form, :meth:`qn_fit`, returns at once.)"""
        import time

        h = self._h
        if not self.qn_eligible():  # (the caller has agreed eligibility over the ranks)
            return None
        key = (self.device.index, self.layout, self.d)
        nb = _lsq_qn_grid.get(key)
        if nb is None:
            nb = _lsq_qn_grid[key] = int(h.lsq_qn_blocks(self.layout, self.d))
        cap = wls_qn_cap(max_iter)
        d, n = self.d, self.n
        work = torch.empty(int(h.lsq_qn_dp_work(d, nb, n)), dtype=torch.float64, device=self.device)
        red_off, ctl_off = int(h.lsq_qn_dp_red_offset(d, nb, n)), int(h.lsq_qn_dp_ctl_offset(d, nb, n))
        red = work[red_off:red_off + d + 2]
        act = work[ctl_off:ctl_off + 1].view(torch.int32)[:1]  # Ctl.act: the struct's first word
        out = torch.zeros(d + 11 + cap, dtype=torch.float64, device=self.device)
        out[d + 1:d + 2].fill_(9.0)  # status "not finished" (evaluation bound reached: the host path re-runs)
        head = head.to(torch.float64).contiguous()
        if head.numel() != 5 + 2 * d:
            raise ValueError("lsq_qn: the summarizer head must hold 5 + 2d values")
        shift = None if self.shift is None else self.shift.dev64.to(self.device).contiguous()
        st = _stream()
        args = (self._xb.data_ptr(), self.layout, d, n, self.y.data_ptr(), self.w.data_ptr(), _ptr(self.scales),
                _ptr(shift), head.data_ptr(), bool(fit_icpt), bool(std_f), float(reg), float(enet), int(max_iter),
                float(tol), cap, work.data_ptr(), nb, out.data_ptr())
        h.lsq_qn_dp(0, *args, st)
        # every line search ends within 21 evaluations and a fit within cap loop passes
        bound = cap * 22 + 2
        flags = torch.empty(2, dtype=torch.int32, pin_memory=True)
        inflight = []  # (event, flag slot) per enqueued batch
        done, k, slot = False, 0, 0
        while not done and k < bound:
            for _ in range(min(batch, bound - k)):
                h.lsq_qn_dp(1, *args, st)
                r = all_reduce(red)
                if r.data_ptr() != red.data_ptr():  # (gloo reduces a host copy)
                    red.copy_(r)
                h.lsq_qn_dp(2, *args, st)
                k += 1
            flags[slot].copy_(act[0], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            inflight.append((ev, slot))
            slot ^= 1
            if len(inflight) == 2:  # the device has the newer batch queued: wait for the older one
                ev0, s0 = inflight.pop(0)
                while not ev0.query():
                    time.sleep(20e-6)
                done = int(flags[s0]) == 3
        self._qn_keep = (work, head, shift, flags)
        return out


_lsq_qn_grid = {}


# ------------------------------------------------------------------------------------------
def wls_small(flat: torch.Tensor, nf: int, fit_intercept: bool, reg: float, enet: float, std_f: bool,
              std_l: bool) -> torch.Tensor:
    """Device WLS Cholesky (k <= 65) from the flat statistics, enqueued on the current stream:
    returns ``[coef(nf), intercept, status, count, wSum, wwSum, bSum, bbSum]`` (no host sync)."""
    h = native.hip()
    _check_dev(flat)
    if flat.dtype != torch.float64 or flat.numel() != 5 + 2 * nf + nf * (nf + 1) // 2:
        raise ValueError("wls_small: flat statistics have the wrong dtype/length")
    out = torch.empty(nf + 7, dtype=torch.float64, device=flat.device)
    h.wls_small(flat.data_ptr(), int(nf), bool(fit_intercept), float(reg), float(enet), bool(std_f), bool(std_l),
                out.data_ptr(), _stream())
    return out


def wls_qn_cap(max_iter: int) -> int:
    """objectiveHistory capacity of ``wls_qn_small``: one entry per loop pass (accepted steps plus
    at most one failed search before each)."""
    return 2 * max(int(max_iter), 0) + 8


def wls_qn_small(flat: torch.Tensor, nf: int, fit_intercept: bool, reg: float, enet: float, std_f: bool,
                 std_l: bool, max_iter: int, tol: float) -> torch.Tensor:
    """Device OWLQN (L1 WLS) from the flat statistics, enqueued on the current stream, no host
    round trip: ``[coef(nf), intercept, status, count, wSum, wwSum, bSum, bbSum, H, reason,
    history...]``.  k <= 128: one wave (``wls_qn_kernel``); up to ``WLS_QN_GRID_MAX_K``: one
    co-resident grid launch (``wls_qn_grid.hip``) with its scratch allocated here."""
    h = native.hip()
    _check_dev(flat)
    k = nf + 1 if fit_intercept else nf
    if flat.dtype != torch.float64 or flat.numel() != 5 + 2 * nf + nf * (nf + 1) // 2:
        raise ValueError("wls_qn_small: flat statistics have the wrong dtype/length")
    if not 1 <= k <= int(h.WLS_QN_GRID_MAX_K):
        raise ValueError(f"wls_qn_small: k = {k} out of range")
    cap = wls_qn_cap(max_iter)
    out = torch.empty(nf + 9 + cap, dtype=torch.float64, device=flat.device)
    if k <= int(h.WLS_QN_MAX_K):
        h.wls_qn_small(flat.data_ptr(), int(nf), bool(fit_intercept), float(reg), float(enet), bool(std_f),
                       bool(std_l), int(max_iter), float(tol), cap, out.data_ptr(), _stream())
        return out
    nb = _qn_grid_blocks(h, k)
    work = torch.empty(int(h.wls_qn_grid_work(k, nb)), dtype=torch.float64, device=flat.device)
    h.wls_qn_grid(flat.data_ptr(), int(nf), bool(fit_intercept), float(reg), float(enet), bool(std_f), bool(std_l),
                  int(max_iter), float(tol), cap, work.data_ptr(), nb, out.data_ptr(), _stream())
    return out


_qn_grid_plan = {}


def _qn_grid_blocks(h, k):
    key = (torch.cuda.current_device(), k)
    nb = _qn_grid_plan.get(key)
    if nb is None:
        nb = _qn_grid_plan[key] = int(h.wls_qn_grid_blocks(int(k)))
    return nb


# control-block layout of wls_large.h (WlsPcgState), checked against the module on first use
PCG_STATE_WORDS, PCG_CONV, PCG_BAD, PCG_OK, PCG_ITERS, PCG_STATUS, PCG_HEAD = 24, 3, 4, 5, 6, 7, 12
PCG_WSUM, PCG_BSTD = 8, 9


@dataclass
class WlsSystem:
    """The standardized dense WLS system on the device (``wls_large.hip``) and its PCG workspace."""
    A: torch.Tensor      # [k, k] f64 row-major (symmetric)
    b: torch.Tensor      # [k]
    minv: torch.Tensor   # [k] Jacobi preconditioner
    aStd: torch.Tensor   # [nf] population std of every feature
    o: torch.Tensor      # control block [state(PCG_STATE_WORDS) | x(k) | coef(nf)]
    k: int
    work: torch.Tensor   # [3k] PCG vectors r | p | Ap


def wls_assemble(flat: torch.Tensor, nf: int, fit_intercept: bool, reg: float, enet: float, std_f: bool,
                 std_l: bool) -> WlsSystem:
    """Standardized dense system of the large-k WLS branch from the flat statistics, enqueued with
    NO host read: the head scalars (wSum, label mean and std, effective L2) and the short-circuit
    status are computed on the device into the control block (``o[PCG_STATUS]`` set: the host
    driver owns the case; ``o[PCG_HEAD:+5]`` the raw head statistics)."""
    h = native.hip()
    _check_dev(flat)
    if (int(h.PCG_STATE_WORDS), int(h.PCG_CONV), int(h.PCG_BAD), int(h.PCG_OK), int(h.PCG_ITERS),
            int(h.PCG_STATUS), int(h.PCG_HEAD), int(h.PCG_WSUM), int(h.PCG_BSTD)) != (
                PCG_STATE_WORDS, PCG_CONV, PCG_BAD, PCG_OK, PCG_ITERS, PCG_STATUS, PCG_HEAD, PCG_WSUM, PCG_BSTD):
        raise RuntimeError("wls_large: control-block layout mismatch between device.py and the HIP module")
    if flat.dtype != torch.float64 or flat.numel() != 5 + 2 * nf + nf * (nf + 1) // 2:
        raise ValueError("wls_assemble: flat statistics have the wrong dtype/length")
    k = nf + 1 if fit_intercept else nf
    dev = flat.device
    A = torch.empty(k, k, dtype=torch.float64, device=dev)
    vec = torch.empty(2 * k + 3 * nf, dtype=torch.float64, device=dev)
    b, minv = vec[:k], vec[k:2 * k]
    aStd, aBar, lam = vec[2 * k:2 * k + nf], vec[2 * k + nf:2 * k + 2 * nf], vec[2 * k + 2 * nf:]
    o = torch.zeros(PCG_STATE_WORDS + k + nf, dtype=torch.float64, device=dev)
    h.wls_assemble(flat.data_ptr(), int(nf), bool(fit_intercept), float(reg), float(enet), bool(std_f), bool(std_l),
                   A.data_ptr(), b.data_ptr(), minv.data_ptr(), aStd.data_ptr(), aBar.data_ptr(), lam.data_ptr(),
                   o.data_ptr(), _stream())
    return WlsSystem(A, b, minv, aStd, o, k, torch.empty(3 * k, dtype=torch.float64, device=dev))


def wls_pcg_enqueue(sysm: WlsSystem, nf: int, rtol: float, iters: int) -> None:
    """Jacobi-PCG start + ``iters`` iterations + the true-residual check, enqueued with no host
    read (iterations after convergence -- or on a STATUS / BAD system -- exit at once)."""
    h = native.hip()
    k = sysm.k
    r, p = sysm.work[:k], sysm.work[k:2 * k]
    h.wls_pcg_init(sysm.b.data_ptr(), sysm.minv.data_ptr(), k, float(rtol), sysm.o.data_ptr(), r.data_ptr(),
                   p.data_ptr(), _stream())
    wls_pcg_more(sysm, nf, iters)


def wls_pcg_more(sysm: WlsSystem, nf: int, iters: int) -> None:
    """``iters`` more PCG iterations (+ the residual check) on the current stream."""
    h = native.hip()
    k = sysm.k
    r, p, Ap = sysm.work[:k], sysm.work[k:2 * k], sysm.work[2 * k:]
    h.wls_pcg_chunk(sysm.A.data_ptr(), sysm.b.data_ptr(), sysm.minv.data_ptr(), sysm.aStd.data_ptr(), k, int(nf),
                    int(iters), sysm.o.data_ptr(), r.data_ptr(), p.data_ptr(), Ap.data_ptr(), _stream())


def wls_pcg_drive(sysm: WlsSystem, nf: int, o: np.ndarray, done: int, chunk: int = 8, max_iter: int = 96) -> np.ndarray:
    """Continue a PCG whose host control block ``o`` (after ``done`` iterations) has not converged:
    ``chunk`` iterations per host check, up to ``max_iter``.  Returns the last host control block."""
    while (o[PCG_CONV] == 0.0 and o[PCG_STATUS] == 0.0 and o[PCG_BAD] == 0.0 and done < max_iter):
        wls_pcg_more(sysm, nf, chunk)
        done += chunk
        o = sysm.o.cpu().numpy()
    return o


def wls_pcg(sysm: WlsSystem, nf: int, rtol: float, chunk: int = 8, max_iter: int = 96) -> np.ndarray:
    """Jacobi-PCG on the assembled system, ``chunk`` iterations per host check (one D2H of the
    control block).  Returns the host control block ``[state | x | coef]``; it holds a usable
    solution iff ``pcg_ok(o)`` -- CG converged AND the true residual passed, no short-circuit
    status, every diagonal entry > 0 (else the caller takes the host driver / Cholesky)."""
    wls_pcg_enqueue(sysm, nf, rtol, chunk)
    return wls_pcg_drive(sysm, nf, sysm.o.cpu().numpy(), chunk, chunk, max_iter)


def pcg_ok(o: np.ndarray) -> bool:
    return o[PCG_STATUS] == 0.0 and o[PCG_BAD] == 0.0 and o[PCG_CONV] != 0.0 and o[PCG_OK] != 0.0


# ------------------------------------------------------------------------------------------
# wide (d > 64) fragment layouts + LDS-tiled MFMA SYRK
# ------------------------------------------------------------------------------------------
def _srcw_desc(h, rows, dev):
    desc = np.zeros((len(rows), 2), dtype=np.int64)  # PackSrcW {ptr, dt, pad}
    for i, r in enumerate(rows):
        desc[i, 0] = r.data_ptr()
        desc[i, 1] = dtype_code(r)
    return _h2d(desc.reshape(-1).view(np.uint8), dev)


def _rows_of(parts):
    rows = []
    for p in parts:
        if p.dim() == 1:
            p = p.unsqueeze(0)
        for i in range(p.shape[0]):
            r = p[i]
            rows.append(r if r.is_contiguous() else r.contiguous())
    return rows


def pack_wide(parts: List[torch.Tensor], eb: int, sel: Optional[torch.Tensor] = None, nt: Optional[int] = None,
              inv_scale: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
              shift="auto") -> TiledWide:
    """Columns -> wide fragment layout (eb 16 = bf16, 8 = fp8 with per-feature scales) of x - s.

    ``shift``: "auto" = the sampled per-column shift (ops/shift.py), the same on every
    data-parallel rank (the banded wide fold all-reduces shifted statistics); None = unshifted; or
    an ``ops.shift.Shift``.  fp8 scales are those of the shifted columns.

    The layout is superstep-major, so row blocks that are multiples of 64 rows pack independently
    into consecutive byte ranges of one image (``out``: a uint8 view of that range) — used to
    stream-ingest matrices larger than one staging copy; such a block-wise ingest must pass the
    whole matrix's ``shift`` (and ``inv_scale``) explicitly."""
    h = native.hip()
    dev = parts[0].device
    rows = _rows_of(parts)
    for r in rows:
        _check_dev(r)
    d, n = len(rows), rows[0].numel()
    if isinstance(shift, str) and out is not None:
        raise ValueError("pack_wide: a block-wise ingest (out=) needs the whole matrix's shift (None or a Shift)")
    shift = _auto_shift(rows, shift, uniform=True)
    desc = _srcw_desc(h, rows, dev)
    if sel is not None:
        sel = sel.contiguous().to(torch.bool)
    scales = None
    if eb == 8 and inv_scale is None:
        amax = torch.empty(d, dtype=torch.float32, device=dev)
        h.feature_amax(desc.data_ptr(), d, n, _ptr(sel), amax.data_ptr(), _stream(), _sptr(shift))
        scales = torch.where(amax > 0, amax / FP8_MAX, torch.ones_like(amax))
        inv_scale = 1.0 / scales
    elif eb == 8:
        scales = 1.0 / inv_scale
    nt = nt or ((d + 255) // 256) * 8
    nbytes = ((n + 63) // 64) * nt * 4 * 64 * eb
    if out is not None:
        if out.dtype != torch.uint8 or out.numel() != nbytes or not out.is_contiguous() or out.device != dev:
            raise ValueError(f"pack_wide: out must be a contiguous uint8 tensor of {nbytes} bytes on {dev}")
        buf = out
    else:
        buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    h.pack_wide(eb, desc.data_ptr(), d, n, nt, _ptr(sel), _ptr(inv_scale), buf.data_ptr(), _stream(), _sptr(shift))
    del rows
    return TiledWide(buf, d, n, eb, scales, shift)


def mask_wide_rows(T: TiledWide, sel: torch.Tensor) -> TiledWide:
    """A copy of ``T`` whose rows with ``sel == False`` are zero (fp8 zero = 0x00, bf16 +0)."""
    h = native.hip()
    _check_dev(T.buf, sel)
    if sel.numel() != T.n:
        raise ValueError("mask_wide_rows: selection length != rows")
    s = sel.contiguous().to(torch.bool)
    if s.data_ptr() % 8:
        s = s.clone()
    out = torch.empty_like(T.buf)
    if out.numel() != int(h.wide_tiled_bytes(T.eb, T.d, T.n)):
        raise ValueError("mask_wide_rows: storage size does not match the wide layout")
    h.wide_mask_rows(T.eb, T.buf.data_ptr(), out.data_ptr(), T.d, T.n, s.data_ptr(), _stream())
    return TiledWide(out, T.d, T.n, T.eb, T.scales, T.shift)


def tile_wide(X: torch.Tensor, eb: int, sel: Optional[torch.Tensor] = None) -> TiledWide:
    return pack_wide([X], eb, sel)


_zero_pages = {}


def _zero_page(h, dev):
    z = _zero_pages.get(dev)
    if z is None:
        z = _zero_pages[dev] = torch.zeros(int(h.WIDE_ZERO_BYTES), dtype=torch.uint8, device=dev)
    return z


def _morton(i: int, j: int) -> int:
    z = 0
    for b in range(16):
        z |= ((i >> b) & 1) << (2 * b + 1) | ((j >> b) & 1) << (2 * b)
    return z


def _wide_pairs(P: int, order: str = "morton"):
    """Upper panel pairs (I <= J) over [0, P] (P = augmentation panel) in launch order.  Blocks
    that one XCD runs together are consecutive in this list (the kernel's XCD remap), so a
    Z-order walk makes them share few panels (~12 per 32 blocks instead of ~18 row-major) and
    those hit that XCD's L2.  Partials are stored by row-major pair index, so order is free."""
    pairs = [(i, j) for i in range(P + 1) for j in range(i, P + 1)]
    if order == "morton":
        pairs.sort(key=lambda p: _morton(*p))
    return pairs


def _wide_splitk(P: int, nsup: int, eb: int) -> int:
    """Split-K so the real (non-augmentation) panel-pair blocks fill whole waves of the 256 CUs
    (1 block/CU at bf16's 128 KiB LDS, 2 at fp8's 64 KiB)."""
    npr = P * (P + 1) // 2 + 0.25 * (P + 1)  # augmentation blocks run at load speed
    slots = 256  # 128 KiB LDS ring: one block per CU
    best, best_eff = 1, 0.0
    for k in range(1, 257):
        if k > nsup:
            break
        blocks = npr * k
        eff = blocks / (-(-blocks // slots) * slots)
        if blocks >= 2 * slots and eff >= 0.9:
            return k
        if eff > best_eff + 1e-9:
            best, best_eff = k, eff
    return best


def _wide_queue_h(nsup: int) -> int:
    """Row ranges per XCD group of the persistent wide schedule (``DQ4ML_WIDE_H``, default 2:
    ~10 units per block keeps the dynamic tail short); 0 = too few rows, use the static grid.
    f32 accumulators count rows exactly only below 2^24 per split."""
    hq = int(os.environ.get("DQ4ML_WIDE_H", "2"))
    if nsup < 8 * 16:
        return 0
    hq = max(hq, -(-nsup * 64 // (8 << 23)))
    return max(1, min(hq, nsup // 16))


def _wide_gang_s(P: int, nsup: int, G: int) -> int:
    """Row ranges per XCD group of the gang schedule (0: not applicable).  The P(P+1)/2 units of a
    range times S must be a multiple of the G blocks of a group, so every block runs the same
    number of equal-cost units (P = 16, G = 32: S = 4, 17 units per block); f32 accumulators
    count rows exactly only below 2^24 per split, and every split keeps >= 16 supersteps."""
    npu = P * (P + 1) // 2
    s_min = max(1, -(-nsup * 64 // (8 << 23)))
    forced = int(os.environ.get("DQ4ML_WIDE_GANG_S", "0"))  # (tests / A/B) a fixed S
    if forced:
        return forced if s_min <= forced and 8 * forced <= nsup else 0
    best, best_eff = 0, 0.0
    for S in range(s_min, s_min + 32):
        if nsup < 8 * S * 16:
            break
        units = npu * S
        eff = units / (-(-units // G) * G)
        if eff > best_eff + 1e-9:
            best, best_eff = S, eff
        if eff == 1.0:
            break
    return best if best_eff >= 0.9 else 0


_wide_grids = {}


def _wide_grid(h) -> int:
    """One block per CU (the ring uses the whole LDS), rounded down to whole XCD groups."""
    dev = torch.cuda.current_device()
    if dev not in _wide_grids:
        cus = int(h.device_info()["multiProcessorCount"])
        _wide_grids[dev] = max(8, cus // 8 * 8)
    return _wide_grids[dev]


@dataclass
class _WideSchedule:
    """Launch constants of one wide Gram shape (cached: a repeated fit re-uses the device tables
    and the split choice instead of rebuilding and re-uploading them)."""
    sched: str            # "gang" | "queue" | "grid"
    splitk: int
    S: int                # gang row ranges per group (0: not the gang schedule)
    hq: int               # queue row ranges per group (0: not the queue schedule)
    pairs_dev: torch.Tensor  # pair list (queue / grid) or the gang's int4 unit table
    units: int = 0        # gang units per group
    tile_base: Optional[torch.Tensor] = None  # gang: [npair + 1] partial-tile prefix per pair
    tiles: int = 0        # partial tiles in all
    pairs_list: Optional[torch.Tensor] = None  # classic gang: off-diagonal pairs, then diagonal ones


# Long gang units (the table form of the gang kernel) only while a row range is short: a long unit
# runs its S ranges back to back with no round barrier inside.  At the 8-GPU shard (610 supersteps
# per range) the 4x smaller fold pays; at 1e7 rows (4883 per range) long units ran 67.1 -> 69.2 ms
# per pass, sclk -2 % at the same board power (same-box A/B, profiles/r6/ab_energy_long_units_fixed.log),
# so long row ranges run the classic gang list (units decoded from u, uniform tile layout).
_LONG_UNIT_MAX_SUP = 1024


def _gang_table(P: int, S: int, G: int, long_units: bool = True):
    """The gang schedule's unit table and per-pair partial-tile prefix (gram_wide.hip
    gram_wide_gang_kernel).  A group of G blocks covers S row ranges of the panel pairs:

    * off-diagonal pairs, as many whole multiples of G as there are: one LONG unit each over all
      S ranges (block l takes G-strided pairs; every block of a round sweeps the same rows, so
      each panel-stage still comes from HBM once per round) -- ONE partial tile per group instead
      of S, so the split-K fold reads up to S x fewer bytes;
    * the remaining off-diagonal pairs, then the diagonal ones (which carry the augmentation
      products), one unit per range, range-major -- the round-5 equal-cost units.
    Every block runs the same number of range-units (the G-multiples keep the long units even,
    the short ones deal round-robin as before).  Returns (int4 rows, units, tile_base, tiles)."""
    pairs = _wide_pairs(P)
    off = [p for p in pairs if p[0] != p[1] and p[1] < P]
    diag = [p for p in pairs if p[0] == p[1] and p[1] < P]
    n_long = (len(off) // G) * G if S > 1 and long_units else 0
    units = [(p, 0, S) for p in off[:n_long]]
    units += [(p, s, 1) for s in range(S) for p in off[n_long:]]
    units += [(p, s, 1) for s in range(S) for p in diag]
    K, kk, rows = {}, {}, []
    for p, _, _ in units:
        K[p] = K.get(p, 0) + 1
    for p, s0, ns in units:
        k = kk.get(p, 0)
        kk[p] = k + 1
        rows.append((p[0], p[1], s0 | (ns << 16), k | (K[p] << 16)))
    # tiles per pair, row-major over I <= J in [0, P]: 8 groups x K; the augmentation column's
    # pairs (I, P) are written by (I, I)'s units, (P, P) by (0, 0)'s
    base, t = [], 0
    for i in range(P + 1):
        for j in range(i, P + 1):
            base.append(t)
            src = (i, j) if j < P else ((i, i) if i < P else (0, 0))
            t += 8 * K.get(src, 0)
    base.append(t)
    return rows, len(units), base, t


_wide_sched_cache = {}
_last_gang_bar = None


def _wide_schedule(h, P: int, nsup: int, eb: int, dev) -> _WideSchedule:
    """Gang (default; equal-cost units, 8 XCD groups x S row ranges) when the unit count fills the
    groups to >= 90 %, else the persistent queue, else the static split-K grid (few rows)."""
    grid = _wide_grid(h)
    forced = os.environ.get("DQ4ML_WIDE_SCHED", "gang")
    key = (dev, P, nsup, eb, grid, forced, os.environ.get("DQ4ML_WIDE_GANG_S"), os.environ.get("DQ4ML_WIDE_H"),
           _LONG_UNIT_MAX_SUP)
    sc = _wide_sched_cache.get(key)
    if sc is not None:
        return sc
    pairs = _wide_pairs(P)
    gs = _wide_gang_s(P, nsup, grid // 8) if forced == "gang" else 0
    hq = _wide_queue_h(nsup) if not gs and forced in ("gang", "queue") else 0
    if gs and nsup // (8 * gs) <= _LONG_UNIT_MAX_SUP:
        # (gram_wide.hip gram_wide_gang_kernel<TABLE>: long off-diagonal units, then equal-cost short ones)
        rows, units, base, tiles = _gang_table(P, gs, grid // 8)
        sc = _WideSchedule("gang", 8 * gs, gs, 0, _h2d(np.asarray(rows, dtype=np.int32).reshape(-1), dev), units,
                           _h2d(np.asarray(base, dtype=np.int32), dev), tiles)
        sc.pairs_list = None
        _wide_sched_cache[key] = sc
        return sc
    if gs:  # the classic gang list: one row range per unit, decoded in the kernel, uniform tile layout
        gp = [p for p in pairs if p[0] != p[1] and p[1] < P] + [p for p in pairs if p[0] == p[1] and p[1] < P]
        sc = _WideSchedule("gang", 8 * gs, gs, 0, None, P * (P + 1) // 2 * gs)
        sc.pairs_list = _h2d(np.asarray(gp, dtype=np.int32).reshape(-1), dev)
        sc.tiles = (P + 1) * (P + 2) // 2 * 8 * gs
        _wide_sched_cache[key] = sc
        return sc
    elif hq:
        sched, splitk = "queue", 8 * hq
    else:
        sched = "grid"
        splitk = _wide_splitk(P, nsup, eb)
        # f32 MFMA accumulators count rows exactly only below 2^24 per split
        splitk = max(1, min(max(splitk, -(-nsup * 64 // (1 << 23))), nsup))
    sc = _WideSchedule(sched, splitk, gs, hq, _h2d(np.asarray(pairs, dtype=np.int32).reshape(-1), dev))
    sc.tiles = (P + 1) * (P + 2) // 2 * splitk
    _wide_sched_cache[key] = sc
    return sc


class DeferredWide:
    """Wide SYRK partials whose split-K fold (+ RCCL all-reduce, band by band) has not been
    enqueued yet: an asynchronous overlapped fit runs it on its side stream with the solve, so the
    compute stream goes on to the next fit's SYRK at once -- the fold kernels (no LDS, 22 VGPRs)
    co-reside with the SYRK's one block per CU in its spare wave slots."""

    is_cuda = True

    def __init__(self, run, keep, out):
        self._run, self._keep, self.out = run, keep, out
        self.device = out.device

    def finish(self) -> torch.Tensor:
        st = faststream.current(faststream.dev_index(self.device))
        for t in self._keep:
            if t is not None:
                t.record_stream(st)
        return self._run()


def _gram_wide(h, T: TiledWide, y, w, sel, x_zero_dead, defer: bool = False):
    """Wide (d > 64) statistics: the LDS-tiled MFMA SYRK over the fragment storage plus the label's
    augmentation panel, folded to the flat WLS layout (band by band under RCCL, each band's
    all-reduce in flight while the next folds).  Enqueued on the current stream with NO host read:
    the label split, its scales and the label shift stay on the device, so an asynchronous fit
    (``dq4ml.fit.async``) runs ahead of the GPU."""
    if w is not None:
        # instance weights: the exact-f32 MFMA SYRK (per-row weight in-kernel) on the stored values
        return _gram_syrk(h, T.to_dense(), y, w, sel, compute_f64=False)
    if sel is not None and not x_zero_dead:
        # the stored tiles still hold the dead rows: zero them in one pass over the fragment
        # storage (wide_mask_rows_kernel), no dequantize / re-pack
        T = mask_wide_rows(T, sel)
    d, n = T.d, T.n
    dev = T.device
    _check_dev(T.buf, y, sel)
    y, _, sel = _prep_rows(y, None, sel, n)
    eb = T.eb
    # the label's augmentation panel, split and packed on the device (gram_wide.hip
    # wide_label_*): aux = [1, s_h, s_l | t, 1/s_h, 1/s_l], no host read
    aux = torch.empty(6, dtype=torch.float64, device=dev)
    lpart = torch.empty(int(h.wide_label_part_doubles()), dtype=torch.float64, device=dev)
    aug = TiledWide(torch.empty(max(1, (n + 63) // 64) * 256 * eb, dtype=torch.uint8, device=dev), 3, n, eb, None,
                    None)  # (one 32-feature tile per 64-row superstep)
    h.wide_label_aug(eb, y.data_ptr(), 0 if y.dtype == torch.float64 else 1, n, _ptr(sel), lpart.data_ptr(),
                     aux.data_ptr(), aug.buf.data_ptr(), _stream())
    aug_scale = aux[:3]
    t_y = aux[3:4] if eb == 8 else None
    P = (d + 255) // 256
    nsup = max(1, (n + 63) // 64)
    sc = _wide_schedule(h, P, nsup, eb, dev)
    splitk = sc.splitk
    out = torch.empty(5 + 2 * d + d * (d + 1) // 2, dtype=torch.float64, device=dev)
    part = torch.empty(sc.tiles * 256 * 256, dtype=torch.float32, device=dev)
    # data-parallel fit over RCCL: fold band by band and all-reduce each band while the next folds
    banded = comm.collectives_active() and comm.backend() == "nccl"
    fold_in = not banded and not defer  # the launch folds into `out` itself
    args = (eb, T.buf.data_ptr(), aug.buf.data_ptr(), _zero_page(h, dev).data_ptr(), T.nt, P, d, nsup)
    if sc.sched == "gang":
        # gang schedule (gram_wide_gang_kernel): 8 groups x S row ranges, static equal-cost units,
        # per-round group barrier (full rounds, bounded: the blocks of an XCD start every round
        # together, profiles/r5_wide_limiter.md)
        bar = torch.empty(256, dtype=torch.int32, device=dev)
        global _last_gang_bar
        _last_gang_bar = bar  # (diagnostics: bar[32 g + 1] != 0 -- group g's barrier timed out and went off)
        h.gram_wide_gang(*args, sc.S, _ptr(sc.pairs_dev), _ptr(sc.pairs_list), sc.units, _ptr(sc.tile_base),
                         part.data_ptr(),
                         aug_scale.data_ptr(), _ptr(T.scales), out.data_ptr(), _wide_grid(h), _stream(), fold_in,
                         bar.data_ptr())
    elif sc.sched == "queue":
        # persistent XCD-grouped schedule (gram_wide_queue_kernel): 8 groups x h row ranges
        heads = torch.empty(8, dtype=torch.int32, device=dev)
        h.gram_wide_queue(*args, sc.hq, sc.pairs_dev.data_ptr(), part.data_ptr(), aug_scale.data_ptr(),
                          _ptr(T.scales), out.data_ptr(), heads.data_ptr(), _wide_grid(h), _stream(), fold_in)
    else:
        h.gram_wide(*args, splitk, sc.pairs_dev.data_ptr(), part.data_ptr(), aug_scale.data_ptr(), _ptr(T.scales),
                    out.data_ptr(), _stream(), 5, fold_in)
    if banded and T.shift is not None and not T.shift.uniform:
        raise ValueError("wide Gram over RCCL: the features' shift must be the same on every rank "
                         "(pack_wide(shift='auto') agrees it; a caller-made Shift needs uniform=True)")
    head_fix = (lambda: h.wide_unshift_label(out.data_ptr(), d, aux.data_ptr(), _stream())) if t_y is not None else None
    fold = functools.partial(h.gram_wide_fold, P, d, splitk, part.data_ptr(), aug_scale.data_ptr(), _ptr(sc.tile_base),
                             _ptr(T.scales))

    def finish():
        if banded:
            _fold_all_reduce(fold, out, P, d, head_fix)  # (the label shift is per rank: un-shifted before the wire)
        else:
            if not fold_in:
                fold(out.data_ptr(), 0, 0, P + 1, _stream())
            if head_fix is not None:
                head_fix()
        # statistics of x - s -> of x (f64, after the banded all-reduce too: pack_wide's shift is the
        # same on every rank, so the un-shift of the sum is the sum of the un-shifts)
        return _unshift(h, out, T.shift, d)
    if defer:
        return DeferredWide(finish, (part, aux, T.scales, out, None if T.shift is None else T.shift.dev, sc.tile_base),
                            out)
    return finish()


def wide_bands(P: int, d: int, bucket_bytes: int, elt: int):
    """Panel-column bands [J0, J1) of the wide fold, each a contiguous slice of the flat WLS layout
    of about ``bucket_bytes`` on the wire: the augmentation column (the head: counts, Σy, aSum,
    abSum) first, then runs of 256-wide Gram columns (column j holds j + 1 packed entries).
    Returns [(J0, J1, flat_lo, flat_hi)]."""
    base = 5 + 2 * d
    bands = [(P, P + 1, 0, base)]
    J0, acc = 0, 0
    for J in range(P):
        lo, hi = J * 256, min(d, (J + 1) * 256)
        acc += (hi * (hi + 1) - lo * (lo + 1)) // 2 * elt
        if acc >= bucket_bytes or J == P - 1:
            a, b = J0 * 256, hi
            bands.append((J0, J + 1, base + a * (a + 1) // 2, base + b * (b + 1) // 2))
            J0, acc = J + 1, 0
    return bands


def _fold_all_reduce(fold, out: torch.Tensor, P: int, d: int, head_fix=None):
    """X1 for the wide Gram, overlapped with its own fold: band i's all-reduce is issued right
    after band i's fold is enqueued, so RCCL (its own stream, ordered after the fold at issue
    time) reduces band i over xGMI while the compute stream folds band i + 1.  Wire format
    ``comm.wire_dtype()`` (default f32: the partials are f32 MFMA accumulators already, half the
    bytes of f64 on every link); bands of ``comm.bucket_bytes()``."""
    import torch.distributed as dist

    wire = comm.wire_dtype()
    f32 = wire == torch.float32
    base = 5 + 2 * d
    buf = torch.empty(out.numel(), dtype=torch.float32, device=out.device) if f32 else out
    stream = _stream()
    works = []
    for J0, J1, lo, hi in wide_bands(P, d, comm.bucket_bytes(), buf.element_size()):
        if f32 and J0 != P:
            fold(0, buf.data_ptr(), J0, J1, stream)
            works.append(dist.all_reduce(buf[lo:hi], op=dist.ReduceOp.SUM, async_op=True))
        else:
            # the head band (count, wSum, wwSum, Σy, Σy², aSum, abSum: 5 + 2d values) is always
            # reduced in f64: counts above 2^24 stay exact and the variances E[x²] - E[x]² keep
            # their digits; only the packed Σxx bands may take the f32 wire
            fold(out.data_ptr(), 0, J0, J1, stream)
            if head_fix is not None and J0 == P:
                head_fix()
            works.append(dist.all_reduce(out[lo:hi], op=dist.ReduceOp.SUM, async_op=True))
    for w in works:
        w.wait()  # the compute stream waits for every band's collective
    if f32:
        out[base:].copy_(buf[base:])
    comm.mark_reduced(out)
