"""The DQ chain in the stream Gram's stage prologue: ONE HBM pass for DQ filter + VectorAssembler
+ normal-equation statistics over in-memory columns (BASELINE config 4).

``LinearRegression.fit`` over ``VectorAssembler(f0..f63)`` over a DQ chain (rule UDFs, filters) on
a columnar source is, in Spark, one stage: the filter and the assembler run inside the
``treeAggregate`` seqOp (``DataQuality4MachineLearningApp.java:68-90, 110-126``).  The two-pass form
(``ops/dqvm.py``'s fused kernel writes a selection vector, the stream Gram re-reads it) reads the
rule inputs once and the selection twice more.  Here the stream kernel of ``gram_stream.hip`` is
compiled by hipRTC with the chain lowered into its per-stage row prologue:

* the chain's input columns (not the features) ride the stage's row-scalar DMA — two
  ``global_load_lds`` wave instructions per 64-row stage, each lane's 16-B / 4-B piece sourced
  from the column region it falls in (a per-lane (base, bytes per row) table, read once per wave);
* ``dq_row_pred`` (generated from the same ``dqvm`` lowering as every fused DQ kernel) runs once
  per row per stage on those LDS bytes and yields the live flag and the label; dead rows get
  weight 0, so the MFMA tiles of the features need no mask;
* the features stream as before (f32 source columns DMA'd into swizzled LDS tiles, bf16 or
  exact-f32 MFMA).

Applies when: gramDtype bf16 / fp32 / fp32split, no weights, 9 <= d <= 64 non-null 16-byte-aligned f32
feature columns passed through unchanged by the chain, a chain that ``dqvm`` can fuse without a
raising rule, and its input columns fit the 1280-byte row-scalar area (<= 20 bytes per row).
"""
from __future__ import annotations

import os
import re
from typing import Optional

import numpy as np
import torch

from ..utils.logging import get_logger

__all__ = ["try_fused_stream", "kernel_source", "raw_layout", "STATS", "ENTRY"]

log = get_logger("streamfuse")
ENTRY = "dq_gram_stream"
STATS = {"stream_grams": 0, "stream_replays": 0}
_HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc", "hip")
_text: Optional[str] = None
_CACHE: dict = {}
_TABS: dict = {}
_CUS: dict = {}
_ROUTES: dict = {}  # (plan skey, features, label, gram dtype) -> _Route of the last such action
_MODES = {"bf16": 2, "fp32": 1, "fp32split": 4}  # gramDtype -> GramMode (its kernel: CMP 1 / 0 / 2)

# the stage's row-scalar area: a 16-B-per-lane DMA instruction (1024 B) and a 4-B one (256 B)
RAW16, RAW4 = 1024, 256


def _device_text() -> str:
    """common.h + gram.h + gram_stream.hip as one hipRTC translation unit (their host parts sit
    behind ``#ifndef __HIPCC_RTC__``)."""
    global _text
    if _text is None:
        parts = []
        for name in ("common.h", "gram.h"):
            with open(os.path.join(_HERE, name)) as f:
                parts.append(f.read().replace("#pragma once\n", ""))
        _text = "\n".join(parts)
    return _text


def _stream_text() -> str:
    with open(os.path.join(_HERE, "gram_stream.hip")) as f:
        return f.read()


def raw_layout(cols):
    """Regions of the row-scalar area for the chain's input columns.  ``cols``: [(column index,
    element bytes, nullable)].  Values first (largest elements first), then validity bytes; a
    region goes to the 16-B instruction's 1024 bytes while it fits, else to the 4-B one's 256.
    Returns [(kind 'v'|'m', column, offset, elem bytes)] or None when they do not fit."""
    regs = [("v", c, s) for c, s, _ in sorted(cols, key=lambda t: -t[1])]
    regs += [("m", c, 1) for c, _, nul in cols if nul]
    out, o16, o4 = [], 0, RAW16
    for kind, c, s in regs:
        size = 64 * s
        if o16 + size <= RAW16:
            out.append((kind, c, o16, s))
            o16 += size
        elif o4 + size <= RAW16 + RAW4:
            out.append((kind, c, o4, s))
            o4 += size
        else:
            return None
    return out


def _lane_table(layout, ptrs, vptrs):
    """[64 lanes][instr 16 B: (base, bytes per row), instr 4 B: (base, bytes per row)] + region
    pointers (the guarded tail's sources), as int64."""
    tab = np.zeros(64 * 4 + len(layout), dtype=np.int64)

    def src(off):
        for kind, c, ro, s in layout:
            if ro <= off < ro + 64 * s:
                p = ptrs[c] if kind == "v" else vptrs[c]
                return p + (off - ro), s
        kind, c, ro, s = layout[0]  # an unused piece re-reads region 0 (lands in unused bytes)
        return (ptrs[c] if kind == "v" else vptrs[c]), s

    for lane in range(64):
        tab[4 * lane + 0], tab[4 * lane + 1] = src(16 * lane)
        tab[4 * lane + 2], tab[4 * lane + 3] = src(RAW16 + 4 * lane)
    for k, (kind, c, ro, s) in enumerate(layout):
        tab[256 + k] = ptrs[c] if kind == "v" else vptrs[c]
    return tab


def kernel_source(g, layout, ctypes: dict, yv: str, NT: int, RING: int, CMP: int, yvalid: str = "true") -> str:
    """The hipRTC source: device headers + the generated row predicate / tail fill + the stream
    kernel + an extern "C" instantiation."""
    loads = []
    for kind, c, off, s in layout:
        if kind == "v":
            loads.append(f"  const {ctypes[c]} fzf{c} = reinterpret_cast<const {ctypes[c]}*>(raw + {off})[lane];")
        else:
            loads.append(f"  const bool fzm{c} = raw[{off} + lane] != 0;")
    body = "\n".join("  " + ln.strip() for ln in g.lines)
    fills = []
    for k, (kind, c, off, s) in enumerate(layout):
        t = ctypes[c] if kind == "v" else "unsigned char"
        fills.append(f"  reinterpret_cast<{t}*>(raw + {off})[lane] = in ? "
                     f"reinterpret_cast<const {t}*>(a.rawtab[{256 + k}])[r] : ({t})0;")
    pred = f"""
namespace dq4ml {{
// the DQ chain on row `lane` of a stage's row-scalar area: live flag and label
__device__ __forceinline__ bool dq_row_pred(const unsigned char* raw, int lane, double& y) {{
{chr(10).join(loads)}
  bool live = true;
{body}
  y = (double)({yv});
  return live && ({yvalid});
}}
// the tail stage (rows >= n zero): the predicate's columns copied with row guards
__device__ __forceinline__ void dq_fill_raw(const GramArgs& a, unsigned char* raw, int lane, int64_t r0) {{
  const int64_t r = r0 + lane;
  const bool in = r < a.n;
{chr(10).join(fills)}
}}
}}  // namespace dq4ml
"""
    prelude = ("#ifndef __HIPCC_RTC__\n#define __HIPCC_RTC__ 1\n#endif\n#define DQ4ML_ROW_PRED 1\n"
               "typedef unsigned char uint8_t;\ntypedef unsigned short uint16_t;\ntypedef unsigned int uint32_t;\n"
               "typedef int int32_t;\ntypedef long long int64_t;\ntypedef unsigned long long uint64_t;\n"
               "typedef unsigned long uintptr_t;\n")
    wrapper = f"""
extern "C" __global__ __launch_bounds__(256) void {ENTRY}(dq4ml::GramArgs a) {{
  dq4ml::gram_stream_f32_body<{NT}, {RING}, {CMP}, 1, 64>(a);
}}
"""
    return prelude + _device_text() + pred + _stream_text() + wrapper


def _wave_bytes(NT: int, ring: int) -> int:
    return ring * (NT * 8192 + RAW16 + RAW4) + 64 * 16


class _Plan:
    def __init__(self, src, layout, d, NT, RING, mode):
        self.src, self.layout, self.d, self.NT, self.RING, self.mode = src, layout, d, NT, RING, mode


def _compile(chain, rel, feat_cols, mode):
    from . import dqvm
    from .scanfuse import _GramNullable, _ScanBase, _scan_gen
    from ..sql.types import VectorUDT

    tbl = rel.table
    schema = tbl.schema
    d = len(feat_cols)
    nullable = [c.valid is not None for c in tbl.columns]
    (parts, udfs), refs = dqvm.nodes_key(chain)
    key = (parts, udfs, tuple(schema.names), tuple(nullable), tuple(str(c.dtype) for c in tbl.columns),
           tuple(feat_cols), mode)
    if key in _CACHE:
        return _CACHE[key]
    plan = None
    try:
        base = _ScanBase(schema, 0, tbl.device)
        g = _scan_gen(base, nullable)
        _, g, _, _ = dqvm.compile_chain(chain, base, False, gen=g)
        if g.has_raise:
            raise dqvm.Unfusable("stream prologue: raising rule")
        vals, valids = {}, {}
        for _t, v, s in g.stores:
            tag = g.recipe[s]
            if tag[0] == "outvalid":
                valids[tag[1]] = v
            if tag[0] == "out":
                vals[tag[1]] = v
        if any(i < d for i in valids):
            raise _GramNullable("nullable feature")
        xs, yv = [vals[i] for i in range(d)], vals[d]
        # a null label drops the row (the unfused fit masks the selection with the label's validity)
        yvalid = valids.get(d, "true")
        for i, v in enumerate(xs):  # every feature a bare, unchanged source column
            m = re.fullmatch(r"\(*(?:\(double\))?\(*fzf(\d+)\)*", v.replace(" ", ""))
            if m is None or int(m.group(1)) != feat_cols[i]:
                raise dqvm.Unfusable("stream prologue: derived feature")
        text = "\n".join(g.lines) + "\n" + yv + "\n" + yvalid
        used = [c for c in sorted(g.used) if re.search(rf"\bfzf{c}\b|\bfzm{c}\b", text)]
        sizes = {}
        for c in used:
            t = tbl.columns[c].values
            if not torch.is_tensor(t) or isinstance(schema.fields[c].dataType, VectorUDT):
                raise dqvm.Unfusable("stream prologue: non-tensor column")
            sizes[c] = t.element_size()
        layout = raw_layout([(c, sizes[c], nullable[c]) for c in used])
        if not used or layout is None:
            raise dqvm.Unfusable("stream prologue: row-scalar area")
        NT = (d + 31) // 32
        RING = 3 if 4 * _wave_bytes(NT, 3) <= 160 * 1024 else 2
        ctypes = {c: dqvm._ctype(schema.fields[c].dataType) for c in used}
        src = kernel_source(g, layout, ctypes, yv, NT, RING, {2: 1, 1: 0, 4: 2}[mode], yvalid)
        plan = _Plan(src, layout, d, NT, RING, mode)
    except (dqvm.Unfusable, _GramNullable, KeyError) as e:
        log.debug("streamfuse: not fusable: %r", e)
        plan = None
    if len(_CACHE) >= 32:
        _CACHE.clear()
    _CACHE[key] = plan
    return plan


class _Route:
    """Everything an action's launch needs once its chain has been analyzed: the source table
    (weakly: a route never keeps 32 GB of columns alive), the compiled plan, the column and lane
    tables, the grid and the feature shift.  Keyed by the action's structural key (sql/skey.py), so
    an action that rebuilt the same chain over the same in-memory relation skips the analysis,
    the pruning and the chain key -- only the launch and its outputs are new."""

    def __init__(self, tbl, cp, feat_cols, rawtab, desc, handle, blocks, lds, P, shift):
        import weakref

        self.tbl = weakref.ref(tbl)
        self.cp, self.feat_cols, self.rawtab, self.desc = cp, feat_cols, rawtab, desc
        self.handle, self.blocks, self.lds, self.P, self.shift = handle, blocks, lds, P, shift
        self.n = tbl.nrows


def replay(route_key):
    """The statistics of an action whose structure an earlier action had (``_Route``), else None."""
    if route_key is None or os.environ.get("DQ4ML_STREAM_DQ", "1") == "0":
        return None
    r = _ROUTES.get(route_key)
    if r is None:
        return None
    tbl = r.tbl()
    if tbl is None or tbl.nrows != r.n or tbl.sel is not None:
        del _ROUTES[route_key]
        return None
    STATS["stream_replays"] += 1
    return _launch(r)


def _launch(r):
    from . import native
    from .scanfuse import FusedGram

    h = native.hip()
    cp, d, n = r.cp, r.cp.d, r.n
    dev = r.rawtab.device
    partials = torch.empty(r.blocks * r.P, dtype=torch.float64, device=dev)
    out = torch.empty(5 + 2 * d + d * (d + 1) // 2, dtype=torch.float64, device=dev)
    from ..utils import tracing

    st = torch.cuda.current_stream(dev).cuda_stream
    shift = r.shift
    with tracing.span("stream_dq_gram"):
        h.gram_stream_rtc(int(r.handle), cp.mode, r.desc.data_ptr(), d, n, r.rawtab.data_ptr(), partials.data_ptr(),
                          r.blocks, int(r.lds), out.data_ptr(), st, 0 if shift is None else shift.dev.data_ptr())
        if shift is not None:
            h.stats_unshift(out.data_ptr(), shift.dev.data_ptr(), d, st)
    tracing.add_rows("stream_dq_gram", n)
    STATS["stream_grams"] += 1
    fg = FusedGram(out, d, [], n)
    # the next step's pass reads only the in-memory columns: the fit tail (all-reduce, solve) may
    # run on the side stream beside it (models/regression.py overlapTail)
    fg.overlap_ok = True
    return fg


def try_fused_stream(plan, features_col: str, label_col: str, session, gram_dtype: str, route_key=None):
    """``LinearRegression.fit``'s statistics in one stream pass with the DQ chain in the stage
    prologue (see the module docstring); a ``scanfuse.FusedGram`` or None (not this shape).
    ``route_key``: the action's structural key -- the analysis is kept for ``replay``."""
    from ..models.feature import VectorAssembleExpr
    from ..sql.expressions import Alias, ColRef
    from ..sql.plan import Filter, LocalRelation, Project, output_name
    if os.environ.get("DQ4ML_STREAM_DQ", "1") == "0" or gram_dtype not in _MODES:
        return None
    if getattr(session, "device", None) is None or session.device.type != "cuda":
        return None
    nodes, p = [], plan
    while isinstance(p, (Project, Filter)) and p._memo is None:
        nodes.append(p)
        p = p.child
    if not nodes or not isinstance(nodes[0], Project) or len(nodes) < 2:
        return None
    if type(p) is not LocalRelation:  # (a CSV relation takes ops/scanfuse.py / ops/scancut.py)
        return None
    tbl = p.table
    if tbl.sel is not None or tbl.device.type != "cuda":
        return None
    top = nodes[0]
    by_name = {output_name(e): e for e in top.exprs}
    fe, le = by_name.get(features_col), by_name.get(label_col)
    if fe is None or le is None or not isinstance(fe, Alias) or not isinstance(fe.child, VectorAssembleExpr):
        return None
    va = fe.child
    d = len(va.inputs)
    if not 9 <= d <= 64:
        return None
    names = tbl.schema.names
    feat_cols = []
    for c in va.inputs:
        if c not in names:
            return None
        k = names.index(c)
        col = tbl.columns[k]
        v = col.values
        if (col.valid is not None or not torch.is_tensor(v) or v.dtype != torch.float32 or not v.is_contiguous()
                or v.data_ptr() % 16):
            return None
        feat_cols.append(k)
    n = tbl.nrows
    if n < 64:
        return None
    lexpr = le.child if isinstance(le, Alias) else le
    gtop = Project(top.child, [Alias(ColRef(c), f"__gx{i}") for i, c in enumerate(va.inputs)] + [Alias(lexpr, "__gy")])
    chain = list(reversed(nodes[1:])) + [gtop]
    mode = _MODES[gram_dtype]
    cp = _compile(chain, p, feat_cols, mode)
    if cp is None:
        return None
    # the chain's input columns: 16-B (4-B) aligned for their DMA instruction
    ptrs, vptrs = {}, {}
    for kind, c, off, s in cp.layout:
        col = tbl.columns[c]
        t = col.values if kind == "v" else col.valid
        if not t.is_contiguous() or t.numel() != n or t.data_ptr() % (16 if off < RAW16 else 4):
            return None
        (ptrs if kind == "v" else vptrs)[c] = t.data_ptr()
    from . import native
    from .device import _h2d, _srcw_desc

    h = native.hip()
    dev = tbl.device
    tkey = (id(tbl), tuple(cp.layout))
    ent = _TABS.get(tkey)
    if ent is None or ent[0] is not tbl:
        rawtab = _h2d(_lane_table(cp.layout, ptrs, vptrs), dev)
        desc = _srcw_desc(h, [tbl.columns[k].values for k in feat_cols], dev)
        if len(_TABS) >= 16:
            _TABS.clear()
        ent = _TABS[tkey] = (tbl, rawtab, desc)
    _, rawtab, desc = ent
    from .dqvm import rtc_handle

    handle = rtc_handle(h, cp, cp.src, ENTRY)
    P = int(h.gram_partial_stride(cp.mode, d))
    lds = max(4 * _wave_bytes(cp.NT, cp.RING), 8 * P)
    cus = _CUS.get(dev.index)
    if cus is None:  # (device properties: a slow query, once per device)
        cus = _CUS[dev.index] = int(h.device_info()["multiProcessorCount"])
    nstage = n // 64
    blocks = int(max(1, min(cus * max(1, (160 * 1024) // lds), (nstage + 15) // 16)))
    from .shift import column_shift

    # off-centre feature columns are shifted in-kernel before the bf16 / f32 rounding (ops/shift.py)
    shift = column_shift([tbl.columns[k].values for k in feat_cols])
    r = _Route(tbl, cp, feat_cols, rawtab, desc, handle, blocks, lds, P, shift)
    if route_key is not None:
        if len(_ROUTES) >= 32:
            _ROUTES.clear()
        _ROUTES[route_key] = r
    return _launch(r)
