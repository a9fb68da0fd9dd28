"""Whole-stage code generation of Project/Filter chains into ONE HIP kernel (the device DQ path).

Spark runs the lab's DQ chain — ``callUDF("minimumPriceRule", price)`` -> ``WHERE price_no_min >
0`` -> ``cast(guest as int)`` -> ``callUDF("priceCorrelationRule", price, guest)`` -> ``WHERE ... >
0`` (DataQuality4MachineLearningApp.java:68-90) — through Janino-compiled whole-stage codegen with
boxed UDF calls per row.  Here the rule UDFs are IR (``dq.rules``), so a whole
chain of plan nodes lowers to straight-line HIP C++:

* one thread per row (grid-stride), every referenced input column loaded once;
* SQL three-valued logic carried as a (value, valid) pair per expression;
* every ``Filter`` ANDs into the row's ``live`` flag -> the output selection vector (no compaction);
* ``RaiseIfNull`` (rule 1's Java NPE) sets a device error flag only for live rows;
* only non-trivial projections are stored; column pass-throughs stay zero-copy.

The source is compiled for gfx950 with hipRTC (``_dq4ml_hip.rtc_compile``, cached per source
text) and launched on the current torch stream.  Chains containing opaque python UDFs or string
expressions are not fused and fall back to the per-node vectorized evaluator.
"""
from __future__ import annotations

import itertools
import os
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ..sql import expressions as E
from ..sql.fn import MathFn
from ..sql.table import ColumnData, Table
from ..sql.types import (BooleanType, DataType, DecimalType, DoubleType, FloatType, IntegerType,
                         LongType, NullType, StringType, StructType, TimestampType, VectorUDT, is_numeric,
                         wider_numeric)

__all__ = ["try_execute_fused", "compile_chain", "Unfusable"]

ENTRY = "dq_fused"
# "vector_deferred": chains ending in VectorAssembler output — the assembler keeps them lazy and
# fuses the pack into the Gram pass (models/feature.py), and the DQ sub-chain below is fused here.
STATS = {"fused_launches": 0, "unfusable": 0, "vector_deferred": 0}


class Unfusable(Exception):
    pass


_CTYPE = {IntegerType: "int", LongType: "long long", DoubleType: "double", FloatType: "float", BooleanType: "bool",
          DecimalType: "double", TimestampType: "long long", NullType: "double"}



def rtc_handle(h, plan, src: str, entry: str, slot: int = 0) -> int:
    """The hipRTC module handle of a cached plan's source, memoized ON the plan object: the native
    cache (``dqvm.cpp``) keys by the whole source text, which costs a copy and a hash of tens of
    KiB per action; a plan's source never changes, so the handle is looked up once per plan."""
    hs = plan.__dict__.setdefault("_rtc", {})
    k = (slot, entry)
    v = hs.get(k)
    if v is None:
        v = hs[k] = int(h.rtc_compile(src, entry)[0])
    return v

_PREWARM = []


def prewarm() -> None:
    """Compile a trivial kernel through hipRTC on a background thread, once per process.  A
    process's first hipRTC compile also loads and initialises the compiler (comgr + LLVM): 0.1 s
    on one box, ~1.8 s on another with a cold page cache (the first action of the 77 GB config-4
    CSV, profiles/r5_first_action.md).  Started with the session, it overlaps the first action's
    upload-bound scan instead of sitting between the scan and the DQ chain.  The native compile
    releases the GIL and holds its cache lock only around lookups (dqvm.cpp)."""
    if _PREWARM:
        return
    import atexit
    import threading

    from . import native

    def run():
        try:
            native.hip().rtc_compile('extern "C" __global__ void dq_prewarm(int* p) { if (p) p[0] = 0; }\n',
                                     "dq_prewarm")
        except Exception as e:  # (a missing compiler surfaces at the first real compile)
            from ..utils.logging import get_logger

            get_logger("dqvm").debug("hipRTC prewarm failed: %s", e)

    t = threading.Thread(target=run, name="dq4ml-rtc-prewarm", daemon=True)
    _PREWARM.append(t)
    t.start()
    atexit.register(t.join, 60.0)  # never tear the runtime down under a compile in flight


def _ctype(t: DataType) -> str:
    c = _CTYPE.get(type(t))
    if c is None:
        raise Unfusable(f"type {t.simpleString()} not fusable")
    return c


def _lit(v, t: DataType) -> str:
    if v is None:
        return "0"
    if isinstance(t, BooleanType):
        return "true" if v else "false"
    if isinstance(t, (IntegerType,)):
        return f"{int(v)}"
    if isinstance(t, (LongType, TimestampType)):
        return f"{int(v)}LL"
    if isinstance(t, FloatType):
        return f"{float(v)!r}f"
    f = float(v)
    if f != f:
        return "__builtin_nan(\"\")"
    if f in (float("inf"), float("-inf")):
        return "__builtin_inf()" if f > 0 else "(-__builtin_inf())"
    return repr(f)


class _Gen:
    def __init__(self, base: Table, check_device: bool = True):
        self.base = base
        self.check_device = check_device
        self.lines: List[str] = []
        self.ptrs: List[int] = []  # device pointers, index = slot
        self.recipe: List[tuple] = []  # what each slot binds to (for the structural chain cache)
        self.loads: List[Tuple[str, str, str, int]] = []  # (C type, var, storage type, slot): row loads
        self.stores: List[Tuple[str, str, int]] = []  # (storage type, value, slot): row stores
        self.keep: List[torch.Tensor] = []
        self.counter = itertools.count()
        self.col_cache: Dict[int, Tuple[str, str, DataType]] = {}
        self.has_raise = False
        self.has_filter = False

    def slot(self, t: Optional[torch.Tensor], tag: tuple) -> int:
        self.ptrs.append(0 if t is None else t.data_ptr())
        self.recipe.append(tag)
        if t is not None:
            self.keep.append(t)
        return len(self.ptrs) - 1

    def tmp(self, prefix="t"):
        return f"{prefix}{next(self.counter)}"

    def emit(self, s):
        self.lines.append("    " + s)

    # -- base column access -------------------------------------------------------------------
    def load_col(self, idx: int):
        if idx in self.col_cache:
            return self.col_cache[idx]
        c: ColumnData = self.base.columns[idx]
        t = c.dtype
        if isinstance(t, (StringType, VectorUDT)) or not torch.is_tensor(c.values) or \
                (self.check_device and not c.values.is_cuda):
            raise Unfusable("non-numeric column")
        vals = c.values.contiguous()
        ct = _ctype(t)
        store_t = {torch.bool: "bool", torch.int32: "int", torch.int64: "long long", torch.float32: "float",
                   torch.float64: "double", torch.uint8: "unsigned char"}.get(vals.dtype)
        if store_t is None:
            raise Unfusable(f"storage {vals.dtype}")
        s = self.slot(vals, ("col", idx))
        v = self.tmp("c")
        self.loads.append((ct, v, store_t, s))
        if c.valid is not None:
            sv = self.slot(c.valid.contiguous(), ("valid", idx))
            m = self.tmp("cm")
            self.loads.append(("bool", m, "bool", sv))
        else:
            m = "true"
        self.col_cache[idx] = (v, m, t)
        return v, m, t


class _Chain:
    """Symbol table for one plan level: name -> ('col', idx) | ('reg', val, valid, dtype, expr)."""

    def __init__(self, names: List[str], syms: List[tuple]):
        self.names = names
        self.syms = syms

    def lookup(self, name: str):
        if name in self.names:
            return self.syms[self.names.index(name)]
        low = [n.lower() for n in self.names]
        if name.lower() in low:
            return self.syms[low.index(name.lower())]
        raise Unfusable(f"unresolved {name}")


def _m_and(*ms: str) -> str:
    """Validity conjunction, folded: constant-true operands drop out (a chain over null-free
    columns then stores no validity at all)."""
    if any(m == "false" for m in ms):
        return "false"
    rest = [m for m in ms if m != "true"]
    return "true" if not rest else " && ".join(f"({m})" for m in rest)


def _compile(g: _Gen, e: E.Expr, chain: _Chain, schema: StructType, live: str) -> Tuple[str, str, DataType]:
    """-> (value C expression/variable, valid C expression/variable, DataType)."""
    if isinstance(e, E.Alias):
        return _compile(g, e.child, chain, schema, live)
    if isinstance(e, E.ColRef):
        sym = chain.lookup(e.name)
        if sym[0] == "col":
            return g.load_col(sym[1])
        return sym[1], sym[2], sym[3]
    if isinstance(e, E.Lit):
        if isinstance(e.dtype, StringType):
            raise Unfusable("string literal")
        t = e.dtype
        return _lit(e.value, t), ("false" if e.value is None else "true"), t
    if isinstance(e, E.UdfCall):
        body = e.expanded()
        if body is None:
            raise Unfusable("opaque udf")
        v, m, t = _compile(g, body, chain, schema, live)
        rt = e._resolved().returnType
        if type(rt) is not type(t):
            return _cast(g, v, m, t, rt)
        return v, m, t
    if isinstance(e, E.RaiseIfNull):
        v, m, t = _compile(g, e.child, chain, schema, live)
        if m != "true":
            g.has_raise = True
            g.emit(f"if (({live}) && !({m})) atomicOr((int*)P[1], 1);")
        return v, "true", t
    if isinstance(e, E.Cast):
        v, m, t = _compile(g, e.child, chain, schema, live)
        return _cast(g, v, m, t, e.to)
    if isinstance(e, E.Not):
        v, m, t = _compile(g, e.child, chain, schema, live)
        return f"(!({v}))", m, BooleanType()
    if isinstance(e, E.Neg):
        v, m, t = _compile(g, e.child, chain, schema, live)
        return f"(-({v}))", m, t
    if isinstance(e, (E.IsNotNull, E.IsNull)):
        v, m, t = _compile(g, e.child, chain, schema, live)
        return (f"({m})" if isinstance(e, E.IsNotNull) else f"(!({m}))"), "true", BooleanType()
    if isinstance(e, E.BinOp):
        return _binop(g, e, chain, schema, live)
    if isinstance(e, E.If):
        cv, cm, _ = _compile(g, e.cond, chain, schema, live)
        av, am, at = _compile(g, e.a, chain, schema, live)
        bv, bm, bt = _compile(g, e.b, chain, schema, live)
        t = wider_numeric(at, bt) if (is_numeric(at) or is_numeric(bt)) else at
        ct = _ctype(t)
        take = g.tmp("k")
        g.emit(f"const bool {take} = {_m_and(cm, cv)};")
        v = g.tmp("v")
        g.emit(f"const {ct} {v} = {take} ? ({ct})({av}) : ({ct})({bv});")
        if am == bm:
            return v, am, t
        m = g.tmp("m")
        g.emit(f"const bool {m} = {take} ? ({am}) : ({bm});")
        return v, m, t
    if isinstance(e, E.CaseWhen):
        return _compile(g, e._chain(), chain, schema, live)
    if isinstance(e, E.Coalesce):
        parts = [_compile(g, a, chain, schema, live) for a in e.args]
        t = parts[0][2]
        for p in parts[1:]:
            t = wider_numeric(t, p[2])
        ct = _ctype(t)
        v, m = g.tmp("v"), g.tmp("m")
        g.emit(f"{ct} {v} = ({ct})({parts[-1][0]}); bool {m} = {parts[-1][1]};")
        for pv, pm, _ in reversed(parts[:-1]):
            g.emit(f"if ({pm}) {{ {v} = ({ct})({pv}); {m} = true; }}")
        return v, m, t
    if isinstance(e, MathFn):
        return _mathfn(g, e, chain, schema, live)
    raise Unfusable(type(e).__name__)


def _cast(g, v, m, src: DataType, to: DataType):
    if isinstance(to, (StringType, VectorUDT)) or isinstance(src, (StringType, VectorUDT)):
        raise Unfusable("string cast")
    ct = _ctype(to)
    out = g.tmp("v")
    if isinstance(to, (IntegerType, LongType)) and isinstance(src, (DoubleType, FloatType, DecimalType)):
        lo, hi = ("-2147483648.0", "2147483647.0") if isinstance(to, IntegerType) else \
            ("-9223372036854775808.0", "9223372036854775807.0")
        g.emit(f"const {ct} {out} = ({v}) != ({v}) ? ({ct})0 : (({v}) <= {lo} ? ({ct}){lo} : "
               f"(({v}) >= {hi} ? ({ct}){hi} : ({ct})({v})));")
    elif isinstance(to, BooleanType):
        g.emit(f"const bool {out} = ({v}) != 0;")
    else:
        g.emit(f"const {ct} {out} = ({ct})({v});")
    return out, m, to


_CMPS = {"<": "<", ">": ">", "<=": "<=", ">=": ">=", "=": "==", "==": "==", "!=": "!=", "<>": "!="}


def _spark_cmp_c(op: str, a: str, b: str) -> str:
    """C form of Spark SQL's NaN-aware float ordering (NaN = NaN, NaN above everything); the
    torch form is ``sql.expressions._spark_cmp``."""
    an, bn = f"__builtin_isnan({a})", f"__builtin_isnan({b})"
    if op in ("=", "==", "!=", "<>"):
        eq = f"(({a} == {b}) || ({an} && {bn}))"
        return eq if op in ("=", "==") else f"(!{eq})"
    return {"<": f"(!{an} && ({bn} || {a} < {b}))",
            ">": f"(!{bn} && ({an} || {a} > {b}))",
            "<=": f"({bn} || (!{an} && {a} <= {b}))",
            ">=": f"({an} || (!{bn} && {a} >= {b}))"}[op]


def _binop(g, e: E.BinOp, chain, schema, live):
    if e.op in ("and", "or"):
        av, am, _ = _compile(g, e.left, chain, schema, live)
        bv, bm, _ = _compile(g, e.right, chain, schema, live)
        v, m = g.tmp("v"), g.tmp("m")
        if e.op == "and":
            g.emit(f"const bool {v} = ({av}) && ({bv});")
            if am == "true" and bm == "true":
                return v, "true", BooleanType()
            g.emit(f"const bool {m} = (({am}) && ({bm})) || (({am}) && !({av})) || (({bm}) && !({bv}));")
        else:
            g.emit(f"const bool {v} = (({am}) && ({av})) || (({bm}) && ({bv}));")
            if am == "true" and bm == "true":
                return v, "true", BooleanType()
            g.emit(f"const bool {m} = (({am}) && ({bm})) || (({am}) && ({av})) || (({bm}) && ({bv}));")
        return v, m, BooleanType()
    av, am, at = _compile(g, e.left, chain, schema, live)
    bv, bm, bt = _compile(g, e.right, chain, schema, live)
    if isinstance(at, StringType) or isinstance(bt, StringType):
        raise Unfusable("string op")
    ot = wider_numeric(at, bt) if not (isinstance(at, BooleanType) and isinstance(bt, BooleanType)) else at
    oc = _ctype(ot)
    a, b = f"(({oc})({av}))", f"(({oc})({bv}))"
    v, m = g.tmp("v"), g.tmp("m")
    both = _m_and(am, bm)
    if both in ("true", "false"):
        m = both
    if e.op in _CMPS:
        if oc in ("double", "float") and not getattr(e, "ieee", False):
            g.emit(f"const bool {v} = {_spark_cmp_c(e.op, a, b)};")
        else:
            g.emit(f"const bool {v} = {a} {_CMPS[e.op]} {b};")
        if m not in ("true", "false"):
            g.emit(f"const bool {m} = {both};")
        return v, m, BooleanType()
    if e.op == "<=>":
        eq = _spark_cmp_c("=", a, b) if oc in ("double", "float") else f"({a} == {b})"
        g.emit(f"const bool {v} = (({am}) && ({bm}) && {eq}) || (!({am}) && !({bm}));")
        return v, "true", BooleanType()
    if e.op in ("+", "-", "*"):
        g.emit(f"const {oc} {v} = {a} {e.op} {b};")
        if m not in ("true", "false"):
            g.emit(f"const bool {m} = {both};")
        return v, m, ot
    if e.op in ("/", "%"):
        m = g.tmp("m")  # these add their own validity condition (no folding)
    if e.op == "/":
        g.emit(f"const double {v} = ((double)({bv})) == 0.0 ? 0.0 : ((double)({av})) / ((double)({bv}));")
        g.emit(f"const bool {m} = ({am}) && ({bm}) && ((double)({bv})) != 0.0;")
        return v, m, DoubleType()
    if e.op == "%":
        if oc in ("double", "float"):
            g.emit(f"const {oc} {v} = ({b}) == 0 ? ({oc})0 : fmod({a}, {b});")
        else:
            g.emit(f"const {oc} {v} = ({b}) == 0 ? ({oc})0 : {a} % {b};")
        g.emit(f"const bool {m} = ({am}) && ({bm}) && ({b}) != 0;")
        return v, m, ot
    raise Unfusable(e.op)


_MATH = {"abs": "fabs", "sqrt": "sqrt", "exp": "exp", "ln": "log", "log10": "log10", "floor": "floor",
         "ceil": "ceil", "ceiling": "ceil", "signum": None}


def _mathfn(g, e: MathFn, chain, schema, live):
    parts = [_compile(g, a, chain, schema, live) for a in e.args]
    t = e.data_type(schema)
    ct = _ctype(t)
    m = " && ".join(f"({p[1]})" for p in parts) or "true"
    v, mm = g.tmp("v"), g.tmp("m")
    x = [f"((double)({p[0]}))" for p in parts]
    n = e.name
    if n == "abs" and not isinstance(t, (DoubleType, FloatType)):
        g.emit(f"const {ct} {v} = ({parts[0][0]}) < 0 ? -({parts[0][0]}) : ({parts[0][0]});")
    elif n in ("sqrt", "ln", "log10") or (n == "log" and len(x) == 1):
        fn = {"sqrt": "sqrt", "ln": "log", "log": "log", "log10": "log10"}[n]
        bad = f"{x[0]} < 0.0" if n == "sqrt" else f"{x[0]} <= 0.0"
        g.emit(f"const {ct} {v} = ({ct}){fn}({x[0]});")
        m = f"({m}) && !({bad})"
    elif n == "log":
        g.emit(f"const {ct} {v} = ({ct})(log({x[1]}) / log({x[0]}));")
    elif n in ("pow", "power"):
        g.emit(f"const {ct} {v} = ({ct})pow({x[0]}, {x[1]});")
    elif n == "round":
        scale = int(e.args[1].value) if len(e.args) > 1 else 0
        f = 10.0 ** scale
        g.emit(f"const {ct} {v} = ({ct})(({x[0]} < 0 ? -1.0 : 1.0) * floor(fabs({x[0]} * {f!r}) + 0.5) / {f!r});")
    elif n == "signum":
        g.emit(f"const {ct} {v} = ({ct})(({x[0]} > 0) - ({x[0]} < 0));")
    elif n in ("greatest", "least"):
        op = "fmax" if n == "greatest" else "fmin"
        acc = x[0]
        for y in x[1:]:
            acc = f"{op}({acc}, {y})"
        g.emit(f"const {ct} {v} = ({ct})({acc});")
    else:
        g.emit(f"const {ct} {v} = ({ct}){_MATH[n]}({x[0]});")
    g.emit(f"const bool {mm} = {m};")
    return v, mm, t


_TORCH = {IntegerType: torch.int32, LongType: torch.int64, DoubleType: torch.float64, FloatType: torch.float32,
          BooleanType: torch.bool, DecimalType: torch.float64, TimestampType: torch.int64, NullType: torch.float64}
_STORE_C = {torch.int32: "int", torch.int64: "long long", torch.float64: "double", torch.float32: "float",
            torch.bool: "bool"}


def _trivial(node) -> bool:
    from ..sql.plan import Project

    return isinstance(node, Project) and all(
        isinstance(x, E.ColRef) or (isinstance(x, E.Alias) and isinstance(x.child, E.ColRef)) for x in node.exprs)


def compile_chain(nodes, base: Table, check_device: bool = True, gen: Optional[_Gen] = None):
    """nodes: bottom-up list of Project/Filter.  Returns (source, gen, outputs) where outputs[i] is
    ('col', base_idx) or ('new', slot, valid_slot_or_None, tensor, valid_tensor, dtype).

    ``gen``: a generator whose base columns are not loaded from memory (the fused CSV scan,
    ``ops/scanfuse.py``: they are parsed into registers): pass-through columns are then stored
    like computed ones, the selection vector is always written and no source is generated here."""
    from ..sql.plan import Filter, Project

    g = gen if gen is not None else _Gen(base, check_device)
    g.slot(base.sel, ("sel",))  # P[0] selection in
    g.slot(None, ("err",))  # P[1] error flag (filled by caller)
    live = "live"
    chain = _Chain(list(base.schema.names), [("col", i) for i in range(len(base.columns))])
    for node in nodes:
        schema = node.child.schema()
        if isinstance(node, Filter):
            v, m, _ = _compile(g, node.cond, chain, schema, live)
            g.emit(f"live = live && ({m}) && ({v});")
            g.has_filter = True
        elif isinstance(node, Project):
            out_schema = node.schema()
            syms = []
            for ex, f in zip(node.exprs, out_schema.fields):
                base_e = ex.child if isinstance(ex, E.Alias) else ex
                if isinstance(base_e, E.Cast) and isinstance(base_e.child, E.ColRef) and \
                        base_e.child.data_type(schema).simpleString() == base_e.to.simpleString():
                    base_e = base_e.child  # SimplifyCasts: a cast to the column's own type is the column
                if isinstance(base_e, E.ColRef):
                    syms.append(chain.lookup(base_e.name))
                    continue
                v, m, t = _compile(g, ex, chain, schema, live)
                if type(t) is not type(f.dataType):
                    v, m, t = _cast(g, v, m, t, f.dataType)
                syms.append(("reg", v, m, f.dataType, ex))
            chain = _Chain(list(out_schema.names), syms)
        else:
            raise Unfusable(type(node).__name__)
    n = base.nrows
    dev = base.device
    outputs = []
    for name, sym in zip(chain.names, chain.syms):
        if sym[0] == "col":
            if gen is None:  # zero-copy pass-through
                outputs.append(("col", sym[1]))
                continue
            v, m, t = g.load_col(sym[1])
        else:
            _, v, m, t, _ = sym
        td = _TORCH[type(t)]
        out = torch.empty(n, dtype=td, device=dev)
        s = g.slot(out, ("out", len(outputs)))
        g.stores.append((_STORE_C[td], v, s))
        vt = None
        if m != "true":
            vt = torch.empty(n, dtype=torch.bool, device=dev)
            sv = g.slot(vt, ("outvalid", len(outputs)))
            g.stores.append(("bool", m, sv))
        outputs.append(("new", out, vt, t))
    sel_out = None
    if g.has_filter or gen is not None:
        sel_out = torch.empty(n, dtype=torch.bool, device=dev)
        s = g.slot(sel_out, ("selout",))
        g.stores.append(("bool", "live", s))
    src = (_kernel_source(g), _kernel_source_vec(g)) if gen is None else None
    return src, g, outputs, sel_out


ROWS_PER_THREAD = 4


def _kernel_source(g: _Gen) -> str:
    """The fused kernel: grid-stride over groups of ROWS_PER_THREAD rows per thread.  All base-column
    loads of a group are issued first (clamped row index, branch-free), then each row's body runs —
    row-independent, so this is exact even when an output aliases an input, and it keeps 4 rows of
    loads in flight per thread (one row at a time left the DQ pass latency-bound at ~2.5 TB/s).
    Slot pointers are copied to registers once (stores through ``P[k]`` could alias the table
    itself, which kept the compiler re-loading it every row)."""
    U = ROWS_PER_THREAD
    ns = len(g.ptrs)
    decl = "".join(f"    {ct} {v}_a[{U}];\n" for ct, v, _, _ in g.loads)
    ld = "".join(f"      {v}_a[u] = ({ct})((const {st}*)p[{s}])[r];\n" for ct, v, st, s in g.loads)
    use = "".join(f"        const {ct} {v} = {v}_a[u];\n" for ct, v, _, _ in g.loads)
    body = "\n".join("    " + ln for ln in g.lines).replace("P[", "p[") + "\n" + "".join(
        f"        (({t}*)p[{s}])[r] = ({t})({v});\n" for t, v, s in g.stores)
    return (ptr_struct(ns) +
            f'extern "C" __global__ __launch_bounds__(256) void {ENTRY}(const DqPtrs P, long long n) {{\n'
            f"  void* p[{ns}];\n"
            f"#pragma unroll\n"
            f"  for (int i = 0; i < {ns}; ++i) p[i] = P.v[i];\n"
            f"  const long long stride = (long long)gridDim.x * blockDim.x;\n"
            f"  for (long long r0 = (long long)blockIdx.x * blockDim.x + threadIdx.x; r0 < n; r0 += {U} * stride) {{\n"
            f"    bool live_a[{U}];\n{decl}"
            f"#pragma unroll\n"
            f"    for (int u = 0; u < {U}; ++u) {{\n"
            f"      const long long rr = r0 + u * stride;\n"
            f"      const long long r = rr < n ? rr : n - 1;\n"
            f"      live_a[u] = p[0] ? ((const bool*)p[0])[r] : true;\n{ld}"
            f"    }}\n"
            f"#pragma unroll\n"
            f"    for (int u = 0; u < {U}; ++u) {{\n"
            f"      const long long r = r0 + u * stride;\n"
            f"      if (r < n) {{\n"
            f"        bool live = live_a[u];\n{use}{body}\n"
            f"      }}\n"
            f"    }}\n"
            f"  }}\n}}\n")


# The generated kernels take their pointer slots BY VALUE (a struct in the kernel-argument segment,
# read with scalar loads): no per-launch pointer table to upload (a pinned staging copy + an H2D
# copy per action, round 3) and no global loads of it in the kernel prologue.  The kernarg segment
# holds 4 KiB: chains with more slots do not fuse.
MAX_SLOTS = 480


def ptr_struct(ns: int) -> str:
    if ns > MAX_SLOTS:
        raise Unfusable("too many pointer slots for the kernel-argument segment")
    return f"struct DqPtrs {{ void* v[{max(ns, 1)}]; }};\n"


def launch(h, handle, grid: int, ptr_list, n: int, stream: int):
    """Launch a generated kernel (``rtc_handle``) with its pointer slots by value."""
    h.rtc_launch_args(int(handle), int(grid), 256, np.asarray(ptr_list, dtype=np.int64), int(n), int(stream))


VEC_ROWS = 4  # consecutive rows per thread, vector form
GRID_CAP = 131072  # grid-stride cap (blocks); config 4 A/B 2x: 8192 5.997 / 5.925, 32768 5.894 / 5.910, 131072 5.872 / 5.859 ms
_VEC_BASE = {"double": "double", "float": "float", "int": "int", "long long": "long long", "bool": "unsigned char",
             "unsigned char": "unsigned char"}
_VEC_NAME = {"double": "f64", "float": "f32", "int": "i32", "long long": "i64", "bool": "u8", "unsigned char": "u8"}


def _vec_t(ct: str, v: int) -> str:
    return f"dq_{_VEC_NAME[ct]}x{v}"


def _vec_types(v: int) -> str:
    return "".join(f"typedef {b} dq_{nm}x{v} __attribute__((ext_vector_type({v})));\n"
                   for b, nm in (("double", "f64"), ("float", "f32"), ("int", "i32"), ("long long", "i64"),
                                 ("unsigned char", "u8")))


def _kernel_source_vec(g: _Gen, V: int = VEC_ROWS) -> str:
    """The same chain for aligned slots (the usual case: whole device allocations): each thread
    owns V CONSECUTIVE rows, so every column is read and every output written with one V-wide
    vector access per thread (the strided form moves 1-8 bytes per lane per instruction); the
    n % V tail rows run the scalar body."""
    ns = len(g.ptrs)
    decl = "".join(f"    {ct} {v}_a[{V}];\n" for ct, v, _, _ in g.loads)
    ldf = "*("  # (non-temporal column loads measured no better)
    ld = "".join(f"    {{ const {_vec_t(st, V)} q = {ldf}(const {_vec_t(st, V)}*)((const {_VEC_BASE[st]}*)p[{s}] + r0));\n"
                 f"      for (int u = 0; u < {V}; ++u) {v}_a[u] = ({ct})q[u]; }}\n" for ct, v, st, s in g.loads)
    use = "".join(f"      const {ct} {v} = {v}_a[u];\n" for ct, v, _, _ in g.loads)
    body = "\n".join("  " + ln for ln in g.lines).replace("P[", "p[")
    odecl = "".join(f"    {_vec_t(t, V)} o{s};\n" for t, _, s in g.stores)
    oset = "".join(f"      o{s}[u] = ({_VEC_BASE[t]})({v});\n" for t, v, s in g.stores)
    ost = "".join(f"    *({_vec_t(t, V)}*)(({_VEC_BASE[t]}*)p[{s}] + r0) = o{s};\n" for t, _, s in g.stores)
    tail_ld = "".join(f"    const {ct} {v} = ({ct})((const {st}*)p[{s}])[r];\n" for ct, v, st, s in g.loads)
    tail_st = "".join(f"    (({t}*)p[{s}])[r] = ({t})({v});\n" for t, v, s in g.stores)
    return (_vec_types(V) + ptr_struct(ns) +
            f'extern "C" __global__ __launch_bounds__(256) void {ENTRY}(const DqPtrs P, long long n) {{\n'
            f"  void* p[{ns}];\n"
            f"#pragma unroll\n"
            f"  for (int i = 0; i < {ns}; ++i) p[i] = P.v[i];\n"
            f"  const long long stride = (long long)gridDim.x * blockDim.x;\n"
            f"  const long long gt = (long long)blockIdx.x * blockDim.x + threadIdx.x;\n"
            f"  const long long nq = n / {V};\n"
            f"  for (long long t = gt; t < nq; t += stride) {{\n"
            f"    const long long r0 = {V} * t;\n"
            f"    bool live_a[{V}];\n{decl}"
            f"    if (p[0]) {{ const dq_u8x{V} q = *(const dq_u8x{V}*)((const unsigned char*)p[0] + r0);\n"
            f"      for (int u = 0; u < {V}; ++u) live_a[u] = q[u] != 0; }}\n"
            f"    else {{ for (int u = 0; u < {V}; ++u) live_a[u] = true; }}\n{ld}{odecl}"
            f"#pragma unroll\n"
            f"    for (int u = 0; u < {V}; ++u) {{\n"
            f"      bool live = live_a[u];\n{use}{body}\n{oset}"
            f"    }}\n{ost}"
            f"  }}\n"
            f"  if (gt < n - {V} * nq) {{\n"
            f"    const long long r = {V} * nq + gt;\n"
            f"    bool live = p[0] ? ((const bool*)p[0])[r] : true;\n{tail_ld}{body}\n{tail_st}"
            f"  }}\n}}\n")


class _ChainPlan:
    """A compiled chain, reusable for any base table of the same structure: the kernel source,
    what each pointer slot binds to, and the output layout."""

    def __init__(self, src, g: _Gen, outputs, sel_out, refs):
        self.src = src
        self.recipe = list(g.recipe)
        self.has_raise, self.has_filter = g.has_raise, g.has_filter
        self.outs = [o if o[0] == "col" else ("new", o[1].dtype, o[2] is not None, o[3]) for o in outputs]
        self.refs = refs  # resolved UDF objects of the key: kept alive so their ids stay unique
        _ = sel_out

    def bind(self, base: Table, err: torch.Tensor):
        n, dev = base.nrows, base.device
        outs = [None if o[0] == "col" else
                (torch.empty(n, dtype=o[1], device=dev), torch.empty(n, dtype=torch.bool, device=dev) if o[2] else None)
                for o in self.outs]
        sel_out = torch.empty(n, dtype=torch.bool, device=dev) if self.has_filter else None
        keep, ptrs = [], []
        for tag in self.recipe:  # noqa: B007
            k = tag[0]
            if k == "sel":
                t = base.sel
            elif k == "err":
                t = err
            elif k == "col":
                t = base.columns[tag[1]].values.contiguous()
            elif k == "valid":
                t = base.columns[tag[1]].valid.contiguous()
            elif k == "out":
                t = outs[tag[1]][0]
            elif k == "outvalid":
                t = outs[tag[1]][1]
            else:
                t = sel_out
            ptrs.append(0 if t is None else t.data_ptr())
            if t is not None:
                keep.append(t)
        return ptrs, outs, sel_out, keep


_CHAIN_CACHE: "Dict[tuple, Optional[_ChainPlan]]" = {}
_CHAIN_CACHE_MAX = 256


def _udfs_of(e, acc):
    if isinstance(e, E.UdfCall):
        body = e.expanded()  # the rule's IR (its constants) is part of the structure too
        acc.append((e._resolved(), None if body is None else body.sql_name()))
    for c in e.children():
        _udfs_of(c, acc)
    return acc


def _storage_tag(c) -> str:
    """A column's storage dtype for the chain key -- without building a device string column's
    Python strings (``DeviceStringColumn.values`` materializes them; string storage is never a
    tensor)."""
    if isinstance(c.dtype, StringType):
        return "-"
    v = c.values
    return str(v.dtype) if torch.is_tensor(v) else "-"


def _chain_key(nodes, base: Table):
    """Structural key of (chain, base layout): expression SQL text + output names per node, the
    resolved UDF objects (a re-registered name is a new object), base column types / storage
    dtypes / validity, selection presence."""
    (parts, udfs), refs = nodes_key(nodes)
    cols = tuple((f.name, f.dataType.simpleString(), _storage_tag(c), c.valid is not None)
                 for f, c in zip(base.schema.fields, base.columns))
    return (parts, cols, base.sel is not None, udfs), refs


def nodes_key(nodes):
    """((per-node structure, UDF identities), resolved UDF objects) of a Project/Filter chain."""
    from ..sql.plan import Filter

    parts, refs = [], []
    for nd in nodes:
        if isinstance(nd, Filter):
            parts.append(("F", nd.cond.sql_name()))
            _udfs_of(nd.cond, refs)
        else:
            parts.append(("P", tuple(x.sql_name() for x in nd.exprs), tuple(nd.schema().names)))
            for x in nd.exprs:
                _udfs_of(x, refs)
    return (tuple(parts), tuple((id(r), b) for r, b in refs)), refs


def try_execute_fused(plan, session) -> Optional[Table]:
    from ..sql.plan import Filter, Project, _maybe_compact, execute

    if session is None or getattr(session, "device", None) is None or session.device.type != "cuda":
        return None
    nodes = []
    p = plan
    while isinstance(p, (Project, Filter)) and (p is plan or p._memo is None):
        nodes.append(p)
        p = p.child
    if not nodes:
        return None
    nodes.reverse()
    if all(_trivial(nd) for nd in nodes):
        return None
    from ..sql.plan import CsvScanRelation

    if isinstance(p, CsvScanRelation) and p._memo is None and p.fused is not None:
        # the chain sits right on a not-yet-scanned CSV relation: scan + chain in one kernel
        from . import scanfuse

        r = scanfuse.try_fused_scan(nodes, p, plan, session)
        if r == "vector":
            STATS["vector_deferred"] += 1
            return None
        if r is not None:
            STATS["fused_launches"] += 1
            return _maybe_compact(r)
    base = execute(p, session)
    if base.nrows == 0 or base.device.type != "cuda":
        return None
    # structural cache: every Spark action re-builds the same DataFrame chain over a new relation
    # (S20) — the Python codegen (~0.3 ms) runs once per chain shape, not once per action
    key, refs = _chain_key(nodes, base)
    if key in _CHAIN_CACHE:
        cp = _CHAIN_CACHE[key]
    else:
        try:
            cp = _ChainPlan(*compile_chain(nodes, base), refs)
        except Unfusable as e:
            cp = "vector" if str(e) == "VectorAssembleExpr" else None
        if len(_CHAIN_CACHE) >= _CHAIN_CACHE_MAX:
            _CHAIN_CACHE.clear()
        _CHAIN_CACHE[key] = cp
    if cp is None or cp == "vector":
        STATS["unfusable" if cp is None else "vector_deferred"] += 1
        return None
    from . import native

    h = native.hip()
    err = torch.zeros(1, dtype=torch.int32, device=base.device)
    ptr_list, outs, sel_out, keep = cp.bind(base, err)
    vec = all(q % (8 * VEC_ROWS) == 0 for q in ptr_list)  # whole allocations: the V-consecutive-rows form
    handle = rtc_handle(h, cp, cp.src[1] if vec else cp.src[0], ENTRY, 1 if vec else 0)
    n = base.nrows
    grid = int(max(1, min((n + 256 * VEC_ROWS - 1) // (256 * VEC_ROWS) if vec else (n + 255) // 256, GRID_CAP)))
    from ..utils import tracing

    with tracing.span("dq_fused"):
        launch(h, handle, grid, ptr_list, int(n), torch.cuda.current_stream().cuda_stream)
    tracing.add_rows("dq_fused", n)
    STATS["fused_launches"] += 1
    checks = []
    if cp.has_raise:
        # a raising rule (RaiseIfNull, MinimumPriceDataQualityUdf.java:11-13) fails the job on the
        # first host read of the action's results (runtime/checks.py): no sync per action
        from .scanfuse import _udf_error_check

        checks = [c for c in (_udf_error_check(nodes, err),) if c is not None]
    schema = plan.schema()
    cols = []
    for o, f, oo in zip(cp.outs, schema.fields, outs):
        if o[0] == "col":
            c = base.columns[o[1]]
            cols.append(ColumnData(c.dtype, c.values, c.valid, dict(c.meta), list(c.checks) + checks))
        else:
            cols.append(ColumnData(f.dataType, oo[0], oo[1], dict(f.metadata), list(checks)))
    sel = sel_out if sel_out is not None else base.sel
    del keep
    return _maybe_compact(Table(schema, cols, n, sel, base.device))


def _find_raise(e):
    if isinstance(e, E.RaiseIfNull):
        return e
    if isinstance(e, E.UdfCall):
        b = e.expanded()
        return _find_raise(b) if b is not None else None
    for c in e.children():
        r = _find_raise(c)
        if r is not None:
            return r
    return None
