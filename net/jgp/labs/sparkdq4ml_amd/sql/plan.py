"""Lazy logical plans and their executor.

Spark builds a lazy lineage and re-executes it from the CSV on every action (the
lab re-scans ``dataset-abstract.csv`` ~10 times).  Here every node memoizes its materialized
:class:`Table` (plans are immutable and all supported expressions are deterministic, so this is
observationally identical) and the executor fuses Project/Filter chains into one device
kernel launch where the expressions allow it (``ops.dqvm``).
"""
from __future__ import annotations

import threading
from typing import List, Optional, Sequence, Tuple

import torch

from .expressions import (Alias, AnalysisException, ColRef, EvalContext, Expr, UdfCall)
from .skey import expr_key, exprs_key, intern
from .table import ColumnData, Table
from .types import BooleanType, StructField, StructType

__all__ = ["LogicalPlan", "LocalRelation", "CsvScanRelation", "Project", "Filter", "Limit", "Union", "execute", "prune_columns"]


class LogicalPlan:
    _memo: Optional[Table] = None
    _skey = 0  # structural key (sql/skey.py): 0 = not computed yet, None = unkeyable

    def children(self) -> List["LogicalPlan"]:
        return []

    def skey(self) -> Optional[int]:
        """Interned structural key: equal for two nodes that denote the same computation over the
        same input (an action's rebuilt chain), None when the node cannot be keyed."""
        return None

    def fresh(self, child: Optional["LogicalPlan"] = None) -> "LogicalPlan":
        """A copy of this (analyzed) node with no execution result, over ``child``: the DataFrame
        layer's structural sharing hands every action its own nodes."""
        n = object.__new__(type(self))
        d = n.__dict__
        d.update(self.__dict__)
        d.pop("_memo", None)
        if child is not None:
            d["child"] = child
        return n

    def schema(self) -> StructType:
        raise NotImplementedError

    def _compute(self, session) -> Table:
        raise NotImplementedError

    def describe(self, indent=0) -> str:
        s = "  " * indent + self._label() + "\n"
        for c in self.children():
            s += c.describe(indent + 1)
        return s

    def _label(self):
        return type(self).__name__


class LocalRelation(LogicalPlan):
    """A materialized relation.  ``sharded``: this process holds one data-parallel shard of it
    (rank order = global row order); defaults to True whenever a multi-process group is up, which
    is the SPMD contract of the engine: every source (reader byte range, ``createDataFrame``,
    ``range``) contributes this rank's rows."""

    def __init__(self, table: Table, label: str = "LocalRelation", sharded: Optional[bool] = None):
        from ..parallel import comm

        self.table = table
        self._memo = table
        self.label = label
        self.sharded = comm.world_size() > 1 if sharded is None else bool(sharded)

    def schema(self):
        return self.table.schema

    def skey(self):
        # one key per relation object (a serial, not the table's id: nothing is pinned); chains
        # rebuilt over the same relation share their analysis
        k = self.__dict__.get("_skey")
        if k is None:
            k = self._skey = intern(("local", next(_SERIAL)))
        return k

    def _compute(self, session):
        return self.table

    def _label(self):
        return f"{self.label} [{', '.join(self.table.schema.names)}]"


class CsvScanRelation(LocalRelation):
    """A device CSV relation scanned lazily, at its first action (Spark also reads the file at
    every action).  Created only when an earlier device scan of the same cached
    bytes already fixed its schema, null columns and line count (``fused``: those facts plus the
    HBM-resident bytes): a Project/Filter chain directly on top then runs fused INTO the scan
    (``ops/scanfuse.py``); any other consumer gets the plain device scan (``scan()``)."""

    def __init__(self, schema: StructType, scan, fused: Optional[dict], label: str = "CsvScan",
                 sharded: Optional[bool] = None):
        from ..parallel import comm

        self._schema = schema
        self._scan = scan
        self.fused = fused
        self.label = label
        self.sharded = comm.world_size() > 1 if sharded is None else bool(sharded)
        self._memo = None

    @property
    def table(self) -> Table:
        if self._memo is None:
            self._memo = self._scan()
        return self._memo

    def schema(self):
        return self._schema

    def _compute(self, session):
        return self._scan()

    def skey(self):
        return self.__dict__.get("_skey")  # set by the reader from the cached input's identity

    def fresh(self, child=None):
        n = super().fresh()
        n._memo = None
        return n

    def _label(self):
        return f"{self.label} [{', '.join(self._schema.names)}]"


_SCHEMAS: dict = {}   # Project skey -> analyzed schema
_SERIAL = __import__("itertools").count(1)
_CHECKED: set = set()  # Filter skeys whose condition type-checked


def is_sharded(plan) -> bool:
    """True when any leaf relation of ``plan`` is a data-parallel shard (actions then combine
    ranks: counts all-reduce, rows gather in rank order)."""
    if isinstance(plan, LocalRelation):
        return plan.sharded
    return any(is_sharded(c) for c in plan.children())


def output_name(e: Expr) -> str:
    if isinstance(e, Alias):
        return e.name
    if isinstance(e, ColRef):
        return e.name
    return e.sql_name()


class Project(LogicalPlan):
    def __init__(self, child: LogicalPlan, exprs: Sequence[Expr]):
        self.child = child
        self.exprs = list(exprs)
        self._schema = None

    def children(self):
        return [self.child]

    def skey(self):
        k = self._skey
        if k == 0:
            ck = self.child.skey()
            ek = exprs_key(self.exprs) if ck is not None else None
            k = self._skey = intern(("Project", ck, ek)) if ek is not None else None
        return k

    def schema(self):
        if self._schema is None:
            k = self.skey()
            s = _SCHEMAS.get(k) if k is not None else None
            if s is not None:
                self._schema = s
                return s
            cs = self.child.schema()
            fields = []
            for e in self.exprs:
                dt = e.data_type(cs)
                meta = {}
                base = e.child if isinstance(e, Alias) else e
                if isinstance(base, ColRef):
                    meta = dict(cs[base._resolve(cs)].metadata)
                elif hasattr(base, "metadata"):
                    meta = base.metadata(cs)
                fields.append(StructField(output_name(e), dt, e.nullable(cs), meta))
            self._schema = StructType(fields)
            if k is not None:
                if len(_SCHEMAS) >= 4096:
                    _SCHEMAS.clear()
                _SCHEMAS[k] = self._schema
        return self._schema

    def _compute(self, session):
        base = execute(self.child, session)
        ctx = EvalContext(base, session)
        cols = []
        schema = self.schema()
        for e, f in zip(self.exprs, schema.fields):
            c = e.eval(ctx)
            if c.dtype != f.dataType:
                from .expressions import cast_column

                c = cast_column(c, f.dataType, base.device)
            if f.metadata and not c.meta:
                c = ColumnData(c.dtype, c.values, c.valid, dict(f.metadata))
            cols.append(c)
        return base.with_columns(schema, cols)

    def _label(self):
        return "Project [" + ", ".join(output_name(e) for e in self.exprs) + "]"


class Filter(LogicalPlan):
    def __init__(self, child: LogicalPlan, cond: Expr):
        self.child = child
        self.cond = cond
        k = self.skey()
        if k is not None and k in _CHECKED:
            return
        dt = cond.data_type(child.schema())
        if not isinstance(dt, BooleanType):
            raise AnalysisException(f"filter expression '{cond.sql_name()}' of type {dt.simpleString()} "
                                    f"is not a boolean.")
        if k is not None:
            if len(_CHECKED) >= 4096:
                _CHECKED.clear()
            _CHECKED.add(k)

    def children(self):
        return [self.child]

    def skey(self):
        k = self._skey
        if k == 0:
            ck = self.child.skey()
            ek = expr_key(self.cond) if ck is not None else None
            k = self._skey = intern(("Filter", ck, ek)) if ek is not None else None
        return k

    def schema(self):
        return self.child.schema()

    def _compute(self, session):
        base = execute(self.child, session)
        c = self.cond.eval(EvalContext(base, session))
        keep = c.values.to(torch.bool)
        if c.valid is not None:
            keep = keep & c.valid
        sel = keep if base.sel is None else (base.sel & keep)
        t = Table(base.schema, base.columns, base.nrows, sel, base.device)
        return _maybe_compact(t)

    def _label(self):
        return f"Filter {self.cond.sql_name()}"


def _maybe_compact(t: Table, threshold: float = 0.25) -> Table:
    """Keep the selection vector unless the live fraction got small (then compact).  Device
    tables keep it unconditionally: every device consumer (DQ VM, pack, Gram, metrics) reads the
    selection natively, and deciding would cost a host sync per filter."""
    if t.sel is None or t.nrows < 4096 or t.sel.is_cuda:
        return t
    live = int(t.sel.sum().item())
    return t.compact() if live < threshold * t.nrows else t


class Limit(LogicalPlan):
    def __init__(self, child: LogicalPlan, n: int):
        self.child, self.n = child, int(n)

    def children(self):
        return [self.child]

    def skey(self):
        k = self._skey
        if k == 0:
            ck = self.child.skey()
            k = self._skey = intern(("Limit", ck, self.n)) if ck is not None else None
        return k

    def schema(self):
        return self.child.schema()

    def _compute(self, session):
        t = execute(self.child, session)
        if not is_sharded(self.child):
            return t.head_rows(self.n)
        # global LIMIT over shards: keep what is left of n after the ranks before this one
        from ..parallel import comm

        counts = comm.all_gather_object(int(t.count()))
        before = sum(counts[:comm.rank()])
        return t.head_rows(max(0, min(self.n - before, counts[comm.rank()])))

    def _label(self):
        return f"Limit {self.n}"


class Union(LogicalPlan):
    def __init__(self, left: LogicalPlan, right: LogicalPlan):
        if len(left.schema()) != len(right.schema()):
            raise AnalysisException("Union can only be performed on tables with the same number of columns")
        self.left, self.right = left, right

    def children(self):
        return [self.left, self.right]

    def schema(self):
        return self.left.schema()

    def _compute(self, session):
        a, b = execute(self.left, session).compact(), execute(self.right, session).compact()
        cols = []
        for ca, cb in zip(a.columns, b.columns):
            if isinstance(ca.values, list):
                vals = ca.values + cb.values
            else:
                dim = 1 if ca.values.dim() == 2 else 0
                vals = torch.cat([ca.values, cb.values.to(ca.values.dtype)], dim=dim)
            if ca.valid is None and cb.valid is None:
                valid = None
            else:
                valid = torch.cat([ca.valid_mask(a.device), cb.valid_mask(b.device)])
            cols.append(ColumnData(ca.dtype, vals, valid, dict(ca.meta)))
        return Table(a.schema, cols, a.nrows + b.nrows, None, a.device)


def prune_columns(plan: LogicalPlan, required) -> LogicalPlan:
    """Catalyst-style ColumnPruning: a plan whose Projects compute only the output columns some
    consumer needs (``required``: column names, case-insensitive; None = all).  Filters keep
    what their condition references; leaves, Limit and Union are not pruned through.  Unchanged
    subtrees are returned as-is, so their memoized tables are reused.

    Spark's ``LinearRegression.train`` selects (label, features, weight) before aggregating and the
    optimizer prunes every other derived column out of the whole-stage code — e.g. a DQ rule
    output only used by a filter is evaluated in registers, never materialized."""
    if required is None:
        return plan
    req = {r.lower() for r in required}
    if isinstance(plan, Project):
        keep = [e for e in plan.exprs if output_name(e).lower() in req]
        child_req = set()
        for e in keep:
            child_req |= e.references()
        child = prune_columns(plan.child, child_req)
        if len(keep) == len(plan.exprs) and child is plan.child:
            return plan
        return Project(child, keep)
    if isinstance(plan, Filter):
        child = prune_columns(plan.child, req | {r.lower() for r in plan.cond.references()})
        f = plan if child is plan.child else Filter(child, plan.cond)
        names = f.schema().names
        if any(n.lower() not in req for n in names):
            # columns only the condition needs: drop them right above the filter, so a fused
            # Project/Filter chain evaluates them in registers and never stores them
            return Project(f, [ColRef(n) for n in names if n.lower() in req])
        return f
    return plan


_exec_lock = threading.RLock()


def execute(plan: LogicalPlan, session=None) -> Table:
    if plan._memo is not None:
        return plan._memo
    with _exec_lock:
        if plan._memo is None:
            from ..ops import dqvm

            fused = dqvm.try_execute_fused(plan, session)
            plan._memo = fused if fused is not None else plan._compute(session)
    return plan._memo


_ = (Tuple, UdfCall)
