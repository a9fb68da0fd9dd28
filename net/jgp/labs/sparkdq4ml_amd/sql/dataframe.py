"""``Dataset<Row>`` façade.

Every DataFrame call the lab makes is here: ``withColumnRenamed`` (``...App.java:58-59``),
``show()``/``show(50)`` (``:63,73,82,94,115,129,137``), ``withColumn`` + ``col``
(``:68-69,86-87,101``), ``printSchema`` (``:72,81,114``) and ``createOrReplaceTempView``
(``:76,88``).  A DataFrame is an immutable handle on a lazy :class:`~.plan.LogicalPlan`.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch

from ..utils.javafmt import java_str
from .column import Column
from .expressions import (Alias, AnalysisException, ColRef, Expr, to_expr)
from .plan import Filter, Limit, LocalRelation, LogicalPlan, Project, Union, execute, is_sharded, output_name
from .skey import expr_key, exprs_key
from .table import Table
from .types import StructType, VectorUDT

__all__ = ["DataFrame", "Row"]


def _rank0() -> bool:
    from ..parallel import comm

    return comm.rank() == 0


class Row(tuple):
    """``pyspark.sql.Row``-like record: a tuple with field names."""

    def __new__(cls, *values, **kw):
        if kw:
            names = list(kw.keys())
            r = tuple.__new__(cls, kw.values())
            r.__fields__ = names
            return r
        r = tuple.__new__(cls, values)
        r.__fields__ = None
        return r

    @classmethod
    def _make(cls, names, values):
        r = tuple.__new__(cls, values)
        r.__fields__ = list(names)
        return r

    def asDict(self):
        return dict(zip(self.__fields__ or [], self))

    def __getattr__(self, item):
        if item.startswith("__"):
            raise AttributeError(item)
        try:
            return self[self.__fields__.index(item)]
        except (ValueError, AttributeError, TypeError):
            raise AttributeError(item) from None

    def __getitem__(self, k):
        if isinstance(k, str):
            return tuple.__getitem__(self, self.__fields__.index(k))
        return tuple.__getitem__(self, k)

    def get(self, i):
        return self[i]

    def getDouble(self, i):
        return float(self[i])

    def getInt(self, i):
        return int(self[i])

    def size(self):
        return len(self)

    def __repr__(self):
        if self.__fields__:
            return "Row(" + ", ".join(f"{n}={v!r}" for n, v in zip(self.__fields__, self)) + ")"
        return "<" + ",".join(repr(v) for v in self) + ">"


def _cell_str(v) -> str:
    if v is None:
        return "null"
    if isinstance(v, str):
        return v
    if isinstance(v, (bytes, bytearray)):
        return "[" + " ".join(f"{b:02X}" for b in v) + "]"
    if hasattr(v, "toString"):
        return v.toString()
    return java_str(v)


def show_string(names: List[str], rows: List[tuple], num_rows: int, truncate: int = 20, vertical=False,
                has_more: bool = False) -> str:
    """``Dataset.showString`` (Spark 2.4): right-aligned cells in ``+---+`` grids, min width 3,
    cells longer than ``truncate`` cut to ``truncate-3`` chars + ``...``."""
    def cut(s):
        if truncate > 0 and len(s) > truncate:
            return s[:truncate] if truncate < 4 else s[: truncate - 3] + "..."
        return s

    header = [cut(n) for n in names]
    body = [[cut(_cell_str(v)) for v in r] for r in rows]
    sb = []
    if not vertical:
        widths = [max(3, len(h)) for h in header]
        for r in body:
            for i, c in enumerate(r):
                widths[i] = max(widths[i], len(c))
        sep = "+" + "+".join("-" * w for w in widths) + "+"

        def line(cells):
            if truncate > 0:
                return "|" + "|".join(c.rjust(w) for c, w in zip(cells, widths)) + "|"
            return "|" + "|".join(c.ljust(w) for c, w in zip(cells, widths)) + "|"

        sb.append(sep)
        sb.append(line(header))
        sb.append(sep)
        for r in body:
            sb.append(line(r))
        sb.append(sep)
        out = "\n".join(sb) + "\n"
    else:
        fw = max([len(h) for h in header] + [0])
        dw = max([len(c) for r in body for c in r] + [0])
        parts = []
        for i, r in enumerate(body):
            head = f"-RECORD {i}"
            parts.append(head.ljust(fw + dw + 3, "-"))
            for h, c in zip(header, r):
                parts.append(h.ljust(fw) + " | " + c.ljust(dw))
        out = "\n".join(parts) + "\n" if parts else "(0 rows)\n"
    if has_more:
        out += f"only showing top {num_rows} {'row' if num_rows == 1 else 'rows'}\n"
    return out


class DataFrameNaFunctions:
    def __init__(self, df):
        self.df = df

    def drop(self, how="any", thresh=None, subset=None):
        from .expressions import IsNotNull, BinOp

        cols = subset or self.df.columns
        conds = [IsNotNull(ColRef(c)) for c in cols]
        if not conds:
            return self.df
        e = conds[0]
        if how == "all":
            for c in conds[1:]:
                e = BinOp("or", e, c)
        else:
            for c in conds[1:]:
                e = BinOp("and", e, c)
        return self.df.filter(Column(e))

    def fill(self, value, subset=None):
        from .functions import coalesce, lit, col

        cols = subset or self.df.columns
        out = self.df
        for c in cols:
            out = out.withColumn(c, coalesce(col(c), lit(value)))
        return out


_DERIVED: dict = {}  # (parent plan skey, transformation) -> analyzed template node (no child)


class DataFrame:
    def __init__(self, plan: LogicalPlan, session):
        self._plan = plan
        self.sparkSession = session
        self._cached = False

    # ---- metadata --------------------------------------------------------------------------
    @property
    def schema(self) -> StructType:
        return self._plan.schema()

    @property
    def columns(self) -> List[str]:
        return self.schema.names

    @property
    def dtypes(self):
        return [(f.name, f.dataType.simpleString()) for f in self.schema.fields]

    def printSchema(self):
        if _rank0():
            print(self.schema.treeString())

    def explain(self, extended=False):
        print("== Physical Plan ==\n" + self._plan.describe())

    # ---- transformations -------------------------------------------------------------------
    def _with(self, plan):
        return DataFrame(plan, self.sparkSession)

    def _derive(self, op, build):
        """Structural sharing of analysis (``sql/skey.py``): the transformation ``op`` of a plan
        with the same structural key was analyzed before -> a fresh copy of that analyzed node over
        this DataFrame's plan (no execution result is shared: the copy has none).  Else ``build()``
        analyzes, and a one-node result over this plan is kept as the template."""
        pk = self._plan.skey() if op is not None else None
        if pk is not None:
            t = _DERIVED.get((pk, op))
            if t is not None:
                return DataFrame(t.fresh(self._plan), self.sparkSession)
        df = build()
        node = df._plan
        if pk is not None and node is not self._plan and getattr(node, "child", None) is self._plan \
                and node.skey() is not None:
            node.schema()  # analyzed before it becomes a template
            t = node.fresh()
            t.child = None  # the template holds no lineage (and so no execution results)
            if len(_DERIVED) >= 4096:
                _DERIVED.clear()
            _DERIVED[(pk, op)] = t
        return df

    def col(self, name: str) -> Column:
        if name != "*" and self.schema.resolve_ci(name) is None:
            raise AnalysisException(f'Cannot resolve column name "{name}" among ({", ".join(self.columns)});')
        return Column(ColRef(name))

    apply = col

    def __getitem__(self, item):
        if isinstance(item, str):
            return self.col(item)
        if isinstance(item, Column):
            return self.filter(item)
        if isinstance(item, (list, tuple)):
            return self.select(*item)
        raise TypeError(item)

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        if name in self.__dict__.get("_plan").schema().names:
            return self.col(name)
        raise AttributeError(name)

    def select(self, *cols) -> "DataFrame":
        if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
            cols = cols[0]
        exprs: List[Expr] = []
        for c in cols:
            if isinstance(c, str):
                if c == "*":
                    exprs += [ColRef(n) for n in self.columns]
                else:
                    exprs.append(ColRef(c))
            else:
                exprs.append(to_expr(c))
        ek = exprs_key(exprs)

        def build():
            self._check_refs(exprs)
            return self._with(Project(self._plan, exprs))
        return self._derive(("select", ek) if ek is not None else None, build)

    def selectExpr(self, *exprs):
        from .parser import parse_select_item

        return self.select(*[Column(parse_select_item(e)) for e in exprs])

    def _check_refs(self, exprs):
        schema = self.schema
        for e in exprs:
            e.data_type(schema)  # raises AnalysisException on unresolved columns

    def withColumn(self, name: str, c: Column) -> "DataFrame":
        e = to_expr(c)
        ek = expr_key(e)
        return self._derive(("withColumn", name, ek) if ek is not None else None, lambda: self._with_column(name, e))

    def _with_column(self, name: str, e) -> "DataFrame":
        names = self.columns
        exprs = []
        replaced = False
        for n in names:
            if n == name or n.lower() == name.lower():
                exprs.append(Alias(e, name))
                replaced = True
            else:
                exprs.append(ColRef(n))
        if not replaced:
            exprs.append(Alias(e, name))
        self._check_refs([e])
        return self._with(Project(self._plan, exprs))

    def withColumnRenamed(self, existing: str, new: str) -> "DataFrame":
        def build():
            names = self.columns
            if existing not in names:
                return self
            return self._with(Project(self._plan, [Alias(ColRef(n), new) if n == existing else ColRef(n)
                                                   for n in names]))
        return self._derive(("withColumnRenamed", existing, new), build)

    def drop(self, *cols):
        drop = {c if isinstance(c, str) else output_name(c._expr) for c in cols}
        return self._with(Project(self._plan, [ColRef(n) for n in self.columns if n not in drop]))

    def filter(self, cond) -> "DataFrame":
        if isinstance(cond, str):
            from .parser import parse_expression

            e = parse_expression(cond)
        else:
            e = to_expr(cond)
        ek = expr_key(e)
        return self._derive(("filter", ek) if ek is not None else None, lambda: self._with(Filter(self._plan, e)))

    where = filter


    def where(self, cond) -> "DataFrame":
        """Alias of :meth:`filter` (Dataset.where)."""
        return self.filter(cond)
    def limit(self, n: int) -> "DataFrame":
        return self._with(Limit(self._plan, n))

    def union(self, other: "DataFrame") -> "DataFrame":
        return self._with(Union(self._plan, other._plan))

    unionAll = union

    @property
    def na(self):
        return DataFrameNaFunctions(self)

    def dropna(self, how="any", thresh=None, subset=None):
        return self.na.drop(how, thresh, subset)

    def fillna(self, value, subset=None):
        return self.na.fill(value, subset)

    def alias(self, name):
        return self

    def toDF(self, *names):
        if len(names) != len(self.columns):
            raise ValueError("number of column names does not match")
        return self._with(Project(self._plan, [Alias(ColRef(o), n) for o, n in zip(self.columns, names)]))

    # ---- persistence -----------------------------------------------------------------------
    def cache(self):
        execute(self._plan, self.sparkSession)
        self._cached = True
        return self

    persist = cache

    def unpersist(self, blocking=False):
        self._cached = False
        return self

    def checkpoint(self, eager=True):
        t = self._table()
        return DataFrame(LocalRelation(t.compact()), self.sparkSession)

    localCheckpoint = checkpoint

    # ---- actions ---------------------------------------------------------------------------
    def _table(self) -> Table:
        return execute(self._plan, self.sparkSession)

    def count(self) -> int:
        n = self._table().count()
        if is_sharded(self._plan):  # X2-style: sum of the shards' counts
            from ..parallel import comm

            return int(sum(comm.all_gather_object(int(n))))
        return n

    def _rows(self, t: Table) -> List[Row]:
        names = t.schema.names
        return [Row._make(names, r) for r in self._gather(t.to_rows())]

    def _gather(self, local_rows, limit: Optional[int] = None):
        """X5: rows of every shard in rank order (= global row order) on every rank."""
        if not is_sharded(self._plan):
            return local_rows
        from ..parallel import comm

        out = []
        for part in comm.all_gather_object([tuple(r) for r in local_rows]):
            out.extend(part)
            if limit is not None and len(out) >= limit:
                return out[:limit]
        return out

    def collect(self) -> List[Row]:
        return self._rows(self._table())

    collectAsList = collect

    def take(self, n: int) -> List[Row]:
        t = self._table().head_rows(n)
        names = t.schema.names
        return [Row._make(names, r) for r in self._gather(t.to_rows(), n)]

    def head(self, n: Optional[int] = None):
        if n is None:
            r = self.take(1)
            return r[0] if r else None
        return self.take(n)

    def first(self):
        return self.head()

    def isEmpty(self):
        return len(self.take(1)) == 0

    def showString(self, n: int = 20, truncate=True, vertical=False) -> str:
        tr = 20 if truncate is True else (0 if truncate is False else int(truncate))
        t = self._table().head_rows(n + 1)
        rows = self._gather(t.to_rows(), n + 1)
        has_more = len(rows) > n
        return show_string(t.schema.names, rows[:n], n, tr, vertical, has_more)

    def show(self, n: int = 20, truncate=True, vertical=False):
        if isinstance(n, bool):
            n, truncate = 20, n
        s = self.showString(n, truncate, vertical)  # collective on sharded data: every rank joins
        if _rank0():
            print(s)

    def toPandas(self):
        import pandas as pd

        if is_sharded(self._plan):
            rows = self.collect()
            return pd.DataFrame([tuple(r) for r in rows], columns=self.columns)
        t = self._table().compact()
        data = {}
        for f, c in zip(t.schema.fields, t.columns):
            data[f.name] = c.to_pylist()
        return pd.DataFrame(data, columns=t.schema.names)

    def foreach(self, f):
        for r in self.collect():
            f(r)

    def describe(self, *cols):
        from .describe import describe

        return describe(self, list(cols) or [f.name for f in self.schema.fields
                                             if not isinstance(f.dataType, VectorUDT)])

    def createOrReplaceTempView(self, name: str):
        self.sparkSession.catalog._views[name.lower()] = self._plan

    def createTempView(self, name: str):
        if name.lower() in self.sparkSession.catalog._views:
            raise AnalysisException(f"Temporary view '{name}' already exists")
        self.createOrReplaceTempView(name)

    registerTempTable = createOrReplaceTempView

    @property
    def write(self):
        from .readwriter import DataFrameWriter

        return DataFrameWriter(self)

    def __repr__(self):
        return "DataFrame[" + ", ".join(f"{n}: {t}" for n, t in self.dtypes) + "]"


_ = (Sequence, torch)
