"""Expression IR.

Every column expression the lab builds — ``col``, literals, the comparison in the DQ clean-up
``WHERE price_no_min > 0`` (``DataQuality4MachineLearningApp.java:77-78``), ``cast(guest as int)``,
aliases and the two DQ rule UDF calls (``...App.java:68-69,86-87``) — is a node of this IR.

Two evaluators consume it:

* ``Expr.eval`` — a vectorized evaluator over :class:`ColumnData` (torch tensors on the session
  device) with SQL three-valued null semantics;
* ``ops.dqvm`` — compiles a fusable sub-tree into the byte-code of the device DQ virtual machine
  (``csrc/hip/dq_vm.hip``), so whole Project/Filter chains run as one HIP kernel.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence

import torch

from .table import ColumnData, Table
from .types import (BooleanType, DataType, DecimalType, DoubleType, FloatType, IntegerType,
                    LongType, NullType, StringType, StructType, TimestampType, VectorUDT,
                    is_numeric, parse_type_name, wider_numeric)

__all__ = [
    "Expr", "ColRef", "Lit", "BinOp", "Not", "Neg", "Cast", "Alias", "IsNull", "IsNotNull",
    "If", "CaseWhen", "Coalesce", "UdfCall", "RaiseIfNull", "AnalysisException", "EvalContext",
    "to_expr",
]


class AnalysisException(Exception):
    """Mirror of ``org.apache.spark.sql.AnalysisException``."""


class EvalContext:
    def __init__(self, table: Table, session=None):
        self.table = table
        self.session = session
        self.device = table.device

    @property
    def n(self):
        return self.table.nrows


def _java_num_str(v):
    from ..utils.javafmt import java_str

    return java_str(v)


class Expr:
    # ---- analysis -------------------------------------------------------------------------
    def children(self) -> List["Expr"]:
        return []

    def data_type(self, schema: StructType) -> DataType:
        raise NotImplementedError

    def nullable(self, schema: StructType) -> bool:
        return any(c.nullable(schema) for c in self.children())

    def sql_name(self) -> str:
        raise NotImplementedError

    def references(self) -> set:
        out = set()
        for c in self.children():
            out |= c.references()
        return out

    def deterministic(self) -> bool:
        return all(c.deterministic() for c in self.children())

    # ---- evaluation -----------------------------------------------------------------------
    def eval(self, ctx: EvalContext) -> ColumnData:
        raise NotImplementedError

    def __repr__(self):
        return self.sql_name()


def to_expr(v) -> Expr:
    if isinstance(v, Expr):
        return v
    e = getattr(v, "_expr", None)  # a Column
    if isinstance(e, Expr):
        return e
    return Lit(v)


# --------------------------------------------------------------------------------------------
# leaves
# --------------------------------------------------------------------------------------------
class ColRef(Expr):
    def __init__(self, name: str):
        self.name = name

    def _field(self, schema):
        try:
            return schema[self._resolve(schema)]
        except KeyError:
            raise AnalysisException(
                f"cannot resolve '`{self.name}`' given input columns: [{', '.join(schema.names)}]") from None

    def _resolve(self, schema):
        if hasattr(schema, "resolve_ci"):
            n = schema.resolve_ci(self.name)
            if n is None:
                raise KeyError(self.name)
            return n
        names = schema.names
        if self.name in names:
            return self.name
        for n in names:
            if n.lower() == self.name.lower():
                return n
        raise KeyError(self.name)

    def data_type(self, schema):
        return self._field(schema).dataType

    def nullable(self, schema):
        return self._field(schema).nullable

    def sql_name(self):
        return self.name

    def references(self):
        return {self.name}

    def eval(self, ctx):
        try:
            return ctx.table.column(self.name)
        except KeyError:
            raise AnalysisException(f"cannot resolve '`{self.name}`' given input columns: "
                                    f"[{', '.join(ctx.table.schema.names)}]") from None


class Lit(Expr):
    def __init__(self, value, dtype: Optional[DataType] = None):
        self.value = value
        if dtype is None:
            if value is None:
                dtype = NullType()
            elif isinstance(value, bool):
                dtype = BooleanType()
            elif isinstance(value, int):
                dtype = IntegerType() if -2 ** 31 <= value < 2 ** 31 else LongType()
            elif isinstance(value, float):
                dtype = DoubleType()
            elif isinstance(value, str):
                dtype = StringType()
            else:
                raise TypeError(f"Unsupported literal type {type(value)}")
        self.dtype = dtype

    def data_type(self, schema):
        return self.dtype

    def nullable(self, schema):
        return self.value is None

    def sql_name(self):
        if self.value is None:
            return "NULL"
        if isinstance(self.value, bool):
            return "true" if self.value else "false"
        if isinstance(self.value, str):
            return self.value
        return _java_num_str(self.value)

    def eval(self, ctx):
        n = ctx.n
        if isinstance(self.dtype, StringType):
            return ColumnData(self.dtype, [self.value] * n, None)
        if self.value is None:
            return ColumnData(NullType(), torch.zeros(n, dtype=torch.float64, device=ctx.device),
                              torch.zeros(n, dtype=torch.bool, device=ctx.device))
        return ColumnData(self.dtype, torch.full((n,), self.value, dtype=self.dtype.torch_dtype, device=ctx.device), None)


# --------------------------------------------------------------------------------------------
# helpers
# --------------------------------------------------------------------------------------------
def _and_valid(*cols: ColumnData):
    v = None
    for c in cols:
        if c.valid is not None:
            v = c.valid if v is None else (v & c.valid)
    return v


def _num(c: ColumnData, target: DataType) -> torch.Tensor:
    if isinstance(c.dtype, StringType):
        raise AnalysisException("string arithmetic is not supported on the device path")
    return c.values.to(target.torch_dtype) if c.values.dtype != target.torch_dtype else c.values


_CMP = {"<": torch.lt, ">": torch.gt, "<=": torch.le, ">=": torch.ge, "=": torch.eq, "==": torch.eq,
        "!=": torch.ne, "<>": torch.ne}
_ARITH = {"+": torch.add, "-": torch.sub, "*": torch.mul}


def _spark_cmp(op: str, a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Spark SQL's NaN-aware float/double ordering (``SQLOrderingUtil``/``NaN semantics``): NaN
    equals NaN and sorts above every other value, including +Infinity.  Integral operands take
    the plain comparison."""
    if not (a.is_floating_point() or b.is_floating_point()):
        return _CMP[op](a, b)
    an, bn = torch.isnan(a), torch.isnan(b)
    if op in ("=", "==", "!=", "<>"):
        eq = torch.eq(a, b) | (an & bn)
        return eq if op in ("=", "==") else ~eq
    if op == "<":
        return ~an & (bn | torch.lt(a, b))
    if op == ">":
        return ~bn & (an | torch.gt(a, b))
    if op == "<=":
        return bn | (~an & torch.le(a, b))
    return an | (~bn & torch.ge(a, b))  # ">="


class BinOp(Expr):
    """Binary operator.  Comparisons follow Spark SQL (NaN = NaN, NaN above everything) unless
    ``ieee=True``: the rule IR of a Java UDF body (``dq/rules.py``) compares primitive doubles
    with Java's IEEE semantics (every comparison with NaN is false), exactly as the reference's
    ``MinimumPriceDataQualityService.java:8`` / ``PriceCorrelationDataQualityService.java:6`` do."""

    def __init__(self, op: str, left: Expr, right: Expr, ieee: bool = False):
        self.op, self.left, self.right = op, to_expr(left), to_expr(right)
        self.ieee = bool(ieee)

    def children(self):
        return [self.left, self.right]

    def operand_type(self, schema):
        lt, rt = self.left.data_type(schema), self.right.data_type(schema)
        if isinstance(lt, StringType) and isinstance(rt, StringType):
            return lt
        if isinstance(lt, TimestampType) and isinstance(rt, TimestampType):
            return lt
        if (isinstance(lt, TimestampType) and isinstance(rt, StringType)) or \
                (isinstance(rt, TimestampType) and isinstance(lt, StringType)):
            # Spark 2.4 findCommonTypeForBinaryComparison: (Timestamp, String) -> StringType, the
            # timestamp side is printed (yyyy-MM-dd HH:mm:ss[.f]) and the two compare as text
            # (casting the string to a timestamp instead is Spark 3.0)
            return StringType()
        if isinstance(lt, StringType) or isinstance(rt, StringType):
            # Spark casts the string side to the numeric type (or double)
            return DoubleType()
        if isinstance(lt, BooleanType) and isinstance(rt, BooleanType):
            return lt
        return wider_numeric(lt, rt)

    def data_type(self, schema):
        if self.op in _CMP or self.op in ("and", "or", "<=>"):
            return BooleanType()
        if self.op == "/":
            return DoubleType()
        return self.operand_type(schema)

    def nullable(self, schema):
        if self.op == "<=>":
            return False
        if self.op == "/":
            return True
        return super().nullable(schema)

    def sql_name(self):
        op = {"and": "AND", "or": "OR", "==": "="}.get(self.op, self.op)
        return f"({self.left.sql_name()} {op} {self.right.sql_name()})"

    def eval(self, ctx):
        l = r = None
        if self.op in ("=", "==", "!=", "<>"):
            # a column against a string constant: a device string column compares in HBM, and the
            # constant is never expanded to a row-length list of Python strings
            if isinstance(self.right, Lit) and isinstance(self.right.value, str):
                l = self.left.eval(ctx)
                eq = _device_string_eq(self, l, None)
            elif isinstance(self.left, Lit) and isinstance(self.left.value, str):
                r = self.right.eval(ctx)
                eq = _device_string_eq(self, None, r)
            else:
                eq = None
            if eq is not None:
                c = l if l is not None else r
                return ColumnData(BooleanType(), eq if self.op in ("=", "==") else ~eq, c.valid)
        l = self.left.eval(ctx) if l is None else l
        r = self.right.eval(ctx) if r is None else r
        schema = ctx.table.schema
        if self.op in ("and", "or"):
            lv = l.values.to(torch.bool)
            rv = r.values.to(torch.bool)
            lm, rm = l.valid_mask(ctx.device), r.valid_mask(ctx.device)
            if self.op == "and":
                false_l, false_r = lm & ~lv, rm & ~rv
                val = lv & rv
                valid = (lm & rm) | false_l | false_r
                val = val & ~(false_l | false_r)
            else:
                true_l, true_r = lm & lv, rm & rv
                val = lv | rv
                valid = (lm & rm) | true_l | true_r
                val = (val & lm & rm) | true_l | true_r
            # (a device mask stays as it is: dropping an all-true one would cost a host sync)
            return ColumnData(BooleanType(), val, None if (not valid.is_cuda and bool(valid.all())) else valid)
        valid = _and_valid(l, r)
        if self.op == "<=>":
            t = self.operand_type(schema)
            lm, rm = l.valid_mask(ctx.device), r.valid_mask(ctx.device)
            eq = _spark_cmp("=", _num(l, t), _num(r, t))
            return ColumnData(BooleanType(), (lm & rm & eq) | (~lm & ~rm), None)
        if isinstance(l.dtype, TimestampType) or isinstance(r.dtype, TimestampType):
            t = self.operand_type(schema)
            if isinstance(t, StringType) and self.op in _CMP:
                l, r = cast_column(l, t, ctx.device), cast_column(r, t, ctx.device)
                return BinOp._string_cmp(self.op, l, r, valid, ctx.device)
            if not isinstance(t, TimestampType) or self.op not in _CMP:
                raise AnalysisException(f"cannot resolve '{self.sql_name()}' due to data type mismatch")
            l = l if isinstance(l.dtype, TimestampType) else _cast_timestamp(l, l.dtype, t, ctx.device)
            r = r if isinstance(r.dtype, TimestampType) else _cast_timestamp(r, r.dtype, t, ctx.device)
            return ColumnData(BooleanType(), _spark_cmp(self.op, l.values, r.values), _and_valid(l, r))
        if self.op in ("=", "==", "!=", "<>"):  # a device string column against a constant
            eq = _device_string_eq(self, l, r)
            if eq is not None:
                return ColumnData(BooleanType(), eq if self.op in ("=", "==") else ~eq, valid)
        if isinstance(l.dtype, StringType) and isinstance(r.dtype, StringType):
            if self.op not in _CMP:
                raise AnalysisException(f"operator {self.op} on strings")
            return BinOp._string_cmp(self.op, l, r, valid, ctx.device)
        t = self.operand_type(schema)
        if isinstance(l.dtype, StringType) or isinstance(r.dtype, StringType):
            l, r = _string_to_double(l, ctx), _string_to_double(r, ctx)
            valid = _and_valid(l, r)
        a, b = _num(l, t), _num(r, t)
        if self.op in _CMP:
            cmp = _CMP[self.op](a, b) if self.ieee else _spark_cmp(self.op, a, b)
            return ColumnData(BooleanType(), cmp, valid)
        if self.op in _ARITH:
            return ColumnData(t, _ARITH[self.op](a, b).to(t.torch_dtype), valid)
        if self.op == "/":
            a64, b64 = a.to(torch.float64), b.to(torch.float64)
            zero = b64 == 0
            out = torch.where(zero, torch.zeros_like(a64), a64 / torch.where(zero, torch.ones_like(b64), b64))
            nv = ~zero if valid is None else (valid & ~zero)
            return ColumnData(DoubleType(), out, None if bool(nv.all()) else nv)
        if self.op == "%":
            zero = b == 0
            out = torch.fmod(a, torch.where(zero, torch.ones_like(b), b))
            nv = ~zero if valid is None else (valid & ~zero)
            return ColumnData(t, out, None if bool(nv.all()) else nv)
        raise AnalysisException(f"unsupported operator {self.op}")

    @staticmethod
    def _string_cmp(op, l: ColumnData, r: ColumnData, valid, device) -> ColumnData:
        """Lexicographic comparison of two string columns (UTF-16 order = code-point order for
        the BMP text the reader produces); a null on either side gives null."""
        py = {"<": lambda a, b: a < b, ">": lambda a, b: a > b, "<=": lambda a, b: a <= b,
              ">=": lambda a, b: a >= b, "=": lambda a, b: a == b, "==": lambda a, b: a == b,
              "!=": lambda a, b: a != b, "<>": lambda a, b: a != b}[op]
        lv, rv = l.to_pylist(), r.to_pylist()
        vals = [bool(py(a, b)) if a is not None and b is not None else False for a, b in zip(lv, rv)]
        vmask = [a is not None and b is not None for a, b in zip(lv, rv)]
        vt = torch.tensor(vmask, dtype=torch.bool, device=device)
        if valid is not None:
            vt = vt & valid
        return ColumnData(BooleanType(), torch.tensor(vals, dtype=torch.bool, device=device), vt)


def _device_string_eq(op: "BinOp", l: ColumnData, r: ColumnData):
    """``col = 'text'`` over a device-scanned string column (``DeviceStringColumn.eq_literal``:
    compared in HBM, the strings never built), else None."""
    from .table import DeviceStringColumn

    for col, other in ((l, op.right), (r, op.left)):
        if col is not None and isinstance(col, DeviceStringColumn) and isinstance(other, Lit) \
                and isinstance(other.value, str):
            return col.eq_literal(other.value)
    return None


def _string_to_double(c: ColumnData, ctx) -> ColumnData:
    if not isinstance(c.dtype, StringType):
        return c
    vals, ok = [], []
    for s in c.values:
        try:
            vals.append(float(s))
            ok.append(s is not None)
        except (TypeError, ValueError):
            vals.append(0.0)
            ok.append(False)
    return ColumnData(DoubleType(), torch.tensor(vals, dtype=torch.float64, device=ctx.device),
                      torch.tensor(ok, dtype=torch.bool, device=ctx.device))


class Not(Expr):
    def __init__(self, child):
        self.child = to_expr(child)

    def children(self):
        return [self.child]

    def data_type(self, schema):
        return BooleanType()

    def sql_name(self):
        return f"(NOT {self.child.sql_name()})"

    def eval(self, ctx):
        c = self.child.eval(ctx)
        return ColumnData(BooleanType(), ~c.values.to(torch.bool), c.valid)


class Neg(Expr):
    def __init__(self, child):
        self.child = to_expr(child)

    def children(self):
        return [self.child]

    def data_type(self, schema):
        return self.child.data_type(schema)

    def sql_name(self):
        return f"(- {self.child.sql_name()})"

    def eval(self, ctx):
        c = self.child.eval(ctx)
        return ColumnData(c.dtype, -c.values, c.valid)


class Cast(Expr):
    def __init__(self, child, to):
        self.child = to_expr(child)
        self.to = parse_type_name(to) if isinstance(to, str) else to

    def children(self):
        return [self.child]

    def data_type(self, schema):
        return self.to

    def nullable(self, schema):
        src = self.child.data_type(schema)
        if isinstance(src, StringType) and not isinstance(self.to, StringType):
            return True
        return self.child.nullable(schema)

    def sql_name(self):
        return f"CAST({self.child.sql_name()} AS {self.to.simpleString().upper()})"

    def eval(self, ctx):
        c = self.child.eval(ctx)
        return cast_column(c, self.to, ctx.device)


def cast_column(c: ColumnData, to: DataType, device) -> ColumnData:
    src = c.dtype
    if type(src) is type(to) and src == to:
        return c
    if isinstance(to, StringType):
        from ..utils.javafmt import java_str

        vals = c.to_pylist()
        return ColumnData(to, [None if v is None else (java_str(v) if not isinstance(v, str) else v) for v in vals],
                          c.valid)
    if isinstance(to, TimestampType) or isinstance(src, TimestampType):
        return _cast_timestamp(c, src, to, device)
    if isinstance(src, StringType):
        vals, ok = [], []
        for s in c.values:
            v, good = None, s is not None
            if good:
                try:
                    st = s.strip()
                    if isinstance(to, (IntegerType, LongType)):
                        v = int(st)
                        if isinstance(to, IntegerType) and not (-2 ** 31 <= v < 2 ** 31):
                            good = False
                    elif isinstance(to, BooleanType):
                        lo = st.lower()
                        if lo in ("true", "t", "yes", "y", "1"):
                            v = True
                        elif lo in ("false", "f", "no", "n", "0"):
                            v = False
                        else:
                            good = False
                    else:
                        v = float(st)
                except ValueError:
                    good = False
            vals.append(v if good else 0)
            ok.append(good)
        td = to.torch_dtype
        return ColumnData(to, torch.tensor(vals, dtype=td, device=device), torch.tensor(ok, dtype=torch.bool, device=device))
    if isinstance(src, NullType):
        return ColumnData(to, torch.zeros(c.n, dtype=to.torch_dtype, device=device),
                          torch.zeros(c.n, dtype=torch.bool, device=device))
    vals = c.values
    if isinstance(to, (IntegerType, LongType)) and vals.is_floating_point():
        # Scala Double.toInt: truncation toward zero, saturating, NaN -> 0
        info = torch.iinfo(to.torch_dtype)
        v = torch.nan_to_num(vals.to(torch.float64), nan=0.0)
        v = torch.clamp(torch.trunc(v), info.min, info.max)
        return ColumnData(to, v.to(to.torch_dtype), c.valid)
    if isinstance(to, BooleanType):
        return ColumnData(to, vals != 0, c.valid)
    return ColumnData(to, vals.to(to.torch_dtype), c.valid)


def _cast_timestamp(c: ColumnData, src: DataType, to: DataType, device) -> ColumnData:
    """Spark 2.4 casts to / from TimestampType (int64 microseconds, UTC): a string parses as the
    CSV reader's timestamps do (``csv_parse_timestamp``; null when it does not); a number is
    seconds since the epoch (integral: exact, fractional: ``(d * 1e6).toLong``); a timestamp as a
    long / int is whole seconds (floor), as a double fractional seconds."""
    if isinstance(src, StringType):
        from ..ops import native

        h = native.host()
        vals, ok = [], []
        for s in c.values:
            us = None if s is None else h.csv_parse_timestamp(s.strip())
            vals.append(0 if us is None else us)
            ok.append(us is not None)
        return ColumnData(to, torch.tensor(vals, dtype=torch.int64, device=device),
                          torch.tensor(ok, dtype=torch.bool, device=device))
    vals = c.values
    if isinstance(to, TimestampType):
        if isinstance(src, BooleanType):
            raise AnalysisException(f"cannot resolve 'CAST(... AS TIMESTAMP)' due to data type mismatch: "
                                    f"cannot cast {src.simpleString()} to timestamp")
        us = vals.to(torch.int64) * 1_000_000 if not vals.is_floating_point() else \
            torch.nan_to_num(vals.to(torch.float64) * 1e6, nan=0.0).to(torch.int64)
        return ColumnData(to, us, c.valid)
    # from a timestamp
    if isinstance(to, (LongType, IntegerType)):
        return ColumnData(to, torch.div(vals, 1_000_000, rounding_mode="floor").to(to.torch_dtype), c.valid)
    if isinstance(to, (DoubleType, FloatType)):
        return ColumnData(to, (vals.to(torch.float64) / 1e6).to(to.torch_dtype), c.valid)
    raise AnalysisException(f"cannot resolve 'CAST(... AS {to.simpleString().upper()})' due to data type "
                            f"mismatch: cannot cast timestamp to {to.simpleString()}")


class Alias(Expr):
    def __init__(self, child, name: str):
        self.child = to_expr(child)
        self.name = name

    def children(self):
        return [self.child]

    def data_type(self, schema):
        return self.child.data_type(schema)

    def nullable(self, schema):
        return self.child.nullable(schema)

    def sql_name(self):
        return self.name

    def eval(self, ctx):
        return self.child.eval(ctx)


class IsNull(Expr):
    def __init__(self, child):
        self.child = to_expr(child)

    def children(self):
        return [self.child]

    def data_type(self, schema):
        return BooleanType()

    def nullable(self, schema):
        return False

    def sql_name(self):
        return f"({self.child.sql_name()} IS NULL)"

    def eval(self, ctx):
        c = self.child.eval(ctx)
        return ColumnData(BooleanType(), ~c.valid_mask(ctx.device), None)


class IsNotNull(IsNull):
    def sql_name(self):
        return f"({self.child.sql_name()} IS NOT NULL)"

    def eval(self, ctx):
        c = self.child.eval(ctx)
        return ColumnData(BooleanType(), c.valid_mask(ctx.device).clone(), None)


class If(Expr):
    """``if(cond, a, b)``: a null condition selects ``b`` (SQL semantics)."""

    def __init__(self, cond, a, b):
        self.cond, self.a, self.b = to_expr(cond), to_expr(a), to_expr(b)

    def children(self):
        return [self.cond, self.a, self.b]

    def data_type(self, schema):
        return wider_numeric(self.a.data_type(schema), self.b.data_type(schema)) \
            if is_numeric(self.a.data_type(schema)) or is_numeric(self.b.data_type(schema)) else self.a.data_type(schema)

    def nullable(self, schema):
        return self.a.nullable(schema) or self.b.nullable(schema)

    def sql_name(self):
        return f"(IF({self.cond.sql_name()}, {self.a.sql_name()}, {self.b.sql_name()}))"

    def eval(self, ctx):
        c, a, b = self.cond.eval(ctx), self.a.eval(ctx), self.b.eval(ctx)
        t = self.data_type(ctx.table.schema)
        take = c.values.to(torch.bool) & c.valid_mask(ctx.device)
        vals = torch.where(take, _num(a, t), _num(b, t))
        if a.valid is None and b.valid is None:
            valid = None
        else:
            valid = torch.where(take, a.valid_mask(ctx.device), b.valid_mask(ctx.device))
        return ColumnData(t, vals, valid)


class CaseWhen(Expr):
    def __init__(self, branches: Sequence, otherwise=None):
        self.branches = [(to_expr(c), to_expr(v)) for c, v in branches]
        self.otherwise = to_expr(otherwise) if otherwise is not None else Lit(None)

    def children(self):
        out = []
        for c, v in self.branches:
            out += [c, v]
        return out + [self.otherwise]

    def _chain(self):
        e = self.otherwise
        for c, v in reversed(self.branches):
            e = If(c, v, e)
        return e

    def data_type(self, schema):
        return self._chain().data_type(schema)

    def nullable(self, schema):
        return True

    def sql_name(self):
        body = " ".join(f"WHEN {c.sql_name()} THEN {v.sql_name()}" for c, v in self.branches)
        return f"CASE {body} ELSE {self.otherwise.sql_name()} END"

    def eval(self, ctx):
        return self._chain().eval(ctx)


class Coalesce(Expr):
    def __init__(self, *args):
        self.args = [to_expr(a) for a in args]

    def children(self):
        return list(self.args)

    def data_type(self, schema):
        t = self.args[0].data_type(schema)
        for a in self.args[1:]:
            t = wider_numeric(t, a.data_type(schema))
        return t

    def nullable(self, schema):
        return all(a.nullable(schema) for a in self.args)

    def sql_name(self):
        return "coalesce(" + ", ".join(a.sql_name() for a in self.args) + ")"

    def eval(self, ctx):
        t = self.data_type(ctx.table.schema)
        cols = [a.eval(ctx) for a in self.args]
        vals = _num(cols[-1], t).clone()
        valid = cols[-1].valid_mask(ctx.device).clone()
        for c in reversed(cols[:-1]):
            m = c.valid_mask(ctx.device)
            vals = torch.where(m, _num(c, t), vals)
            valid = valid | m
        return ColumnData(t, vals, None if bool(valid.all()) else valid)


class RaiseIfNull(Expr):
    """Evaluates to its child, but fails the job if a *live* row is null.

    Models the Java auto-unboxing NPE of ``MinimumPriceDataQualityUdf.call(Double)``
    (``MinimumPriceDataQualityUdf.java:11-13``), which has no null guard."""

    def __init__(self, child, message: str):
        self.child, self.message = to_expr(child), message

    def children(self):
        return [self.child]

    def data_type(self, schema):
        return self.child.data_type(schema)

    def nullable(self, schema):
        return False

    def sql_name(self):
        return self.child.sql_name()

    def eval(self, ctx):
        c = self.child.eval(ctx)
        if c.valid is not None:
            live = ctx.table.sel_mask()
            if bool((live & ~c.valid).any()):
                raise SparkException(self.message)
        return ColumnData(c.dtype, c.values, None)


class SparkException(RuntimeError):
    """Job failure (``org.apache.spark.SparkException``)."""


class UdfCall(Expr):
    """``callUDF(name, cols...)`` — resolved against the session's UDF registry at analysis."""

    def __init__(self, name: str, args: Sequence, udf=None):
        self.name = name
        self.args = [to_expr(a) for a in args]
        self.udf = udf  # resolved registry entry (UserDefinedFunction)

    def children(self):
        return list(self.args)

    def _resolved(self, session=None):
        if self.udf is not None:
            return self.udf
        from .session import SparkSession

        s = session or SparkSession.getActiveSession()
        if s is None:
            raise AnalysisException(f"Undefined function: '{self.name}'")
        self.udf = s.udf.lookup(self.name)
        return self.udf

    def data_type(self, schema):
        return self._resolved().returnType

    def nullable(self, schema):
        return True

    def sql_name(self):
        return f"UDF:{self.name}(" + ", ".join(a.sql_name() for a in self.args) + ")"

    def deterministic(self):
        return self._resolved().deterministic and super().deterministic()

    def expanded(self):
        """The IR body of a fusable rule UDF (None for opaque python UDFs)."""
        u = self._resolved()
        if u.ir_builder is None:
            return None
        return u.ir_builder(*self.args)

    def eval(self, ctx):
        u = self._resolved(ctx.session)
        body = self.expanded()
        if body is not None:
            out = body.eval(ctx)
            return cast_column(out, u.returnType, ctx.device) if out.dtype != u.returnType else out
        return u.eval_opaque([a.eval(ctx) for a in self.args], ctx)


_ = (DecimalType, FloatType, TimestampType, VectorUDT, math)
