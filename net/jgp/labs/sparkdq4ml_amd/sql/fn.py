"""Built-in numeric SQL functions (abs, sqrt, exp, ln/log, pow, floor, ceil, round, greatest, least)."""
from __future__ import annotations

import torch

from .expressions import Expr, _and_valid, _num, to_expr
from .table import ColumnData
from .types import DoubleType, LongType, is_numeric, wider_numeric

__all__ = ["MathFn", "BUILTIN_MATH"]

BUILTIN_MATH = {"abs", "sqrt", "exp", "ln", "log", "log10", "pow", "power", "floor", "ceil", "ceiling",
                "round", "greatest", "least", "signum"}


class MathFn(Expr):
    def __init__(self, name, args):
        self.name = name
        self.args = [to_expr(a) for a in args]

    def children(self):
        return list(self.args)

    def data_type(self, schema):
        if self.name == "abs":
            return self.args[0].data_type(schema)
        if self.name in ("floor", "ceil", "ceiling"):
            return LongType()
        if self.name in ("greatest", "least"):
            t = self.args[0].data_type(schema)
            for a in self.args[1:]:
                t = wider_numeric(t, a.data_type(schema))
            return t
        if self.name == "round":
            t = self.args[0].data_type(schema)
            return t if is_numeric(t) else DoubleType()
        return DoubleType()

    def nullable(self, schema):
        return True if self.name in ("sqrt", "ln", "log", "log10") else super().nullable(schema)

    def sql_name(self):
        return f"{self.name.upper()}(" + ", ".join(a.sql_name() for a in self.args) + ")"

    def eval(self, ctx):
        cols = [a.eval(ctx) for a in self.args]
        t = self.data_type(ctx.table.schema)
        valid = _and_valid(*cols)
        x = [_num(c, DoubleType()) for c in cols]
        n = self.name
        if n == "abs":
            out = torch.abs(cols[0].values)
        elif n == "sqrt":
            out = torch.sqrt(x[0])
            bad = x[0] < 0
            valid = ~bad if valid is None else valid & ~bad
        elif n == "exp":
            out = torch.exp(x[0])
        elif n in ("ln", "log") and len(x) == 1:
            out = torch.log(x[0])
            bad = x[0] <= 0
            valid = ~bad if valid is None else valid & ~bad
        elif n == "log":
            out = torch.log(x[1]) / torch.log(x[0])
        elif n == "log10":
            out = torch.log10(x[0])
            bad = x[0] <= 0
            valid = ~bad if valid is None else valid & ~bad
        elif n in ("pow", "power"):
            out = torch.pow(x[0], x[1])
        elif n == "floor":
            out = torch.floor(x[0])
        elif n in ("ceil", "ceiling"):
            out = torch.ceil(x[0])
        elif n == "round":
            scale = int(self.args[1].value) if len(self.args) > 1 else 0
            f = 10.0 ** scale
            v = x[0] * f
            out = torch.sign(v) * torch.floor(torch.abs(v) + 0.5) / f  # HALF_UP
        elif n == "signum":
            out = torch.sign(x[0])
        elif n in ("greatest", "least"):
            out = x[0]
            for y in x[1:]:
                out = torch.maximum(out, y) if n == "greatest" else torch.minimum(out, y)
        else:
            raise ValueError(n)
        if valid is not None and bool(valid.all()):
            valid = None
        return ColumnData(t, out.to(t.torch_dtype), valid)
