"""Named UDF registry (``spark.udf().register(name, udf, DataTypes.DoubleType)``,
``DataQuality4MachineLearningApp.java:46-49``).

Three kinds of function can be registered:

* **rule objects** exposing ``ir(*arg_exprs) -> Expr`` (the DQ rules of :mod:`..dq`): expanded
  into the expression IR at analysis time, so they are vectorized on the device and fusable into
  the DQ VM kernel — the fast path;
* **Java-style** ``UDF1``/``UDF2`` objects exposing ``call(*args)``: evaluated row by row on the
  live rows with boxed ``None`` for nulls, exactly like Spark's ScalaUDF for Java UDFs;
* plain python callables (pyspark ``udf``): same row-by-row contract; ``vectorized=True`` callables
  receive whole device tensors instead.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch

from .table import ColumnData
from .types import DataType, DoubleType, StringType, parse_type_name

__all__ = ["UserDefinedFunction", "UDFRegistration"]


class UserDefinedFunction:
    def __init__(self, name: str, func: Optional[Callable], returnType: DataType,
                 ir_builder: Optional[Callable] = None, deterministic: bool = True, vectorized: bool = False):
        self.name = name
        self.func = func
        self.returnType = returnType
        self.ir_builder = ir_builder
        self.deterministic = deterministic
        self.vectorized = vectorized

    def __call__(self, *cols):
        from .column import Column
        from .expressions import ColRef, UdfCall, to_expr

        args = [ColRef(c) if isinstance(c, str) else to_expr(c) for c in cols]
        return Column(UdfCall(self.name, args, udf=self))

    def asNondeterministic(self):
        self.deterministic = False
        return self

    def eval_opaque(self, args, ctx) -> ColumnData:
        n = ctx.n
        rt = self.returnType
        dev = ctx.device
        if self.vectorized:
            out = self.func(*[a.values for a in args])
            if not torch.is_tensor(out):
                out = torch.as_tensor(out)
            return ColumnData(rt, out.to(device=dev, dtype=rt.torch_dtype) if rt.torch_dtype else out, None)
        live = ctx.table.sel_mask().detach().cpu().tolist()
        cols = [a.to_pylist() for a in args]
        res = []
        for i in range(n):
            if not live[i]:
                res.append(None)
                continue
            try:
                res.append(self.func(*[c[i] for c in cols]))
            except Exception as e:  # job failure, like an exception inside a Spark task
                from .expressions import SparkException

                raise SparkException(f"Failed to execute user defined function({self.name}: "
                                     f"({', '.join(a.dtype.simpleString() for a in args)}) => "
                                     f"{rt.simpleString()})") from e
        valid = [r is not None for r in res]
        if isinstance(rt, StringType):
            vals = [None if r is None else str(r) for r in res]
            return ColumnData(rt, vals, torch.tensor(valid, dtype=torch.bool, device=dev))
        vals = [0 if r is None else r for r in res]
        t = torch.tensor(vals, dtype=rt.torch_dtype, device=dev)
        vt = torch.tensor(valid, dtype=torch.bool, device=dev)
        return ColumnData(rt, t, None if all(valid) else vt)


class UDFRegistration:
    """``spark.udf()`` (Java) / ``spark.udf`` (python) — both spellings work."""

    def __init__(self, session):
        self._session = session
        self._fns = {}

    def __call__(self):
        return self

    def register(self, name: str, f, returnType=None):
        if isinstance(returnType, str):
            returnType = parse_type_name(returnType)
        if isinstance(f, UserDefinedFunction):
            u = UserDefinedFunction(name, f.func, returnType or f.returnType, f.ir_builder, f.deterministic, f.vectorized)
        else:
            rt = returnType if returnType is not None else getattr(f, "returnType", None) or DoubleType()
            ir = getattr(f, "ir", None)
            fn = getattr(f, "call", None) or f
            if not callable(fn) and ir is None:
                raise TypeError(f"cannot register {f!r} as a UDF")
            u = UserDefinedFunction(name, fn if callable(fn) else None, rt, ir,
                                    vectorized=bool(getattr(f, "vectorized", False)))
        self._fns[name.lower()] = u
        return u

    def lookup(self, name: str) -> UserDefinedFunction:
        u = self._fns.get(name.lower())
        if u is None:
            from .expressions import AnalysisException

            raise AnalysisException(f"Undefined function: '{name}'. This function is neither a registered "
                                    f"temporary function nor a permanent function registered in the database 'default'.")
        return u

    def names(self):
        return sorted(self._fns)
