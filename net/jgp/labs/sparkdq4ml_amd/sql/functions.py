"""``org.apache.spark.sql.functions`` subset (``callUDF`` is imported statically by the lab,
``DataQuality4MachineLearningApp.java:3``)."""
from __future__ import annotations

from .column import Column
from .expressions import CaseWhen, Coalesce, ColRef, IsNull, Lit, UdfCall, to_expr

__all__ = ["col", "column", "lit", "callUDF", "call_udf", "udf", "when", "coalesce", "isnull", "expr"]


def col(name: str) -> Column:
    return Column(ColRef(name))


column = col


def lit(v) -> Column:
    return v if isinstance(v, Column) else Column(Lit(v))


def callUDF(name: str, *cols) -> Column:
    return Column(UdfCall(name, [c._expr if isinstance(c, Column) else ColRef(c) if isinstance(c, str) else to_expr(c)
                                 for c in cols]))


call_udf = callUDF


def when(cond: Column, value) -> Column:
    return Column(CaseWhen([(to_expr(cond), to_expr(value))]))


def coalesce(*cols) -> Column:
    return Column(Coalesce(*[c._expr if isinstance(c, Column) else ColRef(c) for c in cols]))


def isnull(c) -> Column:
    return Column(IsNull(c._expr if isinstance(c, Column) else ColRef(c)))


def expr(text: str) -> Column:
    from .parser import parse_expression

    return Column(parse_expression(text))


def udf(f=None, returnType=None):
    """``pyspark.sql.functions.udf``: wrap a python scalar function as an (anonymous) UDF."""
    from .udf import UserDefinedFunction
    from .types import DoubleType, StringType, parse_type_name

    def wrap(fn):
        rt = returnType if returnType is not None else StringType()
        rt = parse_type_name(rt) if isinstance(rt, str) else rt
        u = UserDefinedFunction(getattr(fn, "__name__", "udf"), fn, rt)
        return u

    if f is None or not callable(f) or isinstance(f, str):
        if f is not None and returnType is None:
            returnType = f
        return wrap
    return wrap(f)
