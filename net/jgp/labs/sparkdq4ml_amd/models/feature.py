"""``org.apache.spark.ml.feature.VectorAssembler`` (``DataQuality4MachineLearningApp.java:110-113``).

Concatenates numeric / boolean / vector input columns into one ``vector`` column.  Physically the
output is a feature-major ``[d, n]`` device matrix produced by the ``pack`` kernel (K4): each
input column becomes one contiguous row of the matrix, cast to ``outputDtype`` (an extension
param; ``float64`` keeps Spark's double semantics, ``float32``/``bfloat16`` feed the fast MFMA Gram
paths).  ``handleInvalid``: ``error`` (default, null -> job failure), ``skip`` (drop rows), ``keep``
(NaN).
"""
from __future__ import annotations

from typing import List

import torch

from ..runtime.checks import defer
from ..utils import tracing
from ..sql.dataframe import DataFrame
from ..sql.expressions import (AnalysisException, ColRef, EvalContext, Expr, IsNotNull, BinOp,
                               SparkException)
from ..sql.plan import Filter, Project
from ..sql.table import ColumnData, LazyVectorColumn
from ..sql.types import (BooleanType, DoubleType, VectorUDT, is_numeric)
from .param import Param, Params, param_accessors

__all__ = ["VectorAssembler", "VectorAssembleExpr"]

_DT = {"float64": torch.float64, "double": torch.float64, "float32": torch.float32, "float": torch.float32,
       "bfloat16": torch.bfloat16, "bf16": torch.bfloat16, "float8": torch.float8_e4m3fn, "fp8": torch.float8_e4m3fn}


class VectorAssembleExpr(Expr):
    def __init__(self, inputs: List[str], handle_invalid: str = "error", out_dtype: str = "float64"):
        self.inputs = list(inputs)
        self.handle_invalid = handle_invalid
        self.out_dtype = out_dtype

    def children(self):
        return [ColRef(c) for c in self.inputs]

    def references(self):
        return set(self.inputs)

    def data_type(self, schema):
        for c in self.inputs:
            t = ColRef(c).data_type(schema)
            if not (is_numeric(t) or isinstance(t, (BooleanType, VectorUDT))):
                raise AnalysisException(f"Data type {t.simpleString()} of column {c} is not supported.")
        return VectorUDT()

    def nullable(self, schema):
        return True

    def num_features(self, schema) -> int:
        d = 0
        for c in self.inputs:
            f = schema[ColRef(c)._resolve(schema)]
            if isinstance(f.dataType, VectorUDT):
                k = f.metadata.get("ml_attr", {}).get("num_attrs")
                if k is None:
                    return -1
                d += int(k)
            else:
                d += 1
        return d

    def metadata(self, schema):
        d = self.num_features(schema)
        return {"ml_attr": {"num_attrs": d}} if d >= 0 else {}

    def sql_name(self):
        return "vecAssembler(" + ", ".join(self.inputs) + ")"

    def eval(self, ctx: EvalContext) -> ColumnData:
        from ..ops import kernels

        cols = [ctx.table.column(c) for c in self.inputs]
        live = ctx.table.sel_mask()
        checks = [ck for c in cols for ck in c.checks]
        if self.handle_invalid == "error":
            # a null input fails the job -- as a device flag read with the first host result
            # (rows shown / fit coefficients), not a host sync here (runtime/checks.py)
            for name, c in zip(self.inputs, cols):
                if c.valid is not None:
                    def exc(name=name):
                        return SparkException(
                            f"Failed to execute user defined function(VectorAssembler$$Lambda: (struct<{name}:double>)"
                            f" => struct<type:tinyint,size:int,indices:array<int>,values:array<double>>) caused by "
                            f"org.apache.spark.SparkException: Values to assemble cannot be null.")
                    checks.append(defer((live & ~c.valid).any(), exc))
        parts = []
        for c in cols:
            if isinstance(c.dtype, VectorUDT):
                parts.append(c.dense())
            else:
                parts.append(c.values.unsqueeze(0) if c.values.dim() == 1 else c.values)
        dt = _DT[self.out_dtype]
        if self.handle_invalid == "keep":
            parts = [p.to(torch.float64) for p in parts]
            parts = [p.unsqueeze(0) if p.dim() == 1 else p for p in parts]
            parts = [torch.where(c.valid_mask(p.device), p, torch.full_like(p, float("nan"))) if c.valid is not None
                     else p for c, p in zip(cols, parts)]
        d = sum(1 if p.dim() == 1 else int(p.shape[0]) for p in parts)
        on_dev = bool(parts) and parts[0].is_cuda
        if dt == torch.bfloat16 and on_dev and d <= 64:
            # MI355X-native storage: MFMA-fragment-ordered tiles, dead rows zeroed (no Gram mask) —
            # produced lazily: a normal-equation fit reads the source columns directly (fused
            # assemble + Gram) and never pays for the pack
            sel = ctx.table.sel

            def _pack(parts=parts, sel=sel):
                with tracing.span("pack"):
                    return kernels.pack_tiled(parts, sel)
            meta = {"ml_attr": {"num_attrs": d}, "zero_dead": sel}
            n = int(parts[0].shape[-1])
            return _with_checks(LazyVectorColumn(VectorUDT(), _pack, n, (parts, sel), meta), checks)
        elif on_dev and (dt == torch.float8_e4m3fn or (dt == torch.bfloat16 and d > 64)):
            # wide fragment layout for the LDS-tiled MFMA SYRK (fp8: per-feature scales)
            with tracing.span("pack"):
                mat = kernels.pack_wide(parts, 8 if dt == torch.float8_e4m3fn else 16, ctx.table.sel)
            meta = {"ml_attr": {"num_attrs": d}, "zero_dead": ctx.table.sel}
        elif on_dev and dt in (torch.float64, torch.float32) and d <= 64:
            # f64 / f32 assembly, produced lazily too: the normal-equation statistics read the
            # source columns directly (gram_skinny_cols for d <= 8, the LDS-DMA stream kernels
            # above); other consumers pack on first use
            def _pack(parts=parts, dt=dt):
                with tracing.span("pack"):
                    return kernels.pack_columns(parts, dt)
            return _with_checks(LazyVectorColumn(VectorUDT(), _pack, int(parts[0].shape[-1]), (parts, ctx.table.sel),
                                                 {"ml_attr": {"num_attrs": d}}), checks)
        elif dt == torch.float8_e4m3fn:  # host engine: fp8 storage is a device layout; keep fp32
            mat = kernels.pack_columns(parts, torch.float32)
            meta = {"ml_attr": {"num_attrs": int(mat.shape[0])}}
        else:
            with tracing.span("pack"):
                mat = kernels.pack_columns(parts, dt)
            meta = {"ml_attr": {"num_attrs": int(mat.shape[0])}}
        return ColumnData(VectorUDT(), mat, None, meta, [c for c in checks if c is not None])


def _with_checks(col, checks):
    col.checks = [c for c in checks if c is not None]
    return col


@param_accessors
class VectorAssembler(Params):
    uid_prefix = "vecAssembler"
    _params = {
        "inputCols": Param("inputCols", "input column names", None, has_default=False),
        "outputCol": Param("outputCol", "output column name", None),
        "handleInvalid": Param("handleInvalid", "how to handle invalid data (NULL values): error, skip or keep",
                               "error", lambda v: v in ("error", "skip", "keep")),
        "outputDtype": Param("outputDtype", "device storage dtype of the assembled matrix "
                                            "(float64 | float32 | bfloat16 | float8)", "float64", lambda v: v in _DT),
    }

    def __init__(self, inputCols=None, outputCol=None, handleInvalid=None, outputDtype=None, uid=None):
        super().__init__(uid)
        self._paramMap["outputCol"] = self.uid + "__output"
        if inputCols is not None:
            self.setInputCols(inputCols)
        if outputCol is not None:
            self.setOutputCol(outputCol)
        if handleInvalid is not None:
            self.setHandleInvalid(handleInvalid)
        if outputDtype is not None:
            self.setOutputDtype(outputDtype)

    def setInputCols(self, cols):
        return self.set("inputCols", list(cols))

    def transform(self, df: DataFrame) -> DataFrame:
        cols = self.getOrDefault("inputCols")
        out = self.getOrDefault("outputCol")
        hi = self.getOrDefault("handleInvalid")
        dt = self.getOrDefault("outputDtype")
        # the same assembly of a structurally equal DataFrame: its analyzed node (sql/skey.py)
        op = ("VectorAssembler", tuple(cols), out, hi, dt) if hi != "skip" else None
        return df._derive(op, lambda: self._transform(df, cols, out, hi))

    def _transform(self, df, cols, out, hi):
        schema = df.schema
        for c in cols:
            ColRef(c).data_type(schema)
        plan = df._plan
        if hi == "skip":
            cond = None
            for c in cols:
                e = IsNotNull(ColRef(c))
                cond = e if cond is None else BinOp("and", cond, e)
            plan = Filter(plan, cond)
        from ..sql.expressions import Alias

        exprs = [ColRef(n) for n in df.columns if n != out] + \
                [Alias(VectorAssembleExpr(cols, hi, self.getOrDefault("outputDtype")), out)]
        return DataFrame(Project(plan, exprs), df.sparkSession)

    def transformSchema(self, schema):
        return Project(_SchemaOnly(schema), [ColRef(n) for n in schema.names] +
                       [VectorAssembleExpr(self.getOrDefault("inputCols"))]).schema()

    # persistence (metadata only, like Spark)
    def save(self, path):
        from .persistence import save_params_only

        save_params_only(self, path, "org.apache.spark.ml.feature.VectorAssembler")

    def write(self):
        from .persistence import ParamsWriter

        return ParamsWriter(self, "org.apache.spark.ml.feature.VectorAssembler")

    @classmethod
    def load(cls, path):
        from .persistence import load_params_only

        return load_params_only(cls, path)


class _SchemaOnly:
    def __init__(self, schema):
        self._s = schema

    def schema(self):
        return self._s


_ = DoubleType
