"""Building device tables from host data (``createDataFrame``, CSV scan results, pandas)."""
from __future__ import annotations

from typing import List, Optional

import numpy as np
import torch

from .table import ColumnData, Table
from .types import (BooleanType, DataType, DecimalType, DoubleType, FloatType, IntegerType,
                    LongType, NullType, StringType, StructField, StructType, TimestampType,
                    VectorUDT, parse_type_name)

__all__ = ["table_from_data", "column_from_pylist", "column_from_numpy"]


def _infer_py(v) -> DataType:
    from ..models.linalg import Vector

    if v is None:
        return NullType()
    if isinstance(v, bool):
        return BooleanType()
    if isinstance(v, (int, np.integer)):
        return LongType()
    if isinstance(v, (float, np.floating)):
        return DoubleType()
    if isinstance(v, str):
        return StringType()
    if isinstance(v, Vector):
        return VectorUDT()
    raise TypeError(f"cannot infer type of {v!r}")


def _merge(a: DataType, b: DataType) -> DataType:
    if isinstance(a, NullType):
        return b
    if isinstance(b, NullType) or a == b:
        return a
    if {type(a), type(b)} <= {LongType, DoubleType, IntegerType}:
        return DoubleType()
    return StringType()


def column_from_pylist(vals: list, dtype: DataType, device) -> ColumnData:
    n = len(vals)
    valid = [v is not None for v in vals]
    vt = None if all(valid) else torch.tensor(valid, dtype=torch.bool, device=device)
    if isinstance(dtype, StringType):
        return ColumnData(dtype, [None if v is None else str(v) for v in vals], vt)
    if isinstance(dtype, VectorUDT):
        d = next((len(v) for v in vals if v is not None), 0)
        arr = np.zeros((d, n), dtype=np.float64)
        for i, v in enumerate(vals):
            if v is not None:
                arr[:, i] = v.toArray()
        return ColumnData(dtype, torch.from_numpy(arr).to(device), vt, {"ml_attr": {"num_attrs": d}})
    if isinstance(dtype, NullType):
        return ColumnData(dtype, torch.zeros(n, dtype=torch.float64, device=device),
                          torch.zeros(n, dtype=torch.bool, device=device))
    td = dtype.torch_dtype
    clean = [(0 if v is None else v) for v in vals]
    return ColumnData(dtype, torch.tensor(clean, dtype=td).to(device), vt)


def column_from_numpy(arr: np.ndarray, valid: Optional[np.ndarray], dtype: DataType, device) -> ColumnData:
    t = torch.from_numpy(np.ascontiguousarray(arr)).to(device=device, dtype=dtype.torch_dtype)
    vt = None
    if valid is not None and not bool(np.all(valid)):
        vt = torch.from_numpy(valid.astype(np.bool_)).to(device)
    return ColumnData(dtype, t, vt)


def _schema_from(schema, names: List[str], types: List[DataType]) -> StructType:
    if isinstance(schema, StructType):
        return schema
    return StructType([StructField(n, t, True) for n, t in zip(names, types)])


def table_from_data(data, schema, device) -> Table:
    device = torch.device(device)
    # pandas
    try:
        import pandas as pd

        if isinstance(data, pd.DataFrame):
            cols, fields = [], []
            for name in data.columns:
                s = data[name]
                if s.dtype.kind in "iu":
                    dt = LongType() if s.dtype.itemsize > 4 else IntegerType()
                    c = column_from_numpy(s.to_numpy(), None, dt, device)
                elif s.dtype.kind == "f":
                    dt = DoubleType() if s.dtype.itemsize == 8 else FloatType()
                    v = s.to_numpy()
                    c = column_from_numpy(np.nan_to_num(v), ~np.isnan(v), dt, device)
                elif s.dtype.kind == "b":
                    dt = BooleanType()
                    c = column_from_numpy(s.to_numpy(), None, dt, device)
                else:
                    vals = [None if (x is None or (isinstance(x, float) and np.isnan(x))) else x for x in s.tolist()]
                    dt = StringType()
                    for v in vals:
                        if v is not None:
                            dt = _infer_py(v)
                            break
                    c = column_from_pylist(vals, dt, device)
                cols.append(c)
                fields.append(StructField(str(name), dt, True))
            return Table(StructType(fields) if not isinstance(schema, StructType) else schema, cols, len(data), None, device)
    except ImportError:  # pragma: no cover
        pass
    # dict of tensors / arrays
    if isinstance(data, dict):
        names = list(data.keys())
        cols, types = [], []
        n = None
        for k in names:
            v = data[k]
            from ..ops.layout import TiledBF16, TiledWide

            valid = None
            if isinstance(v, tuple) and len(v) == 2 and torch.is_tensor(v[0]):  # (values, validity mask)
                v, valid = v
                valid = torch.as_tensor(valid, dtype=torch.bool).to(device)
            if isinstance(v, (TiledBF16, TiledWide)):  # pre-tiled device feature matrix (zero copy)
                c = ColumnData(VectorUDT(), v, None, {"ml_attr": {"num_attrs": int(v.d)}})
            elif torch.is_tensor(v) or isinstance(v, np.ndarray):
                t = torch.as_tensor(v).to(device)
                if t.dim() == 2:
                    dt = VectorUDT()
                    if t.dtype not in (torch.float32, torch.bfloat16, torch.float64):
                        t = t.to(torch.float64)
                    vals = t
                    if t.is_cuda and t.dtype == torch.bfloat16:
                        from ..ops import device as _dev  # ingest into the MFMA-fragment tiled layout

                        vals = _dev.tile_bf16(t) if t.shape[0] <= 64 else _dev.tile_wide(t, 16)
                    c = ColumnData(dt, vals, None, {"ml_attr": {"num_attrs": int(t.shape[0])}})
                else:
                    dt = {torch.float64: DoubleType(), torch.float32: FloatType(), torch.int32: IntegerType(),
                          torch.int64: LongType(), torch.bool: BooleanType()}.get(t.dtype, DoubleType())
                    c = ColumnData(dt, t if t.dtype == dt.torch_dtype else t.to(dt.torch_dtype), valid)
            else:
                vals = list(v)
                dt = NullType()
                for x in vals:
                    dt = _merge(dt, _infer_py(x))
                c = column_from_pylist(vals, dt, device)
            cols.append(c)
            types.append(c.dtype)
            n = c.n
        return Table(_schema_from(schema, names, types), cols, n or 0, None, device)
    # list of rows
    rows = list(data)
    if schema is not None and not isinstance(schema, StructType):
        if isinstance(schema, str):
            fields = []
            for part in schema.split(","):
                nm, _, tp = part.strip().partition(" ")
                if not tp:
                    nm, _, tp = part.strip().partition(":")
                fields.append(StructField(nm.strip(), parse_type_name(tp.strip()), True))
            schema = StructType(fields)
        else:
            names = list(schema)
            schema = None
    else:
        names = None
    if isinstance(schema, StructType):
        names = schema.names
    if rows and isinstance(rows[0], dict):
        names = names or list(rows[0].keys())
        rows = [tuple(r.get(k) for k in names) for r in rows]
    elif rows and hasattr(rows[0], "__fields__") and rows[0].__fields__ and names is None:
        names = list(rows[0].__fields__)
    if not rows:
        if not isinstance(schema, StructType):
            raise ValueError("can not infer schema from empty dataset")
        cols = [column_from_pylist([], f.dataType, device) for f in schema.fields]
        return Table(schema, cols, 0, None, device)
    ncols = len(rows[0])
    names = names or [f"_{i + 1}" for i in range(ncols)]
    colvals = [[r[i] for r in rows] for i in range(ncols)]
    if isinstance(schema, StructType):
        types = [f.dataType for f in schema.fields]
    else:
        types = []
        for vals in colvals:
            t = NullType()
            for v in vals:
                t = _merge(t, _infer_py(v))
            types.append(t if not isinstance(t, NullType) else StringType())
    cols = [column_from_pylist(v, t, device) for v, t in zip(colvals, types)]
    return Table(_schema_from(schema, names, types), cols, len(rows), None, device)


_ = (DecimalType, TimestampType)
