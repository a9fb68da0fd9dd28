"""Physical columnar storage.

A :class:`Table` is the materialized form of a DataFrame: one :class:`ColumnData` per field plus
an optional *selection vector* ``sel`` (bool ``[n]``).  Filters (the DQ clean-up SQL at
``DataQuality4MachineLearningApp.java:77-78,89-90``) only AND into ``sel``; rows are physically
compacted lazily — when rows must be enumerated (``show``/``collect``) or when the live fraction
gets small.  Consumers that reduce over rows (Gram aggregation of ``LinearRegression.fit``,
metrics) take ``sel`` as a 0/1 row weight instead, so the DQ -> assemble -> fit chain never
scatters rows on the device.

Vector columns (``VectorUDT``) are stored **feature-major** ``[d, n]``: every feature is a
contiguous column, which is exactly what the MFMA Gram kernel streams.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np
import torch

from .types import (BooleanType, DataType, DoubleType, IntegerType, LongType, NullType,
                    StringType, StructField, StructType, TimestampType, VectorUDT)

__all__ = ["ColumnData", "DeviceStringColumn", "Table"]


@dataclass
class ColumnData:  # noqa: D101 (dataclass below)
    dtype: DataType
    values: object  # torch.Tensor [n] | [d, n] (VectorUDT) | list (StringType)
    valid: Optional[torch.Tensor] = None  # bool [n]; None => no nulls
    meta: dict = field(default_factory=dict)
    checks: list = field(default_factory=list)  # pending runtime.checks.DeviceCheck (data errors)

    @property
    def n(self) -> int:
        if isinstance(self.values, list):
            return len(self.values)
        return int(self.values.shape[-1])

    def dense(self):
        """Feature-major dense tensor of a vector column (materializes a tiled layout)."""
        from ..ops.layout import TiledBF16, TiledWide

        return self.values.to_dense() if isinstance(self.values, (TiledBF16, TiledWide)) else self.values

    def valid_mask(self, device=None) -> torch.Tensor:
        if self.valid is not None:
            return self.valid
        dev = device if device is not None else (self.values.device if torch.is_tensor(self.values) else "cpu")
        return torch.ones(self.n, dtype=torch.bool, device=dev)

    def has_nulls(self) -> bool:
        return self.valid is not None and not bool(self.valid.all())

    def index(self, idx: torch.Tensor) -> "ColumnData":
        """Gather rows ``idx`` (long tensor)."""
        from ..ops.layout import TiledBF16, TiledWide

        if isinstance(self.values, list):
            il = idx.tolist()
            vals = [self.values[i] for i in il]
        elif isinstance(self.values, (TiledBF16, TiledWide)):
            vals = self.values.gather_rows(idx)
        elif isinstance(self.dtype, VectorUDT):
            vals = self.values.index_select(1, idx.to(self.values.device))
        else:
            vals = self.values.index_select(0, idx.to(self.values.device))
        valid = None if self.valid is None else self.valid.index_select(0, idx.to(self.valid.device))
        return ColumnData(self.dtype, vals, valid, dict(self.meta), list(self.checks))

    def slice(self, start: int, stop: int) -> "ColumnData":
        from ..ops.layout import TiledBF16, TiledWide

        if isinstance(self.values, list):
            vals = self.values[start:stop]
        elif isinstance(self.values, (TiledBF16, TiledWide)):
            vals = self.values.slice_rows(start, stop)
        elif isinstance(self.dtype, VectorUDT):
            vals = self.values[:, start:stop]
        else:
            vals = self.values[start:stop]
        valid = None if self.valid is None else self.valid[start:stop]
        return ColumnData(self.dtype, vals, valid, dict(self.meta), list(self.checks))

    def to_pylist(self) -> list:
        """Host python values (None for null) — used by show/collect.  Raises a pending data
        error of the column (``runtime.checks``) first."""
        if self.checks:
            from ..runtime.checks import verify

            verify(self.checks)
        if isinstance(self.values, list):
            vals = list(self.values)
        elif isinstance(self.dtype, VectorUDT):
            from ..models.linalg import DenseVector

            arr = self.dense().detach().to("cpu", torch.float64).t().contiguous().numpy()
            vals = [DenseVector(row.copy()) for row in arr]
        else:
            t = self.values.detach().cpu()
            if isinstance(self.dtype, BooleanType):
                vals = [bool(v) for v in t.tolist()]
            elif isinstance(self.dtype, TimestampType):
                vals = [micros_to_datetime(v) for v in t.tolist()]
            elif isinstance(self.dtype, (IntegerType, LongType)):
                vals = [int(v) for v in t.tolist()]
            else:
                vals = [float(v) for v in t.to(torch.float64).tolist()]
        if self.valid is not None:
            m = self.valid.detach().cpu().tolist()
            vals = [v if ok else None for v, ok in zip(vals, m)]
        return vals


_EPOCH = None


def micros_to_datetime(us: int):
    """A TimestampType value (microseconds since the epoch, UTC) as the naive ``datetime`` a
    ``collect()`` returns (PySpark: local time; the engine's session time zone is UTC)."""
    import datetime

    global _EPOCH
    if _EPOCH is None:
        _EPOCH = datetime.datetime(1970, 1, 1)
    return _EPOCH + datetime.timedelta(microseconds=int(us))


class LazyVectorColumn(ColumnData):
    """A vector column whose storage is produced on first use (the VectorAssembler's output):
    consumers that can read the SOURCE columns directly (the fused assemble+Gram kernel) never
    materialize it; everything else gets the packed matrix through ``values``."""

    def __init__(self, dtype, materialize, n: int, sources, meta=None):  # noqa: D107
        self.dtype = dtype
        self.valid = None
        self.meta = meta or {}
        self._materialize = materialize
        self._vals = None
        self._n = int(n)
        self.sources = sources  # (parts, sel)
        self.checks = []

    @property
    def values(self):
        if self._vals is None:
            self._vals = self._materialize()
        return self._vals

    @values.setter
    def values(self, v):
        self._vals = v

    @property
    def materialized(self) -> bool:
        return self._vals is not None

    @property
    def n(self) -> int:
        return self._n


class DeviceStringColumn(ColumnData):
    """A string column of a device CSV scan (``ops/csvscan.py``): per row the packed span of its
    field in the scanned input bytes (int64 ``[n]`` in HBM: ``(fs << 25) | (raw << 24) | len``,
    ``csv_scan.h`` kind 4) and its validity.  The Python strings are built on first use of
    ``values`` by the host tokenizer (``_dq4ml_host.csv_strings``: raw -- quoted or escaped --
    fields through ``split_record``, the rest straight from the bytes), so a chain that never
    reads the column (the lab's DQ -> assemble -> fit) never builds them, and row selections
    (``index`` / ``slice``) move only the spans."""

    def __init__(self, spans: torch.Tensor, valid: Optional[torch.Tensor], data, opts: Optional[dict],
                 meta=None, check=None, dbuf: Optional[torch.Tensor] = None):  # noqa: D107
        self.dtype = StringType()
        self.check = check  # () -> None, raises when a mapped input file changed since the scan
        self.dbuf = dbuf  # the same bytes resident in HBM (the file cache's copy), when there is one
        self.spans = spans
        self.valid = valid
        self.data = data  # the scanned bytes (bytes / memoryview / numpy view of the cached file)
        self.opts = dict(opts or {})
        self.meta = meta or {}
        self.checks = []
        self._vals = None

    @property
    def values(self):
        if self._vals is None:
            from ..ops import native

            if self.check is not None:
                self.check()
            o = self.opts
            sp = self.spans.detach().cpu().numpy()
            ok = (self.valid.detach().to("cpu", torch.uint8).numpy() if self.valid is not None
                  else np.ones(sp.shape[0], dtype=np.uint8))
            data = self.data if not isinstance(self.data, (bytes, bytearray)) else memoryview(self.data)
            self._vals = native.host().csv_strings(data, sp, ok, quote=o.get("quote", '"'),
                                                   escape=o.get("escape", "\\"),
                                                   ignore_leading_ws=bool(o.get("trim_lead")),
                                                   ignore_trailing_ws=bool(o.get("trim_trail")))
        return self._vals

    @values.setter
    def values(self, v):
        self._vals = v

    @property
    def materialized(self) -> bool:
        return self._vals is not None

    @property
    def n(self) -> int:
        return int(self.spans.numel())

    def valid_mask(self, device=None) -> torch.Tensor:
        if self.valid is not None:
            return self.valid
        return torch.ones(self.n, dtype=torch.bool, device=device if device is not None else self.spans.device)

    def index(self, idx: torch.Tensor) -> "ColumnData":
        if self._vals is not None:
            return ColumnData.index(self, idx)
        i = idx.to(self.spans.device)
        valid = None if self.valid is None else self.valid.index_select(0, i)
        return DeviceStringColumn(self.spans.index_select(0, i), valid, self.data, self.opts, dict(self.meta),
                                  self.check, self.dbuf)

    def slice(self, start: int, stop: int) -> "ColumnData":
        if self._vals is not None:
            return ColumnData.slice(self, start, stop)
        valid = None if self.valid is None else self.valid[start:stop]
        return DeviceStringColumn(self.spans[start:stop], valid, self.data, self.opts, dict(self.meta), self.check,
                                  self.dbuf)

    def eq_literal(self, lit: str) -> Optional[torch.Tensor]:
        """``column = lit`` on the device (bool [n]; validity is the column's), without building
        the strings: the spans' bytes in HBM are compared with the literal's UTF-8 bytes, and a raw
        (quoted / escaped) field's unescaped text as the kernel produces it (``csv_span_eq``: the
        host tokenizer's rules).  None when the column has no HBM-resident bytes or a whitespace
        trim applies (then the strings are compared on the host)."""
        if self._vals is not None or self.dbuf is None or self.opts.get("trim_lead") or self.opts.get("trim_trail"):
            return None
        from ..ops import native

        dev = self.spans.device
        b = lit.encode("utf-8")
        lt = torch.tensor(list(b) or [0], dtype=torch.uint8).to(dev, non_blocking=True)
        out = torch.empty(self.n, dtype=torch.uint8, device=dev)
        # (the host tokenizer's option bytes: an empty quote disables quoting, the escape defaults
        # to a backslash -- _dq4ml_host.csv_strings)
        q, e = self.opts.get("quote", '"'), self.opts.get("escape", "\\")
        qb, eb = (ord(q[0]) if q else 0), (ord(e[0]) if e else 92)
        if qb > 127 or eb > 127:
            return None  # a quote / escape outside ASCII (several UTF-8 bytes): the host compares
        native.hip().csv_span_eq(self.dbuf.data_ptr(), self.dbuf.numel(), self.spans.data_ptr(), self.n,
                                 lt.data_ptr(), len(b), qb, eb, out.data_ptr(),
                                 torch.cuda.current_stream(dev).cuda_stream)
        return out == 1


class Table:
    def __init__(self, schema: StructType, columns: List[ColumnData], nrows: int,
                 sel: Optional[torch.Tensor] = None, device=None):
        assert len(schema.fields) == len(columns), "schema/column count mismatch"
        self.schema = schema
        self.columns = columns
        self.nrows = int(nrows)
        self.sel = sel
        self.device = torch.device(device) if device is not None else torch.device("cpu")

    # -- structure -------------------------------------------------------------------------
    def column(self, name: str) -> ColumnData:
        idx = self.index_of(name)
        return self.columns[idx]

    def index_of(self, name: str) -> int:
        names = self.schema.names
        if name in names:
            return names.index(name)
        low = [n.lower() for n in names]
        if name.lower() in low:
            return low.index(name.lower())
        raise KeyError(name)

    def has_column(self, name: str) -> bool:
        try:
            self.index_of(name)
            return True
        except KeyError:
            return False

    # -- selection -------------------------------------------------------------------------
    def sel_mask(self) -> torch.Tensor:
        if self.sel is None:
            return torch.ones(self.nrows, dtype=torch.bool, device=self.device)
        return self.sel

    def count(self) -> int:
        """Live rows.  The chain that produced the table ran over every column, so a pending data
        error of ANY column (a raising rule, ``runtime/checks.py``) fails the count too — read
        after the count's own device read, so no extra sync."""
        n = self.nrows if self.sel is None else int(self.sel.sum().item())
        pending = [ck for c in self.columns for ck in getattr(c, "checks", ())]
        if pending:
            from ..runtime.checks import verify

            verify(pending)
        return n

    def compact(self) -> "Table":
        """Materialize the selection vector (stream compaction)."""
        if self.sel is None:
            return self
        from ..ops import kernels

        idx = kernels.selected_indices(self.sel)
        cols = [c.index(idx) for c in self.columns]
        return Table(self.schema, cols, int(idx.numel()), None, self.device)

    def head_rows(self, k: int) -> "Table":
        """First ``k`` live rows (``take``), compacting only what is needed."""
        if self.sel is None:
            k = min(k, self.nrows)
            return Table(self.schema, [c.slice(0, k) for c in self.columns], k, None, self.device)
        from ..ops import kernels

        idx = kernels.selected_indices(self.sel, limit=k)
        return Table(self.schema, [c.index(idx) for c in self.columns], int(idx.numel()), None, self.device)

    def to_rows(self) -> list:
        t = self.compact()
        cols = [c.to_pylist() for c in t.columns]
        return list(zip(*cols)) if cols else [() for _ in range(t.nrows)]

    def with_columns(self, schema: StructType, columns: List[ColumnData]) -> "Table":
        return Table(schema, columns, self.nrows, self.sel, self.device)


def empty_column(dtype: DataType, n: int, device) -> ColumnData:
    if isinstance(dtype, StringType):
        return ColumnData(dtype, [None] * n, torch.zeros(n, dtype=torch.bool, device=device))
    td = dtype.torch_dtype or torch.float64
    return ColumnData(dtype, torch.zeros(n, dtype=td, device=device), torch.zeros(n, dtype=torch.bool, device=device))


def field_for(name: str, data: ColumnData, nullable: bool = True) -> StructField:
    return StructField(name, data.dtype, nullable, dict(data.meta))


_ = (DoubleType, NullType)
