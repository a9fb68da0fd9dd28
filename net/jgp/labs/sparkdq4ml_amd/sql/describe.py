"""``DataFrame.describe(*cols)`` — Spark 2.4's basic statistics summary.

Result: a string-typed DataFrame ``summary | <col>...`` with the rows ``count``, ``mean``,
``stddev`` (sample, ``stddev_samp``: NaN for one value), ``min`` and ``max``, every cell
rendered as Spark casts the aggregate to string (``Double.toString`` for doubles, the column's
own type for min/max).  Numeric columns are reduced on the table's device in ONE pass of
masked reductions (no row compaction); string columns take the host path (mean/stddev of the
strings cast to double, min/max lexicographic).  As in Spark's ``StatFunctions.summary`` only
numeric and string columns are summarized: any other column (boolean, vector, ...) is dropped
silently, named or not.  Floating min/max order NaN above every number (Spark's ordering): ``min``
skips NaN unless every value is NaN, ``max`` is NaN as soon as one value is.
"""
from __future__ import annotations

from typing import List

import torch

from ..utils.javafmt import java_str
from .table import ColumnData
from .types import IntegerType, LongType, StringType, StructField, StructType, is_numeric

__all__ = ["describe"]

_STATS = ("count", "mean", "stddev", "min", "max")


def _fmt(v, integral: bool):
    if v is None:
        return None
    if integral:
        return str(int(v))
    return java_str(float(v))


def _numeric(c: ColumnData, live: torch.Tensor, integral: bool) -> List:
    m = live if c.valid is None else (live & c.valid)
    x = c.values.to(torch.float64)
    n = int(m.sum().item())
    if n == 0:
        return ["0", None, None, None, None]
    xs = x[m]
    mean = float(xs.mean().item())
    sd = float(xs.std(unbiased=True).item()) if n > 1 else float("nan")
    nan = torch.isnan(xs)
    if bool(nan.any()):  # NaN is the largest double in Spark's ordering
        mx = float("nan")
        mn = float("nan") if bool(nan.all()) else xs[~nan].min().item()
    else:
        mn, mx = xs.min().item(), xs.max().item()
    if integral:
        raw = c.values[m]
        mn, mx = int(raw.min().item()), int(raw.max().item())
    return [str(n), java_str(mean), java_str(sd), _fmt(mn, integral), _fmt(mx, integral)]


def _strings(vals: list) -> List:
    vs = [v for v in vals if v is not None]
    if not vs:
        return ["0", None, None, None, None]
    nums = []
    for v in vs:
        try:
            nums.append(float(v.strip()))
        except ValueError:
            pass
    mean = sd = None
    if nums:
        mean = sum(nums) / len(nums)
        sd = (sum((a - mean) ** 2 for a in nums) / (len(nums) - 1)) ** 0.5 if len(nums) > 1 else float("nan")
        mean, sd = java_str(mean), java_str(sd)
    return [str(len(vs)), mean, sd, min(vs), max(vs)]


def describe(df, cols: List[str]):
    from ..parallel import comm  # noqa: F401 - sharded describe gathers rows first

    t = df._table()
    fields = [t.schema[t.index_of(c)] for c in cols]
    # StatFunctions.summary: numeric and string columns only, the rest dropped without an error
    fields = [f for f in fields if is_numeric(f.dataType) or isinstance(f.dataType, StringType)]
    cols = [f.name for f in fields]
    stats = []
    from .plan import is_sharded

    if is_sharded(df._plan):  # rows of every rank, in rank order (X5)
        rows = df.select(*cols).collect()
        for i, f in enumerate(fields):
            vals = [r[i] for r in rows]
            if isinstance(f.dataType, StringType):
                stats.append(_strings(vals))
            else:
                dev = torch.device("cpu")
                valid = torch.tensor([v is not None for v in vals], dtype=torch.bool)
                data = torch.tensor([0 if v is None else v for v in vals],
                                    dtype=torch.int64 if _integral(f) else torch.float64)
                stats.append(_numeric(ColumnData(f.dataType, data, valid), torch.ones(len(vals), dtype=torch.bool,
                                                                                      device=dev), _integral(f)))
    else:
        live = t.sel_mask()
        for f in fields:
            c = t.column(f.name)
            if isinstance(f.dataType, StringType):
                keep = live.cpu().tolist()
                stats.append(_strings([v for v, k in zip(c.values, keep) if k]))
            else:
                stats.append(_numeric(c, live, _integral(f)))
    rows = [tuple([s] + [st[i] for st in stats]) for i, s in enumerate(_STATS)]
    schema = StructType([StructField("summary", StringType(), True)] +
                        [StructField(f.name, StringType(), True) for f in fields])
    return df.sparkSession.createDataFrame(rows, schema)


def _integral(f) -> bool:
    return isinstance(f.dataType, (IntegerType, LongType))
