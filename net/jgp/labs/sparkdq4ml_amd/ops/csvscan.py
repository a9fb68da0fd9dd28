"""Device CSV scan driver (K1/K2, csrc/hip/csv_scan.hip).

``scan_device(data, ...)`` returns a :class:`Table` of typed device columns, or ``None`` when the
input needs the general host scanner (quotes/escapes, string or boolean-mixed columns, integers
beyond int64, decimals outside the exactly-rounded fast path, non-inferred schemas).  The type
lattice masks are merged across data-parallel ranks with an all-reduce (X3) when the file is
sharded by byte range (:func:`shard_byte_range`)."""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch

from ..parallel import comm
from . import native

__all__ = ["scan_device", "merge_type_mask", "shard_byte_range"]

CT_NULL, CT_INT, CT_LONG, CT_DECIMAL, CT_DOUBLE, CT_BOOL, CT_STRING = range(7)
STATS = {"device_scans": 0, "fallbacks": 0}


def merge_type_mask(mask: int) -> int:
    """Tightest common type of the classes present in ``mask`` (bit i = class i seen)."""
    m = int(mask) & ~1  # nulls merge into anything
    if m == 0:
        return CT_STRING  # all-null column -> string (Spark: NullType -> StringType)
    if m & (1 << CT_STRING):
        return CT_STRING
    if m & (1 << CT_BOOL):
        return CT_BOOL if m == (1 << CT_BOOL) else CT_STRING
    return max(i for i in range(1, 5) if m & (1 << i))


def shard_byte_range(data: bytes, rank: int, world: int) -> Tuple[int, int]:
    """Byte range [lo, hi) of ``rank``'s shard, moved forward to row boundaries (a row belongs to
    the shard containing its first byte), like Hadoop's split-straddling LineRecordReader."""
    n = len(data)

    def align(p):
        if p <= 0:
            return 0
        if p >= n:
            return n
        # advance past the terminator that ends the row containing byte p-1
        while p < n and data[p - 1] not in (10, 13):
            p += 1
        if p < n and data[p - 1] == 13 and data[p] == 10:
            p += 1
        return p

    return align(n * rank // world), align(n * (rank + 1) // world)


def scan_device(data: bytes, sep: str = ",", infer: bool = True, device=None, ncols: Optional[int] = None,
                sharded: bool = False):
    from ..sql.localdata import ColumnData
    from ..sql.table import Table
    from ..sql.types import (BooleanType, DoubleType, IntegerType, LongType, StructField, StructType)

    if not infer or len(sep) != 1 or data.find(b'"') >= 0 or data.find(b"\\") >= 0:
        return None
    h = native.hip()
    dev = torch.device(device)
    if ncols is None:
        first = data.split(b"\n", 1)[0].split(b"\r", 1)[0]
        ncols = first.count(sep.encode()) + 1
    if ncols > 256:
        return None
    n = len(data)
    stream = torch.cuda.current_stream(dev).cuda_stream
    host = torch.frombuffer(bytearray(data), dtype=torch.uint8) if n else torch.zeros(0, dtype=torch.uint8)
    buf = host.pin_memory().to(dev, non_blocking=True) if n else torch.zeros(1, dtype=torch.uint8, device=dev)
    nb = int(h.csv_count_blocks(n))
    counts = torch.empty(nb + 1, dtype=torch.int64, device=dev)
    h.csv_line_ends(buf.data_ptr(), n, counts.data_ptr(), 0, stream)
    nterm = int(counts[nb].item())
    trailing = n > 0 and data[-1] not in (10, 13)
    nlines = nterm + (1 if trailing else 0)
    ends = torch.empty(max(nlines, 1), dtype=torch.int64, device=dev)
    if nterm:
        h.csv_line_ends(buf.data_ptr(), n, counts.data_ptr(), ends.data_ptr(), stream)
    if trailing:
        ends[nterm] = n
    dvals = torch.empty(ncols, max(nlines, 1), dtype=torch.float64, device=dev)
    ivals = torch.empty(ncols, max(nlines, 1), dtype=torch.int64, device=dev)
    valid = torch.empty(ncols, max(nlines, 1), dtype=torch.bool, device=dev)
    keep = torch.empty(max(nlines, 1), dtype=torch.bool, device=dev)
    masks = torch.zeros(ncols, dtype=torch.int32, device=dev)
    flags = torch.zeros(1, dtype=torch.int32, device=dev)
    h.csv_parse(buf.data_ptr(), n, ends.data_ptr(), nlines, ncols, ord(sep), dvals.data_ptr(), ivals.data_ptr(),
                valid.data_ptr(), keep.data_ptr(), masks.data_ptr(), flags.data_ptr(), stream)
    if sharded:
        masks = _or_reduce(masks)
        flags = comm.all_reduce_max(flags)
    fl = int(flags.item())
    mk = masks.cpu().numpy().astype(np.int64)
    if fl:
        STATS["fallbacks"] += 1
        return None
    types = [merge_type_mask(m) for m in mk]
    if any(t in (CT_STRING, CT_DECIMAL) for t in types):
        STATS["fallbacks"] += 1
        return None
    STATS["device_scans"] += 1
    fields, cols = [], []
    for c, t in enumerate(types):
        v = valid[c, :nlines]
        vv = None if bool(v.all()) else v.clone()
        if t == CT_INT:
            vals, dt = ivals[c, :nlines].to(torch.int32), IntegerType()
        elif t == CT_LONG:
            vals, dt = ivals[c, :nlines].clone(), LongType()
        elif t == CT_BOOL:
            vals, dt = ivals[c, :nlines] != 0, BooleanType()
        else:
            vals, dt = dvals[c, :nlines].clone(), DoubleType()
        fields.append(StructField(f"_c{c}", dt, True))
        cols.append(ColumnData(dt, vals, vv))
    table = Table(StructType(fields), cols, nlines, None, dev)
    k = keep[:nlines]
    if nlines and not bool(k.all()):  # empty lines are skipped
        table = Table(table.schema, table.columns, nlines, k.clone(), dev).compact()
    return table


def _or_reduce(masks: torch.Tensor) -> torch.Tensor:
    """Bitwise-OR all-reduce of the per-column class masks via MAX over bit planes."""
    if comm.world_size() == 1:
        return masks
    bits = torch.stack([(masks >> i) & 1 for i in range(7)]).to(torch.int32)
    bits = comm.all_reduce_max(bits)
    out = torch.zeros_like(masks)
    for i in range(7):
        out |= bits[i] << i
    return out
