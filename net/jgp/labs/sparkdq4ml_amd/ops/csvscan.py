"""Device CSV scan driver (K1/K2, csrc/hip/csv_scan.hip).

``scan_device(data, ...)`` returns a :class:`Table` of typed device columns, or ``None`` when the
input needs the general host scanner (integers beyond int64, decimals outside the exactly-rounded
fast path, a quoted field whose class only the host tokenizer can tell in a non-string column).
String columns stay on the device as field spans into the input bytes (``csv_scan.h`` kind 4):
:class:`~..sql.table.DeviceStringColumn` builds their Python strings (host C++ ``csv_strings``)
only when a consumer reads them.  The type
lattice masks are merged across data-parallel ranks with an all-reduce (X3) when the file is
sharded by byte range (:func:`shard_byte_range`)."""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch

from ..parallel import comm
from . import native

__all__ = ["scan_device", "merge_type_mask", "shard_byte_range"]

CT_NULL, CT_INT, CT_LONG, CT_DECIMAL, CT_DOUBLE, CT_BOOL, CT_STRING, CT_TIMESTAMP = range(8)
STATS = {"device_scans": 0, "fallbacks": 0, "chunks": 0}


def merge_type_mask(mask: int) -> int:
    """Tightest common type of the classes present in ``mask`` (bit i = class i seen)."""
    m = int(mask) & 0xFE  # nulls merge into anything (bit 8 is the needs-the-host flag)
    if m == 0:
        return CT_STRING  # all-null column -> string (Spark: NullType -> StringType)
    if m & (1 << CT_STRING):
        return CT_STRING
    if m & (1 << CT_BOOL):
        return CT_BOOL if m == (1 << CT_BOOL) else CT_STRING
    if m & (1 << CT_TIMESTAMP):  # a timestamp merges with timestamps only
        return CT_TIMESTAMP if m == (1 << CT_TIMESTAMP) else CT_STRING
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


def _count_fields(line: bytes, sep: int, quote: int, escape: int) -> int:
    """Fields of one record under the univocity tokenizer's quoting (``csrc/host/csv.cpp``
    ``split_record``): a separator inside a quoted field is content."""
    if quote not in line:
        return line.count(sep) + 1
    n, i, fields = len(line), 0, 1
    in_q = quoted = False
    empty = True  # nothing collected in the current field yet
    while i < n:
        c = line[i]
        if in_q:
            if c == escape and escape != quote and i + 1 < n and line[i + 1] in (quote, escape):
                i += 1
            elif c == quote:
                if i + 1 < n and line[i + 1] == quote:
                    i += 1
                else:
                    in_q = False
            empty = False
        elif c == sep:
            fields += 1
            quoted, empty = False, True
        elif c == quote and empty and not quoted:
            in_q = quoted = True
        else:
            if c == escape and escape != quote and i + 1 < n and line[i + 1] == quote:
                i += 1
            empty = False
        i += 1
    return fields


def split_record(line: bytes, sep: int, quote: int, escape: int, null_value: bytes = b"",
                 trim_lead: bool = False, trim_trail: bool = False):
    """[(text bytes, is_null)] of one record, the univocity way (``csrc/host/csv.cpp``
    ``split_record``, which the device parser mirrors): quotes, doubled quotes, the escape before a
    quote, a separator inside quotes kept as content; a quoted field is never null; trims after."""
    out, cur = [], bytearray()
    in_q = quoted = False
    i, n = 0, len(line)
    while i < n:
        c = line[i]
        if in_q:
            if c == escape and escape != quote and i + 1 < n and line[i + 1] in (quote, escape):
                i += 1
                cur.append(line[i])
            elif c == quote:
                if i + 1 < n and line[i + 1] == quote:
                    cur.append(quote)
                    i += 1
                else:
                    in_q = False
            else:
                cur.append(c)
        elif c == sep:
            out.append((bytes(cur), not quoted and bytes(cur) == null_value))
            cur, quoted = bytearray(), False
        elif c == quote and not cur and not quoted:
            in_q = quoted = True
        elif c == escape and escape != quote and i + 1 < n and line[i + 1] == quote:
            i += 1
            cur.append(line[i])
        else:
            cur.append(c)
        i += 1
    out.append((bytes(cur), not quoted and bytes(cur) == null_value))
    res = []
    for t, null in out:
        if not null:
            if trim_lead:
                t = t.lstrip(b" \t")
            if trim_trail:
                t = t.rstrip(b" \t")
        res.append((t, null))
    return res


def _ncols_of(data, sep: str, comment: int = 0, quote: int = 34, escape: int = 92) -> int:
    """Column count from the first line that is neither empty nor a comment line -- Spark drops
    those before it tokenizes the first record (a bounded, growing head search: the input may be
    a multi-GB map with no ``\n`` at all -- the reference data is CR-only)."""
    n, w = len(data), 1 << 16
    while True:
        head = bytes(data[:min(n, w)])
        pos = 0
        while True:
            ends = [x for x in (head.find(b"\n", pos), head.find(b"\r", pos)) if x >= 0]
            if not ends and w < n:
                break  # the line may go on past the head: read more
            e = min(ends) if ends else len(head)
            if e > pos and not (comment and head[pos] == comment):
                return _count_fields(head[pos:e], ord(sep), quote, escape)
            if not ends:  # the whole input holds no such line
                return 1
            pos = e + 1
        w *= 16


_KIND = {CT_INT: (1, torch.int32), CT_LONG: (2, torch.int64), CT_BOOL: (3, torch.bool), CT_STRING: (4, torch.int64),
         CT_TIMESTAMP: (5, torch.int64)}
SLOW_BIT = 0x100  # class-mask bit: a field whose value or class the device could not settle
_SPANNED = (CT_STRING, CT_TIMESTAMP)  # types scanned under a hint only (spans / exact int64 microseconds)


def _opt_args(opts):
    o = opts or {}
    return dict(quote=ord(o.get("quote", '"')), escape=ord(o.get("escape", "\\")), comment=o.get("comment", 0),
                trim_lead=bool(o.get("trim_lead", False)), trim_trail=bool(o.get("trim_trail", False)),
                null_value=o.get("null_value", ""), strict=bool(o.get("strict", False)))


MIN_RESIDENT_CHUNK = 1 << 30  # chunk floor of a scan over HBM-resident bytes (bounds per-chunk outputs only)


class _Planes:
    """Shared column storage of a multi-chunk eager scan: every chunk's parse writes its rows at a
    running offset of ONE allocation per column, so the table's columns are views of these planes
    -- no per-chunk allocations and no concatenation (which read and wrote every parsed byte once
    more and held two copies at the peak: 2 x 65 GB for the 77 GB config-4 CSV).  Sized at the
    first chunk from its line density over the whole input (+3 %); a chunk that does not fit
    gets its own planes and the table falls back to concatenating."""

    def __init__(self, kinds, total_bytes: int, dev):
        self.kinds, self.total, self.dev = kinds, total_bytes, dev
        self.cols = None
        self.off = 0
        self.whole = True  # every chunk so far landed in the planes

    def take(self, nlines: int, chunk_bytes: int):
        """Views for the next ``nlines`` rows, or None (the chunk allocates its own)."""
        if self.cols is None:
            cap = int(nlines * (self.total / max(1, chunk_bytes)) * 1.03) + 4096
            self.cols = [torch.empty(cap, dtype=dt, device=self.dev) for _, dt in self.kinds]
        if not self.whole or self.off + max(nlines, 1) > self.cols[0].numel():
            self.whole = False
            return None
        o = self.off
        self.off += nlines
        return [c[o:o + max(nlines, 1)] for c in self.cols]


class _Shared(list):
    """The chunks' parse outputs (a list, as everywhere) whose column planes are consecutive rows
    of ``planes`` (:class:`_Planes`): ``_finish`` takes each column as one view."""

    def __init__(self, parts, planes):
        super().__init__(parts)
        self.planes = planes


def _scan_chunk(h, buf, n: int, trailing: bool, ncols: int, sep: str, dev, hint=None, opts=None, base: int = 0,
                planes: "Optional[_Planes]" = None):
    """K1 (line ends) + K2 (parse, type masks, null / empty-line counts) over one device byte
    buffer; no host sync except the line count.  Returns (nlines, per-column planes, valid
    [ncols, m], keep [m], stats, base) — stats as documented at ``csv_parse`` (csv_scan.h); ``base``:
    the chunk's offset in the scanned bytes (string spans are relative to the chunk)."""
    from .device import _h2d

    stream = torch.cuda.current_stream(dev).cuda_stream
    nb = int(h.csv_count_blocks(n))
    counts = torch.empty(nb + 1, dtype=torch.int64, device=dev)
    h.csv_line_ends(buf.data_ptr(), n, counts.data_ptr(), 0, stream, -1, 0)
    nterm = int(counts[nb].item())
    nlines = nterm + (1 if trailing else 0)
    # int32 line-end offsets below 2 GiB (half the bytes of the ends pass and of the parse's reads)
    ends = torch.empty(max(nlines, 1), dtype=torch.int32 if h.csv_ends_i32(n) else torch.int64, device=dev)
    # the ends pass also counts, per block, the separators and the terminator kinds (the cutter's
    # scan facts): no whole-chunk torch passes over the bytes / ends afterwards
    facts = torch.empty(nb, 4, dtype=torch.int32, device=dev)
    h.csv_line_ends(buf.data_ptr(), n, counts.data_ptr(), ends.data_ptr(), stream, ord(sep), facts.data_ptr())
    if trailing:
        ends[nterm:].fill_(n)  # a fill kernel: ``ends[nterm] = n`` is a blocking pageable copy
    m = max(nlines, 1)
    # one exact-size allocation per column: a column IS its plane (no copy, and no other
    # column's storage kept alive by it) — f64, or the hinted type (see scan_device)
    kinds = [_KIND.get(t, (0, torch.float64)) for t in (hint or [CT_DOUBLE] * ncols)]
    dcols = planes.take(nlines, n) if planes is not None else None
    if dcols is None:
        dcols = [torch.empty(m, dtype=dt, device=dev) for _, dt in kinds]
    ptrs = _h2d(np.array([t.data_ptr() for t in dcols] + [k for k, _ in kinds], dtype=np.int64), dev)
    valid = torch.empty(ncols, m, dtype=torch.bool, device=dev)
    keep = torch.empty(m, dtype=torch.bool, device=dev)
    # [parse stats (4 + 2 ncols), longest line, separators, shortest line, CR ends, LF ends, CR LF
    # ends]: the facts the byte-parallel cutter (ops/scancut.py) relies on -- the separator count
    # is nlines * (ncols - 1) when every line has exactly ncols fields; line lengths run terminator
    # to terminator; a CR LF pair ends at its CR.  The parse kernel writes the line lengths.
    # (initialised on the device with the ends pass's facts folded in: csv_stats_init)
    stats = torch.empty(10 + 2 * ncols, dtype=torch.int64, device=dev)
    h.csv_stats_init(facts.data_ptr(), nb, stats.data_ptr(), ncols, stream)
    h.csv_parse(buf.data_ptr(), n, ends.data_ptr(), nlines, ncols, ord(sep), ptrs.data_ptr(), valid.data_ptr(),
                keep.data_ptr(), stats.data_ptr(), stream, **_opt_args(opts))
    return nlines, dcols, valid, keep, stats, base


def type_code_of(dt) -> int:
    """Lattice code of a device-scanned column's type (the reader's types_hint)."""
    from ..sql.types import BooleanType, IntegerType, LongType, StringType, TimestampType

    if isinstance(dt, StringType):
        return CT_STRING
    if isinstance(dt, TimestampType):
        return CT_TIMESTAMP
    if isinstance(dt, IntegerType):
        return CT_INT
    if isinstance(dt, LongType):
        return CT_LONG
    if isinstance(dt, BooleanType):
        return CT_BOOL
    return CT_DOUBLE


def _finish(parts, types, st, dev, hinted=False, data=None, opts=None, check=None, dbuf=None):
    """Typed columns from per-chunk parse outputs under the merged types.  ``st``: the chunks'
    stats on the host.  Int / long / boolean values convert exactly from their f64 planes (the
    parser flags integers beyond 2^53 for the host path).  String columns (scanned as spans, always
    hinted) become :class:`DeviceStringColumn` over ``data``, the scanned bytes."""
    from ..sql.localdata import ColumnData
    from ..sql.table import DeviceStringColumn, Table
    from ..sql.types import (BooleanType, DoubleType, IntegerType, LongType, StringType, StructField, StructType,
                             TimestampType)

    fields, cols = [], []
    total = sum(p[0] for p in parts)
    live = [(k, p) for k, p in enumerate(parts) if p[0]]
    for c, t in enumerate(types):
        if t == CT_STRING:
            # spans relative to each chunk -> offsets into ``data`` (fs is bits 25..63)
            sp = [p[1][c][:p[0]] + (p[5] << 25) if p[5] else p[1][c][:p[0]] for _, p in live]
            spans = torch.cat(sp) if len(sp) > 1 else (sp[0] if sp else torch.empty(0, dtype=torch.int64, device=dev))
            vv = None
            if int(st[:, 2 + c].sum()):
                valid_l = [p[2][c, :p[0]] for _, p in live]
                vv = torch.cat(valid_l) if len(valid_l) > 1 else valid_l[0].clone()
            fields.append(StructField(f"_c{c}", StringType(), True))
            cols.append(DeviceStringColumn(spans, vv, data, opts, check=check, dbuf=dbuf))
            continue
        def typed(d):
            if hinted:  # stored as the column's type already
                return d
            if t == CT_INT:
                return d.to(torch.int32)
            if t in (CT_LONG, CT_TIMESTAMP):
                return d.to(torch.int64)
            if t == CT_BOOL:
                return d != 0
            return d
        dt = {CT_INT: IntegerType(), CT_LONG: LongType(), CT_BOOL: BooleanType(),
              CT_TIMESTAMP: TimestampType()}.get(t, DoubleType())
        if isinstance(parts, _Shared) and total:  # the chunks wrote consecutive rows of one plane
            vals = typed(parts.planes.cols[c][:total])
        else:
            vals_l = [typed(dcols[c][:nlines]) for _, (nlines, dcols, _, _, _, _) in live]
            if vals_l:
                vals = torch.cat(vals_l) if len(vals_l) > 1 else vals_l[0]
            else:
                vals = torch.empty(0, dtype=dt.torch_dtype, device=dev)
        vv = None
        if int(st[:, 2 + c].sum()):  # null fields in this column: materialize its validity
            valid_l = [p[2][c, :p[0]] for _, p in live]
            vv = torch.cat(valid_l) if len(valid_l) > 1 else valid_l[0].clone()
        fields.append(StructField(f"_c{c}", dt, True))
        cols.append(ColumnData(dt, vals, vv))
    table = Table(StructType(fields), cols, total, None, dev)
    if total and int(st[:, 1].sum()):  # empty lines are skipped
        keeps = [p[3][:p[0]] for _, p in live]
        k = torch.cat(keeps) if len(keeps) > 1 else keeps[0]
        table = Table(table.schema, table.columns, total, k.clone(), dev).compact()
    table.scan_facts = _facts(st, len(types), int(total))
    return table


def _facts(st: np.ndarray, nc: int, total: int) -> dict:
    """What a later fused scan of the same bytes relies on (ops/scanfuse.py, ops/scancut.py),
    from the chunks' parse stats: line count (empty lines included), the columns holding nulls,
    the fast-path / field-count / line-length / terminator facts."""
    nonempty = int(total) - int(st[:, 1].sum())
    misses, hard = int(st[:, 2 + 2 * nc].sum()), int(st[:, 3 + 2 * nc].sum())
    return {"nlines": int(total), "nullable": [bool(int(st[:, 2 + c].sum())) for c in range(nc)],
            "fast_only": misses == 0,
            # every field off the fast path was a quoted fast-path number: the cutter's QUOTED build
            "quoted_fast": misses > 0 and hard == 0,
            "empty_lines": int(st[:, 1].sum()), "max_line": int(st[:, 4 + 2 * nc].max()),
            "uniform_fields": int(st[:, 5 + 2 * nc].sum()) == nonempty * (nc - 1),
            "min_line": max(1, int(st[:, 6 + 2 * nc].min())) if len(st) else 1,
            "term_kinds": [int(st[:, 7 + 2 * nc + k].sum()) for k in range(3)]}


def infer_streamed(src, sep: str, ncols: Optional[int] = None, sharded: bool = False, opts: Optional[dict] = None,
                   user_types: Optional[list] = None):
    """Schema inference over an input that is not resident in HBM (``runtime.streams.ChunkSource``):
    Spark's inference pass at ``load()`` (``DataQuality4MachineLearningApp.java:53-55``) as one
    streamed device parse whose column planes are dropped chunk by chunk -- only the type masks and
    the facts survive, so memory stays at one chunk.  Returns (type codes, facts) or None (the
    input needs the host scanner)."""
    if len(sep) != 1 or ord(sep) >= 128:  # (the device tokenizer matches one ASCII byte)
        return None
    if user_types:
        if any(t not in STRICT_CODES for t in user_types):
            return None
        opts = dict(opts or {}, strict=True)
        ncols = len(user_types)
    h = native.hip()
    if ncols is None:
        head = bytes(memoryview(src.data)[:min(src.n, 1 << 20)])
        oa = _opt_args(opts)
        ncols = _ncols_of(head, sep, int(oa["comment"] or 0), oa["quote"], oa["escape"])
    if ncols > 256 or not len(src):
        return None
    hint = list(user_types) if user_types else None
    sts, total = [], 0
    for buf, n, trailing in src.chunks():
        nlines, _cols, _valid, _keep, stats, _ = _scan_chunk(h, buf, n, trailing, ncols, sep, src.device, hint, opts)
        total += nlines
        sts.append(stats)
    st = torch.stack(sts).cpu().numpy()
    masks = np.bitwise_or.reduce(st[:, 2 + ncols:2 + 2 * ncols], axis=0)
    if user_types:
        if _strict_flag(masks, int(st[:, 0].max()), user_types, sharded):
            return None
        types = list(user_types)
    else:
        types = _resolve_types(masks, int(st[:, 0].max()), sharded)
        if types is None or any(t in _SPANNED for t in types):  # (the streamed fused Gram: numeric columns)
            return None
    STATS["streamed_inferences"] = STATS.get("streamed_inferences", 0) + 1
    return types, _facts(st, ncols, total)


def _resolve_types(masks: np.ndarray, flag: int, sharded: bool):
    """Merged column types, or None when the host scanner must decide: the slow flag, a decimal,
    or a column holding a field the device could not settle (SLOW_BIT) that its other fields do
    not make a string anyway (a string is the lattice top: no field can change it)."""
    if sharded:
        flag = int(comm.all_reduce_max(torch.tensor([flag], dtype=torch.int64))[0])
        masks = _or_reduce(torch.from_numpy(masks)).numpy()
    if flag:
        return None
    types = [merge_type_mask(int(m)) for m in masks]
    for t, m in zip(types, masks):
        if t == CT_DECIMAL or (int(m) & SLOW_BIT and (t != CT_STRING or not int(m) & 0xFE)):
            return None
    return types


def _strict_flag(masks: np.ndarray, flag: int, user_types, sharded: bool) -> bool:
    """A user-schema scan needs the host: the slow flag, or an unsettled field in a non-string column."""
    bad = int(flag) or any(int(m) & SLOW_BIT and t != CT_STRING for t, m in zip(user_types, masks))
    if sharded:
        bad = int(comm.all_reduce_max(torch.tensor([int(bad)], dtype=torch.int64))[0])
    return bool(bad)


# user-schema type codes the device parser converts (int, long, double, boolean; string: spans)
STRICT_CODES = (CT_INT, CT_LONG, CT_DOUBLE, CT_BOOL, CT_STRING, CT_TIMESTAMP)


def scan_device(data, sep: str = ",", infer: bool = True, device=None, ncols: Optional[int] = None,
                sharded: bool = False, chunk_bytes: Optional[int] = None, pinned: Optional[torch.Tensor] = None,
                device_data: Optional[torch.Tensor] = None, types_hint: Optional[list] = None,
                opts: Optional[dict] = None, user_types: Optional[list] = None, _depth: int = 0,
                source_check=None, device_ready=None):
    """Parse ``data`` on the device.  Inputs larger than ``chunk_bytes`` stream through a
    double-buffered pinned staging ring: chunk k+1's host->device copy runs on a side stream while
    chunk k is parsed, chunks split on row boundaries, type masks OR-merged over
    chunks (and ranks when ``sharded``).

    ``types_hint``: column type codes from an earlier scan of the same bytes (the reader keeps
    them with its cached file): the parser then stores every column as its type directly — no
    f64 plane to convert.  Inference still runs; a hint the masks contradict re-scans unhinted.
    String columns are scanned as spans, which needs the hint: a scan that finds a string column
    without one re-scans once with the inferred types as the hint.  ``source_check``: called before
    their text is built from ``data`` when ``data`` is a map of a file the process does not own
    (raises when the file changed since the scan).

    ``opts``: dialect (quote, escape, comment, trim_lead, trim_trail, null_value; see
    ``csv_parse_dev.h``).  ``user_types``: a user schema (lattice codes in STRICT_CODES): the
    columns are stored as those types, a field that does not convert nulls its record (Spark's
    PERMISSIVE), no inference.

    ``device_ready``: [(end offset, piece)] of a ``device_data`` upload still in flight: each
    chunk waits only for the pieces it covers (runtime.filecache progressive upload)."""
    if len(sep) != 1 or ord(sep) >= 128 or not (infer or user_types):  # (one ASCII separator byte)
        return None
    if user_types:
        if any(t not in STRICT_CODES for t in user_types):
            return None
        opts = dict(opts or {}, strict=True)
        ncols = len(user_types)
        types_hint = list(user_types)
    h = native.hip()
    dev = torch.device(device)
    if ncols is None:
        oa = _opt_args(opts)
        ncols = _ncols_of(data, sep, int(oa["comment"] or 0), oa["quote"], oa["escape"])
    if ncols > 256:
        return None
    hint = list(types_hint) if types_hint is not None and len(types_hint) == ncols else None
    n = len(data)
    if device_data is not None and n > 0:
        # input bytes already resident in HBM (runtime.filecache): chunks are plain slices —
        # no staging, no H2D; chunking only bounds the per-chunk parse outputs
        if device_data.numel() != n:
            raise ValueError("scan_device: device_data does not match data")
        cb = max(int(chunk_bytes or n), MIN_RESIDENT_CHUNK)
        bounds = chunk_bounds(data, cb) if n > cb else [0, n]
        parts = []
        pending = list(device_ready or [])
        cur = torch.cuda.current_stream(dev)
        # (a piece's ``wait(stream)``: a torch event, or a runtime.filecache._Piece whose uploader
        # thread may not have enqueued the DMA yet -- then the host blocks until it has)
        kinds = [_KIND.get(t, (0, torch.float64)) for t in (hint or [CT_DOUBLE] * ncols)]
        # (string spans are chunk-relative: their columns keep the per-chunk form)
        planes = _Planes(kinds, n, dev) if len(bounds) > 2 and all(k != 4 for k, _ in kinds) else None
        for s, e in zip(bounds, bounds[1:]):
            while pending and pending[0][0] < e:  # pieces wholly before this chunk's end
                pending.pop(0)[1].wait(cur)
            if pending:  # the piece holding the chunk's last bytes
                pending[0][1].wait(cur)
            trailing = data[e - 1] not in (10, 13)
            parts.append(_scan_chunk(h, device_data[s:e], e - s, trailing, ncols, sep, dev, hint, opts, s, planes))
        if planes is not None and planes.whole:
            parts = _Shared(parts, planes)
        for _, ev in pending:
            ev.wait(cur)
    elif chunk_bytes is None or n <= chunk_bytes:
        if pinned is not None and n:
            buf = pinned.to(dev, non_blocking=True)  # page-locked mapping: direct DMA
        else:
            host = torch.frombuffer(bytearray(data), dtype=torch.uint8) if n else torch.zeros(0, dtype=torch.uint8)
            buf = host.pin_memory().to(dev, non_blocking=True) if n else torch.zeros(1, dtype=torch.uint8, device=dev)
        trailing = n > 0 and data[-1] not in (10, 13)
        parts = [_scan_chunk(h, buf, n, trailing, ncols, sep, dev, hint, opts)]
    else:
        parts = _scan_chunked(h, data, ncols, sep, dev, int(chunk_bytes), pinned, hint, opts)
    st = torch.stack([p[4] for p in parts]).cpu().numpy()  # the one host read of the parse results
    masks = np.bitwise_or.reduce(st[:, 2 + ncols:2 + 2 * ncols], axis=0)
    if user_types:
        if _strict_flag(masks, int(st[:, 0].max()), user_types, sharded):
            STATS["fallbacks"] += 1
            return None
        STATS["device_scans"] += 1
        return _finish(parts, list(user_types), st, dev, hinted=True, data=data, opts=opts, check=source_check,
                       dbuf=device_data)
    types = _resolve_types(masks, int(st[:, 0].max()), sharded)
    if types is None:
        STATS["fallbacks"] += 1
        return None
    kinds = [_KIND.get(t, (0,))[0] for t in types]
    miss = hint is not None and kinds != [_KIND.get(t, (0,))[0] for t in hint]
    spans = any(t in _SPANNED for t in types) and (hint is None or miss)  # they need the hinted scan
    if sharded:  # every rank takes the same (collective) path
        flags = comm.all_reduce_max(torch.tensor([int(miss), int(spans)], dtype=torch.int64))
        miss, spans = bool(int(flags[0])), bool(int(flags[1]))
    if (miss or spans) and _depth < 2:  # (sharded: ``types`` are the merged ones, equal on every rank)
        STATS["hint_misses" if miss and hint is not None else "span_rescans"] = \
            STATS.get("hint_misses" if miss and hint is not None else "span_rescans", 0) + 1
        return scan_device(data, sep, infer, device, ncols, sharded, chunk_bytes, pinned, device_data,
                           types if spans else None, opts, _depth=_depth + 1, source_check=source_check)
    if miss or spans:
        STATS["fallbacks"] += 1
        return None
    STATS["device_scans"] += 1
    STATS["chunks"] = STATS.get("chunks", 0) + len(parts)
    return _finish(parts, types, st, dev, hinted=hint is not None, data=data, opts=opts, check=source_check,
                   dbuf=device_data)


def chunk_bounds(data: bytes, chunk_bytes: int):
    """Row-aligned chunk boundaries: each cut moves forward to just past a line terminator."""
    n = len(data)
    b = [0]
    while b[-1] < n:
        p = min(n, b[-1] + chunk_bytes)
        if p < n:
            q = p
            while q < n and data[q - 1] not in (10, 13):
                q += 1
            if q < n and data[q - 1] == 13 and data[q] == 10:
                q += 1
            p = q
        b.append(p)
    return b


def _scan_chunked(h, data, ncols: int, sep: str, dev, chunk_bytes: int, pinned: Optional[torch.Tensor] = None,
                  hint=None, opts=None):
    from ..runtime.streams import StagingRing

    bounds = chunk_bounds(data, chunk_bytes)
    spans = [(bounds[i], bounds[i + 1]) for i in range(len(bounds) - 1)]
    ring = StagingRing(max(e - s for s, e in spans), depth=2, device=dev, staging=pinned is None)
    mv = memoryview(data)

    def put(i):
        s, e = spans[i]
        ring.put(i, mv[s:e], pinned=None if pinned is None else pinned[s:e])

    put(0)
    parts = []
    for i, (s, e) in enumerate(spans):
        if i + 1 < len(spans):
            put(i + 1)  # overlaps chunk i's parse
        buf = ring.get(i)
        trailing = data[e - 1] not in (10, 13)
        parts.append(_scan_chunk(h, buf, e - s, trailing, ncols, sep, dev, hint, opts, s))
        ring.release(i)
    return parts


def _or_reduce(masks: torch.Tensor) -> torch.Tensor:
    """Bitwise-OR all-reduce of the per-column class masks via MAX over bit planes."""
    if not comm.collectives_active():
        return masks
    bits = torch.stack([(masks >> i) & 1 for i in range(9)]).to(torch.int32)
    bits = comm.all_reduce_max(bits)
    out = torch.zeros_like(masks)
    for i in range(9):
        out |= bits[i] << i
    return out
