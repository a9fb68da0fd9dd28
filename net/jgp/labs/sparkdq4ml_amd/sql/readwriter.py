"""``DataFrameReader`` / ``DataFrameWriter``.

The lab reads ``data/dataset-abstract.csv`` with ``format("csv").option("inferSchema","true")
.option("header","false")`` (``DataQuality4MachineLearningApp.java:52-55``).  Files are scanned
once at ``load()`` (Spark also runs a schema-inference job there) by

* the device scanner ``csv_scan`` HIP kernel (MI355X sessions, files above
  ``dq4ml.csv.deviceThresholdBytes``, numeric columns), or
* the native host scanner (``_dq4ml_host.csv_scan``) otherwise,

both implementing the contract of SURVEY.md S03.
"""
from __future__ import annotations

import glob
import json
import os
import shutil
import stat
import weakref
from typing import Dict, List, Optional

import numpy as np
import torch

from ..utils import tracing
from ..utils.logging import get_logger
from .localdata import column_from_numpy, column_from_pylist, table_from_data
from .plan import LocalRelation
from .table import ColumnData, Table
from .types import (BooleanType, DecimalType, DoubleType, IntegerType, LongType, StringType,
                    StructField, StructType, TimestampType, parse_type_name)

__all__ = ["DataFrameReader", "DataFrameWriter", "csv_code_to_type"]

# load() of an unchanged cached CSV file: key -> (weak reference to the cache entry, file identity);
# the lazy relation template lives ON the entry (``load_templates``), so an evicted file's template
# (and the HBM bytes its relation points at) goes with it -- nothing here keeps them alive
_LOADS: dict = {}
_LOAD_SERIAL = __import__("itertools").count(1)
_REALPATH: dict = {}
_LOAD_CONF = ("dq4ml.csv.deviceThresholdBytes", "dq4ml.csv.deviceCache", "dq4ml.csv.fuseScan", "dq4ml.chunkBytes",
              "dq4ml.csv.streamThresholdBytes", "dq4ml.shardInput")

log = get_logger("io")

_CODE2TYPE = {1: IntegerType, 2: LongType, 3: lambda: DecimalType(38, 0), 4: DoubleType, 5: BooleanType,
              6: StringType, 7: TimestampType, 0: StringType}


def csv_code_to_type(code: int):
    return _CODE2TYPE[int(code)]()


def _type_to_code(t) -> int:
    if isinstance(t, IntegerType):
        return 1
    if isinstance(t, LongType):
        return 2
    if isinstance(t, DecimalType):
        return 3
    if isinstance(t, DoubleType):
        return 4
    if isinstance(t, BooleanType):
        return 5
    if isinstance(t, TimestampType):
        return 7
    return 6


def _device_csv_opts(o) -> Optional[dict]:
    """The reader options as the device parser's dialect, or None when only the host scanner
    implements them (multi-byte quote / escape / comment, nullValue longer than 16 bytes)."""
    quote, escape = o.get("quote", '"'), o.get("escape", "\\")
    comment, null_value = o.get("comment", ""), o.get("nullvalue", "")
    if len(quote) != 1 or len(escape) != 1 or len(comment) > 1 or len(null_value.encode()) > 16:
        return None
    # the device classifies a field with a quote / escape byte from its raw bytes and compares
    # nullValue with them: exact while neither byte can be part of a number, a boolean or nullValue
    if any(ch.isalnum() or ch in "+-." or ch in null_value for ch in (quote, escape)):
        return None
    return {"quote": quote, "escape": escape, "comment": ord(comment) if comment else 0,
            "trim_lead": _truthy(o.get("ignoreleadingwhitespace", "false")),
            "trim_trail": _truthy(o.get("ignoretrailingwhitespace", "false")),
            "null_value": null_value}


def _split_header(data, sep: str, opts: dict):
    """(column names, byte offset of the first data line) of the header record — the first
    non-empty, non-comment line, split the host scanner's way (quotes included,
    ``ops.csvscan.split_record``) — or None when the file has no data line.  A bounded head
    search: the input may be a multi-GB map."""
    n = len(data)
    pos, w = 0, 1 << 16
    comment = opts["comment"]
    while pos < n:
        head = bytes(data[pos:min(n, pos + w)])
        cut = [x for x in (head.find(b"\n"), head.find(b"\r")) if x >= 0]
        if not cut and pos + len(head) < n:
            w *= 16
            continue
        e = min(cut) if cut else len(head)
        line = head[:e]
        nxt = pos + e + 1 if cut else n
        if cut and head[e:e + 2] == b"\r\n":
            nxt += 1
        if line and not (comment and line[0] == comment):
            if nxt >= n:
                return None
            from ..ops.csvscan import split_record

            fields = split_record(line, ord(sep), ord(opts["quote"]), ord(opts["escape"]),
                                  opts["null_value"].encode(), opts["trim_lead"], opts["trim_trail"])
            return [f"_c{i}" if null else t.decode("utf-8", "replace") for i, (t, null) in enumerate(fields)], nxt
        pos = nxt
    return None


def _map_check(pf):
    """For input read through a file map (``filecache.MappedFile``, ranges above the pinned cache):
    a check run before a device string column builds its text from the map -- it raises if the
    file changed since it was mapped (the bytes under a map are the file's own).  None for owned
    copies (the pinned cache, plain reads)."""
    if pf is None or getattr(pf, "host", None) is not None:
        return None
    path = pf.path
    st = os.stat(path)
    ident = (st.st_size, st.st_mtime_ns, st.st_ino)

    def check():
        s = os.stat(path)
        if (s.st_size, s.st_mtime_ns, s.st_ino) != ident:
            raise RuntimeError(f"{path} changed after it was scanned: its string columns can no longer be read")
    return check


def _csv_cell(v, java_str) -> str:
    """One written CSV value: a timestamp in the CSV source's default ``timestampFormat``
    (``yyyy-MM-dd'T'HH:mm:ss.SSSXXX``, UTC -> ``Z``), which the reader parses back; else Java's
    string form."""
    import datetime

    if isinstance(v, datetime.datetime):
        return v.strftime("%Y-%m-%dT%H:%M:%S.") + f"{v.microsecond // 1000:03d}Z"
    return java_str(v)


def _truthy(v) -> bool:
    return str(v).lower() in ("true", "1", "yes")


_STATS: dict = {}  # path -> its os.stat of this load (one stat per plain file per load)


def _expand(paths) -> List[str]:
    out = []
    _STATS.clear()
    for p in paths:
        if any(ch in p for ch in "*?["):
            out += sorted(glob.glob(p))
            continue
        try:
            st = os.stat(p)
        except OSError:
            from .expressions import AnalysisException

            raise AnalysisException(f"Path does not exist: file:{os.path.abspath(p)};") from None
        if stat.S_ISDIR(st.st_mode):
            out += sorted(f for f in glob.glob(os.path.join(p, "*"))
                          if not os.path.basename(f).startswith(("_", ".")))
        else:
            _STATS[p] = st
            out.append(p)
    return out


class DataFrameReader:
    def __init__(self, session):
        self._session = session
        self._format = "parquet"
        self._options: Dict[str, str] = {}
        self._schema: Optional[StructType] = None

    def __call__(self):
        return self

    def format(self, f: str):
        self._format = f.lower()
        return self

    def option(self, key: str, value):
        self._options[key.lower()] = str(value).lower() if isinstance(value, bool) else str(value)
        return self

    def options(self, **kw):
        for k, v in kw.items():
            self.option(k, v)
        return self

    def schema(self, s):
        if isinstance(s, str):
            fields = []
            for part in s.split(","):
                nm, _, tp = part.strip().partition(" ")
                fields.append(StructField(nm.strip(), parse_type_name(tp.strip()), True))
            s = StructType(fields)
        self._schema = s
        return self

    def load(self, path=None, format=None, **opts):
        from .dataframe import DataFrame

        if format:
            self._format = format.lower()
        for k, v in opts.items():
            self.option(k, v)
        paths = path if isinstance(path, (list, tuple)) else [path]
        files = _expand(paths)
        if self._format == "csv":
            mk = self._load_key(files)
            hit = _LOADS.get(mk[0]) if mk is not None else None
            hpf = hit[0]() if hit is not None else None
            tmpl = getattr(hpf, "load_templates", {}).get(mk[0]) if hpf is not None else None
            if tmpl is not None and hit[1] == mk[1] and hpf.live():
                # the same unchanged bytes with the same options: this action's own (unscanned)
                # copy of the lazy relation the first load built -- the device scan still runs
                # at the action (sql/skey.py)
                return DataFrame(tmpl.fresh(), self._session)
            self._last_pf = None
            table = self._read_csv(files)
            if not isinstance(table, Table):  # a lazily scanned relation (sql.plan.CsvScanRelation)
                table.label = f"Relation[csv] {','.join(paths)}"
                pf = self._last_pf
                if mk is not None and pf is not None and table.fused is not None and table.fused.get("buf") is not None:
                    from .skey import intern

                    table._skey = intern(("csv", next(_LOAD_SERIAL)))
                    if len(_LOADS) >= 64:
                        _LOADS.clear()
                    pf.__dict__.setdefault("load_templates", {})[mk[0]] = table.fresh()
                    _LOADS[mk[0]] = (weakref.ref(pf), mk[1])
                return DataFrame(table, self._session)
        elif self._format == "parquet":
            table = self._read_parquet(files)
        elif self._format == "json":
            table = self._read_json(files)
        else:
            raise ValueError(f"Failed to find data source: {self._format}")
        return DataFrame(LocalRelation(table, f"Relation[{self._format}] {','.join(paths)}"), self._session)

    def _load_key(self, files):
        """(key, file identity) of a load that may reuse an earlier lazy relation: one CSV file on
        one GPU (a sharded read is collective: every rank must take the same path, so no rank
        may skip it), keyed by path, reader options, user schema and the reader's conf."""
        from ..parallel import comm

        dev = self._session.device
        if len(files) != 1 or dev.type != "cuda" or comm.world_size() > 1:
            return None
        st = _STATS.get(files[0])  # (the stat _expand took for this load)
        if st is None:
            try:
                st = os.stat(files[0])
            except OSError:
                return None
        conf = self._session.conf
        ck = tuple(conf.get(k, None) for k in _LOAD_CONF)
        sch = self._schema.simpleString() if self._schema else None
        rp = _REALPATH.get(files[0])
        if rp is None:  # (a path's symlinks are resolved once per process; the stat above is per load)
            if len(_REALPATH) >= 1024:
                _REALPATH.clear()
            rp = _REALPATH[files[0]] = os.path.realpath(files[0])
        key = (rp, tuple(sorted(self._options.items())), sch, ck, str(dev))
        return key, (st.st_size, st.st_mtime_ns, st.st_ino)

    def csv(self, path, schema=None, sep=None, header=None, inferSchema=None, **kw):
        if schema is not None:
            self.schema(schema)
        for k, v in (("sep", sep), ("header", header), ("inferSchema", inferSchema)):
            if v is not None:
                self.option(k, v)
        return self.load(path, format="csv", **kw)

    def parquet(self, *paths):
        return self.load(list(paths), format="parquet")

    def json(self, path):
        return self.load(path, format="json")

    # ---- csv -------------------------------------------------------------------------------
    def _read_csv(self, files: List[str]):
        """CSV -> columnar table.  In a multi-process group (``dq4ml.shardInput``, default on) each
        rank parses only its byte range, moved to row boundaries (Hadoop split semantics), and the
        inferred schema is merged across ranks (tightest common type; names from rank 0, whose
        shard holds the header) — the shards then re-parse under the merged schema if it widened."""
        from ..parallel import comm

        o = self._options
        dev = self._session.device
        thresh = int(self._session.conf.get("dq4ml.csv.deviceThresholdBytes", str(64 << 20)))
        pinned = None
        world, rank = comm.world_size(), comm.rank()
        shard = world > 1 and _truthy(self._session.conf.get("dq4ml.shardInput", "true"))
        presharded = False
        if len(files) == 1 and dev.type == "cuda" and os.path.getsize(files[0]) >= thresh:
            # large single file: pinned host copy cached per (path, size, mtime) (runtime.filecache);
            # every re-scan DMAs it straight to the device — no read(), no bounce buffer.  A rank
            # of a sharded read caches (and reads) only its own row-aligned byte range.
            from ..runtime import filecache

            lo, hi = filecache.shard_range(files[0], rank, world) if shard else (0, os.path.getsize(files[0]))
            presharded = shard
            if hi - lo <= filecache.MAX_BYTES:
                pf = filecache.open_pinned(files[0], lo, hi)
                data, pinned = pf.data, pf.host
            else:
                # larger than the pinned cache may hold: a read-only map, streamed through the
                # pinned staging ring chunk by chunk (no copy of the whole range is ever made); the
                # entry still keeps the range's facts and, if HBM allows, its device-resident bytes
                pf = filecache.open_mapped(files[0], lo, hi)
                data = pf.data
        else:
            pf = None
            data = b"".join(self._read_bytes(f) for f in files)
        self._last_pf = pf
        return self._read_csv_data(data, o, dev, thresh, pinned, pf, presharded)

    def _read_csv_data(self, data, o, dev, thresh, pinned=None, pf=None, presharded=False):
        """A Table, or a lazily scanned ``CsvScanRelation`` for bytes already typed by an earlier
        device scan."""
        from ..parallel import comm

        header = _truthy(o.get("header", "false"))
        infer = _truthy(o.get("inferschema", "false"))
        sep = o.get("sep", o.get("delimiter", ","))
        sep = "\t" if sep == "\\t" else sep
        user_types = [_type_to_code(f.dataType) for f in self._schema.fields] if self._schema else []
        user_names = self._schema.names if self._schema else []
        world, rank = comm.world_size(), comm.rank()
        shard = world > 1 and _truthy(self._session.conf.get("dq4ml.shardInput", "true"))
        lo, hi = 0, len(data)
        if shard and not presharded:
            from ..ops.csvscan import shard_byte_range

            lo, hi = shard_byte_range(data, rank, world)
            data = memoryview(data)[lo:hi] if not isinstance(data, bytes) else data[lo:hi]
            pinned = None if pinned is None else pinned[lo:hi]
        if shard:
            header = header and rank == 0
        if presharded:
            lo, hi = 0, len(data)  # pf holds exactly this rank's bytes
        # the device scanner takes the common dialect options (csv_parse_dev.h): header, a user
        # schema, nullValue, comment, the whitespace trims, any single-byte quote / escape
        dopts = _device_csv_opts(o)
        strict = [c for c in user_types] if user_types else None
        # a user schema of int / long / double / boolean / timestamp / string columns; no schema
        # and no inference: every column a string (Spark's default read)
        all_str = not infer and not strict
        use_dev = (dev.type == "cuda" and dopts is not None and len(sep) == 1 and ord(sep) < 128
                   and (not strict or all(c in (1, 2, 4, 5, 7) or (c == 6 and isinstance(f.dataType, StringType))
                                          for c, f in zip(strict, self._schema.fields))))
        hdr = None
        if use_dev and header:
            hdr = _split_header(data, sep, dopts)
            use_dev = hdr is not None
        if shard:  # every rank must take the same (collective) path
            use_dev = all(comm.all_gather_object(bool(use_dev and len(data) >= thresh)))
        elif use_dev:
            use_dev = len(data) >= thresh
        dev_scan = None
        if use_dev:
            from ..ops import csvscan

            off = hdr[1] if hdr is not None else 0
            names = hdr[0] if hdr is not None else None
            if shard and header is not None:
                # names come from the rank whose shard holds the header (rank 0)
                names = comm.all_gather_object(names)[0]
            body = data[off:] if off else data
            dbytes = None
            dready = None
            if pf is not None and _truthy(self._session.conf.get("dq4ml.csv.deviceCache", "true")):
                from ..runtime import filecache

                if filecache.device_bytes_allowed(hi - lo) or (str(dev), lo, hi) in pf._dev:
                    # HBM-resident input bytes; a first upload is consumed progressively by the
                    # scan below (chunk k parsed while chunk k + 1 is copied)
                    dbytes = pf.device_bytes(dev, lo, hi, progressive=True)
                    dready = [(e - off, ev) for e, ev in pf.take_ready(dev, lo, hi)]
                    dbytes = dbytes[off:] if off else dbytes
            hkey = (lo + off, hi, sep, repr(sorted(dopts.items())))
            fkey = hkey + (tuple(strict) if strict else None,)
            if all_str:
                from ..ops.csvscan import CT_STRING, _ncols_of, _opt_args

                oa = _opt_args(dopts)
                nstr = len(names) if names else _ncols_of(body, sep, int(oa["comment"] or 0), oa["quote"], oa["escape"])
                if shard:  # the first record of the file (rank 0's shard) sets the column count
                    nstr = comm.all_gather_object(nstr)[0]
                strict = [CT_STRING] * nstr
                fkey = hkey + (tuple(strict),)
            ncols = len(strict) if strict else (len(names) if names else None)
            final = (user_names or names) if strict else names

            def dev_scan():
                with tracing.span("csv_scan"):
                    try:
                        t = csvscan.scan_device(body, sep=sep, infer=infer, device=dev, sharded=shard, ncols=ncols,
                                                chunk_bytes=int(self._session.conf.get("dq4ml.chunkBytes",
                                                                                       str(256 << 20))),
                                                pinned=None if pinned is None else pinned[off:], device_data=dbytes,
                                                types_hint=(pf.type_hints.get(hkey) if pf is not None and not strict
                                                            else None), opts=dopts, user_types=strict,
                                                source_check=_map_check(pf), device_ready=dready)
                    finally:
                        if dready is not None:  # every later use of the cached bytes is ordered after the upload
                            pf.wait_ready(dev, lo, hi)
                if t is None:
                    return None
                codes = [csvscan.type_code_of(f.dataType) for f in t.schema.fields]
                if pf is not None:
                    if not strict:  # the next action's scan stores typed columns directly
                        pf.type_hints[hkey] = codes
                    facts = getattr(t, "scan_facts", None)
                    if facts is not None and dbytes is not None:
                        pf.scan_facts[fkey] = dict(facts, types=codes, nbytes=len(body))
                if final:
                    fields = [StructField(nm, f.dataType, True) for nm, f in zip(final, t.schema.fields)]
                    t = Table(StructType(fields), t.columns, t.nrows, t.sel, t.device)
                return t

            # input that cannot stay resident in HBM: one streamed inference pass
            # (types + facts, no column kept), then a lazy relation whose fused Gram action
            # streams the bytes through a chunk ring -- one pass per action at constant memory
            stream_min = int(float(self._session.conf.get("dq4ml.csv.streamThresholdBytes", str(1 << 30))))
            streamed = (pf is not None and dbytes is None and len(body) >= stream_min
                        and _truthy(self._session.conf.get("dq4ml.csv.fuseScan", "true")))
            if shard:  # every rank takes the same (collective) path
                streamed = all(comm.all_gather_object(bool(streamed)))
            if streamed:
                rel = self._streamed_relation(body, pinned, pf, fkey, dopts, sep, strict, ncols, final, shard, dev,
                                              data, header, infer, user_types, user_names)
                if rel is not None:
                    return rel
            # a re-read of bytes an earlier device scan already typed: lazy relation, scanned at
            # the action — fused with the DQ chain on top of it when there is one (ops/scanfuse.py)
            facts = pf.scan_facts.get(fkey) if (pf is not None and dbytes is not None) else None
            # (the per-line fused kernel takes <= 64 columns of lines <= 64 bytes on average; wider
            # rows go through the byte-parallel cutter, ops/scancut.py, or scan eagerly)
            lazy = (facts is not None and len(body) == facts["nbytes"]
                    and _truthy(self._session.conf.get("dq4ml.csv.fuseScan", "true"))
                    and len(facts["types"]) <= 256 and facts["nlines"] > 0
                    and len(body) / facts["nlines"] <= 4096)
            if shard:  # every rank takes the same (collective) path
                lazy = all(comm.all_gather_object(bool(lazy)))
            if lazy:
                from ..ops.csvscan import _KIND, _opt_args
                from ..sql.plan import CsvScanRelation

                if dready:  # (a fresh upload the fused scans will read: order them after it)
                    pf.wait_ready(dev, lo, hi)

                codes = facts["types"]
                fnames = final or [f"_c{i}" for i in range(len(codes))]
                schema = StructType([StructField(nm, csv_code_to_type(c), True) for nm, c in zip(fnames, codes)])
                n = len(body)
                fused = {"buf": dbytes, "n": n, "nlines": facts["nlines"], "device": dev,
                         "trailing": n > 0 and body[-1] not in (10, 13), "mean_line": n / facts["nlines"],
                         "kinds": [_KIND.get(c, (0,))[0] for c in codes], "nullable": list(facts["nullable"]),
                         "fast_only": bool(facts.get("fast_only")),
                         "quoted_fast": bool(facts.get("quoted_fast")),
                         "max_line": int(facts.get("max_line", 1 << 30)),
                         "uniform_fields": bool(facts.get("uniform_fields")),
                         "empty_lines": int(facts.get("empty_lines", 1)),
                         "min_line": int(facts.get("min_line", 1)),
                         "term_kinds": list(facts.get("term_kinds") or (1, 1, 0)),
                         "opts": dict(_opt_args(dopts), sep=sep, strict=bool(strict)), "strict": bool(strict)}
                if fused["opts"]["null_value"] and len(fused["opts"]["null_value"].encode()) > 16:
                    fused = None

                def scan_or_host():
                    t = dev_scan()
                    return t if t is not None else self._host_table(data, header, infer, user_types, user_names,
                                                                   sep, dev, shard)
                return CsvScanRelation(schema, scan_or_host, fused, "Relation[csv]")
            t = dev_scan()
            if t is not None:
                return t
        return self._host_table(data, header, infer, user_types, user_names, sep, dev, shard)

    def _streamed_relation(self, body, pinned, pf, fkey, dopts, sep, strict, ncols, final, shard, dev, data, header,
                           infer, user_types, user_names):
        """Lazy ``CsvScanRelation`` over bytes that stream through the device (``fused["stream"]``:
        a ``runtime.streams.ChunkSource``; ``fused["buf"]`` is None).  The inference pass runs once
        per cached byte range (its types and facts are kept with the file entry)."""
        from ..ops.csvscan import _KIND, _opt_args, infer_streamed
        from ..runtime.streams import ChunkSource
        from ..sql.plan import CsvScanRelation

        chunk = int(float(self._session.conf.get("dq4ml.csv.streamChunkBytes", str(1 << 30))))
        skey = fkey + ("stream", chunk)
        ent = pf.scan_facts.get(skey)
        if ent is None:
            src = ChunkSource(body, None if pinned is None else pinned[len(data) - len(body):], chunk, dev)
            with tracing.span("csv_infer_streamed"):
                r = infer_streamed(src, sep, ncols=ncols, sharded=shard, opts=dopts, user_types=strict)
            if r is None:
                return None
            codes, facts = r
            ent = pf.scan_facts[skey] = (codes, facts, src)
        codes, facts, src = ent
        if facts["nlines"] <= 0 or len(codes) > 256:
            return None
        fnames = final or [f"_c{i}" for i in range(len(codes))]
        schema = StructType([StructField(nm, csv_code_to_type(c), True) for nm, c in zip(fnames, codes)])
        n = len(body)
        fused = {"buf": None, "stream": src, "n": n, "nlines": facts["nlines"], "device": dev,
                 "trailing": n > 0 and body[-1] not in (10, 13), "mean_line": n / facts["nlines"],
                 "kinds": [_KIND.get(c, (0,))[0] for c in codes], "nullable": list(facts["nullable"]),
                 "fast_only": bool(facts.get("fast_only")), "quoted_fast": bool(facts.get("quoted_fast")),
                 "max_line": int(facts.get("max_line", 1 << 30)),
                 "uniform_fields": bool(facts.get("uniform_fields")), "empty_lines": int(facts.get("empty_lines", 1)),
                 "min_line": int(facts.get("min_line", 1)), "term_kinds": list(facts.get("term_kinds") or (1, 1, 0)),
                 "opts": dict(_opt_args(dopts), sep=sep, strict=bool(strict)), "strict": bool(strict)}
        if fused["opts"]["null_value"] and len(fused["opts"]["null_value"].encode()) > 16:
            fused = None

        def scan_eager():  # any action the streamed fused Gram does not cover: the chunked device scan
            from ..ops import csvscan

            with tracing.span("csv_scan"):
                t = csvscan.scan_device(body, sep=sep, infer=infer, device=dev, sharded=shard, ncols=ncols,
                                        chunk_bytes=int(self._session.conf.get("dq4ml.chunkBytes", str(256 << 20))),
                                        pinned=None if pinned is None else pinned[len(data) - len(body):],
                                        types_hint=None if strict else list(codes), opts=dopts, user_types=strict,
                                        source_check=_map_check(pf))
            if t is None:
                return self._host_table(data, header, infer, user_types, user_names, sep, dev, shard)
            fields = [StructField(nm, f.dataType, True) for nm, f in zip(fnames, t.schema.fields)]
            return Table(StructType(fields), t.columns, t.nrows, t.sel, t.device)
        return CsvScanRelation(schema, scan_eager, fused, "Relation[csv]")

    def _host_table(self, data, header, infer, user_types, user_names, sep, dev, shard) -> Table:
        from ..parallel import comm

        if not isinstance(data, bytes):
            data = bytes(data)  # host scanner path (small or fallback): a plain copy
        with tracing.span("csv_scan"):
            nrows, cols = self._host_scan(data, header, infer, user_types, user_names, sep)
            if shard and not user_types:
                from ..ops import native

                h = native.host()
                mine = ([c[0] for c in cols], [int(c[1]) for c in cols])
                parts = comm.all_gather_object(mine)
                names = parts[0][0] or max((p[0] for p in parts), key=len)
                ncol = len(names)
                codes = [0] * ncol
                for _, cs in parts:
                    for i in range(min(ncol, len(cs))):
                        codes[i] = int(h.csv_merge_types(codes[i], cs[i]))
                codes = [c if c else 6 for c in codes] if any(len(p[1]) for p in parts) else codes
                if (list(names), codes) != (mine[0], mine[1]):
                    nrows, cols = self._host_scan(data, header, False, codes, list(names), sep)
        fields, columns = [], []
        for (name, code, vals, valid) in cols:
            dt = self._schema[len(fields)].dataType if self._schema else csv_code_to_type(code)
            if isinstance(vals, list):
                c = column_from_pylist([v if ok else None for v, ok in zip(vals, valid)], StringType(), dev)
            else:
                c = column_from_numpy(vals, valid.astype(bool), dt, dev)
            fields.append(StructField(name, dt, True))
            columns.append(c)
        return Table(StructType(fields), columns, nrows, None, dev)

    def _host_scan(self, data, header, infer, user_types, user_names, sep):
        from ..ops import native

        o = self._options
        return native.host().csv_scan(
            data, sep=sep, quote=o.get("quote", '"'), escape=o.get("escape", "\\"), header=header,
            infer=infer, null_value=o.get("nullvalue", ""), comment=o.get("comment", ""),
            ignore_leading_ws=_truthy(o.get("ignoreleadingwhitespace", "false")),
            ignore_trailing_ws=_truthy(o.get("ignoretrailingwhitespace", "false")),
            user_types=user_types, user_names=user_names)

    @staticmethod
    def _read_bytes(path) -> bytes:
        with open(path, "rb") as f:
            return f.read()

    # ---- parquet / json ----------------------------------------------------------------------
    def _read_parquet(self, files):
        import pyarrow.parquet as pq
        import pyarrow as pa

        tables = [pq.read_table(f) for f in files if f.endswith(".parquet") or os.path.isfile(f)]
        t = pa.concat_tables(tables) if len(tables) > 1 else tables[0]
        return table_from_data(t.to_pandas(), self._schema, self._session.device)

    def _read_json(self, files):
        rows = []
        for f in files:
            with open(f) as fh:
                for line in fh:
                    line = line.strip()
                    if line:
                        rows.append(json.loads(line))
        return table_from_data(rows, self._schema, self._session.device)


class DataFrameWriter:
    def __init__(self, df):
        self._df = df
        self._mode = "errorifexists"
        self._format = "parquet"
        self._options = {}

    def __call__(self):  # ``df.write()`` (the Java API form) as well as ``df.write``
        return self

    def mode(self, m):
        self._mode = m.lower()
        return self

    def format(self, f):
        self._format = f.lower()
        return self

    def option(self, k, v):
        self._options[k.lower()] = str(v)
        return self

    def _prepare(self, path):
        if os.path.exists(path):
            if self._mode in ("overwrite",):
                shutil.rmtree(path) if os.path.isdir(path) else os.remove(path)
            elif self._mode in ("ignore",):
                return False
            elif self._mode != "append":
                from .expressions import AnalysisException

                raise AnalysisException(f"path file:{os.path.abspath(path)} already exists.;")
        os.makedirs(path, exist_ok=True)
        return True

    def save(self, path):
        if not self._prepare(path):
            return
        if self._format == "csv":
            self._write_csv(path)
        elif self._format == "parquet":
            self._write_parquet(path)
        else:
            raise ValueError(self._format)
        open(os.path.join(path, "_SUCCESS"), "w").close()

    def csv(self, path, mode=None, header=None):
        if mode:
            self.mode(mode)
        if header is not None:
            self.option("header", header)
        self._format = "csv"
        self.save(path)

    def parquet(self, path, mode=None):
        if mode:
            self.mode(mode)
        self._format = "parquet"
        self.save(path)

    def _write_csv(self, path):
        from ..utils.javafmt import java_str

        t = self._df._table().compact()
        sep = self._options.get("sep", ",")
        cols = [c.to_pylist() for c in t.columns]
        with open(os.path.join(path, "part-00000.csv"), "w") as f:
            if _truthy(self._options.get("header", "false")):
                f.write(sep.join(t.schema.names) + "\n")
            for r in zip(*cols):
                f.write(sep.join("" if v is None else _csv_cell(v, java_str) for v in r) + "\n")

    def _write_parquet(self, path):
        import pyarrow as pa
        import pyarrow.parquet as pq

        pdf = self._df.toPandas()
        pq.write_table(pa.Table.from_pandas(pdf, preserve_index=False), os.path.join(path, "part-00000.parquet"))


_ = (ColumnData, np, torch)

