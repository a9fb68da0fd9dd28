"""Per-stage tracing: wall-clock + device-time spans for the pipeline stages
(scan / dq / pack / gram / allreduce / solve / metrics / predict), a ``metrics.json`` dump, and
``torch.profiler`` ranges so the stages show up in rocprofv3 / Chrome traces.

Off by default and free when off (``span`` returns a shared no-op context).  Turn on with
``DQ4ML_TRACE=1`` or ``SparkSession.builder().config("dq4ml.trace", "true")``.  Device time is
measured with HIP events recorded on the current stream and resolved lazily at ``report()`` — a
span never synchronizes the device, so tracing does not serialize the pipeline it measures.
"""
from __future__ import annotations

import contextlib
import json
import os
import threading
import time
from collections import OrderedDict
from typing import Dict, Optional

__all__ = ["enabled", "enable", "span", "report", "reset", "dump_json", "add_rows"]

_state = threading.local()
_lock = threading.Lock()
_enabled = os.environ.get("DQ4ML_TRACE", "0") not in ("", "0", "false", "False")
_records: "OrderedDict[str, dict]" = OrderedDict()
_pending = []  # (name, start_event, end_event)


def enabled() -> bool:
    return _enabled


def enable(on: bool = True):
    global _enabled
    _enabled = bool(on)


class _Noop:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


_NOOP = _Noop()


def _rec(name):
    r = _records.get(name)
    if r is None:
        r = _records[name] = {"count": 0, "host_ms": 0.0, "device_ms": 0.0, "rows": 0}
    return r


class _Span:
    __slots__ = ("name", "dev", "t0", "ev0", "rf")

    def __init__(self, name, dev):
        self.name, self.dev = name, dev

    def __enter__(self):
        import torch

        self.rf = None
        try:
            self.rf = torch.profiler.record_function("dq4ml::" + self.name)
            self.rf.__enter__()
        except Exception:  # pragma: no cover - profiler unavailable
            self.rf = None
        self.ev0 = None
        if self.dev and torch.cuda.is_available():
            self.ev0 = torch.cuda.Event(enable_timing=True)
            self.ev0.record()
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        import torch

        dt = (time.perf_counter() - self.t0) * 1e3
        with _lock:
            r = _rec(self.name)
            r["count"] += 1
            r["host_ms"] += dt
            if self.ev0 is not None:
                ev1 = torch.cuda.Event(enable_timing=True)
                ev1.record()
                _pending.append((self.name, self.ev0, ev1))
        if self.rf is not None:
            self.rf.__exit__(*exc)
        return False


def span(name: str, device: bool = True):
    """``with span("gram"): ...`` — records host wall time and (on a GPU) device time."""
    if not _enabled:
        return _NOOP
    return _Span(name, device)


def add_rows(name: str, rows: int):
    if _enabled:
        with _lock:
            _rec(name)["rows"] += int(rows)


def _resolve():
    if not _pending:
        return
    import torch

    torch.cuda.synchronize()
    with _lock:
        for name, e0, e1 in _pending:
            _rec(name)["device_ms"] += e0.elapsed_time(e1)
        _pending.clear()


def report() -> Dict[str, dict]:
    """Per-stage totals: count, host_ms, device_ms, rows, rows_per_s (device time when known)."""
    _resolve()
    out = OrderedDict()
    for k, r in _records.items():
        v = dict(r)
        t = v["device_ms"] or v["host_ms"]
        v["rows_per_s"] = (v["rows"] / (t * 1e-3)) if (v["rows"] and t > 0) else None
        out[k] = v
    return out


def reset():
    _resolve()
    with _lock:
        _records.clear()


def dump_json(path: str, extra: Optional[dict] = None):
    doc = {"stages": report()}
    if extra:
        doc.update(extra)
    with open(path, "w") as f:
        json.dump(doc, f, indent=2)
    return doc


@contextlib.contextmanager
def tracing(on: bool = True):
    """Scoped enable (tests / benchmarks)."""
    prev = _enabled
    enable(on)
    try:
        yield
    finally:
        enable(prev)
