"""Low-overhead stream handling for the asynchronous fit's issue path.

An asynchronous ``LinearRegression.fit`` at the 8-GPU strong-scaling shard is ~0.14 ms of device
work, so its host issue cost decides whether the step stays device-bound.  The public torch stream
API resolves the device on every call (``torch.cuda.current_stream(dev)``, the ``torch.cuda.stream``
context, ``wait_stream``: ``_get_device_index`` -> ``is_available`` chains) and ``wait_stream``
creates a Python ``Event`` per call; a cProfile of the issue loop (``scripts/host_overhead.py``,
``profiles/r3_host_issue.md``) attributed about half of the ~110 us per fit to them.  These helpers
call the torch C entry points with a known device index and order streams through the native event
rings of ``_dq4ml_hip`` (``stream_wait`` / ``event_record`` / ``stream_wait_event``).
"""
from __future__ import annotations

import torch

_C = torch._C


def dev_index(dev) -> int:
    """Device index of a ``torch.device`` / tensor device (no current-device query when set)."""
    i = dev.index
    return _C._cuda_getDevice() if i is None else i


def raw(dev_idx: int) -> int:
    """The current stream's ``hipStream_t`` on device ``dev_idx``."""
    return _C._cuda_getCurrentRawStream(dev_idx)


def current(dev_idx: int) -> "torch.cuda.Stream":
    """``torch.cuda.current_stream(dev_idx)`` without the device resolution."""
    sid, di, dt = _C._cuda_getCurrentStream(dev_idx)
    return torch.cuda.Stream(stream_id=sid, device_index=di, device_type=dt)


class use:
    """``with use(stream):`` — ``torch.cuda.stream(stream)`` for a stream of the current device,
    without the per-call device resolution of the torch context manager."""

    __slots__ = ("s", "prev")

    def __init__(self, s):
        self.s = s
        self.prev = None

    def __enter__(self):
        s = self.s
        self.prev = _C._cuda_getCurrentStream(s.device_index)
        _C._cuda_setStream(stream_id=s.stream_id, device_index=s.device_index, device_type=s.device_type)
        return s

    def __exit__(self, *exc):
        sid, di, dt = self.prev
        _C._cuda_setStream(stream_id=sid, device_index=di, device_type=dt)
        return False


def wait(h, dst: int, src: int) -> None:
    """``dst`` waits for the work enqueued on ``src`` so far (raw stream handles)."""
    h.stream_wait(dst, src)
