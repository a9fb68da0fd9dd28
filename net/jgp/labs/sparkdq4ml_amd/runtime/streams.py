"""HIP stream helpers: a per-device side stream for copies/collectives that
overlap compute on the current stream, and a double-buffered pinned staging ring for streamed
host->device ingest (chunk k+1's H2D copy runs while chunk k is parsed)."""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np
import torch

__all__ = ["side_stream", "StagingRing", "ChunkSource", "cu_masked_stream", "reserved_cu_ids"]

_side: Dict[int, "torch.cuda.Stream"] = {}


def side_stream(device: Optional[torch.device] = None) -> "torch.cuda.Stream":
    idx = torch.cuda.current_device() if device is None or device.index is None else device.index
    s = _side.get(idx)
    if s is None:
        s = _side[idx] = torch.cuda.Stream(device=idx)
    return s


def reserved_cu_ids(reserve: int, cus: int):
    """The CUs held back for the fit tail: the last CU of each 32-CU block of the logical CU order
    (one per XCD when that order is XCD-major), then the next-to-last ones, ... -- any choice is
    correct, the two masks only have to be disjoint."""
    per = max(1, cus // 32)
    ids = []
    k = 0
    while len(ids) < min(reserve, cus):
        for x in range(per):
            c = x * 32 + 31 - k
            if 0 <= c < cus and c not in ids and len(ids) < reserve:
                ids.append(c)
        k += 1
    return ids


_masked: Dict[tuple, "torch.cuda.Stream"] = {}


def cu_masked_stream(cu_ids, cus: int, device=None, tag: int = 0) -> "torch.cuda.Stream":
    """A stream whose kernels dispatch only to the CUs in ``cu_ids`` (``hipExtStreamCreateWithCUMask``),
    cached per (device, CU set, tag).  Used to keep the pipelined fit tail (fold, RCCL kernels'
    neighbours, solve) and the full-chip Gram passes on disjoint CUs (``dq4ml.gram.reserveCUs``)."""
    from ..ops import native

    idx = torch.cuda.current_device() if device is None or torch.device(device).index is None \
        else torch.device(device).index
    key = (idx, tuple(sorted(cu_ids)), tag)
    st = _masked.get(key)
    if st is None:
        words = [0] * ((cus + 31) // 32)
        for c in cu_ids:
            words[c // 32] |= 1 << (c % 32)
        with torch.cuda.device(idx):
            ptr = native.hip().stream_create_cumask(words)
        st = _masked[key] = torch.cuda.ExternalStream(ptr, device=torch.device("cuda", idx))
    return st


_pool = None
_COPY_SLICE = 16 << 20


def _parallel_copy(dst: np.ndarray, src: np.ndarray) -> None:
    """Host memcpy into pinned staging in 16 MiB slices on a thread pool (numpy releases the GIL
    for plain copies): one core's memcpy (~10 GB/s) was the ingest bottleneck, ahead of PCIe."""
    global _pool
    n = src.shape[0]
    if n <= _COPY_SLICE:
        dst[:] = src
        return
    if _pool is None:
        import os
        from concurrent.futures import ThreadPoolExecutor

        _pool = ThreadPoolExecutor(max(1, min(8, (os.cpu_count() or 4))))
    cuts = list(range(0, n, _COPY_SLICE)) + [n]
    list(_pool.map(lambda i: np.copyto(dst[cuts[i]:cuts[i + 1]], src[cuts[i]:cuts[i + 1]]), range(len(cuts) - 1)))


class StagingRing:
    """``depth`` pinned host buffers + device buffers of ``nbytes``; ``put(i, data)`` copies host
    bytes into slot ``i % depth`` and enqueues its H2D on the side stream; ``get(i)`` makes the
    current stream wait for that copy and returns the device view.  A slot is reused only after
    the compute that consumed it has been recorded (event), so the ring never overwrites live data."""

    def __init__(self, nbytes: int, depth: int = 2, device: Optional[torch.device] = None, staging: bool = True):
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        # staging=False: every put() names an already page-locked source (runtime.filecache), so no
        # pinned bounce buffers are needed
        self.host: List[torch.Tensor] = [torch.empty(nbytes if staging else 0, dtype=torch.uint8).pin_memory()
                                         for _ in range(depth)]
        self.dev: List[torch.Tensor] = [torch.empty(nbytes, dtype=torch.uint8, device=self.device)
                                        for _ in range(depth)]
        self.copied = [torch.cuda.Event() for _ in range(depth)]
        self.consumed = [None] * depth
        self.sizes = [0] * depth
        self.depth = depth
        self.stream = side_stream(self.device)

    def put(self, i: int, data, pinned: Optional[torch.Tensor] = None) -> None:
        """Stage chunk ``i``.  ``pinned``: a page-locked host view of the same bytes — then the DMA
        reads it directly (no host memcpy, and the slot's reuse is ordered on the device, not by a
        host wait)."""
        k = i % self.depth
        if pinned is not None:
            n = pinned.numel()
            if n > self.dev[k].numel():
                raise ValueError("StagingRing: chunk larger than the device buffers")
            self.sizes[k] = n
            with torch.cuda.stream(self.stream):
                if self.consumed[k] is not None:
                    self.stream.wait_event(self.consumed[k])
                self.dev[k][:n].copy_(pinned, non_blocking=True)
                self.copied[k].record(self.stream)
            return
        if self.consumed[k] is not None:
            self.consumed[k].synchronize()  # host must not overwrite pinned memory still being copied/used
        n = len(data)
        if n > self.host[k].numel():
            raise ValueError("StagingRing: chunk larger than the staging buffers")
        _parallel_copy(self.host[k][:n].numpy(), np.frombuffer(data, dtype=np.uint8, count=n))
        self.sizes[k] = n
        with torch.cuda.stream(self.stream):
            self.dev[k][:n].copy_(self.host[k][:n], non_blocking=True)
            self.copied[k].record(self.stream)

    def get(self, i: int) -> torch.Tensor:
        k = i % self.depth
        torch.cuda.current_stream().wait_event(self.copied[k])
        return self.dev[k][:self.sizes[k]]

    def release(self, i: int) -> None:
        k = i % self.depth
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream())
        self.consumed[k] = ev


class ChunkSource:
    """An input byte range that is NOT resident in HBM, streamed through the device in row-aligned
    chunks (Spark streams partitions through iterators at constant memory,
    ``DataQuality4MachineLearningApp.java:40, 53-55``).

    ``data``: the bytes on the host (a read-only map or a page-locked copy); ``pinned``: a
    page-locked tensor view of the same bytes when there is one (the DMA then reads it directly).
    :meth:`chunks` yields ``(device view, nbytes, trailing)`` per chunk: chunk k+1's H2D copy runs
    on the side stream while the caller's kernels consume chunk k on the current stream (a
    two-slot ring of ``chunk_bytes`` device buffers, kept across actions)."""

    def __init__(self, data, pinned: Optional[torch.Tensor], chunk_bytes: int, device):
        from ..ops.csvscan import chunk_bounds

        self.data, self.pinned, self.device = data, pinned, torch.device(device)
        self.n = len(data)
        self.bounds = chunk_bounds(data, max(1, int(chunk_bytes)))
        self.spans = [(self.bounds[i], self.bounds[i + 1]) for i in range(len(self.bounds) - 1)]
        self._ring = None

    def __len__(self):
        return len(self.spans)

    def _ring_for(self):
        if self._ring is None:
            width = max((e - s for s, e in self.spans), default=1)
            self._ring = StagingRing(width, depth=2, device=self.device, staging=self.pinned is None)
        return self._ring

    def _put(self, ring, i):
        s, e = self.spans[i]
        if self.pinned is not None:
            ring.put(i, None, pinned=self.pinned[s:e])
            return
        with torch.cuda.device(self.device):  # (runs on the staging thread)
            ring.put(i, memoryview(self.data)[s:e])

    def chunks(self):
        """Chunks in order.  A mapped (not page-locked) source is memcpy'd into the pinned staging
        buffers by one background thread, so chunk k+1's host copy and DMA both overlap the
        consumer's work on chunk k."""
        if not self.spans:
            return
        ring = self._ring_for()
        pool = None
        if self.pinned is None:
            if getattr(self, "_pool", None) is None:
                from concurrent.futures import ThreadPoolExecutor

                self._pool = ThreadPoolExecutor(1)
            pool = self._pool
        pending = {}

        def stage(i):
            if pool is None:
                self._put(ring, i)
            else:
                pending[i] = pool.submit(self._put, ring, i)

        stage(0)
        for i, (s, e) in enumerate(self.spans):
            if i + 1 < len(self.spans):
                stage(i + 1)  # overlaps the consumer's kernels on chunk i
            if i in pending:
                pending.pop(i).result()
            buf = ring.get(i)
            trailing = e > s and self.data[e - 1] not in (10, 13)
            yield buf, e - s, trailing
            ring.release(i)
