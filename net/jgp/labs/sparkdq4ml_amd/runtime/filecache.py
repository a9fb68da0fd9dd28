"""Host (pinned) and device (HBM) caches of input files for CSV ingest.

A large input file is read ONCE into page-locked host memory (parallel ``preadv`` into a pinned
buffer) and kept, keyed by ``(path, size, mtime)``: every Spark action re-scans its input (S20),
and each re-scan then streams the cached bytes to the device by direct DMA (~57 GB/s H2D on the
MI355X box, 1 GB in 17 ms) with no host copy at all.  A rewritten file gets a new entry.

With ``dq4ml.csv.deviceCache`` (default on) the raw bytes of the rank's byte range also stay
resident in HBM (288 GB per MI355X; the cap is derived from the free HBM, ``device_cap_bytes``): a re-scan then parses straight from device memory — the
parse, DQ rules, assembly and fit all still run on every action; only the transfer of unchanged
input bytes is skipped, the way the OS page cache skips the disk read for Spark.

Why a copy and not a registered file mapping: ``hipHostRegister`` of a read-only ``mmap`` works
and avoids even the first copy, but the pinned pages still belong to the file — a truncating
rewrite while registered left ``hipDeviceSynchronize`` hanging (round-1 test).  Our own pinned
buffer cannot change underneath the device."""
from __future__ import annotations

import os
import threading
from collections import OrderedDict
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

__all__ = ["PinnedFile", "MappedFile", "open_pinned", "open_mapped", "shard_range", "map_readonly",
           "device_bytes_allowed", "device_cap_bytes", "clear"]

MAX_FILES = int(os.environ.get("DQ4ML_FILECACHE_FILES", "2"))
MAX_BYTES = int(float(os.environ.get("DQ4ML_FILECACHE_BYTES", str(32 << 30))))
_SLICE = 64 << 20
_cache: "OrderedDict[tuple, PinnedFile]" = OrderedDict()
_lock = threading.Lock()
_pool = None


def _readers() -> ThreadPoolExecutor:
    global _pool
    if _pool is None:
        _pool = ThreadPoolExecutor(max(1, min(8, os.cpu_count() or 4)))
    return _pool


class _Resident:
    """The HBM-resident copies of an input's byte ranges and the pieces of a first upload still
    to be waited on.  A piece is ``(end offset, p)`` where ``p.wait(stream)`` orders ``stream``
    after that piece's DMA (a ``torch.cuda.Event``, or an :class:`_Piece` that a background
    uploader fills)."""

    def take_ready(self, device, lo: int = 0, hi: int = -1):
        """[(end offset, piece)] of an upload still to be waited on by a progressive consumer
        (empty once waited)."""
        hi = self.nbytes if hi < 0 else hi
        return list(self._ready.get((str(device), lo, hi), []))

    def wait_ready(self, device, lo: int = 0, hi: int = -1):
        """Order the current stream after the whole upload of [lo, hi) (a no-op once done)."""
        hi = self.nbytes if hi < 0 else hi
        r = self._ready.pop((str(device), lo, hi), None)
        if r:  # (pieces are copied in order on one stream: the last one's completion covers all)
            r[-1][1].wait(torch.cuda.current_stream(torch.device(device)))


class _Piece:
    """One piece of a background upload: the host learns that its DMA has been ENQUEUED (an
    event set by the uploader thread) and then orders a stream after the DMA itself."""

    def __init__(self):
        self._enq = threading.Event()
        self._ev = None
        self._err = None

    def done(self, ev):
        self._ev = ev
        self._enq.set()

    def fail(self, err):
        self._err = err
        self._enq.set()

    def wait(self, stream):
        self._enq.wait()
        if self._err is not None:
            raise RuntimeError("device upload of the input bytes failed") from self._err
        stream.wait_event(self._ev)


class PinnedFile(_Resident):
    """``host``: pinned uint8 tensor with the file's bytes; ``data``: a numpy view of it (what the
    scanner indexes/slices on the host)."""

    def __init__(self, path: str, lo: int, hi: int):
        """Bytes [lo, hi) of ``path`` (the whole file, or one rank's shard)."""
        self.path = path
        self.lo = lo
        self.nbytes = nbytes = hi - lo
        self._dev = {}  # (device, lo, hi) -> uint8 device tensor
        self._ready = {}  # (device, lo, hi) -> [(end, event)] of an upload not yet waited on
        self.type_hints = {}  # (lo, hi, sep) -> column type codes of the last device scan
        self.scan_facts = {}  # (lo, hi, sep, opts, user types) -> types / nulls / line count (ops/scanfuse)
        self.host = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
        self.data = self.host.numpy()
        fd = os.open(path, os.O_RDONLY)
        try:
            mv = memoryview(self.data)

            def read(off):
                end = min(nbytes, off + _SLICE)
                pos = off
                while pos < end:
                    got = os.preadv(fd, [mv[pos:end]], lo + pos)
                    if got <= 0:
                        raise OSError(f"short read of {path} at {lo + pos}")
                    pos += got

            list(_readers().map(read, range(0, nbytes, _SLICE)))
        finally:
            os.close(fd)

    def live(self) -> bool:
        """Still the cache's entry (not evicted, not superseded by a changed file, not cleared)."""
        return _live(self, _cache)

    def device_bytes(self, device, lo: int = 0, hi: int = -1, progressive: bool = False) -> torch.Tensor:
        """The bytes [lo, hi) resident in HBM (async DMA on first use, then reused).

        The first upload runs in 1 GiB pieces on a side stream (direct DMA from the page-locked
        copy).  ``progressive``: the caller consumes the bytes in order and waits per piece
        (:meth:`take_ready`: the first action's device scan parses piece k while piece k + 1 is
        in flight, instead of after the whole file); otherwise the current stream waits for the
        whole upload here."""
        hi = self.nbytes if hi < 0 else hi
        key = (str(device), lo, hi)
        t = self._dev.get(key)
        if t is None:
            from .streams import side_stream

            dev = torch.device(device)
            t = torch.empty(hi - lo, dtype=torch.uint8, device=dev)
            side = side_stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))  # t's allocation is ordered before the copies
            ready = []
            with torch.cuda.stream(side):
                for a in range(lo, hi, _UPLOAD_PIECE):
                    b = min(hi, a + _UPLOAD_PIECE)
                    t[a - lo:b - lo].copy_(self.host[a:b], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(side)
                    ready.append((b - lo, ev))
            t.record_stream(side)
            self._dev[key] = t
            self._ready[key] = ready
        if not progressive:
            self.wait_ready(device, lo, hi)
        return t


_UPLOAD_PIECE = 1 << 30  # first-upload piece (one event each; the device scan's chunks are >= 1 GiB)

# HBM kept free for everything an action allocates besides the cached input bytes (parsed columns
# of an eager scan, Gram partials, the staging ring, the caching allocator's slack)
HEADROOM_FRACTION = 0.25
HEADROOM_MIN = 24 << 30


def device_cap_bytes(device=None) -> int:
    """Bytes of input the device cache may hold: ``DQ4ML_FILECACHE_DEVICE_BYTES`` if set, else what
    the device has free now (plus what this cache already holds) minus a headroom of 25 % of the
    HBM, at least 24 GiB -- about 190 GB of a 288 GB MI355X; the cap is no longer a fixed 64 GiB."""
    env = os.environ.get("DQ4ML_FILECACHE_DEVICE_BYTES")
    if env:
        return int(float(env))
    if not torch.cuda.is_available():
        return 0
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    free, total = torch.cuda.mem_get_info(dev)
    held = _held(dev)
    return max(0, int(free) + held - max(int(total * HEADROOM_FRACTION), HEADROOM_MIN))


def _held(dev=None) -> int:
    entries = list(_cache.values()) + list(_mapped.values())
    return sum(t.numel() for pf in entries for k, t in pf._dev.items() if dev is None or k[0] == str(dev))


def device_bytes_allowed(nbytes: int, device=None) -> bool:
    """Device residency within the cap, counting the cached entries."""
    return _held(None if device is None else torch.device(device)) + nbytes <= device_cap_bytes(device)


def _live(entry, table) -> bool:
    with _lock:
        return any(v is entry for v in table.values())


class MappedFile(_Resident):
    """A byte range too large for the pinned host cache: a read-only map of the file, plus the same
    per-range facts a ``PinnedFile`` keeps (the device scan's type hints and scan facts) and its
    HBM-resident copy when the device cache allows one (filled piece by piece through two pinned
    bounce buffers, never a whole-range host copy)."""

    host = None  # no page-locked copy: pieces are staged

    def __init__(self, path: str, lo: int, hi: int):
        self.path, self.lo, self.nbytes = path, lo, hi - lo
        self._map = map_readonly(path)
        self.data = memoryview(self._map)[lo:hi]
        self._dev = {}
        self._ready = {}
        self.type_hints = {}
        self.scan_facts = {}

    def live(self) -> bool:
        return _live(self, _mapped)

    def device_bytes(self, device, lo: int = 0, hi: int = -1, progressive: bool = False) -> torch.Tensor:
        """The bytes [lo, hi) resident in HBM.  The first call starts an uploader thread: per
        1 GiB piece, a parallel host memcpy from the map into a pinned bounce buffer, then a DMA
        straight into the resident tensor on the side stream (two bounce buffers: piece k + 1's
        memcpy overlaps piece k's DMA).  ``progressive`` as for :meth:`PinnedFile.device_bytes`:
        the caller's scan parses piece k while later pieces are still being read and copied."""
        hi = self.nbytes if hi < 0 else hi
        key = (str(device), lo, hi)
        t = self._dev.get(key)
        if t is None:
            from .streams import side_stream

            dev = torch.device(device)
            t = torch.empty(hi - lo, dtype=torch.uint8, device=dev)
            side = side_stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))  # t's allocation is ordered before the copies
            t.record_stream(side)
            spans = [(a, min(hi, a + _UPLOAD_PIECE)) for a in range(lo, hi, _UPLOAD_PIECE)]
            pieces = [_Piece() for _ in spans]
            self._dev[key] = t
            self._ready[key] = [(b - lo, p) for (_, b), p in zip(spans, pieces)]
            threading.Thread(target=self._upload, args=(t, dev, side, lo, spans, pieces, key), daemon=True,
                             name="dq4ml-upload").start()
        if not progressive:
            self.wait_ready(device, lo, hi)
        return t

    def _upload(self, t, dev, side, lo, spans, pieces, key):
        from .streams import _parallel_copy

        try:
            with torch.cuda.device(dev):
                width = max(b - a for a, b in spans)
                bounce = [torch.empty(width, dtype=torch.uint8, pin_memory=True) for _ in range(min(2, len(spans)))]
                copied = [None] * len(bounce)
                for i, ((a, b), p) in enumerate(zip(spans, pieces)):
                    k = i % len(bounce)
                    if copied[k] is not None:
                        copied[k].synchronize()  # the bounce buffer's previous DMA has drained
                    _parallel_copy(bounce[k][:b - a].numpy(), np.frombuffer(self.data, dtype=np.uint8, count=b - a,
                                                                            offset=a))
                    with torch.cuda.stream(side):
                        t[a - lo:b - lo].copy_(bounce[k][:b - a], non_blocking=True)
                        ev = torch.cuda.Event()
                        ev.record(side)
                    copied[k] = ev
                    p.done(ev)
                for ev in copied:
                    if ev is not None:
                        ev.synchronize()
        except BaseException as e:  # every waiter raises instead of hanging
            if self._dev.get(key) is t:  # an incomplete copy must never serve a later read
                self._dev.pop(key, None)
                self._ready.pop(key, None)
            for p in pieces:
                if not p._enq.is_set():
                    p.fail(e)


_mapped: "OrderedDict[tuple, MappedFile]" = OrderedDict()


def open_mapped(path: str, lo: int = 0, hi: int = -1) -> MappedFile:
    """The (cached) :class:`MappedFile` of bytes [lo, hi) of ``path``, keyed like ``open_pinned``."""
    st = os.stat(path)
    hi = st.st_size if hi < 0 else hi
    key = (os.path.realpath(path), st.st_size, st.st_mtime_ns, lo, hi)
    with _lock:
        mf = _mapped.get(key)
        if mf is not None:
            _mapped.move_to_end(key)
            return mf
        for k in [k for k in _mapped if k[0] == key[0] and k[1:3] != key[1:3]]:
            del _mapped[k]
        mf = _mapped[key] = MappedFile(path, lo, hi)
        while len(_mapped) > MAX_FILES:
            _mapped.popitem(last=False)
        return mf


def map_readonly(path: str):
    """Read-only shared map of a whole file (for ranges larger than the pinned cache)."""
    import mmap

    with open(path, "rb") as f:
        return mmap.mmap(f.fileno(), 0, flags=mmap.MAP_SHARED, prot=mmap.PROT_READ)


def shard_range(path: str, rank: int, world: int):
    """``ops.csvscan.shard_byte_range`` computed with small reads around the two cut points (a
    row belongs to the shard holding its first byte) — a rank never reads the whole file."""
    n = os.path.getsize(path)

    def align(p, f):
        if p <= 0:
            return 0
        if p >= n:
            return n
        # advance past the terminator that ends the row containing byte p - 1
        pos = p - 1
        while pos < n:
            f.seek(pos)
            win = f.read(1 << 16)
            hits = [x for x in (win.find(b"\n"), win.find(b"\r")) if x >= 0]
            if hits:
                q = pos + min(hits) + 1  # just past the terminator
                if q < n and win[q - 1 - pos:q - pos] == b"\r":
                    f.seek(q)
                    if f.read(1) == b"\n":
                        q += 1
                return min(q, n)
            pos += len(win)
        return n

    with open(path, "rb") as f:
        return align(n * rank // world, f), align(n * (rank + 1) // world, f)


def open_pinned(path: str, lo: int = 0, hi: int = -1) -> PinnedFile:
    st = os.stat(path)
    hi = st.st_size if hi < 0 else hi
    key = (os.path.realpath(path), st.st_size, st.st_mtime_ns, lo, hi)
    with _lock:
        pf = _cache.get(key)
        if pf is not None:
            _cache.move_to_end(key)
            return pf
        # the file changed (size or mtime differ): drop its stale copies; other byte ranges of
        # an unchanged file stay cached
        for k in [k for k in _cache if k[0] == key[0] and k[1:3] != key[1:3]]:
            del _cache[k]
        pf = PinnedFile(path, lo, hi)
        _cache[key] = pf
        while len(_cache) > MAX_FILES or (len(_cache) > 1 and sum(p.nbytes for p in _cache.values()) > MAX_BYTES):
            _cache.popitem(last=False)
        return pf


def clear():
    with _lock:
        _cache.clear()
        _mapped.clear()
