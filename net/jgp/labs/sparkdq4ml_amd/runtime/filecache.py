"""Host (pinned) and device (HBM) caches of input files for CSV ingest.

A large input file is read ONCE into page-locked host memory (parallel ``preadv`` into a pinned
buffer) and kept, keyed by ``(path, size, mtime)``: every Spark action re-scans its input (S20),
and each re-scan then streams the cached bytes to the device by direct DMA (~57 GB/s H2D on the
MI355X box, 1 GB in 17 ms) with no host copy at all.  A rewritten file gets a new entry.

With ``dq4ml.csv.deviceCache`` (default on) the raw bytes of the rank's byte range also stay
resident in HBM (288 GB per MI355X): a re-scan then parses straight from device memory — the
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

import torch

__all__ = ["PinnedFile", "open_pinned", "shard_range", "map_readonly", "device_bytes_allowed", "clear"]

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


class PinnedFile:
    """``host``: pinned uint8 tensor with the file's bytes; ``data``: a numpy view of it (what the
    scanner indexes/slices on the host)."""

    def __init__(self, path: str, lo: int, hi: int):
        """Bytes [lo, hi) of ``path`` (the whole file, or one rank's shard)."""
        self.path = path
        self.lo = lo
        self.nbytes = nbytes = hi - lo
        self._dev = {}  # (device, lo, hi) -> uint8 device tensor
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


    def device_bytes(self, device, lo: int = 0, hi: int = -1) -> torch.Tensor:
        """The bytes [lo, hi) resident in HBM (one async DMA on first use, then reused)."""
        hi = self.nbytes if hi < 0 else hi
        key = (str(device), lo, hi)
        t = self._dev.get(key)
        if t is None:
            t = self._dev[key] = self.host[lo:hi].to(device, non_blocking=True)
        return t


MAX_DEVICE_BYTES = int(float(os.environ.get("DQ4ML_FILECACHE_DEVICE_BYTES", str(64 << 30))))


def device_bytes_allowed(nbytes: int) -> bool:
    """Device residency within the cap, counting the cached entries."""
    used = sum(t.numel() for pf in _cache.values() for t in pf._dev.values())
    return used + nbytes <= MAX_DEVICE_BYTES


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
