"""Page-locked, read-only file mappings for zero-copy CSV ingest.

A large input file is mapped once (``mmap``, pre-faulted) and registered with the HIP runtime as
read-only host memory (``hipHostRegister(..., hipHostRegisterReadOnly)``), so the device DMA
engines read the page cache directly: no ``read()`` copy, no pinned bounce buffer, ~57 GB/s H2D on
the MI355X box (1 GB in 17 ms).  Registration pins the pages once (~0.2 s per GB on first use),
so mappings are cached per ``(path, size, mtime)`` — every Spark action re-scans the file
(S20), and a changed file gets a new mapping.  If registration is unavailable the mapping is
still used through the pinned staging ring (``runtime.streams.StagingRing``)."""
from __future__ import annotations

import mmap
import os
import threading
import warnings
from collections import OrderedDict
from typing import Optional

import numpy as np
import torch

__all__ = ["MappedFile", "open_mapped", "clear"]

_HIP_HOST_REGISTER_READ_ONLY = 0x08
_cache: "OrderedDict[tuple, MappedFile]" = OrderedDict()
_lock = threading.Lock()
MAX_CACHED = int(os.environ.get("DQ4ML_HOSTMAP_FILES", "2"))


class MappedFile:
    def __init__(self, path: str):
        self.path = path
        with open(path, "rb") as f:
            self.mm = mmap.mmap(f.fileno(), 0, flags=mmap.MAP_SHARED | getattr(mmap, "MAP_POPULATE", 0),
                                prot=mmap.PROT_READ)
        self.nbytes = len(self.mm)
        self._ptr = np.frombuffer(self.mm, dtype=np.uint8).ctypes.data if self.nbytes else 0
        self.host: Optional[torch.Tensor] = None  # page-locked view (None: not registered)
        self._registered = False
        if self.nbytes and torch.cuda.is_available():
            try:
                r = torch.cuda.cudart().cudaHostRegister(self._ptr, self.nbytes, _HIP_HOST_REGISTER_READ_ONLY)
                self._registered = int(r) == 0
            except Exception:
                self._registered = False
            if self._registered:
                with warnings.catch_warnings():
                    warnings.simplefilter("ignore")  # the mapping is read-only by design
                    self.host = torch.frombuffer(self.mm, dtype=torch.uint8)

    def close(self):
        self.host = None
        if self._registered:
            torch.cuda.synchronize()  # no DMA may still read the pages
            torch.cuda.cudart().cudaHostUnregister(self._ptr)
            self._registered = False
        try:
            self.mm.close()
        except BufferError:  # a view still alive: unmapped when it is collected
            pass


def open_mapped(path: str) -> MappedFile:
    st = os.stat(path)
    key = (os.path.realpath(path), st.st_size, st.st_mtime_ns)
    with _lock:
        mf = _cache.get(key)
        if mf is not None:
            _cache.move_to_end(key)
            return mf
        for k in [k for k in _cache if k[0] == key[0]]:  # the file changed: drop the stale mapping
            _cache.pop(k).close()
        mf = _cache[key] = MappedFile(path)
        while len(_cache) > MAX_CACHED:
            _cache.popitem(last=False)[1].close()
        return mf


def clear():
    with _lock:
        while _cache:
            _cache.popitem()[1].close()
