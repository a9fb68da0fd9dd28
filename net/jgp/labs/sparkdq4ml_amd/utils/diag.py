"""The one gate of the wrong-result diagnostic builds.

Some code generators can emit timing-only ABLATIONS of their kernels -- phases removed, results
wrong -- to attribute a kernel's time on the GPU box (``DQ4ML_CUT_ABLATE`` for the CSV field
cutter, ``ops/scancut.py``; ``DQ4ML_SCAN_ABL`` for the per-line scan, ``ops/scanfuse.py``).  They
are profiling tools, never product behaviour: an ablation knob is honoured only with
``DQ4ML_DIAG=1`` set as well, and set WITHOUT it the engine refuses to run rather than return wrong
numbers."""
from __future__ import annotations

import os

__all__ = ["ablation", "enabled"]


def enabled() -> bool:
    return os.environ.get("DQ4ML_DIAG", "0") == "1"


def ablation(name: str) -> int:
    """The bit mask of the wrong-result ablation env knob ``name`` (0: the real kernel)."""
    v = int(os.environ.get(name, "0") or 0)
    if v and not enabled():
        raise RuntimeError(f"{name}={v} builds a timing-only kernel with WRONG results; it is honoured only "
                           "for profiling, with DQ4ML_DIAG=1 set as well")
    return v
