"""Loader for the native modules.

``host()`` always works (builds with g++ on first use if the in-tree ``.so`` is missing/stale).
``hip()`` loads the gfx950 kernel module; on a machine with a GPU a missing or broken module is a
hard error — device ops never fall back silently to PyTorch.
"""
from __future__ import annotations

import importlib
import os
import threading

from . import build

_lock = threading.Lock()
_host = None
_hip = None
_hip_err = None


def _import(modname, builder):
    try:
        if build._stale(os.path.join(build.HERE, modname + build.EXT),
                        build._sources("host" if "host" in modname else "hip",
                                       [".cpp", ".hip"])):
            builder()
    except Exception:
        if not os.path.exists(os.path.join(build.HERE, modname + build.EXT)):
            raise
    return importlib.import_module(f"{__package__}.{modname}")


def host():
    global _host
    if _host is None:
        with _lock:
            if _host is None:
                _host = _import("_dq4ml_host", build.build_host)
    return _host


def hip():
    """The gfx950 kernel module.  Raises if it cannot be loaded."""
    global _hip, _hip_err
    if _hip is None:
        with _lock:
            if _hip is None:
                import torch  # noqa: F401  (torch's libamdhip64 must be loaded first)

                try:
                    _hip = _import("_dq4ml_hip", build.build_hip)
                except Exception as e:  # pragma: no cover - exercised on GPU boxes
                    _hip_err = e
                    raise RuntimeError(f"dq4ml HIP extension unavailable: {e}") from e
    return _hip


def hip_available() -> bool:
    try:
        hip()
        return True
    except Exception:
        return False
