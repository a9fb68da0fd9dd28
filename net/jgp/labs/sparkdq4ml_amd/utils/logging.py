"""Logging configuration — the Python analogue of the reference's log4j.properties
(``src/main/resources/log4j.properties:1-11``): application code at DEBUG, engine internals at
WARN, the same console pattern ``%d{yyyy-MM-dd HH:mm:ss.SSS} -%5p --- [%15.15t] %-40.40l: %m%n``.
``DQ4ML_LOG_LEVEL`` overrides the engine level."""
from __future__ import annotations

import logging
import os
import sys

ROOT = "net.jgp.labs.sparkdq4ml_amd"
_configured = False


class _Fmt(logging.Formatter):
    def format(self, r):
        ts = self.formatTime(r, "%Y-%m-%d %H:%M:%S") + f".{int(r.msecs):03d}"
        thread = (r.threadName or "")[-15:].rjust(15)
        loc = f"{r.name}.{r.funcName}({r.filename}:{r.lineno})"[:40].ljust(40)
        return f"{ts} -{r.levelname.replace('WARNING', 'WARN'):>5} --- [{thread}] {loc}: {r.getMessage()}"


def configure_logging():
    global _configured
    if _configured:
        return
    _configured = True
    h = logging.StreamHandler(sys.stderr)
    h.setFormatter(_Fmt())
    root = logging.getLogger(ROOT)
    root.addHandler(h)
    root.propagate = False
    root.setLevel(os.environ.get("DQ4ML_LOG_LEVEL", "ERROR").upper())
    logging.getLogger(ROOT + ".apps").setLevel(logging.DEBUG)


def get_logger(name: str) -> logging.Logger:
    return logging.getLogger(f"{ROOT}.{name}")
