"""``SparkSession`` equivalent (``SparkSession.builder().appName("DQ4ML").master("local[*]")
.getOrCreate()``, ``DataQuality4MachineLearningApp.java:38-41``).

``master`` selects the execution device, mirroring Spark's parallel-width string:

* ``local`` / ``local[N]`` / ``local[*]`` — this node; the session uses the node's MI355X (the
  GPU of this rank, ``LOCAL_RANK``) when one is visible, else host (CPU) execution;
* ``mi355x`` / ``mi355x[*]`` / ``gpu`` — require the GPU;
* ``cpu`` / ``local-cpu[*]`` — force host execution (the unit-test configuration).

Config keys (``.config(k, v)``): ``dq4ml.device``, ``dq4ml.gramDtype`` (fp64|fp32|bf16|fp8: the
default Gram precision of estimators that do not set ``gramDtype``), ``dq4ml.bucketBytes`` (RCCL
all-reduce bucket size), ``dq4ml.trace`` (per-stage tracing, ``utils.tracing``),
``dq4ml.csv.deviceThresholdBytes`` (smallest file the device CSV scanner takes),
``dq4ml.chunkBytes`` (device CSV streaming chunk, default 256 MiB), ``dq4ml.shardInput`` (byte-range
sharded reads across ranks, default true), ``dq4ml.fit.async`` (asynchronous normal-equation fits),
``dq4ml.healthCheck`` (once|always|never rank-health barrier before distributed fits),
``dq4ml.gram.reserveCUs`` (CUs the full-chip Gram passes leave free for the fit tail: fold, RCCL
all-reduce and solve start at once beside the next pass; default 0 on one GPU, see ops/device.py).
"""
from __future__ import annotations

import os
import re
import threading
from typing import Dict, Optional

import torch

from ..utils.logging import configure_logging, get_logger
from .dataframe import DataFrame
from .plan import LocalRelation
from .table import ColumnData, Table
from .types import (BooleanType, DoubleType, IntegerType, LongType, StringType, StructField,
                    StructType, VectorUDT)
from .udf import UDFRegistration

__all__ = ["SparkSession", "Catalog", "RuntimeConfig"]

log = get_logger("session")


class RuntimeConfig:
    def __init__(self, conf: Dict[str, str]):
        self._conf = conf

    def get(self, key, default=None):
        return self._conf.get(key, default)

    def set(self, key, value):
        self._conf[key] = str(value)

    def getAll(self):
        return dict(self._conf)

    def __call__(self):
        return self


class Catalog:
    def __init__(self):
        self._views = {}

    def dropTempView(self, name):
        return self._views.pop(name.lower(), None) is not None

    def listTables(self):
        return sorted(self._views)

    def tableExists(self, name):
        return name.lower() in self._views

    def __call__(self):
        return self


def master_width(master: str, device_type: str) -> int:
    """Parallel width of a master URL: ``mi355x[N]`` / ``gpu[N]`` / ``local[N]`` ->
    N; ``[*]`` -> every visible GPU on a GPU master, every core on a CPU one; no brackets -> 1."""
    m = re.match(r"^[a-z0-9_-]+\[(\*|\d+)(?:\s*,\s*\d+)?\]$", (master or "local[*]").strip().lower())
    if m is None:
        return 1
    if m.group(1) != "*":
        n = int(m.group(1))
        if n < 1:
            raise ValueError(f"invalid master '{master}': width must be >= 1")
        return n
    if device_type == "cuda":
        return max(1, torch.cuda.device_count())  # counting devices does not initialise HIP
    return os.cpu_count() or 1


def _spmd_width(master: str, conf: Dict[str, str], device: torch.device) -> int:
    """Ranks the session runs as: a GPU master's (``mi355x`` / ``gpu`` / ``cuda``) width is one
    process per GPU (RCCL over xGMI); ``local[N]`` and CPU masters keep Spark's meaning, N worker
    threads (``dq4ml.spmd=true`` makes them N gloo / RCCL ranks instead)."""
    width = master_width(master, device.type)
    gpu_master = (master or "").strip().lower().startswith(("mi355x", "gpu", "cuda"))
    spmd = str(conf.get("dq4ml.spmd", "true" if gpu_master else "false")).lower() in ("1", "true", "yes")
    if not spmd:
        if device.type == "cpu" and re.search(r"\[\d+", (master or "")):
            torch.set_num_threads(width)  # local[N]: N worker threads
        return 1
    return width


def _launch_width(master: str, width: int, explicit: bool) -> None:
    """Match the process group to the master's width: inside a launcher the group must have
    exactly ``width`` ranks; outside one an explicit ``[N]`` (N > 1) starts N ranks of THIS
    program (``parallel/launch.py``: children, never an exec) and the parent exits with their
    exit code — Spark's ``local[N]`` gives the app N workers the same way.  ``[*]`` outside a
    launcher stays one process (it must not fork a script that merely wants "whatever is here")."""
    import sys

    from ..parallel import comm

    world_env = int(os.environ.get("WORLD_SIZE", "0") or 0)
    if world_env or comm.is_initialized():
        world = comm.world_size() if comm.is_initialized() else world_env
        if explicit and world != width:
            raise ValueError(f"master '{master}' asks for {width} rank(s) but the process group has {world}")
        if world > 1:
            comm.init()
        return
    if width <= 1 or not explicit:
        return
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        raise RuntimeError(f"master '{master}': cannot start {width} ranks from a process that already "
                           f"initialised the GPU; run it under parallel/launch.py or torchrun")
    from ..parallel.launch import launch

    main = sys.modules.get("__main__")
    spec = getattr(main, "__spec__", None)
    if spec is not None and spec.name:
        argv, module = [spec.name] + sys.argv[1:], True
    elif sys.argv and sys.argv[0] and os.path.exists(sys.argv[0]):
        argv, module = [os.path.abspath(sys.argv[0])] + sys.argv[1:], False
    else:
        raise RuntimeError(f"master '{master}': no script to start {width} ranks of (interactive session); "
                           f"use parallel/launch.py or torchrun")
    raise SystemExit(launch(width, argv, module=module))


def _resolve_device(master: str, conf: Dict[str, str]) -> torch.device:
    forced = conf.get("dq4ml.device") or os.environ.get("DQ4ML_DEVICE")
    m = (master or "local[*]").lower()
    if forced:
        want = forced.lower()
    elif m.startswith("cpu") or m.startswith("local-cpu"):
        want = "cpu"
    elif m.startswith("mi355x") or m.startswith("gpu") or m.startswith("cuda"):
        want = "cuda"
    else:
        want = "auto"
    if want == "auto":
        want = "cuda" if torch.cuda.is_available() else "cpu"
    if want.startswith("cuda"):
        if not torch.cuda.is_available():
            raise RuntimeError(f"master '{master}' requires an MI355X but no GPU is visible")
        idx = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
        if ":" in want:
            idx = int(want.split(":")[1])
        torch.cuda.set_device(idx)
        return torch.device("cuda", idx)
    return torch.device("cpu")


class SparkSession:
    _active: Optional["SparkSession"] = None
    _lock = threading.RLock()

    class Builder:
        def __init__(self):
            self._conf: Dict[str, str] = {}

        def __call__(self):
            return SparkSession.Builder()

        def appName(self, name):
            self._conf["spark.app.name"] = name
            return self

        def master(self, m):
            self._conf["spark.master"] = m
            return self

        def config(self, key=None, value=None, conf=None):
            if conf is not None:
                self._conf.update(conf)
            elif key is not None:
                self._conf[key] = str(value)
            return self

        def enableHiveSupport(self):
            return self

        def getOrCreate(self) -> "SparkSession":
            with SparkSession._lock:
                s = SparkSession._active
                if s is not None and not s._stopped:
                    for k, v in self._conf.items():
                        if k not in ("spark.master",):
                            s.conf.set(k, v)
                    return s
                conf = dict(self._conf)
                master = conf.get("spark.master", "local[*]")
                want_cuda = not (str(conf.get("dq4ml.device") or os.environ.get("DQ4ML_DEVICE") or "").startswith("cpu")
                                 or master.lower().startswith(("cpu", "local-cpu")))
                dtype = "cuda" if want_cuda and torch.cuda.is_available() else "cpu"
                width = _spmd_width(master, conf, torch.device(dtype))
                _launch_width(master, width, bool(re.search(r"\[\d+", master)))
                s = SparkSession(conf)
                s.defaultParallelism = width
                SparkSession._active = s
                return s

    builder = Builder()

    def __init__(self, conf: Dict[str, str]):
        configure_logging()
        self._conf = conf
        self.conf = RuntimeConfig(conf)
        self.master = conf.get("spark.master", "local[*]")
        self.appName = conf.get("spark.app.name", "dq4ml")
        self.device = _resolve_device(self.master, conf)
        if str(conf.get("dq4ml.trace", "")).lower() in ("1", "true", "yes"):
            from ..utils import tracing

            tracing.enable(True)
        if conf.get("dq4ml.bucketBytes"):
            from ..parallel import comm

            comm.set_bucket_bytes(int(conf["dq4ml.bucketBytes"]))
        if conf.get("dq4ml.gram.reserveCUs") is not None:
            from ..ops import device as _dev

            _dev.set_gram_reserve(int(conf["dq4ml.gram.reserveCUs"]))
        if conf.get("dq4ml.allreduceWire"):
            from ..parallel import comm

            comm.set_wire_dtype(str(conf["dq4ml.allreduceWire"]).lower())
        if self.device.type == "cuda" and str(conf.get("dq4ml.rtc.prewarm", "true")).lower() in ("1", "true", "yes"):
            from ..ops import dqvm

            dqvm.prewarm()  # hipRTC's first compile loads the compiler: off the first action's path
        self.udf = UDFRegistration(self)
        self.catalog = Catalog()
        self._stopped = False
        log.debug("session %s on %s (master=%s)", self.appName, self.device, self.master)

    @classmethod
    def getActiveSession(cls):
        return cls._active

    # Java-style accessor spellings ------------------------------------------------------------
    @property
    def read(self):
        from .readwriter import DataFrameReader

        return DataFrameReader(self)

    def sql(self, text: str) -> DataFrame:
        from .parser import plan_sql

        return DataFrame(plan_sql(text, self), self)

    def table(self, name: str) -> DataFrame:
        from .expressions import AnalysisException

        p = self.catalog._views.get(name.lower())
        if p is None:
            raise AnalysisException(f"Table or view not found: {name}")
        return DataFrame(p, self)

    def range(self, start, end=None, step=1):
        if end is None:
            start, end = 0, start
        v = torch.arange(start, end, step, dtype=torch.int64, device=self.device)
        schema = StructType([StructField("id", LongType(), False)])
        return DataFrame(LocalRelation(Table(schema, [ColumnData(LongType(), v)], v.numel(), None, self.device)), self)

    def createDataFrame(self, data, schema=None) -> DataFrame:
        """From a list of rows/tuples/dicts, a pandas DataFrame or a dict of tensors."""
        from .localdata import table_from_data

        return DataFrame(LocalRelation(table_from_data(data, schema, self.device)), self)

    def stop(self):
        self._stopped = True
        if SparkSession._active is self:
            SparkSession._active = None

    close = stop

    def sparkContext(self):
        return self

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.stop()


_ = (BooleanType, DoubleType, IntegerType, StringType, VectorUDT)
