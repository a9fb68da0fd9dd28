"""One-process-per-GPU launcher (SURVEY.md §7b ``dist/launch.py``): a dependency-free equivalent
of ``torch.distributed.run --standalone`` for the SPMD engine.

    python -m net.jgp.labs.sparkdq4ml_amd.parallel.launch --nproc 8 bench.py --gpus 8
    python -m net.jgp.labs.sparkdq4ml_amd.parallel.launch --nproc 8 -m net.jgp.labs.sparkdq4ml_amd.apps.dq4ml_app

Every worker gets RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT (a free
port) and ``HSA_ENABLE_IPC_MODE_LEGACY=0``; workers are started as child processes (never exec'd
from a process that touched the GPU — this launcher itself never initializes HIP).  Fail-fast: the
first worker that exits non-zero takes the whole group down (SIGTERM, then SIGKILL after a grace
period) and its exit code is returned, so a dead rank never leaves the others hanging in a
collective.
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time
from typing import List

__all__ = ["launch", "main"]


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(nproc: int, argv: List[str], module: bool = False, port: int = 0, grace_s: float = 10.0,
           env_extra: dict = None) -> int:
    if nproc < 1:
        raise ValueError("nproc must be >= 1")
    port = port or _free_port()
    procs = []
    for r in range(nproc):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nproc), LOCAL_WORLD_SIZE=str(nproc),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        env.update(env_extra or {})
        cmd = [sys.executable] + (["-m"] if module else []) + list(argv)
        procs.append(subprocess.Popen(cmd, env=env, start_new_session=True))
    rc = 0
    try:
        alive = set(range(nproc))
        while alive:
            for r in list(alive):
                code = procs[r].poll()
                if code is None:
                    continue
                alive.discard(r)
                if code != 0 and rc == 0:
                    rc = code
                    print(f"[launch] rank {r} exited with {code}; stopping the group", file=sys.stderr)
                    _stop([p for i, p in enumerate(procs) if i in alive], grace_s)
                    alive.clear()
            time.sleep(0.05)
    except KeyboardInterrupt:
        _stop(procs, grace_s)
        rc = rc or 130
    return rc


def _stop(procs, grace_s):
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
    deadline = time.time() + grace_s
    for p in procs:
        while p.poll() is None and time.time() < deadline:
            time.sleep(0.05)
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait()


def main(argv=None):
    ap = argparse.ArgumentParser(description="one process per GPU (SPMD)")
    ap.add_argument("--nproc", type=int, default=int(os.environ.get("DQ4ML_NPROC", "1")))
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("-m", dest="module", action="store_true", help="run the target as a module")
    ap.add_argument("target", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    if not a.target:
        ap.error("missing script / module")
    return launch(a.nproc, a.target, module=a.module, port=a.port)


if __name__ == "__main__":
    sys.exit(main())
