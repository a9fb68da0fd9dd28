"""In-tree build of the two native modules.

* ``_dq4ml_host``  — host C++17 runtime (solvers, CSV scanner), g++ -O3.
* ``_dq4ml_hip``   — gfx950 HIP kernels (MFMA Gram, fused DQ VM, compaction, predict/metrics,
  device CSV scan) + their host launchers, ``hipcc --offload-arch=gfx950``.

Both are plain pybind11 extension modules written next to this file, so the built ``.so`` travels
with a ``gpurun`` snapshot and is what ``import`` loads (no JIT cache outside the tree).  The HIP
module links the HIP runtime that PyTorch ships (same SONAME ``libamdhip64.so.7``) so kernels and
torch share one runtime, one device context and the same streams.
"""
from __future__ import annotations

import fcntl
import glob
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
HOST_SO = os.path.join(HERE, "_dq4ml_host" + EXT)
HIP_SO = os.path.join(HERE, "_dq4ml_hip" + EXT)
ARCH = os.environ.get("DQ4ML_OFFLOAD_ARCH", "gfx950")


def _py_includes():
    import pybind11

    return [f"-I{sysconfig.get_paths()['include']}", f"-I{pybind11.get_include()}"]


def _sources(sub, exts):
    out = []
    for e in exts:
        out += glob.glob(os.path.join(CSRC, sub, "*" + e))
    return sorted(out)


def _stale(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    deps = list(sources)
    for sub in ("host", "hip"):
        deps += glob.glob(os.path.join(CSRC, sub, "*.h"))
    return any(os.path.getmtime(s) > t for s in deps)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("native build failed:\n" + " ".join(cmd) + "\n" + r.stdout[-8000:])
    return r.stdout


class _Lock:
    def __init__(self, name):
        self.path = os.path.join(HERE, f".{name}.lock")

    def __enter__(self):
        self.f = open(self.path, "w")
        fcntl.flock(self.f, fcntl.LOCK_EX)
        return self

    def __exit__(self, *a):
        fcntl.flock(self.f, fcntl.LOCK_UN)
        self.f.close()


def build_host(force: bool = False) -> str:
    srcs = _sources("host", [".cpp"])
    with _Lock("host"):
        if force or _stale(HOST_SO, srcs):
            tmp = HOST_SO + f".tmp{os.getpid()}"
            cxx = os.environ.get("CXX", "g++")
            _run([cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden", "-Wall",
                  *_py_includes(), *srcs, "-o", tmp])
            os.replace(tmp, HOST_SO)
    return HOST_SO


def _torch_lib():
    import torch

    return os.path.join(os.path.dirname(torch.__file__), "lib")


def _obj_stale(obj, src, headers):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(s) > t for s in [src, *headers])


def build_hip(force: bool = False) -> str:
    """One object per translation unit under ``ops/.obj/`` (compiled in parallel, only the stale
    ones: a kernel edit recompiles one file, not the module), then one link."""
    srcs = _sources("hip", [".hip", ".cpp"])
    headers = glob.glob(os.path.join(CSRC, "hip", "*.h"))
    objdir = os.path.join(HERE, ".obj")
    with _Lock("hip"):
        if force or _stale(HIP_SO, srcs):
            from concurrent.futures import ThreadPoolExecutor

            os.makedirs(objdir, exist_ok=True)
            hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
            tl = _torch_lib()
            flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden",
                     "-munsafe-fp-atomics", *_py_includes(), f"-I{os.path.join(CSRC, 'hip')}",
                     *os.environ.get("DQ4ML_HIPCC_EXTRA", "").split()]  # A/B builds (-D knobs)
            objs = [os.path.join(objdir, os.path.basename(s) + ".o") for s in srcs]
            todo = [(s, o) for s, o in zip(srcs, objs) if force or _obj_stale(o, s, headers)]

            def cc(so):
                s, o = so
                tmp = o + f".tmp{os.getpid()}"
                _run([hipcc, *flags, "-c", s, "-o", tmp])
                os.replace(tmp, o)

            jobs = max(1, min(len(todo), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16))
            with ThreadPoolExecutor(jobs) as ex:
                list(ex.map(cc, todo))
            tmp = HIP_SO + f".tmp{os.getpid()}"
            _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs,
                  f"-L{tl}", "-lamdhip64", "-lhiprtc", f"-Wl,-rpath,{tl}", "-o", tmp])
            os.replace(tmp, HIP_SO)
    return HIP_SO


def build_all(force: bool = False):
    return build_host(force), build_hip(force)


if __name__ == "__main__":
    force = "--force" in sys.argv
    which = [a for a in sys.argv[1:] if not a.startswith("--")] or ["host", "hip"]
    for w in which:
        print({"host": build_host, "hip": build_hip}[w](force))
