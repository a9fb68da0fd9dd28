"""``pip install -e .`` / ``python setup.py build_ext --inplace``: builds the two in-tree native
modules through ``net/jgp/labs/sparkdq4ml_amd/ops/build.py`` (host C++ runtime with g++, gfx950
HIP kernels with ``hipcc --offload-arch=gfx950``, per-file objects compiled in parallel) — the
same build ``__graft_entry__.build()`` runs.  The Maven POM analogue of the reference (POM:1-65)."""
import os
import sys

from setuptools import setup
from setuptools.command.build_ext import build_ext

ROOT = os.path.dirname(os.path.abspath(__file__))


class BuildNative(build_ext):
    def run(self):
        sys.path.insert(0, ROOT)
        from net.jgp.labs.sparkdq4ml_amd.ops import build as b

        b.build_host(force=self.force)
        b.build_hip(force=self.force)

    def get_outputs(self):
        return []


setup(cmdclass={"build_ext": BuildNative})
