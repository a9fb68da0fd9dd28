"""Print why the generic DQ codegen declines a chain in the config-4 pipeline (diagnostic)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

sys.argv = [sys.argv[0], "--rows-per-gpu", "1e6", "--steps", "1", "--warmup", "0"]
from net.jgp.labs.sparkdq4ml_amd.ops import dqvm

_orig = dqvm.compile_chain


def traced(nodes, base):
    try:
        return _orig(nodes, base)
    except dqvm.Unfusable as e:
        print("UNFUSABLE:", repr(e), [type(n).__name__ for n in nodes], flush=True)
        raise


dqvm.compile_chain = traced
from benchmarks import bench_dq_pipeline  # noqa: E402

bench_dq_pipeline.main()
