"""Host-side profile (cProfile) of one benchmark step: WHICH=cfg4|cfg5|lab, after warm-up."""
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))

which = os.environ.get("WHICH", "cfg4")
if which == "cfg4":
    import bench_dq_pipeline as B
    argv = ["--steps", "1", "--warmup", "1", "--rows-per-gpu", os.environ.get("ROWS", "1.25e8")]
elif which == "lab":
    import bench_csv_pipeline as B
    argv = ["--steps", "1", "--warmup", "1", "--rows", os.environ.get("ROWS", "1e6")]
else:
    import bench_wide as B
    argv = ["--steps", "1", "--warmup", "1", "--rows", os.environ.get("ROWS", "1e7")]

# reuse the benchmark's setup by capturing its step through harness.timed
import harness  # noqa: E402

captured = {}
orig = harness.timed


def grab(step, steps, warmup, dev):
    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step()
    torch.cuda.synchronize()
    print(f"[{which}] step wall ms {1e3 * (time.perf_counter() - t0):.2f}", flush=True)
    reps = int(os.environ.get("REPS", "1"))  # >1: issue REPS steps back to back (host cost per step)
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(reps):
        out = step()
    pr.disable()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"[{which}] {reps} steps issued in {1e3 * (t1 - t0) / reps:.3f} ms each (profiled)", flush=True)
    pstats.Stats(pr).sort_stats(os.environ.get("SORT", "cumulative")).print_stats(int(os.environ.get("TOP", "40")))
    return 1.0, out


B.timed = grab
B.main(argv)
