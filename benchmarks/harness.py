"""Shared timing harness of the BASELINE.json config benchmarks (same contract as ``bench.py``):
W untimed warm-up steps, then exactly K steps bracketed by barrier + device synchronize on both
sides, the MAX over ranks, one JSON line from rank 0."""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


LAST_ISSUE_S = 0.0


def timed(step, steps: int, warmup: int, dev):
    import torch

    from net.jgp.labs.sparkdq4ml_amd.parallel import comm

    on_gpu = dev.type == "cuda"
    out = None
    for _ in range(warmup):
        out = step()
    if on_gpu:
        torch.cuda.synchronize()
    comm.barrier()
    if on_gpu:
        torch.cuda.synchronize()
    prof = None
    if os.environ.get("DQ4ML_BENCH_CPROFILE"):  # host-side profile of the timed steps only
        import cProfile

        prof = cProfile.Profile()
        prof.enable()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = step()
    global LAST_ISSUE_S  # host time to issue the timed steps (async device work: < el unless host-bound)
    LAST_ISSUE_S = time.perf_counter() - t0
    if on_gpu:
        torch.cuda.synchronize()
    if prof is not None:
        prof.disable()
        prof.dump_stats(os.environ["DQ4ML_BENCH_CPROFILE"])
    comm.barrier()
    if on_gpu:
        torch.cuda.synchronize()
    el = time.perf_counter() - t0
    el = float(comm.all_reduce_max(torch.tensor([el], dtype=torch.float64, device=dev)).item())
    return el, out


def emit(line: dict, json_out=None):
    from net.jgp.labs.sparkdq4ml_amd.parallel import comm

    if comm.rank() == 0:
        s = json.dumps(line)
        print(s, flush=True)
        if json_out:
            with open(json_out, "w") as f:
                f.write(s + "\n")
