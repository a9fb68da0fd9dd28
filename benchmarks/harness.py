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


def self_launch(gpus: int, script: str, argv=None):
    """``bench.py``'s ``--gpus`` contract for the config benchmarks.  Returns an exit code the
    caller returns at once -- N ranks were started through ``parallel/launch.py`` (one process per
    GPU, BEFORE this process touches the GPU) or the launcher's world size disagrees (2) -- or None
    when this process is a rank and runs the benchmark."""
    if gpus > 1 and int(os.environ.get("WORLD_SIZE", "1")) != gpus:
        if "WORLD_SIZE" in os.environ:
            print(f"[bench] --gpus {gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}", file=sys.stderr)
            return 2
        from net.jgp.labs.sparkdq4ml_amd.parallel.launch import launch

        return launch(gpus, [os.path.abspath(script)] + list(sys.argv[1:] if argv is None else argv))
    return None


def check_world(gpus: int) -> bool:
    """After ``comm.init()``: the process group has exactly ``--gpus`` ranks (and GPUs exist)."""
    import torch

    from net.jgp.labs.sparkdq4ml_amd.parallel import comm

    if torch.cuda.is_available() and gpus > torch.cuda.device_count():
        print(f"[bench] --gpus {gpus} but only {torch.cuda.device_count()} visible GPU(s)", file=sys.stderr)
        return False
    if comm.world_size() != gpus:
        print(f"[bench] --gpus {gpus} but the process group has {comm.world_size()} rank(s)", file=sys.stderr)
        return False
    return True


def world_info(dev) -> dict:
    """``world`` / ``backend`` / ``rank_devices`` keys of the JSON line (collective: every rank calls)."""
    from net.jgp.labs.sparkdq4ml_amd.parallel import comm

    ranks = comm.all_gather_object({"rank": comm.rank(), "device": str(dev)})
    return {"world": comm.world_size(), "backend": comm.backend() or "none",
            "rank_devices": [r["device"] for r in ranks]}


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
