#!/usr/bin/env python3
"""X1 bucket sweep for the wide Gram all-reduce (config 5: 1e7 x 4096 fp8).

The wide fit folds its f32 SYRK partials band by band and issues each band's RCCL all-reduce as
soon as it is folded (``ops/device.py`` ``_fold_all_reduce``).  The band size is
``dq4ml.bucketBytes``; the wire format ``dq4ml.allreduceWire`` (f32 | f64).  On xGMI every ring
step moves bucket / N bytes per link, so buckets must stay well above the per-step latency while
leaving more than one band to overlap: this script measures the whole statistics pass
(SYRK + banded fold + all-reduce) per (wire, bucket) and prints one JSON line each (rank 0, max over
ranks).  Rows are split over ranks (strong scaling, like the config).

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
        scripts/bucket_sweep.py [--rows 1e7] [--d 4096] [--eb 8] [--reps 3]
    DQ4ML_FORCE_COLLECTIVES=1 python scripts/bucket_sweep.py --rows 1e6     # one GPU, RCCL path
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1e7)
    ap.add_argument("--d", type=int, default=4096)
    ap.add_argument("--eb", type=int, default=8, choices=(8, 16))
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--buckets-mb", default="1,2,4,8,16,32,64")
    ap.add_argument("--wires", default="f32,f64")
    a = ap.parse_args(argv)

    import torch
    import torch.distributed as dist

    from net.jgp.labs.sparkdq4ml_amd.ops import device as devops
    from net.jgp.labs.sparkdq4ml_amd.parallel import comm

    comm.init()
    rank, world = comm.rank(), comm.world_size()
    dev = torch.device("cuda", torch.cuda.current_device())
    n = int(a.rows) // world
    g = torch.Generator(device=dev).manual_seed(11 + rank)
    X = torch.randn(a.d, n, generator=g, device=dev, dtype=torch.float32)
    y = torch.linspace(-1, 1, a.d, device=dev) @ X + 0.25
    T = devops.tile_wide(X, a.eb)
    del X
    compute = "fp8" if a.eb == 8 else "bf16"

    def one():
        return devops.gram_stats(T, y, None, None, compute)

    ref = None
    for wire in a.wires.split(","):
        comm.set_wire_dtype(wire)
        for mb in (float(x) for x in a.buckets_mb.split(",")):
            comm.set_bucket_bytes(int(mb * (1 << 20)))
            out = one()  # warmup (and the numerics check below)
            comm.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                one()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / a.reps * 1e3
            t = torch.tensor([ms], dtype=torch.float64, device=dev)
            if comm.collectives_active():
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
            if ref is None:
                ref = out.clone()
            rel = float(((out - ref).abs().max() / ref.abs().max().clamp_min(1e-300)).item())
            if rank == 0:
                print(json.dumps({"wire": wire, "bucket_mb": mb, "ms_per_pass": float(t.item()), "world": world,
                                  "rows_per_rank": n, "d": a.d, "eb": a.eb,
                                  "bands": len(devops.wide_bands((a.d + 255) // 256, a.d, comm.bucket_bytes(),
                                                                 4 if wire == "f32" else 8)),
                                  "max_rel_diff_vs_first": rel}), flush=True)
    comm.shutdown()


if __name__ == "__main__":
    main()
