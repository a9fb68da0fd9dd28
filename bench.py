#!/usr/bin/env python3
"""Headline benchmark: rows/sec of ``LinearRegression.fit`` on a synthetic 1e8 x 32 dataset
(BASELINE.json config #2/#3), bf16 normal equations, data-parallel over N MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--rows R] [--features D] [--dtype bf16]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One step = one full ``LinearRegression.fit`` through the engine on a DataFrame whose
``features`` column is an assembled (feature-major, bf16) device matrix and ``label`` an f32
column: fused MFMA Gram pass over the rank's shard -> RCCL all-reduce of the f64 statistics over
xGMI -> f64 normal-equation solve -> model.  Rows are sharded across ranks (strong scaling: the
global dataset is fixed at --rows).  Synthetic data, random-init coefficients; nothing is cached
between steps.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def _args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=float, default=1e8, help="global rows (strong scaling)")
    ap.add_argument("--features", type=int, default=32)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32", "fp32split", "fp64"],
                    help="compute precision of the Gram statistics (gramDtype; fp32split: f32 statistics "
                         "from split-bf16 products on f32 storage)")
    ap.add_argument("--storage", default=None, choices=["bf16", "fp32", "fp64", "f32cols"],
                    help="feature storage: an assembled [d, n] matrix of that dtype (default: the "
                         "--dtype; bf16 is ingested into the MFMA-fragment tiled layout), or "
                         "f32cols = d separate f32 columns assembled by VectorAssembler inside "
                         "every fit (fused assemble + Gram, gram_cols_kernel)")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"])
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--sync", dest="use_async", action="store_false",
                    help="synchronous fits (host WLS solve after a D2H of the statistics, every step)")
    ap.add_argument("--async", dest="use_async", action="store_true",
                    help="asynchronous fits (device WLS solve, no host wait per step; the default)")
    ap.set_defaults(use_async=True)
    return ap.parse_args(argv)


def _self_launch(a, argv) -> int:
    """``--gpus N`` without a launcher: start N ranks (one process per GPU) through
    ``parallel/launch.py`` BEFORE anything here touches the GPU, and return their exit code."""
    from net.jgp.labs.sparkdq4ml_amd.parallel.launch import launch

    args = list(sys.argv[1:] if argv is None else argv)
    return launch(a.gpus, [os.path.abspath(__file__)] + args)


def main(argv=None):
    a = _args(argv)
    if a.gpus > 1 and int(os.environ.get("WORLD_SIZE", "1")) != a.gpus:
        if "WORLD_SIZE" in os.environ:
            print(f"[bench] --gpus {a.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}", file=sys.stderr)
            return 2
        return _self_launch(a, argv)
    import torch

    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, SparkSession
    from net.jgp.labs.sparkdq4ml_amd.parallel import comm

    if torch.cuda.is_available() and a.gpus > torch.cuda.device_count():
        print(f"[bench] --gpus {a.gpus} but only {torch.cuda.device_count()} visible GPU(s)", file=sys.stderr)
        return 2
    comm.init()
    rank, world = comm.rank(), comm.world_size()
    if world != a.gpus:
        print(f"[bench] --gpus {a.gpus} but the process group has {world} rank(s)", file=sys.stderr)
        return 2
    # async (default): gram -> RCCL all-reduce -> device WLS solve (wls_small.hip) enqueued back
    # to back, the host never waits inside a step; every fit's solve still runs inside the timed
    # region (the closing synchronize), the model's coefficients materialize on first read.
    # --sync: D2H of the statistics + host solve every step (Spark's driver-side solve).
    # 1x MI355X, d = 32: 1e8 rows 1.043 (async) vs 1.075 (sync) ms; 1.25e7 rows 0.166 vs 0.201 ms.
    spark = SparkSession.builder().appName("bench").master("local[*]") \
        .config("dq4ml.fit.async", "true" if a.use_async else "false").getOrCreate()
    dev = spark.device
    on_gpu = dev.type == "cuda"

    total = int(a.rows)
    if not on_gpu:
        total = min(total, 2_000_000)  # host smoke run
    per_rank = total // world if a.scaling == "strong" else total
    lo = rank * per_rank
    n = per_rank if (a.scaling == "weak" or rank < world - 1) else total - lo
    d = a.features
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    storage = a.storage or ("fp32" if a.dtype == "fp32split" else a.dtype)
    store = {"bf16": torch.bfloat16, "fp32": torch.float32, "fp64": torch.float64,
             "f32cols": torch.float32}[storage]
    ld = (n + 63) // 64 * 64
    Xbuf = torch.empty(d, ld, dtype=store, device=dev)
    beta = torch.linspace(-2.0, 2.0, d, device=dev, dtype=torch.float32)
    y = torch.zeros(n, dtype=torch.float32, device=dev)
    chunk = 1 << 24
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        xc = torch.randn(d, e - s, generator=gen, device=dev, dtype=torch.float32)
        Xbuf[:, s:e] = xc.to(store)
        y[s:e] = beta @ xc + 0.5 + 0.1 * torch.randn(e - s, generator=gen, device=dev, dtype=torch.float32)
    X = Xbuf[:, :n]
    if storage == "f32cols":
        from net.jgp.labs.sparkdq4ml_amd import VectorAssembler

        names = [f"x{i}" for i in range(d)]
        cols = {nm: X[i] for i, nm in enumerate(names)}
        cols["label"] = y
        df = VectorAssembler().setInputCols(names).setOutputCol("features").transform(spark.createDataFrame(cols))
    else:
        df = spark.createDataFrame({"features": X, "label": y})
    lr = LinearRegression(solver="normal", gramDtype=a.dtype)

    def step():
        return lr.fit(df)

    for _ in range(a.warmup):
        model = step()
    if on_gpu:
        torch.cuda.synchronize()
    comm.barrier()
    if on_gpu:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        model = step()
    if on_gpu:
        torch.cuda.synchronize()
    comm.barrier()
    if on_gpu:
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    elapsed = float(comm.all_reduce_max(el).item())
    ranks = comm.all_gather_object({"rank": rank, "device": str(dev),
                                    "device_index": dev.index if on_gpu else None})

    global_rows = total if a.scaling == "strong" else total * world
    ms = elapsed / a.steps * 1e3
    value = global_rows * a.steps / elapsed
    coef = model.coefficients.toArray()
    err = float(abs(coef - beta.double().cpu().numpy()).max())
    if rank == 0:
        line = {
            "metric": "rows/sec LinearRegression.fit, 1e8x32 synthetic, at 1/2/4/8 MI355X",
            "value": value, "unit": "rows/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": ms, "higher_is_better": True, "scaling": a.scaling, "vs_baseline": None,
            "dtype": a.dtype, "data": "synthetic (random-init coefficients, N(0,1) features)",
            "config": {"model": f"LinearRegression(normal equations) d={d}", "global_batch": global_rows,
                       "seq_len": d, "parallelism": f"dp{world}", "rows_per_gpu": n,
                       "device": str(dev), "coef_max_abs_err": err, "storage": storage,
                       "fit_mode": "async" if (a.use_async and on_gpu) else "sync"},
            "world": world, "backend": comm.backend() or "none",
            "rccl_version": comm.rccl_version() if on_gpu else None,
            "rank_devices": [r["device"] for r in ranks],
        }
        s = json.dumps(line)
        print(s, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(s + "\n")
    comm.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
