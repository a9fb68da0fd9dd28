#!/usr/bin/env python3
"""The BASELINE scaling curve in one invocation: every config benchmark at N = 1, 2, 4, 8 ranks
(one process per GPU, launched exactly as the driver launches ``bench.py``:
``python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1``), then
the X1 bucket sweep at the largest N.  Writes one JSON line per run to ``--out`` (JSONL) and prints
a markdown table of value, ms per step and scaling efficiency per config.

    python scripts/scale_curve.py --gpus 1,2,4,8 --out gpurun_out/scale.jsonl     # an 8-GPU node
    python scripts/scale_curve.py --gpus 1,2 --configs headline --quick           # CPU / gloo rehearsal

Efficiency: strong scaling (``bench.py``, config 5, l-bfgs: fixed total rows) = value(N) / (N *
value(1)); weak scaling (config 4: fixed rows per GPU) = value(N) / (N * value(1)) as well, since
``value`` is always the whole-job aggregate rows/s.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# name -> (script, full-size args, quick args for a CPU rehearsal)
CONFIGS = {
    "headline": ("bench.py", ["--steps", "50", "--warmup", "5"], ["--rows", "40000", "--steps", "2", "--warmup", "1"]),
    "cfg4": ("benchmarks/bench_dq_pipeline.py", ["--steps", "5", "--warmup", "2"],
             ["--rows-per-gpu", "20000", "--features", "16", "--steps", "1", "--warmup", "1"]),
    "cfg5": ("benchmarks/bench_wide.py", ["--steps", "12", "--warmup", "3"], ["--steps", "1", "--warmup", "1"]),
    "csv32": ("benchmarks/bench_csv_pipeline.py", ["--features", "32", "--rows", "1e8", "--steps", "5", "--warmup", "1"],
              ["--rows", "40000", "--steps", "1", "--warmup", "1"]),
    "lbfgs": ("benchmarks/bench_lbfgs.py", ["--steps", "2", "--warmup", "1"],
              ["--features", "4100", "--rows", "4000", "--max-iter", "15", "--steps", "1", "--warmup", "1"]),
}


def run_one(name: str, n: int, quick: bool, port: int, timeout: float):
    script, full, small = CONFIGS[name]
    args = (small if quick else full) + ["--gpus", str(n)]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, script)] + args
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    t0 = time.time()
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{") and '"metric"' in ln]
    rec = {"config": name, "n": n, "rc": p.returncode, "wall_s": round(time.time() - t0, 1)}
    if p.returncode == 0 and lines:
        rec["result"] = json.loads(lines[-1])
    else:
        rec["stderr_tail"] = p.stderr[-2000:]
    return rec


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", default="1,2,4,8")
    ap.add_argument("--configs", default=",".join(CONFIGS))
    ap.add_argument("--quick", action="store_true", help="small shapes (CPU / gloo plumbing rehearsal)")
    ap.add_argument("--sweep", action="store_true", help="also run scripts/bucket_sweep.py at the largest N")
    ap.add_argument("--out", default=None)
    ap.add_argument("--timeout", type=float, default=900)
    ap.add_argument("--port", type=int, default=29611)
    a = ap.parse_args(argv)
    ns = [int(x) for x in a.gpus.split(",")]
    recs = []
    port = a.port
    for name in a.configs.split(","):
        for n in ns:
            port += 1
            r = run_one(name, n, a.quick, port, a.timeout)
            recs.append(r)
            print(json.dumps(r), flush=True)
            if a.out:
                with open(a.out, "a") as f:
                    f.write(json.dumps(r) + "\n")
            if r["rc"] != 0:
                break  # a failed N: the larger ones would fail the same way
    if a.sweep:
        n = max(ns)
        port += 1
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "scripts", "bucket_sweep.py")]
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=a.timeout, cwd=ROOT)
        for ln in p.stdout.splitlines():
            if ln.startswith("{"):
                print(ln, flush=True)
                if a.out:
                    with open(a.out, "a") as f:
                        f.write(json.dumps({"config": "bucket_sweep", "n": n, "result": json.loads(ln)}) + "\n")
    # the table
    print("\n| config | N | value | unit | ms/step | efficiency vs N=1 |\n|---|---|---|---|---|---|")
    base = {}
    for r in recs:
        res = r.get("result")
        if res is None:
            print(f"| {r['config']} | {r['n']} | failed (rc {r['rc']}) | | | |")
            continue
        v = float(res["value"])
        if r["n"] == 1 or r["config"] not in base:
            base[r["config"]] = (r["n"], v)
        n0, v0 = base[r["config"]]
        eff = v / (v0 * r["n"] / n0)
        print(f"| {r['config']} | {r['n']} | {v:.4g} | {res.get('unit', '')} | {float(res['ms_per_step']):.4g} | "
              f"{eff:.3f} |")
    return 0 if all(r["rc"] == 0 for r in recs) else 1


if __name__ == "__main__":
    sys.exit(main())
