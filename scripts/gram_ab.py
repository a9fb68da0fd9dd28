"""A/B of Gram kernel variants in ONE process (interleaved rounds), 1e8 x 32 bf16."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from net.jgp.labs.sparkdq4ml_amd.ops import device  # noqa: E402

n = int(float(os.environ.get("N", "1e8")))
d = int(os.environ.get("D", "32"))
rounds = int(os.environ.get("ROUNDS", "5"))
X = torch.randn(d, n, device="cuda").to(torch.bfloat16)
y = torch.randn(n, device="cuda")
T = device.tile_bf16(X)
ref = device.gram_stats(X, y, None, None, "bf16")
got = device.gram_stats(T, y, None, None, "bf16")
print("tiled vs plain max rel diff", float((got - ref).abs().max() / ref.abs().max()))
bytes_x = X.numel() * 2 + y.numel() * 4


def timeit(fn, reps=10):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


variants = {
    "plain": lambda: device.gram_stats(X, y, None, None, "bf16"),
    "tiled": lambda: device.gram_stats(T, y, None, None, "bf16"),
    "read_sum": lambda: torch.sum(T.buf.view(torch.int16), dtype=torch.int64),
    "copy": lambda: T.buf.clone(),
}
res = {k: [] for k in variants}
for r in range(rounds):
    for k, f in variants.items():
        res[k].append(timeit(f))
for k, v in res.items():
    v.sort()
    ms = v[len(v) // 2]
    gbs = (bytes_x if k in ("plain", "tiled") else T.buf.numel() * 2 * (2 if k == "copy" else 1)) / ms / 1e6
    print(f"{k:10s} median {ms:.3f} ms  min {v[0]:.3f}  -> {gbs:.0f} GB/s")
