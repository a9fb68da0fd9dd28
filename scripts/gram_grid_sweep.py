"""Tiled bf16 Gram time vs grid size at a given row count (default: the 8-GPU strong-scaling shard).

    N=1.25e7 D=32 python scripts/gram_grid_sweep.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from net.jgp.labs.sparkdq4ml_amd.ops import device, native  # noqa: E402


def main():
    n, d = int(float(os.environ.get("N", "1.25e7"))), int(os.environ.get("D", "32"))
    g = torch.Generator(device="cuda").manual_seed(0)
    X = torch.randn(d, n, generator=g, device="cuda").to(torch.bfloat16)
    y = torch.randn(n, generator=g, device="cuda")
    T = device.tile_bf16(X)
    del X
    h = native.hip()
    default = int(device._plan_blocks(h, 2, d, n, 2, 0))
    ref = device.gram_stats(T, y, None, None, "bf16")
    print(f"n={n} d={d} default blocks={default}")
    for nb in sorted({default, 256, 512, 768, 1024, 1536, 2048, 3072, 4096, 6144, 8192}):
        out = device.gram_stats(T, y, None, None, "bf16", blocks=nb)
        # f32 MFMA partial sums: a different grid is a different summation order (~1e-8 of n)
        if float((out - ref).abs().max()) > 1e-6 * n:
            bad = (out - ref).abs() > 1e-5 * ref.abs() + 1e-3
            print(f"blocks {nb}: MISMATCH at {bad.nonzero()[:8].flatten().tolist()} out {out[:5].tolist()} ref {ref[:5].tolist()}")
            continue
        for _ in range(5):
            device.gram_stats(T, y, None, None, "bf16", blocks=nb)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 50
        e0.record()
        for _ in range(reps):
            device.gram_stats(T, y, None, None, "bf16", blocks=nb)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        gb = (T.buf.numel() * T.buf.element_size() + y.numel() * 4) / 1e9
        print(f"blocks {nb:6d}: {us:8.1f} us  {gb / us * 1e3:6.2f} TB/s" + ("  (default)" if nb == default else ""))


if __name__ == "__main__":
    main()
