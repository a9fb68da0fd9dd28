"""The same WLS statistics with stock PyTorch-ROCm ops (hipBLASLt GEMM + reductions), for
comparison with the hand-written kernels: 1e8 x 32 bf16 (headline) and f64.

    python scripts/torch_baseline.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from net.jgp.labs.sparkdq4ml_amd.ops import device  # noqa: E402


def stats_torch(X, y):
    """[count, Σw, Σw², Σy, Σy², Σx, Σxy, XᵀX] with unit weights: one augmented GEMM
    [X; y; 1]ᵀ[X; y; 1] (the library's best single call) in the input dtype with fp32 accumulate."""
    A = torch.cat([X, y.to(X.dtype).unsqueeze(0), torch.ones_like(y, dtype=X.dtype).unsqueeze(0)])
    return A @ A.t()


def bench(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    n, d = int(float(os.environ.get("N", "1e8"))), 32
    g = torch.Generator(device="cuda").manual_seed(0)
    Xf = torch.randn(d, n, generator=g, device="cuda")
    y = torch.randn(n, generator=g, device="cuda")
    Xb = Xf.to(torch.bfloat16)
    del Xf
    T = device.tile_bf16(Xb)
    ms_ours = bench(lambda: device.gram_stats(T, y, None, None, "bf16"))
    A = torch.cat([Xb, y.to(torch.bfloat16).unsqueeze(0), torch.ones_like(y, dtype=torch.bfloat16).unsqueeze(0)])
    ms_gemm = bench(lambda: A @ A.t())  # the GEMM alone, operand pre-built
    ms_full = bench(lambda: stats_torch(Xb, y))  # incl. building the augmented operand
    print(f"bf16 n={n:.0e} d={d}: ours {ms_ours:.3f} ms | torch GEMM only {ms_gemm:.3f} ms | "
          f"torch cat+GEMM {ms_full:.3f} ms")
    del A, T
    n2 = n // 4
    X64 = torch.randn(d, n2, generator=g, device="cuda", dtype=torch.float64)
    y64 = torch.randn(n2, generator=g, device="cuda", dtype=torch.float64)
    ms_ours64 = bench(lambda: device.gram_stats(X64, y64, None, None, "fp64"))
    A64 = torch.cat([X64, y64.unsqueeze(0), torch.ones_like(y64).unsqueeze(0)])
    ms_gemm64 = bench(lambda: A64 @ A64.t())
    print(f"f64 n={n2:.1e} d={d}: ours {ms_ours64:.3f} ms | torch GEMM only {ms_gemm64:.3f} ms")


if __name__ == "__main__":
    main()
