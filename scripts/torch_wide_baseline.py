"""Stock PyTorch-ROCm XᵀX for the wide config shape (bf16 GEMM, fp8 torch._scaled_mm), to compare
with the LDS-tiled MFMA SYRK (scripts/wide_bench.py at the same N, D).

    N=2e6 D=4096 python scripts/torch_wide_baseline.py
"""
import os

import torch


def bench(fn, reps=5):
    for _ in range(2):
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
    n, d = int(float(os.environ.get("N", "2e6"))), int(os.environ.get("D", "4096"))
    g = torch.Generator(device="cuda").manual_seed(0)
    X = torch.randn(n, d, generator=g, device="cuda", dtype=torch.bfloat16)  # row-major rows
    flops = 2.0 * n * d * d
    ms = bench(lambda: X.t() @ X)
    print(f"bf16 torch X^T X n={n:.0e} d={d}: {ms:.2f} ms ({flops / ms / 1e9:.0f} TFLOP/s full-GEMM)")
    try:
        X8 = X.to(torch.float8_e4m3fn)
        At = X8.t().contiguous()  # [d, n] row-major
        B = X8  # [n, d] row-major == column-major [d, n]ᵀ view required by _scaled_mm: use .t() of At
        one = torch.ones((), device="cuda")
        fn = lambda: torch._scaled_mm(At, At.t(), scale_a=one, scale_b=one, out_dtype=torch.float32)  # noqa: E731
        ms8 = bench(fn)
        print(f"fp8 torch._scaled_mm n={n:.0e} d={d}: {ms8:.2f} ms ({flops / ms8 / 1e9:.0f} TFLOP/s full-GEMM)")
        del B
    except Exception as e:  # noqa: BLE001
        print(f"fp8 torch._scaled_mm unavailable: {type(e).__name__}: {e}")


if __name__ == "__main__":
    main()
