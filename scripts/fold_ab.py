"""Timing of the Gram slab fold (``gram_reduce`` -> storage-order ``gram_fold_kernel``) on random
partial slabs of the tall bf16 layout (d = 32 / 64) and the f64 layout, checked against a torch
sum of the slabs.  (The first, output-order fold ran 4.4 / 7.9 us at d = 32 / 64; this one
3.8 / 3.9 us back to back.)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from net.jgp.labs.sparkdq4ml_amd.ops import native  # noqa: E402

h = native.hip()
for mode, d in ((2, 32), (2, 64), (0, 32)):
    P = int(h.gram_partial_stride(mode, d))
    nb = 256
    g = torch.Generator(device="cuda").manual_seed(d + mode)
    parts = torch.randn(nb * P, generator=g, device="cuda", dtype=torch.float64)
    out = torch.empty(5 + 2 * d + d * (d + 1) // 2, dtype=torch.float64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for _ in range(20):
        h.gram_reduce(mode, parts.data_ptr(), nb, d, out.data_ptr(), st)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(200):
        h.gram_reduce(mode, parts.data_ptr(), nb, d, out.data_ptr(), st)
    e1.record()
    torch.cuda.synchronize()
    tot = parts.view(nb, P).sum(0)
    head = 5 + 2 * d
    assert torch.allclose(out[:head], tot[:head], rtol=1e-12, atol=1e-9)
    print(f"mode={mode} d={d}: {e0.elapsed_time(e1) / 200 * 1e3:.2f} us/launch (back-to-back)")
