#!/usr/bin/env python3
"""What a per-fit cross-stream ordering point costs between back-to-back Gram passes: 1.25e7 x 32
bf16 tiled Gram (the 8-GPU strong-scaling shard) enqueued 100x on the compute stream, (A) alone,
(B) with an event recorded after each pass and waited by a side stream, (C) as B plus a tiny side
kernel after each wait (what the asynchronous fit tail does)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from net.jgp.labs.sparkdq4ml_amd.ops import device

    dev = torch.device("cuda")
    n, d = 12_500_000, 32
    X = torch.randn(d, n, device=dev).to(torch.bfloat16)
    y = torch.randn(n, device=dev)
    T = device.tile_bf16(X)
    del X
    side = torch.cuda.Stream(dev)
    tiny = torch.zeros(64, device=dev)

    def run(mode, k=100):
        cur = torch.cuda.current_stream(dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            device.gram_stats(T, y, None, None, "bf16")
            if mode >= 1:
                ev = torch.cuda.Event()
                ev.record(cur)
                side.wait_event(ev)
            if mode == 2:
                with torch.cuda.stream(side):
                    tiny.add_(1.0)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k * 1e6

    for _ in range(2):
        for m in (0, 1, 2):
            run(m, 10)
    for rep in range(3):
        print({"rep": rep, "plain_us": round(run(0), 1), "event_us": round(run(1), 1),
               "event_side_kernel_us": round(run(2), 1)}, flush=True)


if __name__ == "__main__":
    main()
