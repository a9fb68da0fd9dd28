"""Fit-tail CU headroom at the 8-GPU strong-scaling shard (VERDICT r4 "next" #3).

Pipelined asynchronous fits of the headline shape at one rank's share (1.25e7 x 32 bf16 by
default).  After every fit's all-reduce a stand-in kernel (``DQ4ML_TAIL_STANDIN`` blocks:usec,
``rowops.hip`` standin: the shape of an RCCL all-reduce's channel blocks) runs on the tail stream;
timing events around it give how long it waited for CUs beside the next fit's Gram pass.
Alternates ``dq4ml.gram.reserveCUs`` 0 / 8 (or REPS x RESERVES) in one process:

    ROWS=1.25e7 FITS=200 python scripts/tail_reserve_probe.py
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, SparkSession
    from net.jgp.labs.sparkdq4ml_amd.models import regression
    from net.jgp.labs.sparkdq4ml_amd.ops import device

    n = int(float(os.environ.get("ROWS", "1.25e7")))
    d = int(os.environ.get("D", "32"))
    fits = int(os.environ.get("FITS", "200"))
    reps = int(os.environ.get("REPS", "2"))
    reserves = [int(v) for v in os.environ.get("RESERVES", "0,8").split(",")]
    standin = os.environ.get("STANDIN", "8:20")
    spark = SparkSession.builder().master("mi355x[*]").config("dq4ml.fit.async", "true").getOrCreate()
    dev = spark.device
    g = torch.Generator(device=dev).manual_seed(7)
    X = torch.randn(d, n, generator=g, device=dev).to(torch.bfloat16)
    y = (torch.linspace(-2, 2, d, device=dev) @ X.float() + 0.5).contiguous()
    df = spark.createDataFrame({"features": X, "label": y})
    lr = LinearRegression(solver="normal", gramDtype="bf16")
    for rep in range(reps):
        for res in reserves:
            device.set_gram_reserve(res)
            for spec in (None, standin):
                regression.set_tail_standin(spec)
                for _ in range(5):
                    lr.fit(df)
                torch.cuda.synchronize()
                regression.STANDIN_EVENTS.clear()
                t0 = time.perf_counter()
                for _ in range(fits):
                    m = lr.fit(df)
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) * 1e3 / fits
                m.coefficients  # noqa: B018 - resolve the last fit
                waits = sorted(e0.elapsed_time(e1) * 1e3 - u for e0, e1, u in regression.STANDIN_EVENTS)
                rec = {"rep": rep, "reserve_cus": res, "standin": spec, "rows": n, "ms_per_fit": round(ms, 4)}
                if waits:
                    rec.update(standin_wait_us_median=round(waits[len(waits) // 2], 1),
                               standin_wait_us_p90=round(waits[int(len(waits) * 0.9)], 1),
                               standin_wait_us_max=round(waits[-1], 1), standin_samples=len(waits))
                print(json.dumps(rec), flush=True)
    regression.set_tail_standin(None)
    device.set_gram_reserve(-1)


if __name__ == "__main__":
    main()
