"""One process of ``test_gpu_wide_async.py``: the wide (k >= 1025, no L1) normal-equation fit
enqueued asynchronously -- device label split, SYRK, split-K fold (+ band-by-band RCCL all-reduce
with ``rccl``), large-k assembly + Jacobi-PCG on the side stream -- with NO host sync, checked
under ``torch.cuda.set_sync_debug_mode("error")``, against a synchronous fit of the same data.

    _gpu_wide_async_worker.py rccl|local <eb>

Prints one JSON line: both models' coefficients / intercepts and the async fit's solver."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, SparkSession
    from net.jgp.labs.sparkdq4ml_amd.ops import device
    from net.jgp.labs.sparkdq4ml_amd.parallel import comm

    mode, eb = sys.argv[1], int(sys.argv[2])
    if mode == "rccl":
        comm.force_collectives(True)
        comm.init(backend="nccl")
    d, n = 1100, 60_001
    g = torch.Generator().manual_seed(7 + eb)
    X = (torch.randn(d, n, generator=g) * (0.5 + torch.rand(d, 1, generator=g)) + 0.3).cuda()
    beta = torch.linspace(-1.0, 1.0, d).cuda()
    y = (beta @ X + 2.5 + 0.05 * torch.randn(n, generator=g).cuda()).double()
    T = device.pack_wide([X if eb == 8 else X.to(torch.bfloat16)], eb, None)
    gd = "fp8" if eb == 8 else "bf16"
    lr = LinearRegression(solver="normal", gramDtype=gd, regParam=0.01, elasticNetParam=0.0)
    sync = SparkSession.builder().master("mi355x[*]").config("dq4ml.fit.async", "false").getOrCreate()
    ref = lr.fit(sync.createDataFrame({"features": T, "label": y}))
    ref_coef = ref.coefficients.toArray().tolist()
    ref_icpt = float(ref.intercept)
    sync.stop()
    spark = SparkSession.builder().master("mi355x[*]").config("dq4ml.fit.async", "true").getOrCreate()
    df = spark.createDataFrame({"features": T, "label": y})
    lr.fit(df).coefficients  # warm-up: communicators, allocator, the PCG budget of this order
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        models = [lr.fit(df) for _ in range(3)]  # back to back: each tail beside the next SYRK
        pending = all(getattr(m, "_pending", None) is not None for m in models)
    finally:
        torch.cuda.set_sync_debug_mode("default")
    assert pending, "the wide fit should be asynchronous"
    out = {"ref_coef": ref_coef, "ref_icpt": ref_icpt,
           "coef": [m.coefficients.toArray().tolist() for m in models],
           "icpt": [float(m.intercept) for m in models], "solver": models[-1].summary.solver}
    print(json.dumps(out))
    comm.barrier()
    comm.shutdown()


if __name__ == "__main__":
    main()
