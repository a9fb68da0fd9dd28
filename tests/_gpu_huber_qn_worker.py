"""One rank of the device Huber L-BFGS-B fit (``huber_qn.hip``) in ``test_gpu_huber_qn.py``,
started with ``subprocess`` (the parent has already initialised the GPU).

    _gpu_huber_qn_worker.py gloo <case>   rank of a 2-process gloo world (RANK/WORLD_SIZE env): this
                                          rank's row shard on cuda:0
    _gpu_huber_qn_worker.py rccl <case>   one process, every collective forced through a one-rank
                                          RCCL communicator, the fit under sync_debug_mode("error")

Prints one JSON line: the model (coefficients, intercept, scale), the device evaluation count and
the objective history."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CASES = {
    "dense": dict(eb=0, d=6, n=20_011, kw=dict(maxIter=100)),
    "bf16": dict(eb=16, d=300, n=30_001, kw=dict(maxIter=60, regParam=0.05)),
    "fp8": dict(eb=8, d=1100, n=20_003, kw=dict(maxIter=40, regParam=0.01, fitIntercept=False)),
}


def data(case, dev):
    """The full data set of a case (the same bits in every process: CPU generator, then upload):
    a linear model with heavy-tailed noise -- every 37th label is an outlier."""
    import torch

    c = CASES[case]
    d, n = c["d"], c["n"]
    g = torch.Generator().manual_seed(d + c["eb"] + 11)
    X = torch.randn(d, n, generator=g, dtype=torch.float64) * (0.5 + torch.rand(d, 1, generator=g,
                                                                                 dtype=torch.float64)) + 0.25
    beta = torch.zeros(d, dtype=torch.float64)
    k = min(d, 30)
    beta[:k] = torch.linspace(-1.0, 2.0, k, dtype=torch.float64)
    y = beta @ X + 0.7 + 0.2 * torch.randn(n, generator=g, dtype=torch.float64)
    y[::37] += 25.0
    return X.to(dev), y.to(dev)


def frame(spark, case, X, y, shift=None):
    from net.jgp.labs.sparkdq4ml_amd.ops import device

    eb = CASES[case]["eb"]
    if eb == 0:
        return spark.createDataFrame({"features": X, "label": y})
    T = device.pack_wide([X.float()], eb, None, shift=shift)
    return spark.createDataFrame({"features": T, "label": y})


def main():
    import torch

    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, SparkSession
    from net.jgp.labs.sparkdq4ml_amd.parallel import comm

    mode, case = sys.argv[1], sys.argv[2]
    c = CASES[case]
    if mode == "rccl":
        comm.force_collectives(True)
        comm.init(backend="nccl")
    else:
        comm.init(backend="gloo")
    r, w = comm.rank(), comm.world_size()
    X, y = data(case, "cuda")
    n = c["n"]
    lo, hi = (n * r // w, n * (r + 1) // w) if mode == "gloo" else (0, n)
    spark = SparkSession.builder().master("mi355x[*]") \
        .config("dq4ml.fit.async", "true" if mode == "rccl" else "false").getOrCreate()
    df = frame(spark, case, X[:, lo:hi].contiguous(), y[lo:hi].contiguous(), None if mode == "gloo" else "auto")
    lr = LinearRegression(loss="huber", tol=1e-9, **c["kw"])
    lr.fit(df).coefficients  # warm-up (communicators, allocator)
    torch.cuda.synchronize()
    if mode == "rccl":
        torch.cuda.set_sync_debug_mode("error")
    try:
        m = lr.fit(df)
        pending = getattr(m, "_pending", None)
    finally:
        torch.cuda.set_sync_debug_mode("default")
    assert mode != "rccl" or pending is not None, "the rccl fit should be asynchronous"
    coef = m.coefficients.toArray().tolist()  # (resolves an asynchronous fit)
    evals = getattr(m, "_huber_evaluations", None)
    if evals is None and pending is not None:
        evals = getattr(pending, "evaluations", None)
    print(json.dumps({"rank": r, "coef": coef, "intercept": float(m.intercept), "scale": float(m.scale),
                      "evaluations": evals, "history": list(map(float, m.summary.objectiveHistory)),
                      "solver": m.summary.solver}))
    comm.barrier()
    comm.shutdown()


if __name__ == "__main__":
    main()
