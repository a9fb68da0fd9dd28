"""One rank of the data-parallel device l-bfgs / OWLQN fit (``lsq_qn.hip`` ``lsq_qn_dp_*``, X4) in
``test_gpu_lsq_qn.py``, started with ``subprocess`` (the parent has already initialised the GPU).

    _gpu_qn_dp_worker.py gloo <solver-case> [empty]
                                              rank of a 2-process gloo world (RANK/WORLD_SIZE env): this
                                              rank's row shard of the wide tiles on cuda:0 (empty: rank 0
                                              holds every row, rank 1 none)
    _gpu_qn_dp_worker.py rccl <solver-case>   one process, every collective forced through a one-rank
                                              RCCL communicator, the fit under sync_debug_mode("error")

Prints one JSON line: the model, the evaluation count of the device fit, the objective history."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CASES = {
    "lbfgs": dict(eb=16, d=300, n=60_001, kw=dict(regParam=0.02, elasticNetParam=0.0)),
    "owlqn": dict(eb=16, d=300, n=60_001, kw=dict(regParam=0.02, elasticNetParam=0.6)),
    "fp8": dict(eb=8, d=1100, n=30_017, kw=dict(regParam=0.01, elasticNetParam=1.0, fitIntercept=False)),
}


def data(case, dev):
    """The full data set of a case (the same bits in every process: CPU generator, then upload)."""
    import torch

    c = CASES[case]
    d, n = c["d"], c["n"]
    g = torch.Generator().manual_seed(d + c["eb"])
    X = torch.randn(d, n, generator=g) * (0.5 + torch.rand(d, 1, generator=g))
    beta = torch.zeros(d)
    k = min(d, 40)
    beta[:k] = torch.linspace(-1.0, 2.0, k)
    y = (beta @ X + 0.5 + 0.1 * torch.randn(n, generator=g)).double()
    return X.to(dev), y.to(dev)


def main():
    import torch

    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, SparkSession
    from net.jgp.labs.sparkdq4ml_amd.ops import device
    from net.jgp.labs.sparkdq4ml_amd.parallel import comm

    mode, case = sys.argv[1], sys.argv[2]
    c = CASES[case]
    os.environ["DQ4ML_LSQ_QN"] = "1"
    if mode == "rccl":
        comm.force_collectives(True)
        comm.init(backend="nccl")
    else:
        comm.init(backend="gloo")
    r, w = comm.rank(), comm.world_size()
    X, y = data(case, "cuda")
    n = c["n"]
    lo, hi = (n * r // w, n * (r + 1) // w) if mode == "gloo" else (0, n)
    if mode == "gloo" and len(sys.argv) > 3 and sys.argv[3] == "empty":
        lo, hi = (0, n) if r == 0 else (n, n)  # the last rank's shard is empty: same branch, zero partials
    # gloo: unshifted bf16 storage, element for element what the parent's single-process reference
    # stores; rccl: the default shift, agreed over the (forced) communicator
    T = device.pack_wide([X[:, lo:hi].contiguous()], c["eb"], None, shift=None if mode == "gloo" else "auto")
    # rccl: an asynchronous fit -- everything is enqueued without a host sync (checked below under
    # sync_debug_mode("error")); the model resolves on first read, after the check
    spark = SparkSession.builder().master("mi355x[*]") \
        .config("dq4ml.fit.async", "true" if mode == "rccl" else "false").getOrCreate()
    df = spark.createDataFrame({"features": T, "label": y[lo:hi].contiguous()})
    lr = LinearRegression(solver="l-bfgs", maxIter=60, tol=1e-9, **c["kw"])
    lr.fit(df)  # warm-up (communicators, allocator)
    torch.cuda.synchronize()
    if mode == "rccl":
        torch.cuda.set_sync_debug_mode("error")
    try:
        m = lr.fit(df)
        pending = getattr(m, "_pending", None) is not None
    finally:
        torch.cuda.set_sync_debug_mode("default")
    assert mode != "rccl" or pending, "the rccl fit should be asynchronous"
    p = getattr(m, "_pending", None)
    coef = m.coefficients.toArray().tolist()  # (resolves an asynchronous fit)
    evals = getattr(m, "_qn_evaluations", None)
    if evals is None and p is not None:
        evals = getattr(p, "evaluations", None)  # set by the device fit's pending result only
    print(json.dumps({"rank": r, "coef": coef, "intercept": float(m.intercept), "evaluations": evals,
                      "history": list(map(float, m.summary.objectiveHistory)), "solver": m.summary.solver}))
    comm.barrier()
    comm.shutdown()


if __name__ == "__main__":
    main()
