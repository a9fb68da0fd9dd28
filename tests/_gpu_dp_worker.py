"""One rank of the 2-process device data-parallel fit in ``test_gpu_distributed.py`` (started
with ``subprocess``, not fork: the parent has already initialised the GPU).  Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def data(d, n):
    import torch

    g = torch.Generator().manual_seed(1234)
    X = torch.randint(-4, 5, (d, n), generator=g).to(torch.float32)
    coef = torch.randint(-2, 3, (d,), generator=g).to(torch.float32)
    noise = torch.randint(-1, 2, (n,), generator=g).to(torch.float32)
    return X, coef @ X + 2.0 + noise  # integers: every partial sum is exact


def main():
    import numpy as np
    import torch

    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, SparkSession
    from net.jgp.labs.sparkdq4ml_amd.parallel import comm

    d, n, fit_async = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    comm.init(backend="gloo")
    r, w = comm.rank(), comm.world_size()
    X, y = data(d, n)
    lo, hi = n * r // w + 3 * r, (n * (r + 1) // w + 3 * (r + 1)) if r < w - 1 else n  # uneven
    spark = SparkSession.builder().master("mi355x[*]").config("dq4ml.fit.async", fit_async).getOrCreate()
    df = spark.createDataFrame({"features": X[:, lo:hi].to(torch.bfloat16).cuda(), "label": y[lo:hi].cuda()})
    lr = LinearRegression(solver="normal", gramDtype="bf16")
    # repeated fits: pipelined streams + the fit replay with collectives active (an all-reduce per fit)
    ms = [lr.fit(df) for _ in range(4)]
    m = ms[-1]
    same = all(np.array_equal(x.coefficients.toArray(), m.coefficients.toArray()) and x.intercept == m.intercept
               for x in ms)
    s = m.summary
    print(json.dumps({"rank": r, "coef": m.coefficients.toArray().tolist(), "intercept": float(m.intercept),
                      "rmse": float(s.rootMeanSquaredError), "r2": float(s.r2), "n": int(s.numInstances), "same": bool(same)}))
    comm.barrier()
    comm.shutdown()


if __name__ == "__main__":
    main()
