"""Data-parallel fit across processes (gloo on CPU here; RCCL on the MI355X node).

Each rank holds a contiguous row shard; the Gram statistics are all-reduced and the
metrics too (X2), so every rank must end with the single-process model."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(n=5000, d=6, seed=0):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(d, n, generator=g, dtype=torch.float64)
    beta = torch.linspace(-1, 1, d, dtype=torch.float64)
    y = beta @ X + 0.3 + 0.05 * torch.randn(n, generator=g, dtype=torch.float64)
    return X, y


def _worker(rank, world, port, q, reg):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), DQ4ML_DEVICE="cpu")
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, SparkSession
    from net.jgp.labs.sparkdq4ml_amd.parallel import comm

    comm.init(backend="gloo")
    X, y = _data()
    n = X.shape[1]
    lo, hi = rank * n // world, (rank + 1) * n // world
    spark = SparkSession.builder().master("cpu").getOrCreate()
    df = spark.createDataFrame({"features": X[:, lo:hi].contiguous(), "label": y[lo:hi].contiguous()})
    m = LinearRegression(regParam=reg, elasticNetParam=0.5 if reg else 0.0).fit(df)
    q.put((rank, m.coefficients.toArray().tolist(), float(m.intercept), float(m.summary.rootMeanSquaredError),
           float(m.summary.r2), int(m.summary.numInstances)))
    comm.barrier()
    comm.shutdown()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("reg", [0.0, 0.1])
def test_dp_fit_matches_single_process(world, reg, cpu_session):
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression

    X, y = _data()
    df = cpu_session.createDataFrame({"features": X, "label": y})
    ref = LinearRegression(regParam=reg, elasticNetParam=0.5 if reg else 0.0).fit(df)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, reg)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, coef, icpt, rmse, r2, nn in res:
        np.testing.assert_allclose(coef, ref.coefficients.toArray(), rtol=1e-9, atol=1e-12)
        assert icpt == pytest.approx(float(ref.intercept), rel=1e-9)
        assert rmse == pytest.approx(float(ref.summary.rootMeanSquaredError), rel=1e-9)
        assert r2 == pytest.approx(float(ref.summary.r2), rel=1e-9)
        assert nn == 5000
    # X6: no coefficient broadcast — every rank solves the same all-reduced Gram, so the
    # coefficients must agree bit for bit across ranks.
    assert all(coef == res[0][1] and icpt == res[0][2] for _, coef, icpt, *_ in res)
