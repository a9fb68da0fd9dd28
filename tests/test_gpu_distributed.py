"""Device data-parallel fit, 2 processes sharing the one MI355X of the test box (SURVEY.md §4,
"Distributed (real)"): each rank runs the HIP Gram over its row shard on ``cuda:0``, the
statistics are all-reduced (X1; gloo here because RCCL refuses two ranks on one GPU — the 8-GPU
RCCL path is the driver's scaling bench) and the metrics too (X2).  Every rank must end with the
single-process device model."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("fit_async", ["true", "false"])
def test_two_rank_device_fit_matches_single_process(gpu_session, fit_async):
    sys.path.insert(0, HERE)
    from _gpu_dp_worker import data

    from net.jgp.labs.sparkdq4ml_amd import LinearRegression

    d, n, world = 32, 400_009, 2
    X, y = data(d, n)
    df = gpu_session.createDataFrame({"features": X.to(torch.bfloat16).cuda(), "label": y.cuda()})
    ref = LinearRegression(solver="normal", gramDtype="bf16").fit(df)

    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r),
                   WORLD_SIZE=str(world), LOCAL_RANK=str(r), DQ4ML_COMM_TIMEOUT="60")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "_gpu_dp_worker.py"), str(d), str(n),
                                       fit_async], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True))
    outs = []
    for p in procs:
        try:
            so, se = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        assert p.returncode == 0, se[-3000:]
        outs.append(json.loads(so.strip().splitlines()[-1]))
    for o in outs:
        assert o["n"] == n
        assert o["same"]  # every repeated fit (replayed, pipelined) equals the first
        np.testing.assert_allclose(o["coef"], ref.coefficients.toArray(), rtol=1e-12, atol=1e-12)
        assert o["intercept"] == pytest.approx(float(ref.intercept), rel=1e-12, abs=1e-12)
        assert o["rmse"] == pytest.approx(float(ref.summary.rootMeanSquaredError), rel=1e-9)
        assert o["r2"] == pytest.approx(float(ref.summary.r2), rel=1e-9)
    assert outs[0]["coef"] == outs[1]["coef"]


def test_two_rank_sharded_device_csv_with_strings(gpu_session, tmp_path):
    """A CSV with string, quoted and timestamp columns read by 2 ranks on the device: each scans its
    row-aligned byte range, the class masks (with the needs-the-host bit) merge across ranks, the
    string / timestamp re-scan is taken by both, and the gathered rows equal the single-process
    read."""
    sys.path.insert(0, HERE)
    from test_gpu_csv_strings import _mixed_csv

    p = tmp_path / "shard.csv"
    p.write_bytes(_mixed_csv(30_001, seed=9))
    gpu_session.conf.set("dq4ml.csv.deviceThresholdBytes", "0")
    ref = gpu_session.read().option("inferSchema", "true").csv(str(p))
    want_types = [t for _, t in ref.dtypes]
    want = [[None if v is None else str(v) for v in row] for row in ref.collect()]
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r),
                   WORLD_SIZE="2", LOCAL_RANK=str(r), DQ4ML_COMM_TIMEOUT="60")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "_gpu_csv_shard_worker.py"), str(p)],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    for q in procs:
        try:
            so, se = q.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for x in procs:
                x.kill()
            raise
        assert q.returncode == 0, se[-3000:]
        outs.append(json.loads(so.strip().splitlines()[-1]))
    assert want_types == ["int", "string", "double", "string", "double", "string"]
    for o in outs:
        assert o["types"] == want_types
        assert o["device_scans"] == 1 and o["fallbacks"] == 0
    assert outs[0]["rows"] == want
