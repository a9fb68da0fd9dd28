"""The lab pipeline as an SPMD data-parallel job (gloo here, RCCL on the MI355X node): every rank
reads its byte-range shard of the CSV (row boundaries, merged inferred schema), DQ rules and
filters run per shard, counts/shows gather across ranks in rank order, the Gram and the metrics
are all-reduced — and the result must equal the single-process oracle, transcript included."""
import contextlib
import io
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import data_path


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, name, transcript):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), DQ4ML_DEVICE="cpu")
    import sys

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from net.jgp.labs.sparkdq4ml_amd import SparkSession, Vectors
    from net.jgp.labs.sparkdq4ml_amd.parallel import comm

    comm.init(backend="gloo")
    try:
        if transcript:
            from net.jgp.labs.sparkdq4ml_amd.apps.dq4ml_app import DataQuality4MachineLearningApp

            buf = io.StringIO()
            with contextlib.redirect_stdout(buf):
                DataQuality4MachineLearningApp(data_path(name), "cpu").start()
            q.put((rank, buf.getvalue()))
        else:
            from test_app_golden import run_pipeline

            spark = SparkSession.builder().master("cpu").getOrCreate()
            counts, model, df = run_pipeline(spark, name)
            s = model.summary
            q.put((rank, counts, float(model.coefficients[0]), float(model.intercept),
                   float(s.rootMeanSquaredError), float(s.r2), float(model.predict(Vectors.dense(40.0))),
                   list(np.asarray(s.objectiveHistory)), int(s.numInstances), len(df.collect()),
                   df.take(3)[0].guest))
        comm.barrier()
    finally:
        comm.shutdown()


def _run(world, name, transcript=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, name, transcript)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("name", ["dataset-abstract.csv", "dataset-full.csv"])
def test_sharded_pipeline_matches_oracle(world, name, cpu_session):
    from test_app_golden import ORACLE, run_pipeline

    ref_counts, ref, ref_df = run_pipeline(cpu_session, name)
    o = ORACLE[name]
    assert ref_counts == o[:3]
    first_guest = ref_df.take(3)[0].guest
    for r in _run(world, name):
        _, counts, coef, icpt, rmse, r2, p40, hist, ninst, ncollect, g0 = r
        assert tuple(counts) == o[:3]
        assert coef == pytest.approx(o[3], rel=1e-9)
        assert icpt == pytest.approx(o[4], rel=1e-9)
        assert rmse == pytest.approx(o[5], rel=1e-9)
        assert r2 == pytest.approx(o[6], rel=1e-9)
        assert p40 == pytest.approx(o[7], rel=1e-9)
        np.testing.assert_allclose(hist, np.asarray(ref.summary.objectiveHistory), rtol=1e-9, atol=1e-15)
        assert ninst == o[2] and ncollect == o[2] and g0 == first_guest


def test_sharded_app_transcript_matches_single_process(cpu_session):
    from net.jgp.labs.sparkdq4ml_amd.apps.dq4ml_app import DataQuality4MachineLearningApp

    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        DataQuality4MachineLearningApp(data_path("dataset-abstract.csv"), "cpu").start()
    res = _run(2, "dataset-abstract.csv", transcript=True)
    assert res[0][1] == buf.getvalue()  # rank 0 prints exactly the single-process transcript
    assert res[1][1] == ""  # other ranks print nothing
