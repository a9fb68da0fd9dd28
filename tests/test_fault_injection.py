"""Failure detection: a rank dying before the Gram all-reduce makes the survivors
fail with an error, not hang; a null where rule 1 has no guard fails the job with R4's NPE
message; a corrupt CSV row is read PERMISSIVE (nulls) and filtered by the null-guarded rule."""
import os
import socket
import time

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), DQ4ML_DEVICE="cpu", DQ4ML_FAULT="before_allreduce:1",
                      DQ4ML_COMM_TIMEOUT="20")
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression, SparkSession
    from net.jgp.labs.sparkdq4ml_amd.parallel import comm

    comm.init(backend="gloo")
    spark = SparkSession.builder().master("cpu").config("dq4ml.healthCheck", "never").getOrCreate()
    X = torch.randn(3, 100, dtype=torch.float64)
    df = spark.createDataFrame({"features": X, "label": X.sum(0)})
    t0 = time.time()
    try:
        LinearRegression(solver="normal").fit(df)
        q.put((rank, "ok", time.time() - t0))
    except Exception as e:  # noqa: BLE001 - the point is that it surfaces
        q.put((rank, type(e).__name__ + ": " + str(e)[:200], time.time() - t0))


def test_dead_rank_before_allreduce_errors_not_hangs():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    rank0 = q.get(timeout=120)  # rank 1 exits hard (code 17) without reporting
    for p in procs:
        p.join(timeout=60)
    assert procs[1].exitcode == 17
    assert rank0[0] == 0 and rank0[1] != "ok", rank0
    assert rank0[2] < 60


def _health_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), DQ4ML_DEVICE="cpu")
    from net.jgp.labs.sparkdq4ml_amd.parallel import comm

    comm.init(backend="gloo")
    if rank == 1:
        time.sleep(8)  # never joins the first check in time
        q.put((rank, "slept"))
        return
    try:
        comm.health_check(timeout_s=2)
        q.put((rank, "ok"))
    except comm.RankFailure as e:
        q.put((rank, "RankFailure: " + str(e)[:120]))


def test_health_check_names_missing_rank():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_health_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res[0].startswith("RankFailure"), res


def test_null_price_fails_rule1_like_npe(cpu_session, tmp_path):
    from net.jgp.labs.sparkdq4ml_amd import callUDF
    from net.jgp.labs.sparkdq4ml_amd.dq.rules import register_lab_rules
    from net.jgp.labs.sparkdq4ml_amd.sql.expressions import SparkException

    f = tmp_path / "nulls.csv"
    f.write_bytes(b"3,25.5\r4,\r5,30.0")
    register_lab_rules(cpu_session)
    df = cpu_session.read().format("csv").option("inferSchema", "true").load(str(f))
    df = df.withColumnRenamed("_c0", "guest").withColumnRenamed("_c1", "price")
    df = df.withColumn("p", callUDF("minimumPriceRule", df.col("price")))
    with pytest.raises(SparkException, match="NullPointerException"):
        df.show()


def test_corrupt_row_is_permissive_and_rule2_filters_it(cpu_session, tmp_path):
    from net.jgp.labs.sparkdq4ml_amd import callUDF
    from net.jgp.labs.sparkdq4ml_amd.dq.rules import register_lab_rules

    f = tmp_path / "corrupt.csv"
    f.write_bytes(b"3,25.5\rabc,xyz\r5\r16,95.0")
    register_lab_rules(cpu_session)
    df = cpu_session.read().format("csv").option("inferSchema", "true").load(str(f))
    assert [f.dataType.simpleString() for f in df.schema.fields] == ["string", "string"]
    df = cpu_session.read().format("csv").schema("guest int, price double").load(str(f))
    rows = df.collect()
    assert rows[1].guest is None and rows[1].price is None  # PERMISSIVE: unparseable -> null
    assert rows[2].price is None  # short row padded with null
    df = df.withColumn("p", callUDF("priceCorrelationRule", df.col("price"), df.col("guest")))
    kept = df.filter(df.col("p") > 0).collect()
    assert [(r.guest, r.price) for r in kept] == [(3, 25.5), (16, 95.0)]
