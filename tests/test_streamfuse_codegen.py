"""The stream-Gram DQ prologue (ops/streamfuse.py) on the CPU: config 4's chain (range + not-null
rule UDFs, their filter, 64 f32 features) lowers to a row predicate over a 4-region row-scalar
layout, and the whole hipRTC translation unit (device parts of common.h / gram.h /
gram_stream.hip + the generated predicate) compiles for gfx950 with hipRTC itself — only the
module load needs the GPU.  Executed against the two-pass path in tests/test_gpu_streamfuse.py."""
import pytest
import torch

from net.jgp.labs.sparkdq4ml_amd import VectorAssembler, callUDF, col
from net.jgp.labs.sparkdq4ml_amd.dq.rules import NotNullRule, RangeRule
from net.jgp.labs.sparkdq4ml_amd.ops import streamfuse
from net.jgp.labs.sparkdq4ml_amd.sql.expressions import Alias, ColRef
from net.jgp.labs.sparkdq4ml_amd.sql.plan import Filter, Project, output_name, prune_columns
from net.jgp.labs.sparkdq4ml_amd.sql.types import DataTypes


def _chain(spark, d=64, n=1000):
    spark.udf().register("rangeRule", RangeRule(0.0, 1e6, name="rangeRule"), DataTypes.DoubleType)
    spark.udf().register("notNullRule", NotNullRule(name="notNullRule"), DataTypes.DoubleType)
    data = {f"f{j}": torch.randn(n) for j in range(d)}
    data["price"] = (torch.randn(n, dtype=torch.float64) + 100, torch.rand(n) > 0.01)
    data["guest"] = (torch.randint(1, 36, (n,), dtype=torch.int32), torch.rand(n) > 0.005)
    df = spark.createDataFrame(data).withColumn("price_ok", callUDF("rangeRule", col("price")))
    df = df.withColumn("guest_ok", callUDF("notNullRule", col("guest")))
    df = df.filter((col("price_ok") > 0) & (col("guest_ok") > 0))
    df = VectorAssembler(inputCols=[f"f{j}" for j in range(d)], outputCol="features").transform(df)
    plan = prune_columns(df._plan, {"features", "price_ok"})
    nodes, p = [], plan
    while isinstance(p, (Project, Filter)) and p._memo is None:
        nodes.append(p)
        p = p.child
    by = {output_name(e): e for e in nodes[0].exprs}
    va, le = by["features"].child, by["price_ok"]
    lexpr = le.child if isinstance(le, Alias) else le
    gtop = Project(nodes[0].child, [Alias(ColRef(c), f"__gx{i}") for i, c in enumerate(va.inputs)]
                   + [Alias(lexpr, "__gy")])
    names = p.table.schema.names
    return list(reversed(nodes[1:])) + [gtop], p, [names.index(c) for c in va.inputs]


def test_row_scalar_layout():
    lay = streamfuse.raw_layout([(64, 8, True), (65, 4, True)])
    assert lay == [("v", 64, 0, 8), ("v", 65, 512, 4), ("m", 64, 768, 1), ("m", 65, 832, 1)]
    # two f64 fill the 16-B instruction's 1024 bytes, an f32 takes the 4-B one's 256
    assert [r[2] for r in streamfuse.raw_layout([(1, 8, False), (2, 8, False), (3, 4, False)])] == [0, 512, 1024]
    assert streamfuse.raw_layout([(1, 8, False), (2, 8, False), (3, 8, False)]) is None  # 1536 B > 1280 B
    lay = streamfuse.raw_layout([(1, 8, False), (2, 4, True), (3, 4, False)])
    assert [r[2] for r in lay] == [0, 512, 768, 1024]  # the validity bytes go to the 4-B instruction


def test_config4_prologue_compiles_with_hiprtc(cpu_session):
    chain, rel, feat = _chain(cpu_session)
    cp = streamfuse._compile(chain, rel, feat, 2)
    assert cp is not None and (cp.NT, cp.RING) == (2, 2)
    assert [r[0] for r in cp.layout] == ["v", "v", "m", "m"]
    assert "dq_row_pred" in cp.src and "gram_stream_f32_body<2, 2, 1, 1, 64>" in cp.src
    from net.jgp.labs.sparkdq4ml_amd.ops import native

    try:
        h = native.hip()
    except Exception as e:  # pragma: no cover - extension not built here
        pytest.skip(f"no native module: {e}")
    try:
        h.rtc_compile(cp.src, streamfuse.ENTRY)
    except Exception as e:  # the compile ran; without a GPU only hipModuleLoadData fails
        assert "compile failed" not in str(e), str(e)[:3000]
