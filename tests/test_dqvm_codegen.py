"""The fused DQ codegen emits valid gfx950 HIP for the lab's chain (compiled offline with hipcc
here; executed against the vectorized evaluator in tests/test_gpu_dqvm.py on the MI355X)."""
import os
import shutil
import subprocess

import pytest

from conftest import data_path
from net.jgp.labs.sparkdq4ml_amd import callUDF
from net.jgp.labs.sparkdq4ml_amd.dq.rules import register_lab_rules
from net.jgp.labs.sparkdq4ml_amd.ops import dqvm
from net.jgp.labs.sparkdq4ml_amd.sql.plan import Filter, Project, execute


def _chain(spark):
    register_lab_rules(spark)
    df = spark.read().format("csv").option("inferSchema", "true").load(data_path("dataset-abstract.csv"))
    df = df.withColumnRenamed("_c0", "guest").withColumnRenamed("_c1", "price")
    df = df.withColumn("price_no_min", callUDF("minimumPriceRule", df.col("price")))
    df.createOrReplaceTempView("price")
    df = spark.sql("SELECT cast(guest as int) guest, price_no_min AS price FROM price WHERE price_no_min > 0")
    df = df.withColumn("price_correct_correl", callUDF("priceCorrelationRule", df.col("price"), df.col("guest")))
    df.createOrReplaceTempView("price")
    df = spark.sql("SELECT guest, price_correct_correl AS price, "
                   "CASE WHEN price_correct_correl > 100 THEN sqrt(guest) ELSE -guest % 3 END AS x "
                   "FROM price WHERE price_correct_correl > 0 AND guest IS NOT NULL")
    return df


def test_codegen_compiles(cpu_session, tmp_path):
    df = _chain(cpu_session)
    nodes, p = [], df._plan
    while isinstance(p, (Project, Filter)):
        nodes.append(p)
        p = p.child
    nodes.reverse()
    base = execute(p, cpu_session)
    (src, src_vec), g, outputs, sel_out = dqvm.compile_chain(nodes, base, check_device=False)
    assert "atomicOr" not in src  # price has no nulls: rule 1 null check elided
    assert src.count("live = live &&") == 2
    assert src_vec.count("live = live &&") == 4  # the 4-row body + the n % 4 tail body
    assert sel_out is not None
    kinds = [o[0] for o in outputs]
    assert kinds == ["col", "new", "new"]  # cast(guest as int) of an int column: the column itself
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("no hipcc")
    for i, code in enumerate((src, src_vec)):
        f = tmp_path / f"k{i}.hip"
        f.write_text("#include <hip/hip_runtime.h>\n" + code)
        r = subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-c", str(f), "-o", str(tmp_path / f"k{i}.o")],
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stderr + "\n" + code


@pytest.mark.parametrize("nullable,fast,ticket", [((False, False), True, "xcd"), ((True, True), False, "global"),
                                                   ((True, False), True, "none")])
def test_scan_fused_codegen_compiles(cpu_session, tmp_path, nullable, fast, ticket):
    """The fused scan + DQ kernel (ops/scanfuse.py) of the lab chain over a CSV relation whose
    facts say: int guest, double price, no nulls — compiles for gfx950, stores only the pruned
    outputs (guest, label) and the selection, and carries no null checks."""
    import torch

    from net.jgp.labs.sparkdq4ml_amd import VectorAssembler
    from net.jgp.labs.sparkdq4ml_amd.ops import scanfuse
    from net.jgp.labs.sparkdq4ml_amd.ops.csvscan import _opt_args
    from net.jgp.labs.sparkdq4ml_amd.sql.dataframe import DataFrame
    from net.jgp.labs.sparkdq4ml_amd.sql.plan import CsvScanRelation, prune_columns
    from net.jgp.labs.sparkdq4ml_amd.sql.types import DoubleType, IntegerType, StructField, StructType

    spark = cpu_session
    register_lab_rules(spark)
    schema = StructType([StructField("_c0", IntegerType(), True), StructField("_c1", DoubleType(), True)])
    fused = {"kinds": [1, 0], "nullable": list(nullable), "strict": False,
             "opts": dict(_opt_args({"comment": 0}), sep=",", strict=False)}
    rel = CsvScanRelation(schema, lambda: None, fused, "Relation[csv]")
    df = DataFrame(rel, spark).withColumnRenamed("_c0", "guest").withColumnRenamed("_c1", "price")
    df = df.withColumn("price_no_min", callUDF("minimumPriceRule", df.col("price")))
    df.createOrReplaceTempView("price")
    df = spark.sql("SELECT cast(guest as int) guest, price_no_min AS price FROM price WHERE price_no_min > 0")
    df = df.withColumn("price_correct_correl", callUDF("priceCorrelationRule", df.col("price"), df.col("guest")))
    df.createOrReplaceTempView("price")
    df = spark.sql("SELECT guest, price_correct_correl AS price FROM price WHERE price_correct_correl > 0")
    df = df.withColumn("label", df.col("price"))
    df = VectorAssembler().setInputCols(["guest"]).setOutputCol("features").transform(df)
    plan = prune_columns(df._plan, {"label", "features"}).child  # the DQ chain below the assembler
    nodes, p = [], plan
    while isinstance(p, (Project, Filter)):
        nodes.append(p)
        p = p.child
    nodes.reverse()
    assert p is rel
    base = scanfuse._ScanBase(rel.schema(), 0, torch.device("cpu"))
    g = scanfuse._scan_gen(base, fused["nullable"])
    _, g, outputs, _ = dqvm.compile_chain(nodes, base, False, gen=g)
    slots = {k: g.slot(None, (k,)) for k in scanfuse._ScanPlan.SCAN_SLOTS}
    src = scanfuse.kernel_source(g, fused["kinds"], fused["nullable"], g.used, fused["opts"], False, 256, slots,
                                 True, fast, ticket)
    if not any(nullable):
        assert [t for t in g.recipe if t[0] in ("out", "outvalid", "selout")] == [("out", 0), ("out", 1), ("selout",)]
    assert ("dq_flag((unsigned int*)p[" in src) == nullable[1]  # RaiseIfNull only when price may be null
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("no hipcc")
    f = tmp_path / "scan.hip"
    f.write_text("#include <hip/hip_runtime.h>\n" + src)
    r = subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", str(f), "-o", str(tmp_path / "scan.o")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@pytest.mark.parametrize("string_col", [False, True])
def test_scan_fused_gram_codegen_compiles(cpu_session, tmp_path, string_col):
    """Gram mode of the fused scan kernel (``scanfuse.try_fused_gram``'s shape): the lab chain,
    then ``VectorAssembler([guest])`` + label as the kernel's d = 1 feature / label outputs —
    no row store, per-window f64 statistics in the ``gram_width`` layout; compiles for gfx950.
    ``string_col``: a third, string column the chain does not read (kind 4: the kernel only cuts
    past its field, ``csv_field_span``)."""
    import torch

    from net.jgp.labs.sparkdq4ml_amd import VectorAssembler
    from net.jgp.labs.sparkdq4ml_amd.ops import scanfuse
    from net.jgp.labs.sparkdq4ml_amd.ops.csvscan import _opt_args
    from net.jgp.labs.sparkdq4ml_amd.sql.dataframe import DataFrame
    from net.jgp.labs.sparkdq4ml_amd.sql.expressions import Alias, ColRef
    from net.jgp.labs.sparkdq4ml_amd.sql.plan import CsvScanRelation, prune_columns
    from net.jgp.labs.sparkdq4ml_amd.sql.types import DoubleType, IntegerType, StringType, StructField, StructType

    spark = cpu_session
    register_lab_rules(spark)
    fields = [StructField("_c0", IntegerType(), True), StructField("_c1", DoubleType(), True)]
    fused = {"kinds": [1, 0], "nullable": [False, False], "strict": False,
             "opts": dict(_opt_args({"comment": 0}), sep=",", strict=False)}
    if string_col:
        fields.append(StructField("_c2", StringType(), True))
        fused["kinds"].append(4)
        fused["nullable"].append(True)
    schema = StructType(fields)
    rel = CsvScanRelation(schema, lambda: None, fused, "Relation[csv]")
    df = DataFrame(rel, spark).withColumnRenamed("_c0", "guest").withColumnRenamed("_c1", "price")
    df = df.withColumn("price_no_min", callUDF("minimumPriceRule", df.col("price")))
    df.createOrReplaceTempView("price")
    df = spark.sql("SELECT cast(guest as int) guest, price_no_min AS price FROM price WHERE price_no_min > 0")
    df = df.withColumn("label", df.col("price"))
    df = VectorAssembler().setInputCols(["guest"]).setOutputCol("features").transform(df)
    plan = prune_columns(df._plan, {"label", "features"})
    nodes, p = [], plan
    while isinstance(p, (Project, Filter)):
        nodes.append(p)
        p = p.child
    assert p is rel
    top = nodes[0]
    gtop = Project(top.child, [Alias(ColRef("guest"), "__gx0"), Alias(ColRef("label"), "__gy")])
    chain = list(reversed(nodes[1:])) + [gtop]
    base = scanfuse._ScanBase(rel.schema(), 0, torch.device("cpu"))
    g = scanfuse._scan_gen(base, fused["nullable"])
    _, g, outputs, _ = dqvm.compile_chain(chain, base, False, gen=g)
    slots = {k: g.slot(None, (k,)) for k in scanfuse._ScanPlan.SCAN_SLOTS + ("gpart",)}
    fast = not string_col  # (a string column is never on the numeric fast path)
    src = scanfuse.kernel_source(g, fused["kinds"], fused["nullable"], g.used, fused["opts"], False, 256, slots,
                                 True, fast, "xcd", 1)
    assert scanfuse.gram_width(1) == 6 and "gred[4][6]" in src
    assert ("= !csv_field_span(" in src) == string_col
    assert "[li] =" not in src  # no row is stored
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("no hipcc")
    f = tmp_path / "scan_gram.hip"
    f.write_text("#include <hip/hip_runtime.h>\n" + src)
    r = subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", str(f), "-o", str(tmp_path / "g.o")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    # the default Gram-mode build: no global line numbering (no ticket, no look-back, no nalloc check)
    src2 = scanfuse.kernel_source(g, fused["kinds"], fused["nullable"], g.used, fused["opts"], False, 256, slots,
                                  True, fast, "xcd", 1, nolb=True)
    assert "__hip_atomic_fetch_add" not in src2 and "sgl0 = pre" not in src2 and "li >= nalloc" not in src2
    assert "const long long blk = blockIdx.x;" in src2 and "sgl0 = pre" in src
    f2 = tmp_path / "scan_gram_nolb.hip"
    f2.write_text("#include <hip/hip_runtime.h>\n" + src2)
    r = subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", str(f2), "-o", str(tmp_path / "g2.o")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
