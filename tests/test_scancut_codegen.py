"""The byte-parallel CSV cutter's codegen (ops/scancut.py) on the CPU: the generated persistent
kernel compiles for gfx950 for the lab chain (d = 1, register sums) and for a wide row (d = 12,
the 4 x 4 blocked LDS Gram), and the augmented-Gram slot map covers the ``gram_width`` layout
exactly once.  Executed against fp64 oracles in tests/test_gpu_scancut.py on the MI355X."""
import os
import shutil
import subprocess

import pytest

from net.jgp.labs.sparkdq4ml_amd import VectorAssembler, callUDF, col
from net.jgp.labs.sparkdq4ml_amd.dq.rules import RangeRule, register_lab_rules
from net.jgp.labs.sparkdq4ml_amd.ops import dqvm, scancut, scanfuse
from net.jgp.labs.sparkdq4ml_amd.sql.plan import Filter, Project


@pytest.mark.parametrize("d", [1, 2, 3, 8, 9, 33])
def test_gram_index_covers_layout_once(d):
    seen = {}
    for j in range(d + 2):
        for i in range(j + 1):
            k = scancut._gram_index(i, j, d)
            if (i, j) == (d, d):
                assert k == 0  # the intercept column's square is the live count
                continue
            assert k is not None and k not in seen, (i, j, k)
            seen[k] = (i, j)
    assert sorted(seen) == list(range(1, scancut.gram_width(d)))
    # the d <= 8 register path emits the same slots (column-major packed upper)
    code = scanfuse._gram_code([f"v{i}" for i in range(d)], "vy")
    for j in range(d):
        for i in range(j + 1):
            assert f"acc[{scancut._gram_index(i, j, d)}] += gx{i} * gx{j};" in code


@pytest.mark.parametrize("d", [9, 32, 64])
def test_tile_slot_map_covers_layout_once(d):
    """The [x | y | 1] row tile (the label column stored at slot d by the converter) maps every
    upper entry of the tile onto the gram_width layout exactly once, like [x | 1 | y]."""
    class Sh:
        pass

    for yfirst in (False, True):
        sh = Sh()
        sh.d, sh.yfirst = d, yfirst
        seen = {}
        for j in range(d + 2):
            for i in range(j + 1):
                k = scancut._tile_slot(sh, i, j)
                assert k is not None and k not in seen, (yfirst, i, j, k)
                seen[k] = (i, j)
        assert sorted(seen) == list(range(scancut.gram_width(d)))
        assert scancut._tile_slot(sh, d + 1, d) is None  # the tile's lower half is not read
    sh = Sh()
    sh.d, sh.yfirst = d, True
    assert scancut._tile_slot(sh, d, d) == 2 and scancut._tile_slot(sh, d + 1, d + 1) == 0  # Σy², count
    assert scancut._tile_slot(sh, d, d + 1) == 1 and scancut._tile_slot(sh, 0, d) == 3 + d  # Σy, Σx0y


def _cut_source(spark, d, lab, stamps=False, quoted=False, max_line=None):
    import torch

    from net.jgp.labs.sparkdq4ml_amd.ops.csvscan import _opt_args
    from net.jgp.labs.sparkdq4ml_amd.sql.dataframe import DataFrame
    from net.jgp.labs.sparkdq4ml_amd.sql.expressions import Alias, ColRef
    from net.jgp.labs.sparkdq4ml_amd.sql.plan import CsvScanRelation, prune_columns
    from net.jgp.labs.sparkdq4ml_amd.sql.types import DataTypes, DoubleType, IntegerType, StructField, StructType

    ncol = 2 if lab else d + 1
    kinds = [1, 0] if lab else [0] * ncol
    schema = StructType([StructField(f"_c{i}", IntegerType() if k == 1 else DoubleType(), True)
                         for i, k in enumerate(kinds)])
    fused = {"kinds": kinds, "nullable": [False] * ncol, "strict": False, "fast_only": True, "empty_lines": 0,
             "uniform_fields": True, "max_line": max_line or (10 if lab else 11 * ncol), "device": torch.device("cpu"),
             "min_line": 6 if lab else 9 * ncol, "term_kinds": [100, 0, 0],
             "opts": dict(_opt_args({"comment": 0}), sep=",", strict=False)}
    rel = CsvScanRelation(schema, lambda: None, fused, "Relation[csv]")
    df = DataFrame(rel, spark)
    if lab:
        register_lab_rules(spark)
        df = df.withColumnRenamed("_c0", "guest").withColumnRenamed("_c1", "price")
        df = df.withColumn("price_no_min", callUDF("minimumPriceRule", df.col("price")))
        df.createOrReplaceTempView("price")
        df = spark.sql("SELECT cast(guest as int) guest, price_no_min AS price FROM price WHERE price_no_min > 0")
        df = df.withColumn("price_correct_correl", callUDF("priceCorrelationRule", df.col("price"), df.col("guest")))
        df.createOrReplaceTempView("price")
        df = spark.sql("SELECT guest, price_correct_correl AS price FROM price WHERE price_correct_correl > 0")
        df = df.withColumn("label", df.col("price"))
        inputs = ["guest"]
    else:
        spark.udf().register("rangeRule", RangeRule(0.0, 150.0, name="rangeRule"), DataTypes.DoubleType)
        df = df.withColumn("y_ok", callUDF("rangeRule", col(f"_c{d}"))).filter(col("y_ok") > 0)
        df = df.withColumn("label", col("y_ok"))
        inputs = [f"_c{i}" for i in range(d)]
    df = VectorAssembler().setInputCols(inputs).setOutputCol("features").transform(df)
    plan = prune_columns(df._plan, {"label", "features"})
    nodes, p = [], plan
    while isinstance(p, (Project, Filter)):
        nodes.append(p)
        p = p.child
    assert p is rel
    gtop = Project(nodes[0].child, [Alias(ColRef(c), f"__gx{i}") for i, c in enumerate(inputs)]
                   + [Alias(ColRef("label"), "__gy")])
    chain = list(reversed(nodes[1:])) + [gtop]
    H = scancut.applicable(fused)
    assert H == scancut.head_for(fused["max_line"])
    base = scanfuse._ScanBase(rel.schema(), 0, torch.device("cpu"))
    g = scanfuse._scan_gen(base, fused["nullable"])
    _, g, _, _ = dqvm.compile_chain(chain, base, False, gen=g)
    slots = {k: g.slot(None, (k,)) for k in ("buf", "nwin", "trailing", "vflag", "gpart") + (("dbg",) if stamps else ())}
    ml = fused["max_line"]
    src, sh = scancut.kernel_source(g, kinds, g.used, fused["opts"], H, slots, d, 13, False, fused["min_line"],
                                    scancut.blocks_per_cu(scancut.kernel_source(g, kinds, g.used, fused["opts"], H,
                                                                                slots, d, 13, False,
                                                                                fused["min_line"], 0, ml, quoted)[1].lds),
                                    ml, quoted)
    return src


@pytest.mark.parametrize("d,lab,stamps,quoted", [(1, True, False, False), (12, False, False, False),
                                                 (40, False, True, False), (12, False, False, True)])
def test_cut_kernel_compiles_for_gfx950(cpu_session, tmp_path, monkeypatch, d, lab, stamps, quoted):
    if stamps:  # the diagnostic phase-clock build
        monkeypatch.setenv("DQ4ML_CUT_STAMPS", "1")
    src = _cut_source(cpu_session, d, lab, stamps, quoted)
    assert ("qany" in src) == quoted  # quoted fast-path numbers: bounds inside the quotes
    assert ("s_memtime" in src) == stamps
    assert f"void {scancut.ENTRY}(" in src
    assert "for (int r = tid; r < nr; r += 256)" in src  # a row tile larger than the block is covered
    assert ("DQ_TIDX" in src) == (d > 8)  # the MFMA Gram of the row tile
    assert ("csv_num_r<2>(stage, end" in src) == lab  # 8-byte converter frame for the lab's short fields
    assert ("gt[q_ga] = dv;" in src) == (d > 8)  # every column stored straight into its row-tile slot
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("no hipcc")
    f = tmp_path / "cut.hip"
    f.write_text("#include <hip/hip_runtime.h>\n" + src)
    r = subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", str(f), "-o", str(tmp_path / "c.o")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]


def test_cutter_preconditions():
    base = {"fast_only": True, "strict": False, "nullable": [False, False], "empty_lines": 0, "uniform_fields": True,
            "kinds": [1, 0], "max_line": 300, "term_kinds": [7, 0, 0], "opts": {"sep": ",", "null_value": "", "trim_lead": 0, "trim_trail": 0,
                                                       "comment": 0}}
    assert scancut.applicable(base) == 512
    for k, v in (("fast_only", False), ("nullable", [True, False]), ("empty_lines", 2), ("uniform_fields", False),
                 ("kinds", [2, 0]), ("max_line", 5000), ("term_kinds", [4, 3, 0]), ("term_kinds", [4, 0, 3])):
        assert scancut.applicable(dict(base, **{k: v})) is None, k
    assert scancut.applicable(dict(base, opts=dict(base["opts"], sep="."))) is None
    # every off-fast-path field a quoted fast-path number: the QUOTED build takes it
    assert scancut.applicable(dict(base, fast_only=False, quoted_fast=True)) == 512
    assert scancut.term_of(dict(base, term_kinds=[0, 9, 0])) == (10, False)
    assert scancut.term_of(dict(base, term_kinds=[9, 0, 9])) == (13, True)


@pytest.mark.parametrize("d", [9, 32, 40, 64])
def test_vstrip_tables_cover_gram_width_once(cpu_session, d):
    """With the [y | 1] strip on the VALU, the MFMA tiles' index table writes only the x x^T
    slots and the strip's table the 2 d + 3 others: together every gram_width slot once."""
    import re

    src = _cut_source(cpu_session, d, False)
    tab = {}
    for name in ("DQ_TIDX", "DQ_SSLOT"):
        m = re.search(name + r"\[\d+\] = \{([^}]*)\}", src)
        assert m is not None, name
        tab[name] = [int(v) for v in m.group(1).split(",") if int(v) >= 0]
    GW = scancut.gram_width(d)
    assert sorted(tab["DQ_SSLOT"]) == list(range(3 + 2 * d))
    assert sorted(tab["DQ_TIDX"]) == list(range(3 + 2 * d, GW))
    assert "sn_ += live ? 1.0 : 0.0;" in src  # the count, Σy and Σy² from the row phase
