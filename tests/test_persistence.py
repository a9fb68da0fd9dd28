"""Spark-ML save/load format."""
import json
import os

import numpy as np
import pyarrow.parquet as pq
import pytest
import torch

from net.jgp.labs.sparkdq4ml_amd import LinearRegression, LinearRegressionModel, VectorAssembler, Vectors


def _model(spark):
    g = torch.Generator().manual_seed(0)
    X = torch.randn(3, 200, generator=g, dtype=torch.float64)
    y = torch.tensor([1.0, -2.0, 0.5], dtype=torch.float64) @ X + 4.0
    df = spark.createDataFrame({"features": X, "label": y})
    return LinearRegression().setMaxIter(40).setRegParam(0.1).setElasticNetParam(0.3).fit(df), df


def test_lr_model_roundtrip_and_layout(cpu_session, tmp_path):
    m, df = _model(cpu_session)
    path = str(tmp_path / "lrm")
    m.write().save(path)
    assert os.path.exists(os.path.join(path, "metadata", "_SUCCESS"))
    assert os.path.exists(os.path.join(path, "data", "_SUCCESS"))
    meta = json.loads(open(os.path.join(path, "metadata", "part-00000")).readline())
    assert meta["class"] == "org.apache.spark.ml.regression.LinearRegressionModel"
    assert meta["uid"] == m.uid and meta["uid"].startswith("linReg_")
    assert meta["paramMap"]["regParam"] == 0.1 and meta["paramMap"]["maxIter"] == 40
    assert meta["defaultParamMap"]["tol"] == 1e-6 and meta["defaultParamMap"]["solver"] == "auto"
    files = [f for f in os.listdir(os.path.join(path, "data")) if f.endswith(".snappy.parquet")]
    assert len(files) == 1
    t = pq.read_table(os.path.join(path, "data", files[0]))
    assert t.column_names == ["intercept", "coefficients", "scale"]
    assert str(t.schema.field("coefficients").type) == \
        "struct<type: int8 not null, size: int32, indices: list<element: int32 not null>, values: list<element: double not null>>"
    assert b"org.apache.spark.sql.parquet.row.metadata" in t.schema.metadata
    row = t.to_pylist()[0]
    assert row["coefficients"]["type"] == 1
    np.testing.assert_array_equal(row["coefficients"]["values"], m.coefficients.toArray())
    m2 = LinearRegressionModel.load(path)
    assert m2.uid == m.uid
    assert m2.getRegParam() == 0.1 and m2.getElasticNetParam() == 0.3
    np.testing.assert_array_equal(m2.coefficients.toArray(), m.coefficients.toArray())
    assert m2.intercept == m.intercept
    assert m2.predict(Vectors.dense(1.0, 2.0, 3.0)) == m.predict(Vectors.dense(1.0, 2.0, 3.0))
    p1 = [r.prediction for r in m.transform(df).select("prediction").collect()]
    p2 = [r.prediction for r in m2.transform(df).select("prediction").collect()]
    assert p1 == p2
    with pytest.raises(IOError):
        m.write().save(path)
    m.write().overwrite().save(path)


def test_metadata_version_matches_data_layout(cpu_session, tmp_path):
    """sparkVersion 2.4.4 goes with the 3-column (scale) layout; a pre-2.3 directory (2 columns,
    sparkVersion 2.2.x) still loads with scale 1.0, as Spark's reader version split does."""
    import pyarrow as pa

    m, _ = _model(cpu_session)
    path = str(tmp_path / "lrm")
    m.write().save(path)
    meta_file = os.path.join(path, "metadata", "part-00000")
    meta = json.loads(open(meta_file).readline())
    assert meta["sparkVersion"] == "2.4.4"
    data_dir = os.path.join(path, "data")
    fname = [f for f in os.listdir(data_dir) if f.endswith(".parquet")][0]
    t = pq.read_table(os.path.join(data_dir, fname))
    assert t.column_names[-1] == "scale" and t.column("scale").to_pylist() == [1.0]
    # rewrite as a Spark 2.2 directory: drop the scale column, stamp 2.2.0
    pq.write_table(pa.Table.from_arrays([t.column("intercept"), t.column("coefficients")],
                                        names=["intercept", "coefficients"]), os.path.join(data_dir, fname))
    meta["sparkVersion"] = "2.2.0"
    open(meta_file, "w").write(json.dumps(meta) + "\n")
    m2 = LinearRegressionModel.load(path)
    np.testing.assert_array_equal(m2.coefficients.toArray(), m.coefficients.toArray())
    assert m2.scale == 1.0
    # a 2.3+ stamp on 2-column data is inconsistent and refused
    meta["sparkVersion"] = "2.4.4"
    open(meta_file, "w").write(json.dumps(meta) + "\n")
    with pytest.raises(ValueError):
        LinearRegressionModel.load(path)


def test_params_only_stages(tmp_path):
    va = VectorAssembler().setInputCols(["a", "b"]).setOutputCol("features").setHandleInvalid("skip")
    p = str(tmp_path / "va")
    va.save(p)
    va2 = VectorAssembler.load(p)
    assert va2.uid == va.uid and va2.getInputCols() == ["a", "b"] and va2.getHandleInvalid() == "skip"
    lr = LinearRegression().setMaxIter(7).setSolver("normal")
    p = str(tmp_path / "lr")
    lr.save(p)
    lr2 = LinearRegression.load(p)
    assert lr2.getMaxIter() == 7 and lr2.getSolver() == "normal" and lr2.uid == lr.uid
