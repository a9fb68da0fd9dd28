"""Spark-ML persistence format (BASELINE.json "Spark-ML model save format").

``LinearRegressionModel.write().save(path)`` produces the directory layout Spark's
``DefaultParamsWriter`` + ``LinearRegressionModelWriter`` produce:

    path/metadata/part-00000      one JSON line: class, timestamp, sparkVersion, uid, paramMap,
                                  defaultParamMap
    path/metadata/_SUCCESS
    path/data/part-00000-<uuid>-c000.snappy.parquet   one row (intercept: double,
                                  coefficients: VectorUDT struct<type:tinyint,size:int,
                                  indices:array<int>,values:array<double>>, scale: double)
    path/data/_SUCCESS

The target version is the reference's Spark 2.4.4 (``pom.xml``).  ``sparkVersion: "2.4.4"`` and
the ``scale`` column agree: the Huber loss (and with it the model's ``scale``) arrived in Spark 2.3,
whose ``LinearRegressionModelReader`` branches on the metadata version — "2.2 and before" reads
``(intercept, coefficients)``, "2.3 and later" reads ``(intercept, coefficients, scale)``.  The
reader below follows the same version split, so pre-2.3 directories still load (scale = 1.0).

The parquet footer carries ``org.apache.spark.sql.parquet.row.metadata`` (Spark's JSON schema,
including the VectorUDT annotation) so Spark itself can read the files back.  Params-only stages
(``VectorAssembler``) write metadata only; ``Pipeline``/``PipelineModel`` write a stage list.
"""
from __future__ import annotations

import json
import os
import shutil
import time
import uuid

import numpy as np

__all__ = ["MLWriter", "ParamsWriter", "LinearRegressionModelWriter", "LinearRegressionModelReader",
           "save_params_only", "load_params_only", "read_metadata", "write_metadata", "SPARK_VERSION"]

SPARK_VERSION = "2.4.4"

_VECTOR_SQL_TYPE = {
    "type": "struct",
    "fields": [
        {"name": "type", "type": "byte", "nullable": False, "metadata": {}},
        {"name": "size", "type": "integer", "nullable": True, "metadata": {}},
        {"name": "indices", "type": {"type": "array", "elementType": "integer", "containsNull": False},
         "nullable": True, "metadata": {}},
        {"name": "values", "type": {"type": "array", "elementType": "double", "containsNull": False},
         "nullable": True, "metadata": {}},
    ],
}
_VECTOR_UDT = {"type": "udt", "class": "org.apache.spark.ml.linalg.VectorUDT",
               "pyClass": "pyspark.ml.linalg.VectorUDT", "sqlType": _VECTOR_SQL_TYPE}


def _jsonable(v):
    if isinstance(v, (np.floating,)):
        return float(v)
    if isinstance(v, (np.integer,)):
        return int(v)
    if isinstance(v, np.ndarray):
        return v.tolist()
    return v


def _prepare_dir(path: str, overwrite: bool):
    if os.path.exists(path):
        if not overwrite:
            raise IOError(f"Path {path} already exists. To overwrite it, please use write.overwrite().save(path) "
                          f"for Scala and use write().overwrite().save(path) for Java and Python.")
        shutil.rmtree(path)
    os.makedirs(path)


def write_metadata(instance, path: str, cls_name: str, extra: dict = None):
    meta_dir = os.path.join(path, "metadata")
    os.makedirs(meta_dir, exist_ok=True)
    plist = instance.params_list()
    param_map = {k: _jsonable(v) for k, v in instance._paramMap.items() if k in plist and _spark_param(k)}
    default_map = {k: _jsonable(p.default) for k, p in plist.items() if p.has_default and _spark_param(k)
                   and p.default is not None}
    meta = {"class": cls_name, "timestamp": int(time.time() * 1000), "sparkVersion": SPARK_VERSION,
            "uid": instance.uid, "paramMap": param_map, "defaultParamMap": default_map}
    # engine-specific params ride in their own key so Spark ignores them
    ext = {k: _jsonable(v) for k, v in instance._paramMap.items() if k in plist and not _spark_param(k)}
    if ext:
        meta["dq4mlParamMap"] = ext
    if extra:
        meta.update(extra)
    with open(os.path.join(meta_dir, "part-00000"), "w") as f:
        f.write(json.dumps(meta, separators=(",", ":")) + "\n")
    open(os.path.join(meta_dir, "_SUCCESS"), "w").close()


def _spark_param(name: str) -> bool:
    return name not in ("gramDtype", "outputDtype")


def read_metadata(path: str) -> dict:
    meta_dir = os.path.join(path, "metadata")
    parts = sorted(f for f in os.listdir(meta_dir) if f.startswith("part-"))
    with open(os.path.join(meta_dir, parts[0])) as f:
        return json.loads(f.readline())


def apply_metadata(instance, meta: dict):
    plist = instance.params_list()
    for src in (meta.get("paramMap", {}), meta.get("dq4mlParamMap", {})):
        for k, v in src.items():
            if k in plist:
                instance.set(k, v)
    return instance


class MLWriter:
    def __init__(self):
        self._overwrite = False

    def overwrite(self):
        self._overwrite = True
        return self

    def session(self, _):
        return self

    def save(self, path: str):
        _prepare_dir(path, self._overwrite)
        self.save_impl(path)

    def save_impl(self, path: str):
        raise NotImplementedError


class ParamsWriter(MLWriter):
    def __init__(self, instance, cls_name: str):
        super().__init__()
        self.instance, self.cls_name = instance, cls_name

    def save_impl(self, path):
        write_metadata(self.instance, path, self.cls_name)


def save_params_only(instance, path: str, cls_name: str, overwrite: bool = True):
    w = ParamsWriter(instance, cls_name)
    if overwrite:
        w.overwrite()
    w.save(path)


def load_params_only(cls, path: str):
    meta = read_metadata(path)
    inst = cls(uid=meta["uid"])
    return apply_metadata(inst, meta)


# ---- LinearRegressionModel ----------------------------------------------------------------
LR_MODEL_CLASS = "org.apache.spark.ml.regression.LinearRegressionModel"


def _spark_schema_json():
    return json.dumps({"type": "struct", "fields": [
        {"name": "intercept", "type": "double", "nullable": False, "metadata": {}},
        {"name": "coefficients", "type": _VECTOR_UDT, "nullable": True, "metadata": {}},
        {"name": "scale", "type": "double", "nullable": False, "metadata": {}},
    ]}, separators=(",", ":"))


class LinearRegressionModelWriter(MLWriter):
    def __init__(self, model):
        super().__init__()
        self.model = model

    def save_impl(self, path):
        import pyarrow as pa
        import pyarrow.parquet as pq

        write_metadata(self.model, path, LR_MODEL_CLASS)
        data_dir = os.path.join(path, "data")
        os.makedirs(data_dir)
        coef = np.asarray(self.model._coefficients.toArray(), dtype=np.float64)
        vec_type = pa.struct([pa.field("type", pa.int8(), nullable=False), pa.field("size", pa.int32()),
                              pa.field("indices", pa.list_(pa.field("element", pa.int32(), nullable=False))),
                              pa.field("values", pa.list_(pa.field("element", pa.float64(), nullable=False)))])
        vec = pa.array([{"type": 1, "size": None, "indices": None, "values": coef.tolist()}], type=vec_type)
        schema = pa.schema([pa.field("intercept", pa.float64(), nullable=False),
                            pa.field("coefficients", vec_type),
                            pa.field("scale", pa.float64(), nullable=False)],
                           metadata={"org.apache.spark.sql.parquet.row.metadata": _spark_schema_json()})
        table = pa.Table.from_arrays([pa.array([float(self.model._intercept)]), vec,
                                      pa.array([float(getattr(self.model, "scale", 1.0))])], schema=schema)
        fname = f"part-00000-{uuid.uuid4()}-c000.snappy.parquet"
        pq.write_table(table, os.path.join(data_dir, fname), compression="snappy")
        open(os.path.join(data_dir, "_SUCCESS"), "w").close()


def _vector_from_struct(s) -> np.ndarray:
    if s["type"] == 1:
        return np.asarray(s["values"], dtype=np.float64)
    out = np.zeros(int(s["size"]), dtype=np.float64)
    out[np.asarray(s["indices"], dtype=np.int64)] = np.asarray(s["values"], dtype=np.float64)
    return out


class LinearRegressionModelReader:
    def load(self, path: str):
        import pyarrow.parquet as pq

        from .linalg import DenseVector
        from .regression import LinearRegressionModel

        meta = read_metadata(path)
        if meta.get("class") != LR_MODEL_CLASS:
            raise ValueError(f"Error loading metadata: Expected class name {LR_MODEL_CLASS} but found class name "
                             f"{meta.get('class')}")
        data_dir = os.path.join(path, "data")
        files = sorted(f for f in os.listdir(data_dir) if f.endswith(".parquet"))
        row = pq.read_table(os.path.join(data_dir, files[0])).to_pylist()[0]
        major, minor = (int(x) for x in str(meta.get("sparkVersion", SPARK_VERSION)).split(".")[:2])
        if (major, minor) <= (2, 2):  # Spark 2.2 and before: (intercept, coefficients)
            scale = 1.0
        else:  # Spark 2.3 and later: (intercept, coefficients, scale)
            if "scale" not in row:
                raise ValueError(f"model data written by Spark {meta.get('sparkVersion')} lacks the scale column")
            scale = float(row["scale"])
        m = LinearRegressionModel(meta["uid"], DenseVector(_vector_from_struct(row["coefficients"])),
                                  float(row["intercept"]), scale)
        return apply_metadata(m, meta)
