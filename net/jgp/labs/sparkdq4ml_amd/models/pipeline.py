"""``org.apache.spark.ml.Pipeline`` / ``PipelineModel``: chain the lab's VectorAssembler and
LinearRegression (DataQuality4MachineLearningApp.java:106-126) as one estimator, with Spark's
persistence layout (metadata with ``stageUids`` + ``stages/<idx>_<uid>/``)."""
from __future__ import annotations

import os
from typing import List

from .param import Param, Params

__all__ = ["Pipeline", "PipelineModel"]

_CLASS_OF = {
    "VectorAssembler": "org.apache.spark.ml.feature.VectorAssembler",
    "LinearRegression": "org.apache.spark.ml.regression.LinearRegression",
    "LinearRegressionModel": "org.apache.spark.ml.regression.LinearRegressionModel",
    "Pipeline": "org.apache.spark.ml.Pipeline",
    "PipelineModel": "org.apache.spark.ml.PipelineModel",
}


def _stage_loader(cls_name: str):
    from .feature import VectorAssembler
    from .regression import LinearRegression, LinearRegressionModel

    return {
        "org.apache.spark.ml.feature.VectorAssembler": VectorAssembler,
        "org.apache.spark.ml.regression.LinearRegression": LinearRegression,
        "org.apache.spark.ml.regression.LinearRegressionModel": LinearRegressionModel,
        "org.apache.spark.ml.Pipeline": Pipeline,
        "org.apache.spark.ml.PipelineModel": PipelineModel,
    }[cls_name]


def _save_stages(stages, path):
    sdir = os.path.join(path, "stages")
    os.makedirs(sdir, exist_ok=True)
    n = len(stages)
    width = len(str(n))
    for i, st in enumerate(stages):
        st.write().save(os.path.join(sdir, f"{str(i).zfill(width)}_{st.uid}"))


def _load_stages(path, uids):
    from .persistence import read_metadata

    sdir = os.path.join(path, "stages")
    width = len(str(len(uids)))
    out = []
    for i, uid in enumerate(uids):
        p = os.path.join(sdir, f"{str(i).zfill(width)}_{uid}")
        meta = read_metadata(p)
        out.append(_stage_loader(meta["class"]).load(p))
    return out


class _PipelineWriter:
    def __init__(self, inst, cls_name):
        from .persistence import MLWriter

        self._w = MLWriter()
        self.inst, self.cls_name = inst, cls_name

    def overwrite(self):
        self._w.overwrite()
        return self

    def save(self, path):
        from .persistence import _prepare_dir, write_metadata

        _prepare_dir(path, self._w._overwrite)
        stages = self.inst.getStages() if hasattr(self.inst, "getStages") else self.inst.stages
        write_metadata(self.inst, path, self.cls_name, {"paramMap": {"stageUids": [s.uid for s in stages]}})
        _save_stages(stages, path)


class Pipeline(Params):
    uid_prefix = "pipeline"
    _params = {"stages": Param("stages", "stages of the pipeline", None, has_default=False)}

    def __init__(self, stages=None, uid=None):
        super().__init__(uid)
        if stages is not None:
            self.setStages(stages)

    def setStages(self, stages):
        self._paramMap["stages"] = list(stages)
        return self

    def getStages(self) -> List:
        return list(self._paramMap.get("stages", []))

    def fit(self, df):
        stages = self.getStages()
        last_est = max([i for i, s in enumerate(stages) if hasattr(s, "fit")], default=-1)
        fitted = []
        cur = df
        for i, s in enumerate(stages):
            if hasattr(s, "fit"):
                m = s.fit(cur)
                fitted.append(m)
                if i < last_est:
                    cur = m.transform(cur)
            else:
                fitted.append(s)
                if i < last_est:
                    cur = s.transform(cur)
        return PipelineModel(fitted, uid=self.uid)

    def write(self):
        return _PipelineWriter(self, _CLASS_OF["Pipeline"])

    def save(self, path):
        self.write().save(path)

    @classmethod
    def load(cls, path):
        from .persistence import read_metadata

        meta = read_metadata(path)
        return Pipeline(_load_stages(path, meta["paramMap"]["stageUids"]), uid=meta["uid"])


class PipelineModel(Params):
    uid_prefix = "pipeline"

    def __init__(self, stages, uid=None):
        super().__init__(uid)
        self.stages = list(stages)

    def transform(self, df):
        for s in self.stages:
            df = s.transform(df)
        return df

    def write(self):
        return _PipelineWriter(self, _CLASS_OF["PipelineModel"])

    def save(self, path):
        self.write().save(path)

    @classmethod
    def load(cls, path):
        from .persistence import read_metadata

        meta = read_metadata(path)
        return PipelineModel(_load_stages(path, meta["paramMap"]["stageUids"]), uid=meta["uid"])
