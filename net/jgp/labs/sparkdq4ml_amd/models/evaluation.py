"""``org.apache.spark.ml.evaluation.RegressionEvaluator`` (rmse | mse | r2 | mae | var) over the
prediction/label columns, through the fused device metrics reduction (K8: the prediction column
is fed as a one-feature matrix with coefficient 1)."""
from __future__ import annotations

import numpy as np
import torch

from ..ops import kernels
from ..parallel import comm
from .param import Param, Params, param_accessors

__all__ = ["RegressionEvaluator"]


@param_accessors
class RegressionEvaluator(Params):
    uid_prefix = "regEval"
    _params = {
        "metricName": Param("metricName", "metric name in evaluation (mse|rmse|r2|mae|var)", "rmse",
                            lambda v: v in ("mse", "rmse", "r2", "mae", "var")),
        "labelCol": Param("labelCol", "label column name", "label"),
        "predictionCol": Param("predictionCol", "prediction column name", "prediction"),
        "throughOrigin": Param("throughOrigin", "whether the regression is through the origin", False),
    }

    def __init__(self, predictionCol=None, labelCol=None, metricName=None, uid=None):
        super().__init__(uid)
        for k, v in (("predictionCol", predictionCol), ("labelCol", labelCol), ("metricName", metricName)):
            if v is not None:
                self.set(k, v)

    def isLargerBetter(self):
        return self.getOrDefault("metricName") in ("r2", "var")

    def evaluate(self, df, params=None) -> float:
        ev = self.copy(params) if params else self
        tbl = df._table()
        p = tbl.column(ev.getOrDefault("predictionCol"))
        y = tbl.column(ev.getOrDefault("labelCol"))
        sel = tbl.sel
        for c in (p, y):
            if c.valid is not None:
                sel = c.valid if sel is None else (sel & c.valid)
        pv = p.values.to(torch.float64).unsqueeze(0)
        sums = kernels.regression_metrics(pv, y.values, np.ones(1), 0.0, sel, 0.0)
        sums = comm.all_reduce_sum(sums).cpu().numpy()
        n, sy, syy, _, srr, sabs, sp, spp = (float(v) for v in sums)
        mean_y = sy / n
        name = ev.getOrDefault("metricName")
        if name == "mse":
            return srr / n
        if name == "rmse":
            return float(np.sqrt(srr / n))
        if name == "mae":
            return sabs / n
        if name == "var":  # explained variance: SSreg / n
            return (spp - 2 * mean_y * sp + n * mean_y ** 2) / n
        if ev.getOrDefault("throughOrigin"):
            return 1.0 - srr / syy
        return 1.0 - srr / (syy - n * mean_y ** 2)
