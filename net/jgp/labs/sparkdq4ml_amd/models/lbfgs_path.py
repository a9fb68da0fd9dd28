"""Iterative l-bfgs path of LinearRegression (solver=l-bfgs, numFeatures > 4096, huber loss)."""


def train_lbfgs(est, df, tbl, X, y, d):
    raise NotImplementedError("l-bfgs path")
