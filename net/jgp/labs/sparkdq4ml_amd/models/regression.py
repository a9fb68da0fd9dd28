"""``LinearRegression`` / ``LinearRegressionModel`` / training summary.

The lab builds ``new LinearRegression().setMaxIter(40).setRegParam(1).setElasticNetParam(1)``,
calls ``fit`` (``DataQuality4MachineLearningApp.java:120-126``), ``model.transform(df).show()``
(``:129``), reads ``summary().totalIterations/objectiveHistory/residuals/rootMeanSquaredError/r2``
(``:132-139``), ``intercept/getRegParam/getTol`` (``:141-146``) and ``predict(Vectors.dense(40.0))``
(``:149-151``).

Execution of ``fit`` (normal-equation path):

1. ``gram_stats`` — one fused device pass over the feature matrix, label, weights and the DQ
   selection vector (HIP MFMA kernel; f64/f32/bf16/fp8 compute selectable through
   ``gramDtype``) producing Spark's WLS aggregator statistics;
2. one RCCL all-reduce of that flat f64 buffer across data-parallel ranks (``parallel.comm``);
3. the f64 normal-equation solve (native host library / device for large k);
4. the summary is lazy: predictions and metrics are one more fused device pass on first access.
"""
from __future__ import annotations

from typing import Optional

import os

import numpy as np
import torch

from ..ops import device, kernels, native, scanfuse, streamfuse
from ..ops.layout import TiledBF16
from ..parallel import comm
from ..sql.dataframe import DataFrame
from ..runtime import faststream, streams
from ..runtime.checks import defer, verify
from ..sql.expressions import AnalysisException, ColRef, EvalContext, Expr, SparkException
from ..sql.plan import Filter, Project, execute, prune_columns
from ..sql.table import ColumnData
from ..sql.types import DoubleType, VectorUDT, is_numeric
from ..utils.logging import get_logger
from .linalg import DenseVector, Vector, Vectors
from ..utils import tracing
from .optim import DEVICE_SOLVE_MIN_K, MAX_NUM_FEATURES, PCG_RTOL, GramStats, fit_wls_flat
from .param import Param, Params, param_accessors

__all__ = ["LinearRegression", "LinearRegressionModel", "LinearRegressionTrainingSummary",
           "LinearRegressionSummary"]

log = get_logger("regression")


class _JavaFloat(float):
    """A float that can also be *called* — lets both ``summary.r2`` (pyspark) and
    ``summary.r2()`` (Java, as in the reference app) work."""

    def __call__(self):
        return float(self)


class _JavaInt(int):
    def __call__(self):
        return int(self)


class _JavaArray(np.ndarray):
    def __call__(self):
        return np.asarray(self)


def _jarr(a):
    return np.asarray(a, dtype=np.float64).view(_JavaArray)


_GRAM_DTYPES = ("fp64", "fp32", "fp32split", "bf16", "fp8")


class _LRParams(Params):
    _params = {
        "featuresCol": Param("featuresCol", "features column name", "features"),
        "labelCol": Param("labelCol", "label column name", "label"),
        "predictionCol": Param("predictionCol", "prediction column name", "prediction"),
        "maxIter": Param("maxIter", "maximum number of iterations (>= 0)", 100, lambda v: v >= 0, converter=int),
        "regParam": Param("regParam", "regularization parameter (>= 0)", 0.0, lambda v: v >= 0, converter=float),
        "elasticNetParam": Param("elasticNetParam", "the ElasticNet mixing parameter, in range [0, 1]", 0.0,
                                 lambda v: 0 <= v <= 1, converter=float),
        "tol": Param("tol", "the convergence tolerance for iterative algorithms (>= 0)", 1e-6, lambda v: v >= 0, converter=float),
        "fitIntercept": Param("fitIntercept", "whether to fit an intercept term", True),
        "standardization": Param("standardization", "whether to standardize the training features before fitting "
                                                    "the model", True),
        "weightCol": Param("weightCol", "weight column name. If this is not set or empty, we treat all instance "
                                        "weights as 1.0", None, has_default=False),
        "solver": Param("solver", "The solver algorithm for optimization. Supported options: auto, normal, l-bfgs",
                        "auto", lambda v: v in ("auto", "normal", "l-bfgs")),
        "aggregationDepth": Param("aggregationDepth", "suggested depth for treeAggregate (>= 2)", 2, lambda v: v >= 2, converter=int),
        "loss": Param("loss", "The loss function to be optimized. Supported options: squaredError, huber",
                      "squaredError", lambda v: v in ("squaredError", "huber")),
        "epsilon": Param("epsilon", "The shape parameter to control the amount of robustness. Must be > 1.0.", 1.35,
                         lambda v: v > 1.0, converter=float),
        "gramDtype": Param("gramDtype", "device compute precision of the normal-equation Gram pass "
                                        "(fp64 | fp32 | fp32split | bf16 | fp8; fp32split: f32 statistics "
                                        "from split-bf16 products, exact-f32-class error at the bf16 MFMA "
                                        "rate)", "fp64", lambda v: v in _GRAM_DTYPES),
    }


def _weight_of(params, tbl):
    if params.isSet("weightCol") and params.getOrDefault("weightCol"):
        w = tbl.column(params.getOrDefault("weightCol"))
        return w.values.to(torch.float64) if w.values.dtype != torch.float32 else w.values
    return None


def _fit_checks(params, tbl, X) -> list:
    """Data errors of a fit as pending device flags (``runtime/checks.py``; no host sync): the
    features' own pending checks (``VectorAssembler`` nulls), a null feature vector, and a null
    weight -- Spark 2.4 fails the job on the latter (``Row(label: Double, weight: Double, ...)``
    pattern in ``LinearRegression.train`` -> ``scala.MatchError``)."""
    checks = list(getattr(X, "checks", []))
    live = None
    if X.valid is not None:
        live = tbl.sel_mask()
        checks.append(defer((live & ~X.valid).any(), lambda: ValueError("features column contains nulls")))
    if params.isSet("weightCol") and params.getOrDefault("weightCol"):
        name = params.getOrDefault("weightCol")
        wc = tbl.column(name)
        if wc.valid is not None:
            live = tbl.sel_mask() if live is None else live
            checks.append(defer((live & ~wc.valid).any(), lambda: SparkException(
                f"Job aborted due to stage failure: scala.MatchError: [null weight in column {name}] "
                f"(of class org.apache.spark.sql.catalyst.expressions.GenericRowWithSchema)")))
        checks.extend(wc.checks)
    return [c for c in checks if c is not None]


_FL_CHECKED: dict = {}  # (id(schema), features, label) -> the schema that passed (rebuilt actions share it)


def _check_features_label(params, df: DataFrame):
    schema = df.schema
    fc, lc = params.getOrDefault("featuresCol"), params.getOrDefault("labelCol")
    if _FL_CHECKED.get((id(schema), fc, lc)) is schema:
        return fc, lc
    try:
        ft = ColRef(fc).data_type(schema)
    except AnalysisException:
        raise ValueError(f"Field \"{fc}\" does not exist.\nAvailable fields: {', '.join(schema.names)}") from None
    if not isinstance(ft, VectorUDT):
        raise ValueError(f"requirement failed: Column {fc} must be of type struct<type:tinyint,size:int,"
                         f"indices:array<int>,values:array<double>> but was actually {ft.simpleString()}.")
    lt = ColRef(lc).data_type(schema)
    if not is_numeric(lt):
        raise ValueError(f"requirement failed: Column {lc} must be of type numeric but was actually of type "
                         f"{lt.simpleString()}.")
    if len(_FL_CHECKED) >= 256:
        _FL_CHECKED.clear()
    _FL_CHECKED[(id(schema), fc, lc)] = schema
    return fc, lc


def _fused_scan_stats(params, df: DataFrame):
    """The fit's statistics computed inside ONE pass over the source with the DQ chain fused in:
    the CSV scan kernel itself for f64 statistics (``scanfuse.try_fused_gram`` / the cutter:
    scan + DQ chain + VectorAssembler + Gram, no row ever stored), or the stream Gram with the
    chain in its stage prologue for bf16 / f32 statistics over in-memory columns
    (``streamfuse.try_fused_stream``), when the DataFrame is that shape and the fit is an
    unweighted normal-equation one; else None."""
    p0 = df._plan  # both fused paths need an unevaluated Project / Filter chain on top
    if not isinstance(p0, (Project, Filter)) or p0._memo is not None:
        return None
    if params.getOrDefault("loss") != "squaredError" or params.getOrDefault("solver") not in ("auto", "normal"):
        return None
    if params.isSet("weightCol") and params.getOrDefault("weightCol"):
        return None
    gd = _gram_dtype(params, df)
    sess = getattr(df, "sparkSession", None)
    if sess is None or getattr(sess, "device", None) is None or sess.device.type != "cuda":
        return None
    fc, lc = _check_features_label(params, df)
    if gd == "fp64":
        # an action that rebuilt a chain of the same structure over the same cached input replays
        # the lowered kernel (sql/skey.py): only the launch and its outputs are new
        rk = scanfuse.route_key(p0.skey(), fc, lc, sess)
        fused = scanfuse.replay(rk, p0, sess)
        if fused is not None:
            return fused
        return scanfuse.try_fused_gram(prune_columns(df._plan, {fc, lc}), fc, lc, sess, route_key=rk)
    # bf16 / exact-f32 statistics over in-memory columns: the DQ chain in the stream Gram's
    # stage prologue, one HBM pass (ops/streamfuse.py); a rebuilt chain of the same structure
    # replays the analyzed launch
    sk = p0.skey()
    rk = (sk, fc, lc, gd, sess.device.index) if sk is not None else None
    fused = streamfuse.replay(rk)
    if fused is not None:
        return fused
    return streamfuse.try_fused_stream(prune_columns(df._plan, {fc, lc}), fc, lc, sess, gd, route_key=rk)


def _features_label(params, df: DataFrame):
    fc, lc = _check_features_label(params, df)
    # only (features, label, weight) are read: prune every other derived column (ColumnPruning)
    need = {fc, lc}
    if params.isSet("weightCol") and params.getOrDefault("weightCol"):
        need.add(params.getOrDefault("weightCol"))
    tbl = execute(prune_columns(df._plan, need), df.sparkSession)
    X = tbl.column(fc)
    y = tbl.column(lc)
    return tbl, X, y



def _gram_dtype(est, df) -> str:
    """Explicit ``gramDtype`` param, else the session's ``dq4ml.gramDtype``, else fp64."""
    if est.isSet("gramDtype"):
        return est.getOrDefault("gramDtype")
    sess = getattr(df, "sparkSession", None)
    v = sess.conf.get("dq4ml.gramDtype", None) if sess is not None else None
    return v if v in _GRAM_DTYPES else est.getOrDefault("gramDtype")

@param_accessors
class LinearRegression(_LRParams):
    uid_prefix = "linReg"

    def __init__(self, uid=None, **kw):
        super().__init__(uid)
        for k, v in kw.items():
            self.set(k, v)

    def fit(self, dataset: DataFrame, params=None) -> "LinearRegressionModel":
        est = self.copy(params) if params else self
        return est._train(dataset)

    # persistence (params only, DefaultParamsWriter layout) -----------------------------------
    def write(self):
        from .persistence import ParamsWriter

        return ParamsWriter(self, "org.apache.spark.ml.regression.LinearRegression")

    def save(self, path):
        self.write().save(path)

    @classmethod
    def load(cls, path):
        from .persistence import load_params_only

        return load_params_only(cls, path)

    def _train(self, df: DataFrame) -> "LinearRegressionModel":
        reps = df.__dict__.get("_fit_replays")
        rp = reps.get(self.uid) if reps else None
        if rp is not None:
            if rp.valid(self, df):
                return rp.issue(self, df)
            del reps[self.uid]
        fused = _fused_scan_stats(self, df)
        if fused is not None:
            return self._train_wls(df, None, None, None, fused.d, fused)
        tbl, X, y = _features_label(self, df)
        d = _num_features(X)
        if d <= 0:
            raise ValueError("requirement failed: The number of features must be positive.")
        loss, solver = self.getOrDefault("loss"), self.getOrDefault("solver")
        if loss == "huber" and solver == "normal":
            raise ValueError("requirement failed: LinearRegression with huber loss only supports L-BFGS solver.")
        if loss == "squaredError" and ((solver == "auto" and d <= MAX_NUM_FEATURES) or solver == "normal"):
            return self._train_wls(df, tbl, X, y, d)
        from .lbfgs_path import train_lbfgs

        return train_lbfgs(self, df, tbl, X, y, d)

    def _train_wls(self, df, tbl, X, y, d, fused=None):
        self.__dict__.pop("_tiled_plan", None)  # set by THIS fit's _wls_stats only
        sess = getattr(df, "sparkSession", None)
        overlap = sess is not None and str(sess.conf.get("dq4ml.fit.overlapTail", "true")).lower() in ("1", "true")
        if fused is not None:  # statistics already reduced by the fused scan / stream kernel
            flat, checks = fused.flat, list(fused.checks)
            tracing.add_rows("gram", fused.nrows)
            # a fused CSV scan keeps its tail on the compute stream (the next action's scan waits for
            # this solve, see scanfuse.try_fused_gram); the in-memory stream route (config 4) puts it
            # on the side stream beside the next step's pass -- at N > 1 its all-reduce too
            overlap = overlap and bool(getattr(fused, "overlap_ok", False))
        else:
            # (not the wide SYRK: two of them co-running would split the CUs, each block of the
            # one-block-per-CU grid needs a whole CU's LDS)
            pipe = _pipe_stream(df, tbl) if overlap and d <= 64 else None
            if pipe is not None:
                caller = faststream.current(faststream.dev_index(df.sparkSession.device))
                with faststream.use(pipe):
                    flat, checks = self._wls_stats(df, tbl, X, y, d, overlap, caller)
                    hc = _rank_health(df)
                    model = self._wls_finish(df, flat, d, checks + ([hc] if hc is not None else []), overlap)
                plan = self.__dict__.pop("_tiled_plan", None)
                if plan is not None and model.__dict__.get("_pending") is not None:
                    # kept by the DataFrame (its lifetime bounds the plan's tensors), per estimator;
                    # the plan's row operands were made on `pipe`: replays on the other pipeline
                    # streams wait for that once
                    ready = torch.cuda.Event()
                    ready.record(pipe)
                    df.__dict__.setdefault("_fit_replays", {})[self.uid] = _FitReplay(self, df, plan, checks, d,
                                                                                       (ready, pipe))
                return model
            flat, checks = self._wls_stats(df, tbl, X, y, d, overlap)
            self.__dict__.pop("_tiled_plan", None)
        hc = _rank_health(df)  # (a deferred flag: read with the fit's first host read)
        return self._wls_finish(df, flat, d, checks + ([hc] if hc is not None else []), overlap)

    def _wls_stats(self, df, tbl, X, y, d, overlap, caller=None):
        checks = _fit_checks(self, tbl, X)
        w = _weight_of(self, tbl)
        sel = tbl.sel
        yv, yvalid = y.values, y.valid
        if yvalid is not None:
            sel = yvalid if sel is None else (sel & yvalid)
        zd = X.meta.get("zero_dead", False)
        x_zero_dead = yvalid is None and (tbl.sel is None or (zd is not False and zd is tbl.sel))
        with tracing.span("gram"):
            gd = _gram_dtype(self, df)
            flat = None
            if _fusable_assembly(X, w, gd, yvalid):
                parts, asel = X.sources  # fused VectorAssembler + Gram: the features are never packed
                flat = kernels.gram_cols(parts, yv, sel if sel is not None else asel)
            elif _skinny_cols(X, gd):
                flat = kernels.gram_skinny_cols(X.sources[0], yv, w, sel)  # f64, no pack
            elif _lazy_sources(X):
                # f64 / f32 statistics of 9..64 same-dtype source columns: LDS-DMA stream kernel
                # over the columns themselves (None: mixed / unaligned sources -> pack below)
                parts, asel = X.sources
                flat = kernels.gram_stream_cols(parts, yv, w, sel if sel is not None else asel, gd)
            if flat is None:
                # a single-GPU overlapped asynchronous fit folds the Gram partials on its side
                # stream too.  Not with N > 1: co-running with the next Gram pass the fold's loads
                # queue behind its HBM stream (8 us alone, ~100 us co-running), and the side stream
                # must still fit the all-reduce and the solve into one Gram period
                defer = overlap and _async_conf(df) and d <= 64 and not comm.collectives_active()
                # the wide (MFMA-bound) SYRK: its fold, all-reduce and solve go to the side stream
                # with the solve at any world size -- the memory-bound fold co-runs with the next
                # fit's SYRK instead of following it
                if d > 64 and overlap and _async_fit(df, _DEVICE_FLAT, d, _wls_args(self, d)):
                    defer = True
                Xv = _values(X, caller)
                if _replayable(Xv, w):
                    # resolve the launch once: a repeated fit of this DataFrame replays it
                    plan = device.TiledGramPlan(native.hip(), Xv, yv, None, sel, x_zero_dead)
                    flat = plan.launch(device._stream(), defer)
                    self._tiled_plan = (plan, defer)
                else:
                    flat = kernels.gram_stats(Xv, yv, w, sel, gd, x_zero_dead=x_zero_dead, defer=defer)
        tracing.add_rows("gram", tbl.nrows)
        return flat, checks

    def _wls_finish(self, df, flat, d, checks, overlap):
        args = (flat,) + _wls_args(self, d)[1:]
        if _async_fit(df, flat, d, args):
            # dq4ml.fit.overlapTail: fit tail (Gram fold + X1 all-reduce + device solve) on a side
            # stream, so it overlaps whatever the caller enqueues next on the compute stream (the
            # next fit's Gram pass) instead of following it (in-process A/B, 1x MI355X, d = 32:
            # 159.3 -> 151.7 us per fit at 1.25e7 rows, 1033 -> 1025 us at 1e8; scripts/overlap_ab.py)
            # (the tail stays on the side stream for a pipelined fit too: on its pipeline stream the
            # one-workgroup solve co-runs with the next fit's whole-GPU Gram, gets a sliver of a CU
            # and holds up the fit after that -- same-box A/B 0.142-0.184 vs 0.137 ms per fit)
            with tracing.span("solve"):
                pending = _PendingWLS(args, overlap=overlap, checks=checks)  # resolved on first read
            return _async_model(self, df, pending)
        if hasattr(flat, "finish"):
            flat = flat.finish()
        with tracing.span("allreduce"):
            flat = comm.all_reduce_sum(flat)  # X1: data-parallel Gram all-reduce (RCCL over xGMI)
        args = (flat,) + args[1:]
        # host bookkeeping first, while the Gram kernels run; the solve's D2H is the only sync
        model = LinearRegressionModel(self.uid, None, 0.0)
        self.copyValues(model)
        with tracing.span("solve"):
            wls, stats = fit_wls_flat(*args)
        verify(checks)  # the solve has synchronised: reading the flags costs one small copy
        model._coefficients = DenseVector(wls.coefficients)
        model._intercept = float(wls.intercept)
        model._set_summary(LinearRegressionTrainingSummary(model, df, wls, wls.objectiveHistory,
                                                           stats=stats, solver=wls.solver))
        return model


def _values(X, caller):
    """``X.values``.  In a pipelined fit (``caller``: the caller's stream, the current stream being
    a pipeline stream) a lazily assembled column is materialized on the CALLER's stream -- the
    column memoizes the matrix for every later reader of the DataFrame, which runs there -- and
    the pipeline stream waits for it (no cross-stream read of a pipe-made tensor)."""
    from ..sql.table import LazyVectorColumn

    if caller is None or not isinstance(X, LazyVectorColumn) or X.materialized:
        return X.values
    pipe = faststream.raw(caller.device_index)
    with faststream.use(caller):
        v = X.values
    native.hip().stream_wait(pipe, caller.cuda_stream)
    return v


def _wls_args(est, d):
    """``fit_wls_flat`` arguments after ``flat``, from the estimator's params."""
    return (None, d, est.getOrDefault("fitIntercept"), float(est.getOrDefault("regParam")),
            float(est.getOrDefault("elasticNetParam")), bool(est.getOrDefault("standardization")), True,
            "auto", int(est.getOrDefault("maxIter")), float(est.getOrDefault("tol")))


def _async_model(est, df, pending) -> "LinearRegressionModel":
    """The model of an asynchronous fit: coefficients and summary resolve on first read."""
    model = LinearRegressionModel(est.uid, None, 0.0)
    model._pending = pending
    est.copyValues(model)
    model._set_summary(LinearRegressionTrainingSummary(model, df, pending, None, stats=pending, solver=pending))
    return model


def _replay_env():
    # the knobs that change what a replayed fit would enqueue (DQ4ML_FORCE_COLLECTIVES acts
    # through comm.collectives_active(), compared separately)
    return os.environ.get("DQ4ML_FIT_REPLAY"), os.environ.get("DQ4ML_FIT_PIPELINE")


def _replayable(Xv, w) -> bool:
    """The fit's Gram pass can be captured as a :class:`ops.device.TiledGramPlan`: bf16 fragment
    tiles on the GPU, no weights."""
    return (isinstance(Xv, TiledBF16) and w is None and Xv.buf.is_cuda and Xv.d <= 64
            and os.environ.get("DQ4ML_FIT_REPLAY", "1") != "0")


class _FitReplay:
    """A repeated asynchronous fit of the SAME DataFrame by the same estimator (the benchmark loop,
    cross-validation folds over one cached table, a refit after ``transform``): the table, its
    columns, the checks and the Gram launch are those of the first fit, so the replay only
    allocates outputs and enqueues the pass, the fold, the all-reduce and the solve -- none of the
    plan walking, schema resolution, column pruning and operand preparation of ``_train``.

    Held by the DataFrame (``df._fit_replays[estimator uid]``), so the plan's tensors live exactly
    as long as the data they describe.  Valid while the estimator's params, the session conf, the
    collectives state and the dispatch-relevant ``DQ4ML_*`` knobs equal those of the recorded fit,
    and tracing is off (a traced fit takes the full path to record its spans); anything else
    drops the replay."""

    __slots__ = ("pmap", "conf", "env", "coll", "plan", "defer", "checks", "d", "args", "ring", "dev", "ready",
                 "waited")

    def __init__(self, est, df, plan_defer, checks, d, ready=None):
        self.pmap = dict(est._paramMap)
        self.conf = dict(df.sparkSession.conf._conf)
        self.env = _replay_env()
        self.coll = comm.collectives_active()
        self.plan, self.defer = plan_defer
        self.checks, self.d = list(checks), d
        self.args = _wls_args(est, d)[1:]
        self.dev = faststream.dev_index(df.sparkSession.device)
        dev = df.sparkSession.device
        self.ring = _pipe_streams[(dev, _tail_masks(dev) is not None)]
        # (event, stream) after the recorded fit's operands were made: every other pipeline
        # stream waits for it before its first replay
        self.ready = ready
        self.waited = set() if ready is None else {ready[1].cuda_stream}

    def valid(self, est, df) -> bool:
        return (est._paramMap == self.pmap and df.sparkSession.conf._conf == self.conf
                and _replay_env() == self.env and comm.collectives_active() == self.coll
                and not tracing.enabled())

    def issue(self, est, df):
        ring = self.ring  # the pipeline streams (_pipe_stream without the conf / env reads)
        pipe = ring[1][ring[0] % len(ring[1])]
        ring[0] += 1
        ps = pipe.cuda_stream
        if self.ready is not None and ps not in self.waited:
            pipe.wait_event(self.ready[0])
            self.waited.add(ps)
        native.hip().stream_wait(ps, faststream.raw(self.dev))
        with faststream.use(pipe):
            flat = self.plan.launch(ps, self.defer)
            pending = _PendingWLS((flat,) + self.args, overlap=True, checks=self.checks)
        return _async_model(est, df, pending)


def _num_features(X) -> int:
    """Feature count without materializing a lazily assembled column."""
    from ..sql.table import LazyVectorColumn

    if isinstance(X, LazyVectorColumn) and not X.materialized:
        return int(X.meta["ml_attr"]["num_attrs"])
    return int(X.values.shape[0])


def _fusable_assembly(X, w, gram_dtype, yvalid) -> bool:
    from ..sql.table import LazyVectorColumn

    if not isinstance(X, LazyVectorColumn) or X.materialized or w is not None or gram_dtype != "bf16":
        return False
    parts, _ = X.sources
    return all(p.is_cuda and p.dtype in (torch.float32, torch.float64, torch.bfloat16, torch.int32, torch.int64,
                                          torch.bool, torch.uint8) for p in parts)


def _lazy_sources(X) -> bool:
    from ..sql.table import LazyVectorColumn

    return isinstance(X, LazyVectorColumn) and not X.materialized


def _skinny_cols(X, gram_dtype) -> bool:
    """f64 statistics of a lazily assembled narrow vector, straight from its source columns."""
    from ..sql.table import LazyVectorColumn

    if not isinstance(X, LazyVectorColumn) or X.materialized or gram_dtype != "fp64":
        return False
    parts, _ = X.sources
    d = sum(1 if p.dim() == 1 else int(p.shape[0]) for p in parts)
    return 1 <= d <= 8 and all(p.is_cuda and p.dtype in (torch.float32, torch.float64, torch.bfloat16, torch.int32,
                                                         torch.int64, torch.bool, torch.uint8) for p in parts)


def _rank_health(df):
    """Rank-health barrier before the first distributed fit of a session (``dq4ml.healthCheck``:
    ``once`` (default) | ``always`` | ``never``) — a dead rank surfaces as ``RankFailure``."""
    if not comm.collectives_active():
        return
    sess = getattr(df, "sparkSession", None)
    mode = str(sess.conf.get("dq4ml.healthCheck", "once")).lower() if sess is not None else "once"
    if mode == "never" or (mode == "once" and getattr(sess, "_health_checked", False)):
        return None
    chk = comm.health_check(float(sess.conf.get("dq4ml.healthCheckTimeout", "30")) if sess is not None else 30.0,
                            deferred=True)
    if sess is not None:
        sess._health_checked = True
    return chk


def _async_conf(df) -> bool:
    sess = getattr(df, "sparkSession", None)
    return sess is not None and str(sess.conf.get("dq4ml.fit.async", "false")).lower() in ("1", "true", "yes")


def _async_fit(df, flat, d, args) -> bool:
    """Asynchronous normal-equation fit (session config ``dq4ml.fit.async``): device statistics
    and a device solver for the branch -- Cholesky (no L1) for <= 64 features, OWLQN (L1) up to
    k = QN_DEVICE_MAX_K, the large-k assembly + Jacobi-PCG (no L1, k >= DEVICE_SOLVE_MIN_K: the
    wide config-5 fit) -> the solve is enqueued on the device and the host does not wait for the
    fit; coefficients, summary and any Spark warning/exception materialize on first read (edge
    cases re-solve on the host with identical semantics)."""
    sess = getattr(df, "sparkSession", None)
    if sess is None or str(sess.conf.get("dq4ml.fit.async", "false")).lower() not in ("1", "true", "yes"):
        return False
    if not (getattr(flat, "is_cuda", False) and d >= 1):
        return False
    _, _, fit_icpt, reg, enet = args[:5]
    # L1 (OWLQN, the lab's own regParam=1 / elasticNetParam=1) runs on the device too: one wave
    # for k <= 128, one co-resident grid launch up to QN_DEVICE_MAX_K (wls_qn_grid.hip)
    from .optim import QN_DEVICE_MAX_K

    if enet != 0.0 and reg != 0.0:
        return d + (1 if fit_icpt else 0) <= QN_DEVICE_MAX_K
    return d <= 64 or d + (1 if fit_icpt else 0) >= DEVICE_SOLVE_MIN_K


class _DeviceFlat:  # (_async_fit's eligibility probe before the statistics exist)
    is_cuda = True


_DEVICE_FLAT = _DeviceFlat()
_tail_streams = {}
_pipe_streams = {}


def _pipe_stream(df, tbl):
    """Compute stream for this asynchronous fit's statistics pass (``dq4ml.fit.pipeline``, default
    2, or 3 with collectives): consecutive fits alternate over that many streams, each ordered after
    the caller's stream, so fit k+1's Gram blocks start on the CUs that fit k's drain frees instead
    of waiting for fit k's last block (the drain and launch are most of the ~25 us fixed cost of a
    pass).  Data-parallel fits fold on their compute stream before the all-reduce, which holds that
    stream ~100 us while the next pass streams HBM: a third stream keeps a pass in flight meanwhile
    (forced-RCCL shard 0.151 -> 0.143 ms per fit; without collectives depth 3 loses, 0.130 -> 0.133,
    profiles/r6/pipeline_depth_ab.log).  Every fit still runs its whole pass; results are per fit
    and unchanged.  None: the caller's stream."""
    if not _async_conf(df):
        return None
    sess = df.sparkSession
    depth = int(os.environ.get("DQ4ML_FIT_PIPELINE")
                or sess.conf.get("dq4ml.fit.pipeline", "3" if comm.collectives_active() else "2"))
    dev = getattr(sess, "device", None)
    if depth < 2 or dev is None or dev.type != "cuda":
        return None
    masks = _tail_masks(dev)
    key = (dev, masks is not None)
    ring = _pipe_streams.get(key)
    if ring is None or len(ring[1]) != depth:
        if masks is not None:  # Gram passes off the CUs reserved for the fit tail
            ring = [0, [streams.cu_masked_stream(masks[0], masks[2], dev, tag=i) for i in range(depth)]]
        else:
            ring = [0, [torch.cuda.Stream(device=dev) for _ in range(depth)]]
        _pipe_streams[key] = ring
    st = ring[1][ring[0] % depth]
    ring[0] += 1
    native.hip().stream_wait(st.cuda_stream, faststream.raw(faststream.dev_index(dev)))
    return st


# DQ4ML_TAIL_STANDIN=blocks:usec -- after each overlapped fit's all-reduce, a stand-in kernel of
# `blocks` workgroups holding a CU slot for `usec` us (rowops.hip standin) runs on the tail
# stream, bracketed by timing events: (end - start) - usec is how long the emulated collective
# waited for CUs beside the next fit's Gram pass (tests/test_gpu_pipeline.py, ops/device.py
# set_gram_reserve).  None: off.
_STANDIN = None
STANDIN_EVENTS = []


def set_tail_standin(spec):
    global _STANDIN
    _STANDIN = None if not spec else tuple(int(v) for v in str(spec).split(":"))
    STANDIN_EVENTS.clear()


def _standin(h, side):
    blocks, usec = _STANDIN
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(side)
    h.standin(blocks, usec, side.cuda_stream)
    e1.record(side)
    STANDIN_EVENTS.append((e0, e1, usec))


set_tail_standin(os.environ.get("DQ4ML_TAIL_STANDIN"))


def _tail_masks(dev):
    """(Gram CUs, tail CUs, CU count) when ``dq4ml.gram.reserveCUs`` > 0 and CU masking is asked
    for (``DQ4ML_CU_MASK=1``), else None: the pipelined Gram passes and the fit tail then run on
    disjoint CUs.  Off by default: measured, the masked Gram pass ran 0.46-0.49 ms instead of
    0.14 ms and the masked tail waited 100-136 us (profiles/r5_tail_reserve.md); unmasked, a
    tail kernel starts within ~6 us beside a running pass."""
    reserve = device.gram_reserve()
    if reserve <= 0 or os.environ.get("DQ4ML_CU_MASK", "0") != "1" or dev is None or dev.type != "cuda":
        return None
    cus = device._cus(native.hip())
    tail = streams.reserved_cu_ids(reserve, cus)
    keep = [c for c in range(cus) if c not in set(tail)]
    return keep, tail, cus


def _tail_stream(dev, wide: bool = False) -> "torch.cuda.Stream":
    """The fit tail's side stream.  ``wide``: the large-k tail (fold, all-reduce, assembly, PCG) of
    the MFMA-bound wide SYRK gets a HIGH-priority stream of its own.  HIP deals the streams of a
    process round-robin over its few hardware queues, and a plain side stream landed on the
    compute stream's queue, where the tail serialized behind the next fit's prologue (10.5 ->
    9.5 ms per 1.25e6 x 4096 fit once the host reads were gone).  A separate queue at normal
    priority (a CU-masked stream over every CU) lost in a same-process A/B, 10.45-10.51 against
    8.97-9.01 ms per fit (profiles/r6/wide_tail_ab.log, profiles/r6_wide_async.md): the tail's fold
    then interleaves with the next fit's SYRK and stalls its gang rounds; at high priority the
    fold drains first, and the LDS-free PCG runs beside the SYRK.

    The tall (d <= 64) fits' tail gets a high-priority stream too: with every collective forced
    through RCCL the 1.25e7-row shard ran 0.158 -> 0.149-0.152 ms per fit, single-GPU 0.130 -> 0.129
    and 1e8 rows 1.018-1.026 -> 1.018 (same-box A/B, profiles/r6/tall_tail_prio_ab.log)."""
    masks = _tail_masks(dev)
    key = (dev, masks is not None, wide)
    st = _tail_streams.get(key)
    if st is None:
        if masks is not None:
            st = streams.cu_masked_stream(masks[1], masks[2], dev, tag=98 if wide else 99)
        else:
            st = torch.cuda.Stream(device=dev, priority=-1)
        _tail_streams[key] = st
    return st



class _PendingWLS:
    """A WLS solve enqueued on the device (``ops.device.wls_small``); ``resolve()`` syncs once.

    ``overlap=True``: the fit tail — X1 all-reduce of the flat statistics (RCCL) and the solve —
    runs on a per-device side stream ordered after the Gram pass, so the compute stream is free
    for the next launch at once (the Gram kernel leaves CU slots for the one-workgroup solve and
    the RCCL kernel).  ``resolve()`` orders the caller's stream after the tail before reading."""

    pending_fit = True

    def __init__(self, args, overlap: bool = False, checks=None):
        flat, d, fit_icpt, reg, enet, std_f, std_l = args[:7]
        max_iter, tol = args[8], args[9]
        self._done = None
        self._checks = list(checks or [])
        self._qn = enet != 0.0 and reg != 0.0  # OWLQN branch (wls_qn_kernel) instead of Cholesky
        self._sysm = None  # large-k branch: the assembled system (wls_large.hip)

        def solve(flat):
            if self._qn:
                return device.wls_qn_small(flat, d, fit_icpt, reg, enet, std_f, std_l, max_iter, tol)
            if d > 64:  # large k: assembly + Jacobi-PCG, budgeted from the last solve of this order
                self._sysm = device.wls_assemble(flat, d, fit_icpt, reg, enet, std_f, std_l)
                self._budget = _pcg_budget.get(self._sysm.k, 16)
                device.wls_pcg_enqueue(self._sysm, d, PCG_RTOL, self._budget)
                return self._sysm.o
            return device.wls_small(flat, d, fit_icpt, reg, enet, std_f, std_l)
        if hasattr(flat, "finish") and not overlap:
            flat = flat.finish()
        if overlap:
            h = native.hip()
            self._dev = faststream.dev_index(flat.device)
            side = _tail_stream(flat.device, wide=d > 64)
            h.stream_wait(side.cuda_stream, faststream.raw(self._dev))
            with faststream.use(side):
                if hasattr(flat, "finish"):
                    flat = flat.finish()  # Gram partial slabs -> flat statistics, on the side stream
                flat.record_stream(side)  # produced on the compute stream, consumed here
                with tracing.span("allreduce"):
                    flat = comm.all_reduce_sum(flat)
                if _STANDIN is not None:  # (diagnostics) a collective's channel blocks, emulated
                    _standin(h, side)
                self.out = solve(flat)
                self._done = h.event_record(side.cuda_stream)  # a native ring event of the side stream
        else:
            flat = comm.all_reduce_sum(flat)
            self.out = solve(flat)
        self.args = (flat,) + tuple(args[1:])
        self._res = None

    def resolve(self):
        if self._res is None:
            flat, d = self.args[0], self.args[1]
            if self._done is not None:
                native.hip().stream_wait_event(faststream.raw(self._dev), self._done)
            host = self.out.cpu().numpy()
            verify(self._checks)  # data errors of the fit surface here, on first read
            if self._sysm is not None:
                self._res = self._resolve_large(host)
                return self._res
            if self._qn:
                from .optim import owlqn_result

                r = owlqn_result(host, d)
                # handed back (label / weight short-circuits, history capacity): the native driver,
                # not a second device solve
                self._res = r if r is not None else fit_wls_flat(*self.args, host_only=True)
                return self._res
            if int(host[d + 1]) != 0:  # edge case: the host driver owns warnings/errors/fallbacks
                self._res = fit_wls_flat(*self.args, host_only=True)
            else:
                from .optim import WLSModel

                args = self.args

                def diag_inv():
                    return fit_wls_flat(*args)[0].diagInvAtWA
                wls = WLSModel(host[:d].copy(), float(host[d]), diag_inv, np.zeros(1), "cholesky")
                self._res = (wls, GramStats.scalars_only(host[d + 2:d + 7], d))
        return self._res


    def _resolve_large(self, o):
        """The large-k solve's control block -> model: PCG not done within the enqueued budget
        continues from its state (host-checked chunks); every fallback is ``wls_large_result``'s."""
        from .optim import wls_large_result

        flat, d = self.args[0], self.args[1]
        sysm = self._sysm
        if self._done is not None:  # the continuation chunks run on the caller's (now ordered) stream
            cur = torch.cuda.current_stream(flat.device)
            for t in (sysm.A, sysm.b, sysm.minv, sysm.aStd, sysm.o, sysm.work):
                t.record_stream(cur)
        o = device.wls_pcg_drive(sysm, d, o, self._budget)
        if o[device.PCG_CONV] != 0.0 and o[device.PCG_STATUS] == 0.0:
            # the next fit of this order enqueues what this one needed (+2): converged iterations
            # after that are no-op launches, too few only costs a host-checked continuation
            _pcg_budget[sysm.k] = int(min(96, max(8, o[device.PCG_ITERS] + 2)))
        return wls_large_result(flat, sysm, o, d, *self.args[2:])


# Jacobi-PCG iterations to enqueue for an asynchronous large-k solve, per system order k
_pcg_budget = {}


class PredictExpr(Expr):
    """``prediction = features . coef + intercept`` (K7, fused device GEMV)."""

    def __init__(self, features: str, coef: np.ndarray, intercept: float):
        self.features, self.coef, self.intercept = features, coef, intercept

    def children(self):
        return [ColRef(self.features)]

    def data_type(self, schema):
        return DoubleType()

    def nullable(self, schema):
        return False

    def sql_name(self):
        return "prediction"

    def eval(self, ctx: EvalContext) -> ColumnData:
        X = ctx.table.column(self.features)
        with tracing.span("predict"):
            return ColumnData(DoubleType(), kernels.predict(X.values, self.coef, self.intercept), X.valid,
                              checks=list(X.checks))


@param_accessors
class LinearRegressionModel(_LRParams):
    uid_prefix = "linReg"

    def __init__(self, uid: Optional[str], coefficients: Vector, intercept: float, scale: float = 1.0):
        super().__init__(uid)
        self._pending = None  # _PendingWLS of an asynchronous fit
        self._coef_v = None if coefficients is None else (
            coefficients if isinstance(coefficients, Vector) else DenseVector(coefficients))
        self._icpt_v = _JavaFloat(intercept)
        self._scale_v = scale
        self._summary = None

    def _materialize(self):
        if self._pending is not None:
            wls, _ = self._pending.resolve()
            self._coef_v = DenseVector(np.asarray(wls.coefficients, dtype=np.float64))
            self._icpt_v = _JavaFloat(float(wls.intercept))
            self._scale_v = float(getattr(wls, "scale", self._scale_v))  # (huber: sigma)
            self._pending = None

    @property
    def scale(self):
        self._materialize()
        return self._scale_v

    @scale.setter
    def scale(self, v):
        self._materialize()
        self._scale_v = v

    @property
    def _coefficients(self) -> Vector:
        self._materialize()
        return self._coef_v

    @_coefficients.setter
    def _coefficients(self, v):
        self._pending, self._coef_v = None, v if isinstance(v, Vector) else DenseVector(v)

    @property
    def _intercept(self):
        self._materialize()
        return self._icpt_v

    @_intercept.setter
    def _intercept(self, v):
        self._materialize()
        self._icpt_v = _JavaFloat(v)

    # pyspark-style properties that are also callable (Java spelling) -----------------------------
    @property
    def coefficients(self):
        return _CallableVector(self._coefficients.toArray())

    @property
    def intercept(self):
        return self._intercept

    @property
    def numFeatures(self):
        return _JavaInt(len(self._coefficients))

    def _set_summary(self, s):
        self._summary = s
        return self

    @property
    def hasSummary(self):
        return self._summary is not None

    @property
    def summary(self) -> "LinearRegressionTrainingSummary":
        if self._summary is None:
            raise RuntimeError(f"No training summary available for this {type(self).__name__}")
        return self._summary

    def predict(self, features) -> float:
        v = features.toArray() if isinstance(features, Vector) else np.asarray(features, dtype=np.float64)
        return _JavaFloat(float(np.dot(self._coefficients.toArray(), v)) + float(self._intercept))

    def transform(self, df: DataFrame) -> DataFrame:
        fc, pc = self.getOrDefault("featuresCol"), self.getOrDefault("predictionCol")
        if not pc:
            return df
        ColRef(fc).data_type(df.schema)
        from ..sql.expressions import Alias

        exprs = [ColRef(n) for n in df.columns if n != pc] + \
                [Alias(PredictExpr(fc, self._coefficients.toArray(), float(self._intercept)), pc)]
        return DataFrame(Project(df._plan, exprs), df.sparkSession)

    def evaluate(self, df: DataFrame) -> "LinearRegressionSummary":
        return LinearRegressionSummary(self, df)

    # persistence ---------------------------------------------------------------------------
    def write(self):
        from .persistence import LinearRegressionModelWriter

        return LinearRegressionModelWriter(self)

    def save(self, path):
        self.write().save(path)

    @classmethod
    def read(cls):
        from .persistence import LinearRegressionModelReader

        return LinearRegressionModelReader()

    @classmethod
    def load(cls, path):
        return cls.read().load(path)

    def __repr__(self):
        return f"LinearRegressionModel: uid={self.uid}, numFeatures={len(self._coefficients)}"


class _CallableVector(DenseVector):
    def __call__(self):
        return self


class LinearRegressionSummary:
    """Metrics over ``model.transform(df)`` (``RegressionMetrics`` semantics of Spark 2.4): one fused
    predict + reduction pass on the device (K7+K8), lazily, shared by every metric."""

    def __init__(self, model: LinearRegressionModel, df: DataFrame, diag_inv=None, stats: GramStats = None):
        self._model = model
        self._df = df
        self._diag_src = diag_inv  # WLSModel (lazy), array, or None
        self._stats = stats
        self._m = None
        self._pred_df = None

    def __call__(self):  # Java spelling: model.summary()
        return self

    @property
    def predictions(self) -> DataFrame:
        if self._pred_df is None:
            self._pred_df = self._model.transform(self._df)
        return self._pred_df

    @property
    def predictionCol(self):
        return self._model.getOrDefault("predictionCol")

    @property
    def labelCol(self):
        return self._model.getOrDefault("labelCol")

    @property
    def featuresCol(self):
        return self._model.getOrDefault("featuresCol")

    def _resolve_fit(self):
        pass

    def _metrics(self):
        if self._m is None:
            self._resolve_fit()
            tbl = self._df._table()
            X = tbl.column(self.featuresCol)
            y = tbl.column(self.labelCol)
            sel = tbl.sel
            if y.valid is not None:
                sel = y.valid if sel is None else (sel & y.valid)
            shift = float(self._stats.bBar) if self._stats is not None else 0.0
            with tracing.span("metrics"):
                sums = kernels.regression_metrics(X.values, y.values, self._model._coefficients.toArray(),
                                                  float(self._model._intercept), sel, shift)
                sums = comm.all_reduce_sum(sums)
            self._m = _Metrics(sums.cpu().numpy(), shift, not self._model.getOrDefault("fitIntercept"))
        return self._m

    @property
    def numInstances(self):
        return _JavaInt(int(round(self._metrics().n)))

    @property
    def degreesOfFreedom(self):
        k = len(self._model._coefficients)
        return _JavaInt(self.numInstances - k - (1 if self._model.getOrDefault("fitIntercept") else 0))

    @property
    def explainedVariance(self):
        return _JavaFloat(self._metrics().ss_reg / self._metrics().n)

    @property
    def meanAbsoluteError(self):
        return _JavaFloat(self._metrics().sum_abs_err / self._metrics().n)

    @property
    def meanSquaredError(self):
        return _JavaFloat(self._metrics().ss_err / self._metrics().n)

    @property
    def rootMeanSquaredError(self):
        return _JavaFloat(np.sqrt(self._metrics().ss_err / self._metrics().n))

    @property
    def r2(self):
        m = self._metrics()
        return _JavaFloat(1.0 - m.ss_err / (m.ss_y if m.through_origin else m.ss_tot))

    @property
    def r2adj(self):
        icpt = 1 if self._model.getOrDefault("fitIntercept") else 0
        n = self.numInstances
        return _JavaFloat(1 - (1 - self.r2) * (n - icpt) / (n - len(self._model._coefficients) - icpt))

    @property
    def residuals(self) -> DataFrame:
        from ..sql.expressions import Alias, BinOp, Cast

        p = self.predictions
        e = Alias(BinOp("-", Cast(ColRef(self.labelCol), "double"), ColRef(self.predictionCol)), "residuals")
        return _CallableDF(Project(p._plan, [e]), p.sparkSession)

    @property
    def devianceResiduals(self):
        r = self.residuals._table()
        col = r.columns[0]
        live = r.sel_mask() & col.valid_mask(r.device)
        v = col.values[live]
        if self._model.isSet("weightCol") and self._model.getOrDefault("weightCol"):
            w = self.predictions._table().column(self._model.getOrDefault("weightCol")).values[live]
            v = v * torch.sqrt(w.to(torch.float64))
        return _jarr([float(v.min()), float(v.max())])

    @property
    def _diag_inv(self):
        self._resolve_fit()
        src = self._diag_src
        if src is None:
            return np.zeros(1)
        return np.asarray(src.diagInvAtWA if hasattr(src, "diagInvAtWA") else src)

    def _require_std_errors(self):
        if self._diag_inv.shape[0] == 1 and self._diag_inv[0] == 0:
            raise RuntimeError("No Std. Error of coefficients available for this LinearRegressionModel")

    @property
    def coefficientStandardErrors(self):
        self._require_std_errors()
        rss = self.meanSquaredError * self.numInstances
        sigma2 = rss / self.degreesOfFreedom
        return _jarr(np.sqrt(self._diag_inv * sigma2))

    @property
    def tValues(self):
        se = self.coefficientStandardErrors
        est = self._model._coefficients.toArray()
        if self._model.getOrDefault("fitIntercept"):
            est = np.concatenate([est, [float(self._model._intercept)]])
        return _jarr(est / se)

    @property
    def pValues(self):
        from scipy.stats import t as student_t

        return _jarr(2.0 * (1.0 - student_t.cdf(np.abs(self.tValues), self.degreesOfFreedom)))


class _CallableDF(DataFrame):
    def __call__(self):
        return self


class LinearRegressionTrainingSummary(LinearRegressionSummary):
    def __init__(self, model, df, diag_inv, objective_history, stats=None, solver="auto"):
        if getattr(diag_inv, "pending_fit", False):  # asynchronous fit: everything resolves on first read
            self._pending_fit = diag_inv
            super().__init__(model, df, None, None)
            self._hist_v, self._solver_v = None, None
            return
        self._pending_fit = None
        super().__init__(model, df, diag_inv, stats)
        self._hist_v = np.asarray(objective_history, dtype=np.float64)
        self._solver_v = solver

    def _resolve_fit(self):
        if self._pending_fit is not None:
            wls, stats = self._pending_fit.resolve()
            self._diag_src, self._stats = wls, stats
            self._hist_v, self._solver_v = np.asarray(wls.objectiveHistory, dtype=np.float64), wls.solver
            self._pending_fit = None

    @property
    def _history(self):
        self._resolve_fit()
        return self._hist_v

    @property
    def solver(self):
        self._resolve_fit()
        return self._solver_v

    @property
    def objectiveHistory(self):
        return _jarr(self._history)

    @property
    def totalIterations(self):
        """Spark 2.4: ``objectiveHistory.length``."""
        return _JavaInt(len(self._history))


class _Metrics:
    """RegressionMetrics from the fused reduction: sums over live rows of
    [n, y-s, (y-s)^2, r, r^2, |r|, p-s, (p-s)^2] with shift s (numerically stable SStot/SSreg)."""

    def __init__(self, sums, shift, through_origin):
        n, sy, syy, sr, srr, sabs, sp, spp = (float(v) for v in sums[:8])
        self.n = n
        self.through_origin = through_origin
        mean_y_shifted = sy / n
        self.mean_y = shift + mean_y_shifted
        self.ss_err = srr
        self.sum_abs_err = sabs
        self.ss_tot = syy - n * mean_y_shifted ** 2
        # SSy = sum(y^2) = sum((y-s)^2) + 2 s sum(y-s) + n s^2
        self.ss_y = syy + 2 * shift * sy + n * shift * shift
        # SSreg = sum((p - ybar)^2) = sum((p-s)^2) - 2 (ybar-s) sum(p-s) + n (ybar-s)^2
        self.ss_reg = spp - 2 * mean_y_shifted * sp + n * mean_y_shifted ** 2


_ = (execute, Vectors)
