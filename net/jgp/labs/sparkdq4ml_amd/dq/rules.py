"""DQ rules as fusable expression IR.

Each rule is a UDF object with both contracts of :mod:`..sql.udf`:

* ``call(*boxed)`` — the Java ``UDF1``/``UDF2`` row contract (``MinimumPriceDataQualityUdf.java:
  11-13``, ``PriceCorrelationDataQualityUdf.java:11-16``), including their null policies:
  rule 1 has **no** null guard (a null price unboxes -> NPE -> job failure), rule 2 maps a null
  price or guest to ``-1.0`` (then filtered out by ``WHERE ... > 0``);
* ``ir(*arg_exprs)`` — the same rule as IR, which the engine evaluates vectorized on the device
  and compiles into the fused DQ VM kernel together with the clean-up filters.

``RangeRule`` / ``NotNullRule`` / ``ThresholdRule`` generalize them for user pipelines (the
"null/range UDF filters" of the 1e9-row DQ config).
"""
from __future__ import annotations

from ..sql.expressions import (BinOp, Cast, If, IsNull, Lit, RaiseIfNull, to_expr)
from ..sql.types import DataTypes
from . import services


class DQRule:
    returnType = DataTypes.DoubleType
    name = "rule"

    def call(self, *args):
        raise NotImplementedError

    def ir(self, *args):
        raise NotImplementedError

    def __call__(self, *cols):
        from ..sql.udf import UserDefinedFunction

        return UserDefinedFunction(self.name, self.call, self.returnType, self.ir)(*cols)


class MinimumPriceDataQualityUdf(DQRule):
    """``UDF1<Double, Double>`` — ``MinimumPriceDataQualityUdf.java:7-14``."""

    serialVersionUID = -201966159201746851
    name = "minimumPriceRule"

    def call(self, price):
        if price is None:  # Java auto-unboxing of a null Double
            raise TypeError("java.lang.NullPointerException")
        return services.check_minimum_price(price)

    def ir(self, price):
        p = RaiseIfNull(Cast(to_expr(price), "double"),
                        "Failed to execute user defined function(MinimumPriceDataQualityUdf: (double) => double)"
                        " caused by java.lang.NullPointerException")
        return If(BinOp("<", p, Lit(float(services.MIN_PRICE)), ieee=True), Lit(-1.0), p)


class PriceCorrelationDataQualityUdf(DQRule):
    """``UDF2<Double, Integer, Double>`` — ``PriceCorrelationDataQualityUdf.java:7-18``."""

    serialVersionUID = 4949954702581973224
    name = "priceCorrelationRule"

    def call(self, price, guest):
        if price is None or guest is None:
            return -1.0
        return services.check_price_range(price, int(guest))

    def ir(self, price, guest):
        p = Cast(to_expr(price), "double")
        g = Cast(to_expr(guest), "int")
        bad = BinOp("and", BinOp("<", g, Lit(services.CORRELATION_MAX_GUESTS), ieee=True),
                    BinOp(">", p, Lit(float(services.CORRELATION_MAX_PRICE)), ieee=True))
        null = BinOp("or", IsNull(p), IsNull(g))
        return If(null, Lit(-1.0), If(bad, Lit(-1.0), p))


class RangeRule(DQRule):
    """``lo <= x <= hi ? x : sentinel`` (null -> sentinel)."""

    def __init__(self, lo=None, hi=None, sentinel=-1.0, name="rangeRule"):
        self.lo, self.hi, self.sentinel, self.name = lo, hi, sentinel, name

    def call(self, x):
        if x is None or (self.lo is not None and x < self.lo) or (self.hi is not None and x > self.hi):
            return self.sentinel
        return float(x)

    def ir(self, x):
        v = Cast(to_expr(x), "double")
        bad = IsNull(v)
        if self.lo is not None:
            bad = BinOp("or", bad, BinOp("<", v, Lit(float(self.lo)), ieee=True))
        if self.hi is not None:
            bad = BinOp("or", bad, BinOp(">", v, Lit(float(self.hi)), ieee=True))
        return If(bad, Lit(float(self.sentinel)), v)


class NotNullRule(RangeRule):
    def __init__(self, sentinel=-1.0, name="notNullRule"):
        super().__init__(None, None, sentinel, name)


def register_lab_rules(session):
    """The two registrations of ``DataQuality4MachineLearningApp.java:46-49``."""
    session.udf().register("minimumPriceRule", MinimumPriceDataQualityUdf(), DataTypes.DoubleType)
    session.udf().register("priceCorrelationRule", PriceCorrelationDataQualityUdf(), DataTypes.DoubleType)
