"""Java-compatible text formatting of numbers.

The reference prints every number through the JVM: ``System.out.println("RMSE: " + d)``
(``DataQuality4MachineLearningApp.java:138``), ``Dataset.show()`` cells and
``Vectors.dense(...).toString`` (``DataQuality4MachineLearningApp.java:136``) all go through
``java.lang.Double.toString``.  Transcript parity therefore needs the
exact Java rendering:

* ``1.0e-3 <= |x| < 1.0e7``  -> plain decimal with at least one fractional digit (``120.0``)
* otherwise                  -> computerized scientific notation ``d.dddE[-]n`` (``1.0E-6``)
* shortest digit string that round-trips (the JDK>=19 / Ryu behaviour; Python ``repr`` gives
  the same digits).
"""
from __future__ import annotations

import datetime as _dt
import math
from decimal import Decimal

import numpy as np

__all__ = ["java_double_str", "java_float_str", "java_str", "format_vector", "timestamp_str"]


def _digits_exp(shortest: str):
    """Return (digit string without leading/trailing zeros, decimal exponent E) so that
    value = 0.d1d2d3... * 10^(E+1)  i.e. d1.d2d3... * 10^E."""
    t = Decimal(shortest).as_tuple()
    digits = "".join(str(d) for d in t.digits).lstrip("0")
    exp = t.exponent
    stripped = digits.rstrip("0")
    exp += len(digits) - len(stripped)
    digits = stripped or "0"
    sci_e = len(digits) - 1 + exp
    return digits, sci_e


def _render(neg: bool, digits: str, e: int, a: float) -> str:
    sign = "-" if neg else ""
    if 1e-3 <= a < 1e7:
        if e >= 0:
            ip = digits[: e + 1].ljust(e + 1, "0")
            fp = digits[e + 1:] or "0"
        else:
            ip = "0"
            fp = "0" * (-e - 1) + digits
        return f"{sign}{ip}.{fp}"
    frac = digits[1:] or "0"
    return f"{sign}{digits[0]}.{frac}E{e}"


def java_double_str(x) -> str:
    """``java.lang.Double.toString(x)``."""
    x = float(x)
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    if x == 0.0:
        return "-0.0" if math.copysign(1.0, x) < 0 else "0.0"
    a = abs(x)
    digits, e = _digits_exp(repr(a))
    return _render(x < 0, digits, e, a)


def java_float_str(x) -> str:
    """``java.lang.Float.toString(x)`` (shortest float32 digits)."""
    f = np.float32(x)
    if np.isnan(f):
        return "NaN"
    if np.isinf(f):
        return "Infinity" if f > 0 else "-Infinity"
    if f == 0:
        return "-0.0" if np.signbit(f) else "0.0"
    a = abs(f)
    s = np.format_float_scientific(a, unique=True)
    digits, e = _digits_exp(s)
    return _render(bool(f < 0), digits, e, float(a))


def java_str(v) -> str:
    """String concatenation semantics of Java for the value kinds the framework prints."""
    if v is None:
        return "null"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (int, np.integer)):
        return str(int(v))
    if isinstance(v, np.float32):
        return java_float_str(v)
    if isinstance(v, (float, np.floating)):
        return java_double_str(v)
    if isinstance(v, _dt.datetime):
        return timestamp_str(v)
    return str(v)


def timestamp_str(v) -> str:
    """Spark 2.4 ``DateTimeUtils.timestampToString``: ``yyyy-MM-dd HH:mm:ss`` plus the fraction of a
    second without its trailing zeros."""
    s = v.strftime("%Y-%m-%d %H:%M:%S")
    return s + ("." + f"{v.microsecond:06d}".rstrip("0") if v.microsecond else "")


def format_vector(values) -> str:
    """``DenseVector.toString``: ``[v0,v1,...]`` with Java doubles."""
    return "[" + ",".join(java_double_str(v) for v in values) + "]"
