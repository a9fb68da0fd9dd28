"""Java-compatible text formatting of numbers.

The reference prints every number through the JVM: ``System.out.println("RMSE: " + d)``
(``DataQuality4MachineLearningApp.java:138``), ``Dataset.show()`` cells and
``Vectors.dense(...).toString`` (``DataQuality4MachineLearningApp.java:136``) all go through
``java.lang.Double.toString``.  The reference compiles for Java 1.8 (``pom.xml:59-60``) on Spark
2.4.4, so the digits are those of JDK 8's ``sun.misc.FloatingDecimal`` -- NOT the shortest
round-trip string of JDK >= 19 (Raffaello Giulietti's Ryu-like rewrite):

* ``1.0e-3 <= |x| < 1.0e7``  -> plain decimal with at least one fractional digit (``120.0``)
* otherwise                  -> computerized scientific notation ``d.dddE[-]n`` (``1.0E-6``)
* digits: :func:`_fd_dtoa`, a transcription of the JDK 8 digit generator's contract --
  integers below 2^63 print exactly (low insignificant digits rounded off:
  ``2^60 -> 1.15292150460684698E18``), everything else by the Steele & White / dtoa free-format
  loop with a SYMMETRIC half-ULP stopping test, Java int / long arithmetic where the JDK uses it
  (including its wrap-around) and exact big-integer arithmetic elsewhere, and at least two digits
  in E-form.  Java 8's output always parses back to the same double, but is sometimes one digit
  longer than the shortest string (``2.82879384806159E17`` prints as ``2.82879384806159008E17``).

Parity is pinned to the algorithm's own invariants and known JDK 8 outputs
(``tests/test_javafmt.py``); no JVM is available here to diff against.
"""
from __future__ import annotations

import datetime as _dt
import math
import struct
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


# ---- JDK 8 sun.misc.FloatingDecimal.BinaryToASCIIBuffer.dtoa ---------------------------------
_EXP_SHIFT = 52
_FRACT_HOB = 1 << _EXP_SHIFT
_SIGNIF_MASK = _FRACT_HOB - 1
_MAX_SMALL_BIN_EXP, _MIN_SMALL_BIN_EXP = 62, -(63 // 3)
_SMALL_5_POW = [5 ** i for i in range(14)]
_LONG_5_POW = [5 ** i for i in range(27)]
_N_5_BITS = [0] + [(5 ** i).bit_length() for i in range(1, 27)]  # ceil(log2(5^i))


def _i32(v: int) -> int:  # Java int wrap-around
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v >> 31 else v


def _i64(v: int) -> int:  # Java long wrap-around
    v &= 0xFFFFFFFFFFFFFFFF
    return v - (1 << 64) if v >> 63 else v


def _insignificant_digits_for_pow2(p2: int) -> int:
    # insignificantDigitsNumber[p2] = floor(p2 * log10(2)) for 1 < p2 < 64
    return int(p2 * 0.30102999566398119521) if 1 < p2 < 64 else 0


def _estimate_dec_exp(fract_bits: int, bin_exp: int) -> int:
    d2 = struct.unpack("<d", struct.pack("<Q", 0x3FF0000000000000 | (fract_bits & _SIGNIF_MASK)))[0]
    d = (d2 - 1.5) * 0.289529654 + 0.176091259 + float(bin_exp) * 0.301029995663981
    return math.floor(d)


def _develop_long_digits(dec_exp: int, lvalue: int, insignificant: int):
    if insignificant:
        pow10 = 10 ** insignificant
        residue = lvalue % pow10
        lvalue //= pow10
        dec_exp += insignificant
        if residue >= pow10 >> 1:
            lvalue += 1
    s = str(lvalue)
    t = s.rstrip("0")
    dec_exp += len(s) - len(t)
    return t, dec_exp + len(t)  # (digits, decExponent)


def _roundup(digits: list, dec_exponent: int) -> int:
    i = len(digits) - 1
    q = digits[i]
    if q == 9:
        while q == 9 and i > 0:
            digits[i] = 0
            i -= 1
            q = digits[i]
        if q == 9:  # carry out: a high-order 1, the rest 0s, larger exponent
            digits[0] = 1
            return dec_exponent + 1
    digits[i] = q + 1
    return dec_exponent


def _fd_dtoa(bin_exp: int, fract_bits: int, n_significant_bits: int):
    """(digit string, decExponent) of JDK 8 ``dtoa(binExp, fractBits, nSignificantBits, true)``:
    value = 0.d1d2... * 10^decExponent.  ``fract_bits`` is normalized (bit 52 set)."""
    tail_zeros = (fract_bits & -fract_bits).bit_length() - 1
    n_fract_bits = _EXP_SHIFT + 1 - tail_zeros
    n_tiny_bits = max(0, n_fract_bits - bin_exp - 1)
    if _MIN_SMALL_BIN_EXP <= bin_exp <= _MAX_SMALL_BIN_EXP and n_tiny_bits == 0:
        # an integer below 2^63: its exact digits, insignificant low-order ones rounded off
        insignificant = (_insignificant_digits_for_pow2(bin_exp - n_significant_bits - 1)
                         if bin_exp > n_significant_bits else 0)
        v = fract_bits << (bin_exp - _EXP_SHIFT) if bin_exp >= _EXP_SHIFT else fract_bits >> (_EXP_SHIFT - bin_exp)
        return _develop_long_digits(0, v, insignificant)
    dec_exp = _estimate_dec_exp(fract_bits, bin_exp)
    B5 = max(0, -dec_exp)
    B2 = B5 + n_tiny_bits + bin_exp
    S5 = max(0, dec_exp)
    S2 = S5 + n_tiny_bits
    M5 = B5
    M2 = B2 - n_significant_bits
    fract_bits >>= tail_zeros
    B2 -= n_fract_bits - 1
    common2 = min(B2, S2)
    B2 -= common2
    S2 -= common2
    M2 -= common2
    if n_fract_bits == 1:  # exact power of two: the next smaller double is half as far
        M2 -= 1
    if M2 < 0:
        B2 -= M2
        S2 -= M2
        M2 = 0
    b_bits = n_fract_bits + B2 + (_N_5_BITS[B5] if B5 < len(_N_5_BITS) else B5 * 3)
    ten_s_bits = S2 + 1 + (_N_5_BITS[S5 + 1] if S5 + 1 < len(_N_5_BITS) else (S5 + 1) * 3)
    digits = []
    e_form = dec_exp < -3 or dec_exp >= 8  # (decided on the first estimate, as the JDK does)
    if b_bits < 64 and ten_s_bits < 64:
        # Java int (b_bits, ten_s_bits < 32) or long arithmetic, wrap-around included
        w = _i32 if (b_bits < 32 and ten_s_bits < 32) else _i64
        p5 = _SMALL_5_POW if w is _i32 else _LONG_5_POW
        mask = 31 if w is _i32 else 63
        b = w(w(w(fract_bits) * p5[B5]) << (B2 & mask))
        s = w(p5[S5] << (S2 & mask))
        m = w(p5[M5] << (M2 & mask))
        tens = w(s * 10)
        q = int(b / s) if b * s >= 0 else -int(abs(b) // abs(s))
        b = w(10 * (b - q * s))
        m = w(m * 10)
        low = b < m
        high = w(b + m) > tens
        if q == 0 and not high:
            dec_exp -= 1  # the estimate was one too high: drop the leading zero
        else:
            digits.append(q)
        if e_form or dec_exp < -3 or dec_exp >= 8:
            high = low = False
        while not low and not high:
            q = b // s
            b = w(10 * (b % s))
            m = w(m * 10)
            if m > 0:
                low = b < m
                high = w(b + m) > tens
            else:  # m overflowed: certainly > b, and b + m > tens overflowed too
                low = high = True
            digits.append(q)
        low_diff = w(w(b << 1) - tens)
    else:
        # FDBigInteger: exact
        S = (5 ** S5) << S2
        B = (fract_bits * 5 ** B5) << B2
        M = (5 ** (M5 + 1)) << (M2 + 1)
        tenS = (5 ** (S5 + 1)) << (S2 + 1)
        q, B = B // S, 10 * (B % S)
        low = B < M
        high = B + M > tenS
        if q == 0 and not high:
            dec_exp -= 1
        else:
            digits.append(q)
        if dec_exp < -3 or dec_exp >= 8:
            high = low = False
        while not low and not high:
            q, B = B // S, 10 * (B % S)
            M *= 10
            low = B < M
            high = B + M > tenS
            digits.append(q)
        low_diff = ((B << 1) > tenS) - ((B << 1) < tenS) if (high and low) else 0
    dec_exponent = dec_exp + 1
    if high:
        if low:
            if low_diff == 0:
                if digits[-1] & 1:
                    dec_exponent = _roundup(digits, dec_exponent)
            elif low_diff > 0:
                dec_exponent = _roundup(digits, dec_exponent)
        else:
            dec_exponent = _roundup(digits, dec_exponent)
    return "".join(str(x) for x in digits), dec_exponent


def _java_chars(neg: bool, digits: str, dec_exponent: int) -> str:
    """JDK 8 ``BinaryToASCIIBuffer.getChars`` (the Double.toString layout of dtoa's digits)."""
    sign = "-" if neg else ""
    nd = len(digits)
    if 0 < dec_exponent < 8:
        n = min(nd, dec_exponent)
        if n < dec_exponent:
            return f"{sign}{digits[:n]}{'0' * (dec_exponent - n)}.0"
        return f"{sign}{digits[:n]}.{digits[n:] if n < nd else '0'}"
    if -3 < dec_exponent <= 0:
        return f"{sign}0.{'0' * -dec_exponent}{digits}"
    e = dec_exponent - 1
    return f"{sign}{digits[0]}.{digits[1:] if nd > 1 else '0'}E{e}"


def _java8_digits(bits: int, exp_bits: int, mant_bits: int):
    """(neg, digits, decExponent) of a finite non-zero IEEE value's bit pattern (JDK 8
    ``getBinaryToASCIIConverter``: normalization of subnormals, nSignificantBits)."""
    bias = (1 << (exp_bits - 1)) - 1
    neg = bool(bits >> (exp_bits + mant_bits))
    fract = bits & ((1 << mant_bits) - 1)
    bin_exp = (bits >> mant_bits) & ((1 << exp_bits) - 1)
    if bin_exp == 0:  # subnormal: normalize
        width = 64 if mant_bits == 52 else 32
        leading = width - fract.bit_length()
        shift = leading - (width - 1 - mant_bits)
        fract <<= shift
        bin_exp = 1 - shift
        n_sig = width - leading
    else:
        fract |= 1 << mant_bits
        n_sig = mant_bits + 1
    bin_exp -= bias
    digits, dec_exponent = _fd_dtoa(bin_exp, fract << (_EXP_SHIFT - mant_bits), n_sig)
    return neg, digits, dec_exponent


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
    bits = struct.unpack("<Q", struct.pack("<d", x))[0]
    return _java_chars(*_java8_digits(bits, 11, 52))


def java_double_str_shortest(x) -> str:
    """The JDK >= 19 rendering (shortest round-trip digits, Python ``repr``'s) -- kept for
    comparison with :func:`java_double_str` (Java 8)."""
    x = float(x)
    if math.isnan(x) or math.isinf(x) or x == 0.0:
        return java_double_str(x)
    a = abs(x)
    digits, e = _digits_exp(repr(a))
    return _render(x < 0, digits, e, a)


def java_float_str(x) -> str:
    """``java.lang.Float.toString(x)`` (JDK 8: the same digit generator at float precision)."""
    f = np.float32(x)
    if np.isnan(f):
        return "NaN"
    if np.isinf(f):
        return "Infinity" if f > 0 else "-Infinity"
    if f == 0:
        return "-0.0" if np.signbit(f) else "0.0"
    return _java_chars(*_java8_digits(int(np.asarray(f, dtype=np.float32).view(np.uint32)), 8, 23))


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
