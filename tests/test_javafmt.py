import numpy as np

from net.jgp.labs.sparkdq4ml_amd.utils.javafmt import java_double_str, java_float_str, format_vector


def test_java_double_plain_and_scientific():
    cases = [(23.1, "23.1"), (120.0, "120.0"), (-1.0, "-1.0"), (1e-6, "1.0E-6"), (0.001, "0.001"), (1e7, "1.0E7"), (9999999.0, "9999999.0"), (0.0, "0.0"), (-0.0, "-0.0"), (1.5e-4, "1.5E-4"), (218.0035110637381, "218.0035110637381"), (123456789.0, "1.23456789E8"), (0.5, "0.5"), (2.8021924953004715, "2.8021924953004715"), (float("nan"), "NaN"), (float("inf"), "Infinity"), (float("-inf"), "-Infinity"), (1e21, "1.0E21"), (100.0, "100.0"), (12345.678, "12345.678")]
    for v, s in cases:
        assert java_double_str(v) == s, (v, java_double_str(v), s)


def test_java_float():
    assert java_float_str(np.float32(0.1)) == "0.1"
    assert java_float_str(np.float32(1e-5)) == "1.0E-5"


def test_vector_format():
    assert format_vector([14.0]) == "[14.0]"
    assert format_vector([0.5, 1e-6]) == "[0.5,1.0E-6]"


# ---- JDK 8 FloatingDecimal (the reference's pom.xml:59-60 targets Java 1.8) -----------------
# Known JDK <= 18 renderings where the digit string is not the shortest one (the anomalies the
# JDK 19 rewrite removed, JDK-4511638): the free-format loop's symmetric half-ULP test stops one
# digit late, and exact integers below 2^63 print every significant digit.
JDK8_KNOWN = [
    (2e23, "1.9999999999999998E23"),
    (8.41e21, "8.409999999999999E21"),
    (2.0 ** -44, "5.6843418860808015E-14"),
    (2.0 ** 60, "1.15292150460684698E18"),
    (2.82879384806159e17, "2.82879384806159008E17"),
    (1e23, "9.999999999999999E22"),
    (5e-324, "4.9E-324"),
    (1.7976931348623157e308, "1.7976931348623157E308"),
    (2.2250738585072014e-308, "2.2250738585072014E-308"),
]


def test_java8_known_outputs():
    for v, s in JDK8_KNOWN:
        assert java_double_str(v) == s, (v, java_double_str(v), s)
        assert java_double_str(-v) == "-" + s


def _parse_java(s: str) -> float:
    return float(s)  # Java's E-notation is Python-parsable


def test_java8_invariants_random_doubles():
    """The algorithm's own contract on 20 000 random doubles over the whole exponent range and on
    boundary values: (1) the string parses back to the same double; (2) it is the shortest string
    or at most ONE digit longer (the symmetric stop test's slack); (3) layout: F-form exactly for
    1e-3 <= |x| < 1e7, at least one fractional digit, E-form mantissa in [1, 10)."""
    from net.jgp.labs.sparkdq4ml_amd.utils.javafmt import java_double_str_shortest

    rng = np.random.default_rng(8)
    bits = rng.integers(0, 0x7FEFFFFFFFFFFFFF, size=20_000, dtype=np.int64)
    vals = list(bits.view(np.float64)) + [1e-3, 1e7, 9999999.999999998, 0.0009999999999999998, 1e-4, 1e22, 2.0 ** 63,
                                          2.0 ** 62 + 2048.0, 123456789012345680.0, 1.0 / 3.0, 4.35, 0.1 + 0.2]
    longer = 0
    for v in vals:
        v = float(v)
        s = java_double_str(v)
        assert _parse_java(s) == v, (v, s)
        mant = s.split("E")[0].lstrip("-")
        nd = len(mant.replace(".", "").lstrip("0").rstrip("0")) or 1
        short = java_double_str_shortest(v).split("E")[0].lstrip("-")
        ns = len(short.replace(".", "").lstrip("0").rstrip("0")) or 1
        assert nd <= ns + 1 or abs(v) < 2.0 ** 63 and v == int(v), (v, s, java_double_str_shortest(v))
        longer += nd > ns
        assert "." in mant and not mant.endswith(".")
        if 1e-3 <= abs(v) < 1e7:
            assert "E" not in s, (v, s)
        else:
            assert "E" in s and 1.0 <= abs(float(mant)) < 10.0, (v, s)
    assert longer < len(vals) // 20  # the anomalies are rare


def test_java8_float_invariants():
    rng = np.random.default_rng(9)
    vals = rng.integers(1, 0x7F7FFFFF, size=5000, dtype=np.int64).astype(np.uint32).view(np.float32)
    for f in vals:
        s = java_float_str(f)
        assert np.float32(float(s)) == f, (f, s)
    assert java_float_str(np.float32(3.4028235e38)) == "3.4028235E38"
    assert java_float_str(np.float32(1.4e-45)) == "1.4E-45"
    assert java_float_str(np.float32(1e10)) == "1.0E10"


def test_lab_transcript_values():
    """The numbers the lab prints -- Java 8 renders them as their shortest
    strings."""
    for v, s in [(2.8021924953004755, "2.8021924953004755"), (0.9965340953376102, "0.9965340953376102"),
                 (20.979190460591617, "20.979190460591617"), (218.00351106373807, "218.00351106373807"),
                 (1.0, "1.0"), (1e-6, "1.0E-6"), (40.0, "40.0"), (0.5, "0.5")]:
        assert java_double_str(v) == s
