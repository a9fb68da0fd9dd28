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
