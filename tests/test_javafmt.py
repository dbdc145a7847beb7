"""JDK 8 number formatting (linkerd_amd.javafmt) pinned by the reference's fixture.

The admin dashboard fixture (admin/.../js/spec/fixtures/metrics.js) is real
/admin/metrics.json output of a JDK-8 linkerd: every stat.avg text there is
Double.toString(sum / (double) count) and every gauge text Float.toString(gauge).
The texts are committed as data by tests/golden/make_p5_fixture.py.
"""
import json
import os

import numpy as np
import pytest

from linkerd_amd.javafmt import double_to_string, float_to_string

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _texts():
    return json.load(open(os.path.join(GOLDEN, "p5_number_texts.json")))["texts"]


def test_fixture_avg_texts_are_jdk8_double_to_string():
    """All 142 stat.avg texts, and their sum/count consistency (P5)."""
    avgs = [t["text"] for t in _texts() if t["key"] == "stat.avg"]
    assert len(avgs) == 142
    for a in avgs:
        assert double_to_string(float(a)) == a
    summ = json.load(open(os.path.join(GOLDEN, "p5_fixture_summaries.json")))["summaries"]
    for s in summ:
        if s["count"]:
            assert double_to_string(s["sum"] / s["count"]) == double_to_string(s["avg"])


def test_fixture_gauge_texts_are_jdk8_float_to_string():
    """Gauges print through FloatingDecimal's float path, which keeps digits the
    shortest round-trip form drops: 1.48832833E12 (JDK 8) vs 1.4883283E12."""
    gauges = [t["text"].replace("E+", "E") for t in _texts() if t["key"] == "gauge"]
    assert len(gauges) > 200
    for g in gauges:
        assert float_to_string(float(g)) == g
    shortest = np.format_float_scientific(np.float32(1.48832833e12), unique=True)
    assert shortest.startswith("1.4883283e") and float_to_string(1.48832833e12) == "1.48832833E12"


@pytest.mark.parametrize("x,want", [
    (1.0, "1.0"), (1.5, "1.5"), (3030.0, "3030.0"), (1e7, "1.0E7"), (1e-4, "1.0E-4"), (0.001, "0.001"),
    (281.7352941176471, "281.7352941176471"), (0.0, "0.0"), (-0.0, "-0.0"), (9999999.0, "9999999.0"),
    (12345678.0, "1.2345678E7"), (float("nan"), "NaN"), (float("inf"), "Infinity"), (-float("inf"), "-Infinity"),
    (5e-324, "4.9E-324"), (1.7976931348623157e308, "1.7976931348623157E308"),
    # JDK-4511638 (public OpenJDK bug): JDK <= 18 FloatingDecimal anomalies
    (2.82879384806159e17, "2.82879384806159008E17"), (1e23, "9.999999999999999E22"),
])
def test_double_to_string_known_answers(x, want):
    assert double_to_string(x) == want


def test_double_to_string_round_trips():
    rng = np.random.default_rng(7)
    xs = np.concatenate([rng.integers(1, 10 ** 12, 20000) / rng.integers(1, 10 ** 6, 20000),
                         rng.standard_normal(5000) * 10.0 ** rng.integers(-30, 30, 5000)])
    for x in xs:
        assert float(double_to_string(float(x))) == float(x)


def test_float_to_string_round_trips():
    rng = np.random.default_rng(8)
    for x in (rng.standard_normal(5000) * 10.0 ** rng.integers(-30, 30, 5000)).astype(np.float32):
        assert np.float32(float(float_to_string(float(x)))) == x
