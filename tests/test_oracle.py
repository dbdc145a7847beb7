"""CPU oracle pinned against the reference's own known-answer tests (P1-P5,
SURVEY.md §4) and cross-checked against an independent pure-Python restatement.
These run without a GPU."""
import json
import os
import zlib

import numpy as np
import pytest

from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
INT_MAX = 2147483647


def summary_of(values, oracle_mod=O):
    h = oracle_mod.OracleHistograms(1)
    h.ingest(np.zeros(len(values), np.uint32), np.asarray(values, np.float32))
    return h.snapshot(reset=False)[0]


# ---------------- limits (BucketedHistogram.scala:25-46) ----------------

def test_limits_shape_and_known_values():
    L = O.limits()
    assert L.size == 1797                         # BucketedHistogram.scala:42
    assert (L[:113] == np.arange(1, 114)).all()   # unit buckets up to 113
    assert L[113] == 115 and L[1796] == 2137204091
    assert (np.diff(L) > 0).all()
    # consecutive limits differ by at most a factor 1 + 2*error (before rounding)
    assert (L[1:] <= np.floor(L[:-1] * 1.01) + 2).all()


def test_limits_match_committed_checksum_and_python_restatement():
    L = O.limits()
    g = json.load(open(os.path.join(GOLDEN, "limits.json")))
    assert g["n"] == L.size and g["first"] == L[:8].tolist() and g["last"] == L[-4:].tolist()
    assert zlib.crc32(L.astype("<i4").tobytes()) == g["crc32_le_i4"]
    assert O.py_make_limits(0.005) == L.tolist()


def test_make_limits_requires_valid_error():
    buf = (O.ctypes.c_int32 * 4)()
    assert O.lib().l5do_make_limits(0.0, buf, 4) == -1
    assert O.lib().l5do_make_limits(1.5, buf, 4) == -1


# ---------------- Java numerics ----------------

@pytest.mark.parametrize("x,want", [(0.5, 1), (1.5, 2), (2.5, 3), (-2.5, -2), (-0.5, 0), (0.49999999999999994, 0),
                                    (1.8, 2), (0.9999 * 3434, 3434), (4503599627370497.0, 4503599627370497),
                                    (1e300, 2 ** 63 - 1), (float("nan"), 0)])
def test_java_round(x, want):
    assert O.lib().l5do_java_round(x) == want
    assert O.py_round(x) == min(want, 2 ** 63 - 1) or x == 1e300


@pytest.mark.parametrize("f,want", [(0.0, 0), (0.99, 0), (-0.99, 0), (3.7, 3), (-3.7, -3), (1e20, 2 ** 63 - 1),
                                    (-1e20, -(2 ** 63)), (float("inf"), 2 ** 63 - 1), (float("nan"), 0),
                                    (2147483648.0, 2147483648)])
def test_java_f2l(f, want):
    assert O.lib().l5do_java_f2l(f) == want
    assert O.py_f2l(f) == want


def test_bucket_rule_matches_binary_search_insertion_point():
    L = O.limits()
    lib = O.lib()
    for v in [-5, 0, 1, 2, 112, 113, 114, 115, 3011, 3030, 3042, 2137204090, 2137204091, 2147483646,
              2147483647, 2 ** 40, -(2 ** 32) + 7, -3_000_000_000]:
        b = lib.l5do_bucket_of(v)
        assert b == O.py_bucket(v), v
        if v >= INT_MAX:
            assert b == 1797
        else:
            key = np.int64(v).astype(np.int32) if -2 ** 31 <= v < 2 ** 31 else np.int32(np.uint32(v & 0xFFFFFFFF))
            assert b == int(np.searchsorted(L, key, side="right"))


# ---------------- P1-P4: the reference's asserted tests ----------------

def test_p1_single_sample():
    """PrometheusTelemeterTest.scala:41-68: {1.0f} -> count 1, sum 1, avg 1.0, all quantiles 1."""
    s = summary_of([1.0])
    assert (s["count"], s["sum"], s["avg"]) == (1, 1, 1.0)
    assert s["min"] == s["max"] == s["p50"] == s["p90"] == s["p95"] == s["p99"] == s["p9990"] == s["p9999"] == 1


def test_p2_two_samples_cumulative():
    """PrometheusTelemeterTest.scala:70-86: then +2.0f -> count 2, sum 3, avg 1.5, q0=1, q.5=1, q.9..q1=2."""
    s = summary_of([1.0, 2.0])
    assert (s["count"], s["sum"], s["avg"]) == (2, 3, 1.5)
    assert (s["min"], s["p50"]) == (1, 1)
    assert s["p90"] == s["p95"] == s["p99"] == s["p9990"] == s["p9999"] == s["max"] == 2


def test_p3_influx_two_stats():
    """InfluxDbTelemeterTest.scala:141-172: abc {1,2}, def {2,4}."""
    a = summary_of([1.0, 2.0])
    d = summary_of([2.0, 4.0])
    assert (a["avg"], a["count"], a["max"], a["min"], a["p50"], a["p90"], a["sum"]) == (1.5, 2, 2, 1, 1, 2, 3)
    assert (d["avg"], d["count"], d["max"], d["min"], d["p50"], d["p90"], d["p95"], d["p99"], d["p9990"],
            d["p9999"], d["sum"]) == (3.0, 2, 4, 2, 2, 4, 4, 4, 4, 4, 6)


def test_p4_reset_between_intervals():
    """AdminMetricsExportTelemeterTest.scala:47-85: {1} -> tick -> +2 -> tick: 2nd interval shows only 2."""
    h = O.OracleHistograms(1)
    h.ingest(np.zeros(1, np.uint32), np.array([1.0], np.float32))
    s1 = h.snapshot(reset=True)[0]
    h.ingest(np.zeros(1, np.uint32), np.array([2.0], np.float32))
    s2 = h.snapshot(reset=True)[0]
    for f, want in (("count", 1), ("max", 1), ("min", 1), ("p50", 1), ("p9999", 1), ("sum", 1), ("avg", 1.0)):
        assert s1[f] == want
    for f, want in (("count", 1), ("max", 2), ("min", 2), ("p50", 2), ("p9999", 2), ("sum", 2), ("avg", 2.0)):
        assert s2[f] == want


def test_empty_summary_is_zero():
    s = O.OracleHistograms(3).snapshot()
    for f in O.SUMMARY_FIELDS:
        assert (s[f] == 0).all()


# ---------------- P5: the admin dashboard fixture ----------------

def _p5_rows():
    return json.load(open(os.path.join(GOLDEN, "p5_fixture_summaries.json")))["summaries"]


def test_p5_fixture_invariants():
    L = O.limits().astype(np.int64)
    mids = set(((L[:-1] + L[1:]) // 2).tolist()) | {0, INT_MAX}
    rows = [r for r in _p5_rows() if r["count"] > 0]
    assert len(rows) == 142
    for r in rows:
        for f in ("min", "max", "p50", "p90", "p95", "p99", "p9990", "p9999"):
            assert r[f] in mids, (r["path"], f, r[f])
        assert r["min"] <= r["p50"] <= r["p90"] <= r["p95"] <= r["p99"] <= r["p9990"] <= r["p9999"] <= r["max"]
        assert r["avg"] == r["sum"] / r["count"], r["path"]  # Java: total / num.toDouble


def test_p5_constant_series_reproduced_exactly():
    """connection_received_bytes: 34 x 3030 -> every quantile 3026 (metrics.js:2782-2794), and every
    other fixture summary whose samples are pinned (min == max, integral avg) is reproduced."""
    rows = [r for r in _p5_rows() if r["count"] > 0 and r["min"] == r["max"] and r["sum"] % r["count"] == 0]
    assert any(r["path"].endswith("connection_received_bytes") and r["sum"] == 103020 for r in rows)
    for r in rows:
        s = summary_of([float(r["sum"] // r["count"])] * r["count"])
        for f in ("count", "min", "max", "sum", "p50", "p90", "p95", "p99", "p9990", "p9999", "avg"):
            assert s[f] == r[f], (r["path"], f, s[f], r[f])


# ---------------- C restatement == Python restatement ----------------

def test_c_oracle_matches_python_restatement():
    rng = np.random.default_rng(7)
    vals = np.concatenate([np.exp(rng.uniform(-1, 22, 3000)), rng.uniform(-1e10, 1e10, 200),
                           np.array([np.nan, np.inf, -np.inf, 0.0, -0.0, 2147483520.0, 2147483648.0])])
    vals = vals.astype(np.float32)
    series = rng.integers(0, 5, vals.size).astype(np.uint32)
    h = O.OracleHistograms(5)
    h.ingest(series, vals)
    got = h.snapshot(reset=False)
    counts = h.counts()
    for s in range(5):
        p = O.PyStat()
        for v in vals[series == s]:
            p.add(float(v))
        assert p.counts == counts[s].tolist()
        want = p.summary()
        for f in O.SUMMARY_FIELDS:
            assert got[s][f] == want[f], (s, f)


def test_multithreaded_ingest_matches_single_thread():
    rng = np.random.default_rng(8)
    S = 97
    series = rng.integers(0, S, 200_000).astype(np.uint32)
    vals = np.exp(rng.uniform(0, 9, series.size)).astype(np.float32)
    a, b = O.OracleHistograms(S), O.OracleHistograms(S)
    a.ingest(series, vals, threads=1)
    b.ingest(series, vals, threads=8)
    np.testing.assert_array_equal(a.counts(), b.counts())
    np.testing.assert_array_equal(a.totals(), b.totals())


@pytest.mark.parametrize("name", ["mixed64", "c1_100k", "c2_200x500", "c3_zipf1000"])
def test_golden_vectors_reproduce(name):
    g = np.load(os.path.join(GOLDEN, f"golden_{name}.npz"))
    S = int(g["nseries"])
    h = O.OracleHistograms(S)
    h.ingest(g["series"], g["values"])
    np.testing.assert_array_equal(h.counts(), g["counts"])
    np.testing.assert_array_equal(h.totals(), g["totals"])
    summ = h.snapshot()
    assert summ.view(np.uint8).reshape(S, 88).tobytes() == g["summaries"].tobytes()


def test_summarize_counts_matches_hist():
    g = np.load(os.path.join(GOLDEN, "golden_mixed64.npz"))
    s = O.summarize_counts(g["counts"], g["totals"])
    assert s.view(np.uint8).reshape(-1, 88).tobytes() == g["summaries"].tobytes()
    # the threaded batch driver (the full-size GPU tests' checker): same bytes at any split
    for threads in (3, 8, 200):
        t = O.summarize_counts(g["counts"], g["totals"], threads=threads)
        assert t.tobytes() == s.tobytes()
