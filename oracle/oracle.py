"""CPU ORACLE loader (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module, and only as the checker.  The product package (linkerd_amd) never does.

Two restatements of the reference's histogram path live here:

* ``C`` -- ctypes binding of oracle/hist_oracle.c (fast; used for big cases and
  as the CPU baseline).
* ``py_*`` -- an independent pure-Python restatement (small cases only), used to
  cross-check the C restatement.

Reference lines restated (paths relative to the reference checkout):
  telemetry/core/src/main/scala/com/twitter/finagle/stats/buoyant/BucketedHistogram.scala:25-46
  telemetry/core/src/main/scala/io/buoyant/telemetry/Metric.scala:22-88
  finagle-stats 6.45.0 BucketedHistogram (third-party jar, not vendored)
"""
from __future__ import annotations

import ctypes
import math
import os
import struct
import subprocess
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libl5d_oracle.so")
NLIMITS = 1797
NBUCKETS = 1798
INT_MAX = 2147483647
PERCENTILES = (0.50, 0.90, 0.95, 0.99, 0.999, 0.9999)
SUMMARY_FIELDS = ("count", "min", "max", "sum", "p50", "p90", "p95", "p99", "p9990", "p9999", "avg")

SUMMARY_DTYPE = np.dtype([(f, "<i8") for f in SUMMARY_FIELDS[:-1]] + [("avg", "<f8")])
assert SUMMARY_DTYPE.itemsize == 88


class _Summary(ctypes.Structure):
    _fields_ = [(f, ctypes.c_int64) for f in SUMMARY_FIELDS[:-1]] + [("avg", ctypes.c_double)]


class _Hist(ctypes.Structure):
    _fields_ = [("counts", ctypes.c_int32 * NBUCKETS), ("num", ctypes.c_int64), ("total", ctypes.c_int64)]


HIST_DTYPE = np.dtype({"names": ["counts", "num", "total"],
                       "formats": [("<i4", (NBUCKETS,)), "<i8", "<i8"],
                       "offsets": [0, 7192, 7200], "itemsize": 7208})

_lock = threading.Lock()
_lib = None


def build(force: bool = False) -> str:
    """Compile oracle/hist_oracle.c (make) if the .so is missing."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    with _lock:
        if _lib is None:
            build()
            L = ctypes.CDLL(LIB_PATH)
            L.l5do_default_limits.restype = ctypes.POINTER(ctypes.c_int32)
            L.l5do_java_f2l.restype = ctypes.c_int64
            L.l5do_java_f2l.argtypes = [ctypes.c_float]
            L.l5do_java_round.restype = ctypes.c_int64
            L.l5do_java_round.argtypes = [ctypes.c_double]
            L.l5do_bucket_of.restype = ctypes.c_int
            L.l5do_bucket_of.argtypes = [ctypes.c_int64]
            L.l5do_midpoint.restype = ctypes.c_int64
            L.l5do_midpoint.argtypes = [ctypes.c_int]
            L.l5do_make_limits.restype = ctypes.c_int
            L.l5do_make_limits.argtypes = [ctypes.c_double, ctypes.POINTER(ctypes.c_int32), ctypes.c_int]
            L.l5do_ingest.restype = ctypes.c_int
            L.l5do_ingest.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_size_t, ctypes.c_int]
            L.l5do_snapshot_all.restype = None
            L.l5do_snapshot_all.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int]
            L.l5do_summary_of_counts.restype = None
            L.l5do_summary_of_counts.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
            L.l5do_summarize_counts_n.restype = ctypes.c_int
            L.l5do_summarize_counts_n.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                                  ctypes.c_void_p, ctypes.c_int]
            L.l5do_export.restype = None
            L.l5do_export.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
            L.l5do_hist_size.restype = ctypes.c_size_t
            assert L.l5do_hist_size() == HIST_DTYPE.itemsize
            _lib = L
        return _lib


def limits() -> np.ndarray:
    return np.ctypeslib.as_array(lib().l5do_default_limits(), shape=(NLIMITS,)).copy()


class OracleHistograms:
    """S finagle BucketedHistograms in one numpy structured array (C oracle)."""

    def __init__(self, nseries: int):
        self.nseries = int(nseries)
        self.h = np.zeros(self.nseries, dtype=HIST_DTYPE)

    def ingest(self, series: np.ndarray, values: np.ndarray, threads: int = 1) -> int:
        series = np.ascontiguousarray(series, dtype=np.uint32)
        values = np.ascontiguousarray(values, dtype=np.float32)
        assert series.shape == values.shape
        return lib().l5do_ingest(self.h.ctypes.data, self.nseries, series.ctypes.data,
                                 values.ctypes.data, series.size, int(threads))

    def snapshot(self, reset: bool = True) -> np.ndarray:
        out = np.zeros(self.nseries, dtype=SUMMARY_DTYPE)
        lib().l5do_snapshot_all(self.h.ctypes.data, self.nseries, out.ctypes.data, int(reset))
        return out

    def counts(self) -> np.ndarray:
        return self.h["counts"].copy()

    def totals(self) -> np.ndarray:
        return self.h["total"].copy()

    def nums(self) -> np.ndarray:
        return self.h["num"].copy()


def summarize_counts(counts: np.ndarray, totals: np.ndarray, threads: int = 1) -> np.ndarray:
    """Summaries for dense int32 count rows + int64 totals (num = sum of counts):
    l5do_summary_of_counts per row, rows split over `threads` workers (one C call)."""
    counts = np.ascontiguousarray(counts, dtype=np.int32).reshape(-1, NBUCKETS)
    totals = np.ascontiguousarray(totals, dtype=np.int64).reshape(-1)
    assert totals.shape[0] == counts.shape[0]
    out = np.zeros(counts.shape[0], dtype=SUMMARY_DTYPE)
    rc = lib().l5do_summarize_counts_n(counts.ctypes.data, totals.ctypes.data, counts.shape[0],
                                       out.ctypes.data, int(threads))
    assert rc == 0, f"l5do_summarize_counts_n: {rc}"
    return out


# --------------------------------------------------------------------------
# Independent pure-Python restatement (small cases only)
# --------------------------------------------------------------------------

def py_make_limits(error: float = 0.005) -> list:
    """BucketedHistogram.scala:25-40."""
    assert 0.0 < error <= 1.0
    max_value = float(INT_MAX)
    factor = 1.0 + (error * 2)
    vals = []
    n = 1.0
    while True:
        nxt = n * factor
        if nxt >= max_value:
            break
        v = int(nxt) + 1
        if v not in vals[-1:]:
            vals.append(v)
        n = nxt
    return [1] + vals


_PY_LIMITS = None


def _py_limits():
    global _PY_LIMITS
    if _PY_LIMITS is None:
        _PY_LIMITS = py_make_limits()
    return _PY_LIMITS


def py_f2l(f: float) -> int:
    """Java (long) cast of a float (JLS 5.1.3)."""
    f = struct.unpack("<f", struct.pack("<f", f))[0]
    if math.isnan(f):
        return 0
    if f >= 2.0 ** 63:
        return 2 ** 63 - 1
    if f <= -(2.0 ** 63):
        return -(2 ** 63)
    return int(f)  # Python int() truncates toward zero


def py_round(x: float) -> int:
    """java.lang.Math.round(double): floor(x + 1/2) evaluated exactly."""
    from fractions import Fraction
    if math.isnan(x):
        return 0
    return math.floor(Fraction(x) + Fraction(1, 2))


def _wrap64(v: int) -> int:
    return (v + 2 ** 63) % 2 ** 64 - 2 ** 63


def py_bucket(v: int) -> int:
    import bisect
    if v >= INT_MAX:
        return NLIMITS
    key = _wrap64(v) & 0xFFFFFFFF
    if key >= 2 ** 31:
        key -= 2 ** 32
    return bisect.bisect_right(_py_limits(), key)


def py_mid(b: int) -> int:
    L = _py_limits()
    if b == 0:
        return 0
    if b >= NLIMITS:
        return INT_MAX
    return (L[b - 1] + L[b]) // 2


class PyStat:
    """Metric.Stat over a restated finagle BucketedHistogram (Metric.scala:22-70)."""

    def __init__(self):
        self.clear()
        self.snapshotted = None

    def clear(self):
        self.counts = [0] * NBUCKETS
        self.num = 0
        self.total = 0

    def add(self, value: float):
        v = py_f2l(value)
        if v >= INT_MAX:
            self.total = _wrap64(self.total + INT_MAX)
            b = NLIMITS
        else:
            self.total = _wrap64(self.total + v)
            b = py_bucket(v)
        self.counts[b] += 1
        self.num += 1

    def percentile(self, p: float) -> int:
        target = py_round(p * float(self.num))
        total = 0
        i = 0
        while i < NBUCKETS and total < target:
            total += self.counts[i]
            i += 1
        if i == 0:
            return 0
        if i == NBUCKETS:
            return INT_MAX
        return py_mid(i - 1)

    def summary(self) -> dict:
        nz = [b for b, c in enumerate(self.counts) if c > 0]
        mn = 0 if self.num == 0 else py_mid(nz[0])
        if self.num == 0:
            mx = 0
        elif self.counts[NBUCKETS - 1] > 0:
            mx = INT_MAX
        else:
            mx = py_mid(nz[-1])
        pct = [self.percentile(p) for p in PERCENTILES]
        avg = 0.0 if self.num == 0 else float(self.total) / float(self.num)
        return dict(zip(SUMMARY_FIELDS, [self.num, mn, mx, self.total] + pct + [avg]))

    def snapshot(self) -> dict:
        self.snapshotted = self.summary()
        return self.snapshotted

    def bucket_and_counts(self) -> list:
        L = _py_limits()
        out = []
        for b, c in enumerate(self.counts):
            if c > 0:
                lower = 0 if b == 0 else L[b - 1]
                upper = L[b] if b < NLIMITS else INT_MAX
                out.append((lower, upper, c))
        return out

    def reset(self) -> list:
        buckets = self.bucket_and_counts()
        self.clear()
        return buckets
