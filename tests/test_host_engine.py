"""Host logic around the engine, on CPU: the StatEngine registry (id reclamation on
MetricsTree.prune), Stat.reset atomicity under concurrent Stat.add, and the buffer
checks HistogramEngine applies before anything reaches the C-ABI.

The engine underneath is OracleEngine: the C oracle behind HistogramEngine's
method signatures (test infrastructure only; the product has no CPU fallback).
"""
import threading

import numpy as np
import pytest

from linkerd_amd import _native as N
from linkerd_amd.engine import HistogramEngine
from linkerd_amd.telemetry import MetricsTree, MetricsTreeStatsReceiver, StatEngine


class OracleEngine:
    """HistogramEngine's snapshot/peek/ingest over the C oracle (one lock, like the
    C-ABI's per-context mutex)."""

    def __init__(self, S, oracle):
        self.max_series = S
        self.O = oracle
        self.h = oracle.OracleHistograms(S)
        self.lock = threading.Lock()
        self.ingested = 0

    def ingest(self, series, values):
        with self.lock:
            assert self.h.ingest(np.asarray(series, np.uint32), np.asarray(values, np.float32)) == 0
            self.ingested += len(series)

    def snapshot(self, first=0, count=None, reset=True, with_counts=False):
        with self.lock:
            count = self.max_series - first if count is None else count
            sl = slice(first, first + count)
            counts = self.h.h["counts"][sl].copy()
            out = self.O.summarize_counts(counts, self.h.h["total"][sl])
            if reset:
                self.h.h[sl] = 0
        return (out, counts) if with_counts else out

    def peek(self, sid):
        with self.lock:
            row = self.h.h["counts"][sid]
            L = self.O.limits()
            nz = np.flatnonzero(row > 0)
            out = np.zeros(nz.size, dtype=N.BUCKET_COUNT_DTYPE)
            out["lower"] = np.where(nz == 0, 0, L[np.maximum(nz - 1, 0)])
            out["upper"] = np.where(nz < 1797, L[np.minimum(nz, 1796)], 2147483647)
            out["count"] = row[nz]
            return out


@pytest.fixture
def limits_from_oracle(monkeypatch, oracle):
    # StatEngine.reset_series reads the limits from the C-ABI (l5dh_limits); the
    # library may be built here, but use the oracle's to keep this a host-only test
    monkeypatch.setattr(N, "limits", oracle.limits)


def test_prune_reclaims_series_ids(oracle, limits_from_oracle):
    """More Stats than the engine holds, created and pruned in turn (client churn,
    MetricsPruningModule.scala:14-39): ids are reused and a reused id starts empty."""
    eng = StatEngine(engine=OracleEngine(8, oracle), batch=4)
    tree = MetricsTree(eng)
    stats = MetricsTreeStatsReceiver(tree)
    for gen in range(5):
        ss = [stats.scope("rt", "r", "client", f"c{gen}_{i}").stat("request_latency_ms") for i in range(8)]
        for i, s in enumerate(ss):
            for v in range(i + 1):
                s.add(float(v + 1))
        assert eng.registered == 8
        assert [s.summary.count for s in ss] == list(range(1, 9))
        with pytest.raises(RuntimeError, match="full"):
            stats.stat("one_too_many")
        stale = ss[0]
        stats.scope("rt", "r").prune()
        assert eng.registered == 0
        stale.add(5.0)  # a pruned Stat still accepts samples, which go nowhere
        assert stale.summary.count == 0 and stale.peek() == []
    fresh = stats.stat("fresh")
    assert fresh.summary.count == 0 and fresh.peek() == []


def test_stat_reset_is_atomic_under_concurrent_adds(oracle, limits_from_oracle):
    """Metric.Stat.reset (Metric.scala:44-51) while 8 threads add: every sample ends
    up in exactly one returned bucket list or in the final summary."""
    eng = StatEngine(engine=OracleEngine(4, oracle), batch=64)
    tree = MetricsTree(eng)
    stat = MetricsTreeStatsReceiver(tree).stat("lat")
    per_thread = 20_000
    returned = []
    stop = threading.Event()

    def producer(k):
        for i in range(per_thread):
            stat.add(float(1 + (i + k) % 200))

    def resetter():
        while not stop.is_set():
            buckets, _ = stat.reset()
            returned.append(sum(b.count for b in buckets))

    threads = [threading.Thread(target=producer, args=(k,)) for k in range(8)]
    r = threading.Thread(target=resetter)
    r.start()
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    stop.set()
    r.join()
    final = stat.summary.count
    assert sum(returned) + final == 8 * per_thread
    assert eng.engine.ingested == 8 * per_thread


def _bare_engine(S=100, device=0):
    e = HistogramEngine.__new__(HistogramEngine)  # no context: only the host-side checks run
    e.max_series, e.device, e._stream, e._events = S, device, None, []
    return e


def test_buffer_checks_reject_wrong_dtype_size_and_device():
    import torch
    e = _bare_engine()
    ok = e._buf(np.zeros(10, np.uint32), (np.uint32, np.int32), "series")
    assert ok
    with pytest.raises(TypeError, match="dtype"):
        e._buf(np.zeros(10, np.int64), (np.uint32, np.int32), "series")
    with pytest.raises(TypeError, match="dtype"):
        e._buf(torch.zeros(10, dtype=torch.float64), (np.float32,), "values")
    with pytest.raises(ValueError, match="at least"):
        e._buf(np.zeros(100 * 1798 - 1, np.int32), (np.int32,), "counts", 100 * 1798)
    with pytest.raises(ValueError, match="contiguous"):
        e._buf(np.zeros((10, 2), np.int32)[:, 0], (np.int32,), "counts")
    with pytest.raises(ValueError, match="read-only"):
        a = np.zeros(10, np.int64)
        a.flags.writeable = False
        e._buf(a, (np.int64,), "out", writable=True)
    with pytest.raises(ValueError, match="outside"):
        e._range(90, 20)
    with pytest.raises(ValueError, match="at least"):
        e._summ_buf(np.zeros(99 * 11, np.int64), 100, "summaries")
    assert e._summ_buf(np.zeros(100, N.SUMMARY_DTYPE), 100, "summaries")


def test_ingest_rejects_ids_outside_uint32():
    e = _bare_engine()
    with pytest.raises(ValueError, match="uint32"):
        e.ingest(np.array([-1, 2]), np.array([1.0, 2.0], np.float32))
