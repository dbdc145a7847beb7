"""Host-side mirror of io.buoyant.telemetry (reference: telemetry/core/src/main/scala/
io/buoyant/telemetry/{Metric,MetricsTree,MetricsTreeStatsReceiver}.scala), with
Metric.Stat backed by the MI355X engine instead of a per-Stat BucketedHistogram.

Names, argument meaning and error behaviour follow the reference:
  * MetricsTree.resolve / try_resolve / children / metric / mk_counter / mk_stat /
    register_gauge / deregister_gauge / prune (MetricsTree.scala:10-120); a type
    conflict raises ValueError ("non-stat metric already exists"), the analogue of
    IllegalArgumentException (MetricsTree.scala:82,92,103,112).
  * Metric.Stat.add / peek / snapshot / reset / summary / snapshotted_summary /
    starting_at (Metric.scala:22-70); HistogramSummary has the 11 fields of
    Metric.scala:76-88.
What changes is *where* the arithmetic runs: Stat.add appends (series id, value)
to a per-thread staging batch; batches go to the GPU through the C-ABI
(l5dh_ingest); StatEngine.snapshot_all is the batched form of the timer's
per-Stat snapshot()+reset() walk (AdminMetricsExportTelemeter.scala:154-162).
"""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

from .javamap import reference_child_order


@dataclass(frozen=True)
class HistogramSummary:
    """Metric.HistogramSummary (Metric.scala:76-88)."""
    count: int
    min: int
    max: int
    sum: int
    p50: int
    p90: int
    p95: int
    p99: int
    p9990: int
    p9999: int
    avg: float

    @staticmethod
    def from_record(rec) -> "HistogramSummary":
        return HistogramSummary(int(rec["count"]), int(rec["min"]), int(rec["max"]), int(rec["sum"]),
                                int(rec["p50"]), int(rec["p90"]), int(rec["p95"]), int(rec["p99"]),
                                int(rec["p9990"]), int(rec["p9999"]), float(rec["avg"]))


@dataclass(frozen=True)
class BucketAndCount:
    """finagle-core BucketAndCount(lowerLimit, upperLimit, count)."""
    lower: int
    upper: int
    count: int


class StatEngine:
    """Series registry + batched ingest in front of one HistogramEngine (one GPU).

    Each thread stages Stat.add calls in its own (ids, values) batch; a full batch,
    or any snapshot/peek/reset, flushes every thread's batch to the GPU.
    """

    def __init__(self, capacity: int = 1 << 16, device: int = 0, batch: int = 1 << 16, engine=None):
        if engine is None:
            from .engine import HistogramEngine
            engine = HistogramEngine(capacity, device)
        self.engine = engine
        self.capacity = int(engine.max_series)
        self.batch = int(batch)
        self._lock = threading.Lock()
        self._next = 0
        self._free: List[int] = []
        self._limits = None
        self._tls = threading.local()
        self._buffers: List["_Staging"] = []

    # registry (MetricsTree.mkStat assigns the id; MetricsTree.prune releases it)
    def register(self) -> int:
        with self._lock:
            if self._free:
                return self._free.pop()
            if self._next >= self.capacity:
                raise RuntimeError(f"histogram engine full: {self.capacity} series")
            sid = self._next
            self._next += 1
            return sid

    def release(self, sid: int) -> None:
        """Return a pruned Stat's id (MetricsPruningModule.scala:14-39 prunes closed
        clients' subtrees).  Its staged samples are flushed and its row is cleared
        on the GPU before the id can be handed out again, so a new Stat starts empty."""
        self.flush()
        self.engine.snapshot(first=sid, count=1, reset=True)
        with self._lock:
            self._free.append(sid)

    @property
    def registered(self) -> int:
        """Series ids currently held by Stats."""
        return self._next - len(self._free)

    def _staging(self) -> "_Staging":
        st = getattr(self._tls, "st", None)
        if st is None:
            st = _Staging(self.batch)
            self._tls.st = st
            with self._lock:
                self._buffers.append(st)
        return st

    def add(self, sid: int, value: float) -> None:
        st = self._staging()
        with st.lock:
            st.ids[st.n] = sid
            st.vals[st.n] = value
            st.n += 1
            if st.n == self.batch:
                self._flush_locked(st)

    def _flush_locked(self, st: "_Staging") -> None:
        if st.n:
            n, st.n = st.n, 0  # cleared first: a failed call is never re-sent (no double count)
            self.engine.ingest(st.ids[:n], st.vals[:n])

    def flush(self) -> None:
        with self._lock:
            bufs = list(self._buffers)
        for st in bufs:
            with st.lock:
                self._flush_locked(st)

    # snapshot paths
    def summary(self, sid: int, reset: bool = False) -> HistogramSummary:
        self.flush()
        rec = self.engine.snapshot(first=sid, count=1, reset=reset)[0]
        return HistogramSummary.from_record(rec)

    def peek(self, sid: int) -> List[BucketAndCount]:
        self.flush()
        return [BucketAndCount(int(b["lower"]), int(b["upper"]), int(b["count"])) for b in self.engine.peek(sid)]

    def reset_series(self, sid: int) -> List[BucketAndCount]:
        """Metric.Stat.reset (Metric.scala:44-51): bucketAndCounts + clear as ONE
        engine call (snapshot of one series with its counts and reset), so no sample
        flushed by another thread can fall between the two."""
        self.flush()
        _, counts = self.engine.snapshot(first=sid, count=1, reset=True, with_counts=True)
        if self._limits is None:
            from . import _native
            self._limits = _native.limits()
        L = self._limits
        row = counts[0]
        return [BucketAndCount(0 if b == 0 else int(L[b - 1]), int(L[b]) if b < len(L) else 2147483647, int(row[b]))
                for b in np.flatnonzero(row > 0)]

    def snapshot_all(self, reset: bool = True) -> np.ndarray:
        """Summaries of every series in one fused GPU pass (snapshot + reset)."""
        self.flush()
        return self.engine.snapshot(first=0, count=self.capacity, reset=reset)


class _Staging:
    def __init__(self, n: int):
        self.lock = threading.Lock()
        self.ids = np.zeros(n, dtype=np.uint32)
        self.vals = np.zeros(n, dtype=np.float32)
        self.n = 0


class Metric:
    """sealed trait Metric (Metric.scala:8-89)."""

    class _None:
        def __repr__(self):
            return "Metric.None"

    NONE = _None()

    class Counter:
        """Metric.Counter (Metric.scala:14-20): AtomicLong."""

        def __init__(self):
            self._lock = threading.Lock()
            self._value = 0

        def incr(self, delta: int = 1) -> None:
            with self._lock:
                self._value += int(delta)

        def get(self) -> int:
            return self._value

    class Stat:
        """Metric.Stat (Metric.scala:22-70) over the GPU engine."""

        def __init__(self, engine: Optional[StatEngine] = None):
            self._engine = engine
            # the per-Stat monitor of Metric.scala:30-33: add() reads the id and stages
            # its sample under it, and _release() takes the id away under it, so once
            # _release has run no add can stage the old id (which may be re-issued)
            self._lock = threading.Lock()
            self.series_id = engine.register() if engine is not None else None
            self._summary_snapshot: Optional[HistogramSummary] = None
            self._reset_time = time.time()

        def _eng(self) -> StatEngine:
            if self._engine is None:
                from ._native import NativeLibraryMissing
                raise NativeLibraryMissing("Metric.Stat needs a StatEngine (GPU); none attached")
            return self._engine

        @property
        def starting_at(self) -> float:
            return self._reset_time

        def add(self, value: float) -> None:
            with self._lock:
                sid = self.series_id  # read once
                if sid is None and self._engine is not None:
                    return  # pruned: like adding to a histogram no exporter reads any more
                self._eng().add(sid, value)

        def peek(self) -> List[BucketAndCount]:
            if self.series_id is None and self._engine is not None:
                return []
            return self._eng().peek(self.series_id)

        def _release(self) -> None:
            """MetricsTree.prune: hand the series id back to the engine.  The id is
            taken under the Stat's lock, so every add that saw it has already staged its
            sample; StatEngine.release then flushes those and clears the row before the
            id is handed out again."""
            with self._lock:
                sid, self.series_id = self.series_id, None
            if self._engine is not None and sid is not None:
                self._engine.release(sid)

        def snapshot(self) -> HistogramSummary:
            self._summary_snapshot = self.summary
            return self._summary_snapshot

        def reset(self) -> Tuple[List[BucketAndCount], float]:
            eng = self._eng()
            buckets = [] if self.series_id is None else eng.reset_series(self.series_id)
            now = time.time()
            delta = now - self._reset_time
            self._reset_time = now
            return buckets, delta

        @property
        def summary(self) -> HistogramSummary:
            if self.series_id is None and self._engine is not None:
                return HistogramSummary(0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0.0)
            return self._eng().summary(self.series_id, reset=False)

        @property
        def snapshotted_summary(self) -> Optional[HistogramSummary]:
            return self._summary_snapshot

        def _set_snapshot(self, summary: HistogramSummary, reset_time: Optional[float] = None) -> None:
            """Used by the batched snapshot driver (one GPU pass for all Stats)."""
            self._summary_snapshot = summary
            if reset_time is not None:
                self._reset_time = reset_time

    class Gauge:
        """Metric.Gauge (Metric.scala:72-74)."""

        def __init__(self, f: Callable[[], float]):
            self._f = f

        def get(self) -> float:
            return float(np.float32(self._f()))


class MetricsTree:
    """MetricsTree.Impl (MetricsTree.scala:38-120)."""

    def __init__(self, engine: Optional[StatEngine] = None):
        self._engine = engine
        self._trees: Dict[str, "MetricsTree"] = {}  # insertion order
        self._order: Optional[List[str]] = None
        self._tlock = threading.Lock()
        self._mlock = threading.Lock()
        self._metric = Metric.NONE

    @property
    def children(self) -> Dict[str, "MetricsTree"]:
        """Children in the reference's iteration order (ConcurrentHashMap ->
        immutable Map, MetricsTree.scala:44-45; linkerd_amd.javamap)."""
        with self._tlock:
            if self._order is None or len(self._order) != len(self._trees):
                self._order = reference_child_order(list(self._trees))
            return {k: self._trees[k] for k in self._order}

    def _get_or_mk(self, k: str) -> "MetricsTree":
        with self._tlock:
            t = self._trees.get(k)
            if t is None:
                t = MetricsTree(self._engine)
                self._trees[k] = t
            return t

    def resolve(self, scope: Sequence[str]) -> "MetricsTree":
        t = self
        for name in scope:
            t = t._get_or_mk(name)
        return t

    def try_resolve(self, scope: Sequence[str]) -> Optional["MetricsTree"]:
        t = self
        for name in scope:
            with t._tlock:
                t = t._trees.get(name)
            if t is None:
                return None
        return t

    @property
    def metric(self):
        return self._metric

    def mk_counter(self) -> Metric.Counter:
        with self._mlock:
            m = self._metric
            if isinstance(m, Metric.Counter):
                return m
            if m is Metric.NONE:
                self._metric = Metric.Counter()
                return self._metric
            raise ValueError("non-counter metric already exists")

    def mk_stat(self) -> Metric.Stat:
        with self._mlock:
            m = self._metric
            if isinstance(m, Metric.Stat):
                return m
            if m is Metric.NONE:
                self._metric = Metric.Stat(self._engine)
                return self._metric
            raise ValueError("non-stat metric already exists")

    def register_gauge(self, f: Callable[[], float]) -> None:
        with self._mlock:
            if self._metric is Metric.NONE or isinstance(self._metric, Metric.Gauge):
                self._metric = Metric.Gauge(f)
                return
            raise ValueError("non-gauge metric already exists")

    def deregister_gauge(self) -> None:
        with self._mlock:
            if self._metric is Metric.NONE:
                return
            if isinstance(self._metric, Metric.Gauge):
                self._metric = Metric.NONE
                return
            raise ValueError("non-gauge metric already exists")

    def prune(self) -> None:
        with self._tlock:
            kids = list(self._trees.values())
            self._trees.clear()
            self._order = None
        for k in kids:
            k.prune()
        with self._mlock:
            m, self._metric = self._metric, Metric.NONE
        if isinstance(m, Metric.Stat):
            m._release()

    def walk(self, prefix: Tuple[str, ...] = ()):
        """Depth-first (path, tree) pairs."""
        yield prefix, self
        for name, child in self.children.items():
            yield from child.walk(prefix + (name,))


class MetricsTreeStatsReceiver:
    """MetricsTreeStatsReceiver (MetricsTreeStatsReceiver.scala:8-28)."""

    def __init__(self, tree: MetricsTree):
        self.tree = tree

    def counter(self, *name: str) -> Metric.Counter:
        return self.tree.resolve(name).mk_counter()

    def stat(self, *name: str) -> Metric.Stat:
        return self.tree.resolve(name).mk_stat()

    def add_gauge(self, *name: str, f: Callable[[], float]):
        self.tree.resolve(name).register_gauge(f)

    def remove_gauge(self, *name: str) -> None:
        self.tree.resolve(name).deregister_gauge()

    def prune(self, *name: str) -> None:
        self.tree.resolve(name).prune()

    def scope(self, *namespaces: str) -> "MetricsTreeStatsReceiver":
        return MetricsTreeStatsReceiver(self.tree.resolve(namespaces))


def snapshot_histograms(tree: MetricsTree, engine: StatEngine) -> int:
    """Batched AdminMetricsExportTelemeter.snapshotHistograms (:154-162): one fused
    GPU snapshot + reset of every series, then each Stat's snapshottedSummary is set.
    Returns the number of Stats updated."""
    now = time.time()
    summaries = engine.snapshot_all(reset=True)
    n = 0
    for _, t in tree.walk():
        m = t.metric
        if isinstance(m, Metric.Stat) and m.series_id is not None:
            m._set_snapshot(HistogramSummary.from_record(summaries[m.series_id]), now)
            n += 1
    return n
