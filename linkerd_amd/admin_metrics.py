"""/admin/metrics.json from GPU-produced summaries, plus the histogram snapshot
driver.

Restates AdminMetricsExportTelemeter
(reference: telemetry/admin-metrics-export/src/main/scala/io/buoyant/telemetry/admin/
AdminMetricsExportTelemeter.scala):
  * handler (:31-54): `pretty`, `tree` and `q` query parameters; an unknown
    subtree answers 404 with {"error": "No such subtree: <q>"};
  * writeJsonMetric (:81-104): counters as Java long, gauges as Java float,
    stats as `<name>.count` and -- only when count > 0 -- max, min, p50, p90,
    p95, p99, p9990, p9999, sum (longs) and avg (Java double); nothing for a Stat
    that has not been snapshotted yet;
  * writeFlatJson (:106-116): one object of `a/b/c` keys in tree-walk order
    (sorted by key when pretty); writeJsonTree (:118-136): nested objects with
    the metric under "counter" / "gauge" / "stat";
  * run / snapshotHistograms (:65-77, :153-162): every snapshot interval, every
    Stat is snapshotted and reset.  Here that walk is ONE fused GPU snapshot +
    reset of all series (telemetry.snapshot_histograms), not a per-Stat DFS.
Output bytes follow jackson-core 2.8 JsonGenerator defaults (string escapes,
non-finite numbers quoted, DefaultPrettyPrinter layout); child order is the
reference's (linkerd_amd.javamap).
"""
from __future__ import annotations

import math
import threading
from typing import List, Optional, Tuple
from urllib.parse import parse_qs, urlsplit

from .javafmt import double_to_string, float_to_string, long_to_string
from .telemetry import Metric, MetricsTree, StatEngine, snapshot_histograms

STAT_FIELDS = ("max", "min", "p50", "p90", "p95", "p99", "p9990", "p9999", "sum")

_SHORT_ESCAPES = {'"': '\\"', "\\": "\\\\", "\b": "\\b", "\t": "\\t", "\f": "\\f", "\n": "\\n", "\r": "\\r"}


def json_string(s: str) -> str:
    """JsonGenerator.writeString / writeFieldName quoting (CharTypes.sOutputEscapes128)."""
    out = []
    for ch in s:
        e = _SHORT_ESCAPES.get(ch)
        if e is not None:
            out.append(e)
        elif ord(ch) < 0x20:
            out.append("\\u%04X" % ord(ch))
        else:
            out.append(ch)
    return '"' + "".join(out) + '"'


def _json_float(x: float, to_string) -> str:
    # QUOTE_NON_NUMERIC_NUMBERS (on by default): NaN / Infinity are written as strings
    if math.isnan(x) or math.isinf(x):
        return json_string(to_string(x))
    return to_string(x)


class _Gen:
    """The subset of a jackson JsonGenerator the exporter uses (compact or
    DefaultPrettyPrinter: two-space indent, " : " separator, "{ }" when empty)."""

    def __init__(self, pretty: bool = False):
        self.pretty = pretty
        self.out: List[str] = []
        self.counts: List[int] = []  # entries written per open object

    def _before_entry(self):
        n = self.counts[-1]
        if n:
            self.out.append(",")
        if self.pretty:
            self.out.append("\n" + "  " * len(self.counts))
        self.counts[-1] = n + 1

    def start_object(self):
        self.out.append("{")
        self.counts.append(0)

    def end_object(self):
        n = self.counts.pop()
        if self.pretty:
            self.out.append(("\n" + "  " * len(self.counts)) if n else " ")
        self.out.append("}")

    def field_name(self, name: str):
        self._before_entry()
        self.out.append(json_string(name))
        self.out.append(" : " if self.pretty else ":")

    def number_field(self, name: str, text: str):
        self.field_name(name)
        self.out.append(text)

    def text(self) -> str:
        return "".join(self.out)


def _write_metric(jg: _Gen, name: str, m) -> None:
    """writeJsonMetric (AdminMetricsExportTelemeter.scala:81-104)."""
    if isinstance(m, Metric.Counter):
        jg.number_field(name, long_to_string(m.get()))
    elif isinstance(m, Metric.Gauge):
        jg.number_field(name, _json_float(m.get(), float_to_string))
    elif isinstance(m, Metric.Stat):
        s = m.snapshotted_summary
        if s is not None:
            jg.number_field(f"{name}.count", long_to_string(s.count))
            if s.count > 0:
                for f in STAT_FIELDS:
                    jg.number_field(f"{name}.{f}", long_to_string(getattr(s, f)))
                jg.number_field(f"{name}.avg", _json_float(s.avg, double_to_string))


def flatten_metrics_tree(tree: MetricsTree, prefix: str = "", acc=None) -> List[Tuple[str, object]]:
    """flattenMetricsTree (:138-151): (a/b/c, metric) for every node, root included."""
    if acc is None:
        acc = []
    acc.append((prefix, tree.metric))
    for name, child in tree.children.items():
        flatten_metrics_tree(child, name if not prefix else f"{prefix}/{name}", acc)
    return acc


def _utf16_key(s: str):
    return s.encode("utf-16-be", "surrogatepass")


def write_flat_json(tree: MetricsTree, pretty: bool = False) -> str:
    jg = _Gen(pretty)
    jg.start_object()
    flat = flatten_metrics_tree(tree)
    if pretty:
        flat = sorted(flat, key=lambda kv: _utf16_key(kv[0]))  # Seq.sortBy(_._1): stable, String ordering
    for name, m in flat:
        _write_metric(jg, name, m)
    jg.end_object()
    return jg.text()


def _write_tree(jg: _Gen, tree: MetricsTree) -> None:
    jg.start_object()
    m = tree.metric
    if isinstance(m, Metric.Counter):
        _write_metric(jg, "counter", m)
    elif isinstance(m, Metric.Gauge):
        _write_metric(jg, "gauge", m)
    elif isinstance(m, Metric.Stat):
        _write_metric(jg, "stat", m)
    for name, child in tree.children.items():
        jg.field_name(name)
        _write_tree(jg, child)
    jg.end_object()


def write_json_tree(tree: MetricsTree) -> str:
    jg = _Gen(False)
    _write_tree(jg, tree)
    return jg.text()


def _bool_param(params, name: str, default: bool) -> bool:
    """finagle Request.getBooleanParam: 1/t/true and 0/f/false (any case)."""
    v = params.get(name)
    if not v:
        return default
    x = v[0].lower()
    if x in ("1", "t", "true"):
        return True
    if x in ("0", "f", "false"):
        return False
    return default


def _java_split_slash(q: str) -> List[str]:
    parts = q.split("/")
    while len(parts) > 1 and parts[-1] == "":  # String.split drops trailing empty strings
        parts.pop()
    return parts


class AdminMetricsExportTelemeter:
    """AdminMetricsExportTelemeter (:25-164): /admin/metrics.json and the
    histogram snapshot driver."""

    path = "/admin/metrics.json"

    def __init__(self, metrics: MetricsTree, snapshot_interval: float = 60.0, engine: Optional[StatEngine] = None):
        self.metrics = metrics
        self.snapshot_interval = float(snapshot_interval)
        self.engine = engine if engine is not None else metrics._engine
        self._started = False
        self._lock = threading.Lock()
        self._timer: Optional[threading.Timer] = None
        self._closed = threading.Event()

    def handle(self, uri: str) -> Tuple[int, str, str]:
        """(status, media type, body) for a request URI such as
        /admin/metrics.json?q=foo/bar&tree=1."""
        params = parse_qs(urlsplit(uri).query, keep_blank_values=True)
        pretty = _bool_param(params, "pretty", False)
        tree = _bool_param(params, "tree", False)
        q = params["q"][0] if "q" in params else None
        sub = self.metrics.try_resolve(_java_split_slash(q)) if q is not None else self.metrics
        if sub is None:
            return 404, "application/json", '{"error": "No such subtree: %s"}' % q
        body = write_json_tree(sub) if tree else write_flat_json(sub, pretty)
        return 200, "application/json", body

    # -- snapshot driver -----------------------------------------------------
    def tick(self) -> int:
        """One snapshot interval: snapshot + reset every Stat (one fused GPU pass).
        Returns the number of Stats updated."""
        if self.engine is None:
            return 0
        return snapshot_histograms(self.metrics, self.engine)

    def run(self) -> "AdminMetricsExportTelemeter":
        """Start the periodic snapshot task (at most once, as run() at :65-67)."""
        with self._lock:
            if self._started:
                return self
            self._started = True
        self._schedule()
        return self

    def _schedule(self):
        if self._closed.is_set():
            return
        self._timer = threading.Timer(self.snapshot_interval, self._fire)
        self._timer.daemon = True
        self._timer.start()

    def _fire(self):
        if self._closed.is_set():
            return
        self.tick()
        self._schedule()

    def close(self) -> None:
        self._closed.set()
        if self._timer is not None:
            self._timer.cancel()
