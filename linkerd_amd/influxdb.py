"""InfluxDB LINE protocol export from GPU-produced summaries.

Restates InfluxDbTelemeter.writeMetrics
(reference: telemetry/influxdb/src/main/scala/io/buoyant/telemetry/influxdb/
InfluxDbTelemeter.scala:17-130): the prefix segments rt/<router>,
rt/service/<path>, rt/client/<id>, rt/client/service/<path>, rt/server/<srv>
become tags (:63-75); the metrics directly under one parent are written as the
fields of one measurement, after the lines of their own subtrees (:78-108);
counters print as Java Long, gauges as Java Float, and a snapshotted Stat as
<name>_count/_sum/_avg/_min/_max/_p50/_p90/_p95/_p99/_p999/_p9999 (avg as Java
Double); tags and fields are sorted by key (:46-50); top-level metrics go under
the measurement "root" (:36, :111-118); the measurement name is escaped with
[^a-zA-Z0-9:] -> _ (:42-43).  Tag and field values are not escaped (as in the
reference).
"""
from __future__ import annotations

import re
from typing import List, Sequence, Tuple

from .javafmt import double_to_string, float_to_string, long_to_string
from .telemetry import Metric, MetricsTree

_DISALLOWED = re.compile(r"[^a-zA-Z0-9:]")
ROOT_PREFIX = ("root",)

Tags = Tuple[Tuple[str, str], ...]


def escape_key(key: str) -> str:
    return _DISALLOWED.sub("_", key)


def _utf16_key(kv):
    return kv[0].encode("utf-16-be", "surrogatepass")


def format_labels(labels: Sequence[Tuple[str, str]]) -> str:
    return ",".join(f"{k}={v}" for k, v in sorted(labels, key=_utf16_key))  # stable sortBy(_._1)


def _label_exists(tags: Tags, name: str) -> bool:
    return any(k == name for k, _ in tags)


def _rewrite(prefix: Tuple[str, ...], tags: Tags):
    if len(prefix) == 2 and prefix[0] == "rt" and not _label_exists(tags, "rt"):
        return ("rt",), tags + (("rt", prefix[1]),)
    if len(prefix) == 3 and prefix[:2] == ("rt", "service") and not _label_exists(tags, "service"):
        return ("rt", "service"), tags + (("service", prefix[2]),)
    if len(prefix) == 3 and prefix[:2] == ("rt", "client") and not _label_exists(tags, "client"):
        return ("rt", "client"), tags + (("client", prefix[2]),)
    if len(prefix) == 4 and prefix[:3] == ("rt", "client", "service") and not _label_exists(tags, "service"):
        return ("rt", "client", "service"), tags + (("service", prefix[3]),)
    if len(prefix) == 3 and prefix[:2] == ("rt", "server") and not _label_exists(tags, "server"):
        return ("rt", "server"), tags + (("server", prefix[2]),)
    return prefix, tags


def _fields(name: str, m) -> List[Tuple[str, str]]:
    if isinstance(m, Metric.Counter):
        return [(name, long_to_string(m.get()))]
    if isinstance(m, Metric.Gauge):
        return [(name, float_to_string(m.get()))]
    if isinstance(m, Metric.Stat):
        s = m.snapshotted_summary
        if s is None:
            return []
        return [(name + "_count", long_to_string(s.count)), (name + "_sum", long_to_string(s.sum)),
                (name + "_avg", double_to_string(s.avg)), (name + "_min", long_to_string(s.min)),
                (name + "_max", long_to_string(s.max)), (name + "_p50", long_to_string(s.p50)),
                (name + "_p90", long_to_string(s.p90)), (name + "_p95", long_to_string(s.p95)),
                (name + "_p99", long_to_string(s.p99)), (name + "_p999", long_to_string(s.p9990)),
                (name + "_p9999", long_to_string(s.p9999))]
    return []


def write_metrics(tree: MetricsTree, out: List[str], prefix0: Tuple[str, ...] = (), tags0: Tags = ()) -> None:
    prefix1, tags1 = _rewrite(prefix0, tags0)
    fields: List[Tuple[str, str]] = []
    for name, child in tree.children.items():
        write_metrics(child, out, prefix1 + (name,), tags1)  # deeper lines first (side effect)
        fields.extend(_fields(name, child.metric))
    if fields:
        prefix = prefix1 if prefix1 else ROOT_PREFIX
        line = escape_key(":".join(prefix))
        if tags1:
            line += "," + format_labels(tags1)
        out.append(line + " " + format_labels(fields) + "\n")


class InfluxDbTelemeter:
    """InfluxDbTelemeter (:17-40): /admin/metrics/influxdb."""

    path = "/admin/metrics/influxdb"

    def __init__(self, metrics: MetricsTree):
        self.metrics = metrics

    def render(self, host: str = "none") -> str:
        """The handler body; `host` is the request's Host header ("none" if absent)."""
        out: List[str] = []
        write_metrics(self.metrics, out, (), (("host", host),))
        return "".join(out)
