"""Prometheus text export from GPU-produced summaries.

Restates PrometheusTelemeter.writeMetrics
(reference: telemetry/prometheus/src/main/scala/io/buoyant/telemetry/prometheus/
PrometheusTelemeter.scala:37-135): prefix segments rt/<router>, rt/service/<path>,
rt/client/<id>, rt/client/service/<path>, rt/server/<srv> are rewritten into labels;
counters print as Java Long, gauges as Java Float, stats print _count/_sum/_avg
(avg as Java Double) plus 8 quantile lines from `snapshotted_summary`, and nothing
before the first snapshot.  Child order follows the tree's map order (the
reference's immutable-Map hash order), so compare outputs as line multisets.
"""
from __future__ import annotations

import re
from typing import List, Sequence, Tuple

from .javafmt import double_to_string, float_to_string, long_to_string
from .telemetry import Metric, MetricsTree

_METRIC_NAME_DISALLOWED = re.compile(r"[^a-zA-Z0-9:]")
_LABEL_KEY_DISALLOWED = re.compile(r"[^a-zA-Z0-9_]")
_LABEL_VAL_DISALLOWED = re.compile(r'(\\|"|\n)')

Labels = Tuple[Tuple[str, str], ...]


def escape_key(key: str) -> str:
    return _METRIC_NAME_DISALLOWED.sub("_", key)


def escape_label_key(key: str) -> str:
    return _LABEL_KEY_DISALLOWED.sub("_", key)


def escape_label_val(v: str) -> str:
    # replaceAllIn(key, """\\\\""") : each of \ " newline becomes two backslashes
    return _LABEL_VAL_DISALLOWED.sub(lambda m: "\\\\", v)


def format_labels(labels: Labels) -> str:
    if not labels:
        return ""
    return "{" + ", ".join(f'{escape_label_key(k)}="{escape_label_val(v)}"' for k, v in labels) + "}"


def _label_exists(labels: Labels, name: str) -> bool:
    return any(k == name for k, _ in labels)


def _rewrite(prefix: Tuple[str, ...], labels: Labels):
    if len(prefix) == 2 and prefix[0] == "rt" and not _label_exists(labels, "rt"):
        return ("rt",), labels + (("rt", prefix[1]),)
    if len(prefix) == 3 and prefix[:2] == ("rt", "service") and not _label_exists(labels, "service"):
        return ("rt", "service"), labels + (("service", prefix[2]),)
    if len(prefix) == 3 and prefix[:2] == ("rt", "client") and not _label_exists(labels, "client"):
        return ("rt", "client"), labels + (("client", prefix[2]),)
    if len(prefix) == 4 and prefix[:3] == ("rt", "client", "service") and not _label_exists(labels, "service"):
        return ("rt", "client", "service"), labels + (("service", prefix[3]),)
    if len(prefix) == 3 and prefix[:2] == ("rt", "server") and not _label_exists(labels, "server"):
        return ("rt", "server"), labels + (("server", prefix[2]),)
    return prefix, labels


QUANTILES = (("0", "min"), ("0.5", "p50"), ("0.9", "p90"), ("0.95", "p95"), ("0.99", "p99"),
             ("0.999", "p9990"), ("0.9999", "p9999"), ("1", "max"))


def write_metrics(tree: MetricsTree, out: List[str], prefix0: Tuple[str, ...] = (), labels0: Labels = ()) -> None:
    prefix1, labels1 = _rewrite(prefix0, labels0)
    key = escape_key(":".join(prefix1))
    m = tree.metric
    if isinstance(m, Metric.Counter):
        out.append(f"{key}{format_labels(labels1)} {long_to_string(m.get())}\n")
    elif isinstance(m, Metric.Gauge):
        out.append(f"{key}{format_labels(labels1)} {float_to_string(m.get())}\n")
    elif isinstance(m, Metric.Stat):
        s = m.snapshotted_summary
        if s is not None:
            lab = format_labels(labels1)
            out.append(f"{key}_count{lab} {long_to_string(s.count)}\n")
            out.append(f"{key}_sum{lab} {long_to_string(s.sum)}\n")
            out.append(f"{key}_avg{lab} {double_to_string(s.avg)}\n")
            for q, field in QUANTILES:
                out.append(f"{key}{format_labels(labels1 + (('quantile', q),))} {long_to_string(getattr(s, field))}\n")
    for name, child in tree.children.items():
        write_metrics(child, out, prefix1 + (name,), labels1)


class PrometheusTelemeter:
    """PrometheusTelemeter (PrometheusTelemeter.scala:17-35): /admin/metrics/prometheus."""

    path = "/admin/metrics/prometheus"

    def __init__(self, metrics: MetricsTree):
        self.metrics = metrics

    def render(self) -> str:
        out: List[str] = []
        write_metrics(self.metrics, out)
        return "".join(out)


def line_multiset(text: str) -> dict:
    from collections import Counter
    return Counter(l for l in text.split("\n") if l)
