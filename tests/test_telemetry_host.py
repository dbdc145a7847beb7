"""Host-side mirror of io.buoyant.telemetry and the Prometheus exporter, on CPU.

Mirrors the reference's own tests: MetricsTree type conflicts
(MetricsTree.scala:82,92,103,112), PrometheusTelemeterTest.scala (counter, gauge,
stat lines, label escaping, path labelling).  Stat summaries are injected the way
the batched snapshot driver sets them (no GPU needed here); the full GPU flow is in
tests/test_gpu_telemetry.py.
"""
import pytest

from linkerd_amd.javafmt import double_to_string, float_to_string
from linkerd_amd.prometheus import PrometheusTelemeter, escape_label_val, line_multiset
from linkerd_amd.telemetry import HistogramSummary, Metric, MetricsTree, MetricsTreeStatsReceiver


def _receiver():
    tree = MetricsTree()
    return tree, MetricsTreeStatsReceiver(tree), PrometheusTelemeter(tree)


def test_tree_resolve_and_conflicts():
    tree = MetricsTree()
    c = tree.resolve(["a", "b"]).mk_counter()
    assert tree.resolve(["a", "b"]).mk_counter() is c
    with pytest.raises(ValueError, match="non-stat metric already exists"):
        tree.resolve(["a", "b"]).mk_stat()
    with pytest.raises(ValueError, match="non-gauge metric already exists"):
        tree.resolve(["a", "b"]).register_gauge(lambda: 1.0)
    assert tree.try_resolve(["a", "x"]) is None
    assert tree.try_resolve(["a", "b"]) is tree.resolve(["a", "b"])
    tree.resolve(["g"]).register_gauge(lambda: 3.0)
    tree.resolve(["g"]).register_gauge(lambda: 4.0)  # gauge may be re-registered
    assert tree.resolve(["g"]).metric.get() == 4.0
    tree.resolve(["g"]).deregister_gauge()
    assert tree.resolve(["g"]).metric is Metric.NONE
    tree.resolve(["a"]).prune()
    assert tree.resolve(["a"]).children == {}


def test_stat_without_engine_fails_loudly():
    from linkerd_amd._native import NativeLibraryMissing
    s = MetricsTree().resolve(["s"]).mk_stat()
    with pytest.raises(NativeLibraryMissing):
        s.add(1.0)


def test_prometheus_counter_and_gauge():
    """PrometheusTelemeterTest: counter -> 'foo:bar:bas 1'; gauge -> 'foo:bar:bas 1.0'."""
    tree, stats, prom = _receiver()
    stats.scope("foo", "bar").counter("bas").incr()
    assert prom.render() == "foo:bar:bas 1\n"
    tree2, stats2, prom2 = _receiver()
    v = {"x": 1.0}
    stats2.scope("foo", "bar").add_gauge("bas", f=lambda: v["x"])
    assert prom2.render() == "foo:bar:bas 1.0\n"
    v["x"] = 2.0
    assert prom2.render() == "foo:bar:bas 2.0\n"


def test_prometheus_stat_lines_p1_p2():
    """PrometheusTelemeterTest.scala:41-86 (summaries as the GPU produces them)."""
    tree, stats, prom = _receiver()
    stat = stats.scope("foo", "bar").stat("bas")
    assert prom.render() == ""  # no data before the first snapshot
    stat._set_snapshot(HistogramSummary(1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1.0))
    assert prom.render() == (
        "foo:bar:bas_count 1\nfoo:bar:bas_sum 1\nfoo:bar:bas_avg 1.0\n"
        'foo:bar:bas{quantile="0"} 1\nfoo:bar:bas{quantile="0.5"} 1\nfoo:bar:bas{quantile="0.9"} 1\n'
        'foo:bar:bas{quantile="0.95"} 1\nfoo:bar:bas{quantile="0.99"} 1\nfoo:bar:bas{quantile="0.999"} 1\n'
        'foo:bar:bas{quantile="0.9999"} 1\nfoo:bar:bas{quantile="1"} 1\n')
    stat._set_snapshot(HistogramSummary(2, 1, 2, 3, 1, 2, 2, 2, 2, 2, 1.5))
    assert prom.render() == (
        "foo:bar:bas_count 2\nfoo:bar:bas_sum 3\nfoo:bar:bas_avg 1.5\n"
        'foo:bar:bas{quantile="0"} 1\nfoo:bar:bas{quantile="0.5"} 1\nfoo:bar:bas{quantile="0.9"} 2\n'
        'foo:bar:bas{quantile="0.95"} 2\nfoo:bar:bas{quantile="0.99"} 2\nfoo:bar:bas{quantile="0.999"} 2\n'
        'foo:bar:bas{quantile="0.9999"} 2\nfoo:bar:bas{quantile="1"} 2\n')


def test_prometheus_label_escaping_and_path_labels():
    """PrometheusTelemeterTest: labels are escaped; rt/service/client/server paths become labels."""
    tree, stats, prom = _receiver()
    svc = '\\x5b\\x31\\x32\\x33\\x2e\\x31\\x32\\x33\\x2e\\x31\\x32\\x33\\x2e\\x31\\x32\\x33\\x5dun"esc'
    stats.scope("rt", "incoming", "service", svc).counter("requests").incr()
    want = ('rt:service:requests{rt="incoming", service="\\\\x5b\\\\x31\\\\x32\\\\x33\\\\x2e\\\\x31\\\\x32\\\\x33'
            '\\\\x2e\\\\x31\\\\x32\\\\x33\\\\x2e\\\\x31\\\\x32\\\\x33\\\\x5dun\\\\esc"} 1\n')
    assert prom.render() == want
    for scope, want in [
        (("rt", "incoming", "service", "/svc/foo"), 'rt:service:requests{rt="incoming", service="/svc/foo"} 1\n'),
        (("rt", "incoming", "client", "/#/bar"), 'rt:client:requests{rt="incoming", client="/#/bar"} 1\n'),
        (("rt", "incoming", "client", "/#/bar", "service", "/svc/foo"),
         'rt:client:service:requests{rt="incoming", client="/#/bar", service="/svc/foo"} 1\n'),
        (("rt", "incoming", "server", "127.0.0.1/4141"),
         'rt:server:requests{rt="incoming", server="127.0.0.1/4141"} 1\n'),
    ]:
        tree, stats, prom = _receiver()
        stats.scope(*scope).counter("requests").incr()
        assert prom.render() == want


def test_escape_label_val_rule():
    assert escape_label_val('a\\b"c\nd') == "a\\\\b\\\\c\\\\d"


def test_java_number_strings():
    assert [double_to_string(x) for x in (1.0, 1.5, 3030.0, 1e7, 1e-4, 281.7352941176471, 0.0)] == \
        ["1.0", "1.5", "3030.0", "1.0E7", "1.0E-4", "281.7352941176471", "0.0"]
    assert float_to_string(4008938.8) == "4008938.8" and float_to_string(1.48832833e12) == "1.48832833E12"  # JDK 8 (tests/test_javafmt.py)


def test_line_multiset_compare():
    a = "x 1\ny 2\n"
    b = "y 2\nx 1\n"
    assert line_multiset(a) == line_multiset(b)
