"""/admin/metrics.json and InfluxDB LINE exporters on CPU,
mirroring the reference's own tests:
AdminMetricsExportTelemeterTest.scala:11-141 and InfluxDbTelemeterTest.scala:19-204.
Stat summaries are injected the way the batched snapshot driver sets them (the
values the GPU produces for {1} and {1, 2}, pinned end to end in
tests/test_gpu_telemetry.py); child order is checked against the reference's
tree-mode fixture (tests/golden/metrics_key_order.json).
"""
import json
import os

from linkerd_amd.admin_metrics import AdminMetricsExportTelemeter, json_string, write_flat_json
from linkerd_amd.influxdb import InfluxDbTelemeter
from linkerd_amd.javamap import chm_order, java_string_hash, reference_child_order
from linkerd_amd.telemetry import HistogramSummary, MetricsTree, MetricsTreeStatsReceiver

ONE = HistogramSummary(1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1.0)
ONE_TWO = HistogramSummary(2, 1, 2, 3, 1, 2, 2, 2, 2, 2, 1.5)
TWO = HistogramSummary(1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2.0)
TWO_FOUR = HistogramSummary(2, 2, 4, 6, 2, 4, 4, 4, 4, 4, 3.0)


def _admin():
    tree = MetricsTree()
    return tree, MetricsTreeStatsReceiver(tree), AdminMetricsExportTelemeter(tree, 60.0)


def _get(tel, uri="/admin/metrics.json"):
    status, media, body = tel.handle(uri)
    assert media == "application/json"
    return status, body


def mk_histo_json(name, datum):
    """AdminMetricsExportTelemeterTest.mkHistoJson (:128-141)."""
    parts = [f'"{name}.count":1'] + [f'"{name}.{f}":{datum}' for f in
                                     ("max", "min", "p50", "p90", "p95", "p99", "p9990", "p9999", "sum")]
    return "{" + ",".join(parts + [f'"{name}.avg":{datum}.0']) + "}"


def test_admin_counters_updated_immediately():
    tree, stats, tel = _admin()
    c = stats.scope("foo", "bar").counter("bas")
    c.incr()
    assert _get(tel) == (200, '{"foo/bar/bas":1}')
    c.incr()
    assert _get(tel) == (200, '{"foo/bar/bas":2}')


def test_admin_gauges_updated_immediately():
    tree, stats, tel = _admin()
    v = {"x": 1.0}
    stats.scope("foo", "bar").add_gauge("bas", f=lambda: v["x"])
    assert _get(tel) == (200, '{"foo/bar/bas":1.0}')
    v["x"] = 2.0
    assert _get(tel) == (200, '{"foo/bar/bas":2.0}')


def test_admin_histograms_served_from_last_snapshot():
    """:47-85 -- nothing before the first snapshot, then the last snapshot's summary."""
    tree, stats, tel = _admin()
    stat = stats.scope("foo", "bar").stat("bas")
    assert _get(tel) == (200, "{}")
    stat._set_snapshot(ONE)
    assert _get(tel) == (200, mk_histo_json("foo/bar/bas", 1))
    stat._set_snapshot(TWO)
    assert _get(tel) == (200, mk_histo_json("foo/bar/bas", 2))


def test_admin_empty_snapshot_writes_count_only():
    """:89-90 -- a snapshotted Stat with count 0 emits only `.count`."""
    tree, stats, tel = _admin()
    stats.scope("a").stat("s")._set_snapshot(HistogramSummary(0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0.0))
    assert _get(tel) == (200, '{"a/s.count":0}')


def test_admin_tree_mode():
    tree, stats, tel = _admin()
    stats.scope("foo", "bar").counter("bas").incr()
    assert _get(tel, "/admin/metrics.json?tree=1") == (200, '{"foo":{"bar":{"bas":{"counter":1}}}}')


def test_admin_subtree_selector():
    tree, stats, tel = _admin()
    stats.scope("foo", "bar").counter("bas").incr()
    stats.scope("foo", "bar").counter("bass").incr()
    stats.scope("x", "y").counter("z").incr()
    assert _get(tel, "/admin/metrics.json?q=foo/bar") == (200, '{"bass":1,"bas":1}')
    assert _get(tel, "/admin/metrics.json?q=foo/bar&tree=1") == (200, '{"bass":{"counter":1},"bas":{"counter":1}}')
    assert _get(tel, "/admin/metrics.json?q=nope") == (404, '{"error": "No such subtree: nope"}')


def test_admin_pretty_and_stat_tree_mode():
    tree, stats, tel = _admin()
    stats.scope("b").counter("c").incr(3)
    stats.scope("a").stat("s")._set_snapshot(ONE_TWO)
    status, body = _get(tel, "/admin/metrics.json?pretty=true")
    lines = body.split("\n")
    assert lines[0] == "{" and lines[-1] == "}"
    keys = [json.loads("{" + l.rstrip(",") + "}") for l in lines[1:-1]]
    names = [next(iter(k)) for k in keys]
    assert names[0] == "a/s.count" and names[-2] == "a/s.avg" and names[-1] == "b/c"  # sorted by metric path
    assert lines[1] == '  "a/s.count" : 2,'
    assert write_flat_json(MetricsTree(), pretty=True) == "{ }"
    status, body = _get(tel, "/admin/metrics.json?tree=1&q=a")
    assert json.loads(body) == {"s": {"stat.count": 2, "stat.max": 2, "stat.min": 1, "stat.p50": 1, "stat.p90": 2,
                                      "stat.p95": 2, "stat.p99": 2, "stat.p9990": 2, "stat.p9999": 2, "stat.sum": 3,
                                      "stat.avg": 1.5}}


def test_json_string_escapes():
    assert json_string('a"b\\c\n\t\x01/é') == '"a\\"b\\\\c\\n\\t\\u0001/é"'


def test_reference_child_order_pinned_by_fixture():
    """Child order of every node of the reference's tree-mode fixture (P5).  Nodes
    the fixture's authors extended by hand (one inserted key, or invented names)
    are recognised as such; every generated node matches exactly."""
    path = os.path.join(os.path.dirname(__file__), "golden", "metrics_key_order.json")
    nodes = json.load(open(path))["child_key_orders"]
    exact = one_inserted = hand = 0
    for keys in nodes:
        if len(keys) <= 4:  # Map1..Map4: ConcurrentHashMap bin order (ties keep insertion order)
            bins = [(java_string_hash(k) ^ ((java_string_hash(k) & 0xFFFFFFFF) >> 16)) & 15 for k in keys]
            exact += bins == sorted(bins)
            hand += bins != sorted(bins)
            continue
        if reference_child_order(keys) == keys:
            exact += 1
        elif any(reference_child_order([y for y in keys if y != x]) == [y for y in keys if y != x] for x in keys):
            one_inserted += 1
        else:
            hand += 1
            assert keys[0].startswith("$/inet/127.1/") or keys[0] == "subtractor", keys
    assert exact >= 130 and one_inserted == 15 and hand <= 10, (exact, one_inserted, hand)


def test_chm_order_examples():
    assert chm_order(["bas", "bass"]) == ["bass", "bas"]  # AdminMetricsExportTelemeterTest.scala:111
    keys = [f"k{i}" for i in range(40)]  # crosses two resizes
    assert sorted(chm_order(keys)) == sorted(keys)


# ---- InfluxDbTelemeterTest ------------------------------------------------------
def _influx():
    tree = MetricsTree()
    return tree, MetricsTreeStatsReceiver(tree), InfluxDbTelemeter(tree)


def test_influx_counter_and_no_scope():
    tree, stats, tel = _influx()
    c = stats.scope("foo", "bar").counter("bas")
    c.incr()
    assert tel.render() == "foo:bar,host=none bas=1\n"
    c.incr()
    assert tel.render() == "foo:bar,host=none bas=2\n"
    tree, stats, tel = _influx()
    c1, c2 = stats.counter("abc"), stats.counter("def")
    c1.incr()
    c2.incr(2)
    assert tel.render() == "root,host=none abc=1,def=2\n"


def test_influx_gauges():
    tree, stats, tel = _influx()
    v = {"x": 1.0}
    stats.scope("foo", "bar").add_gauge("bas", f=lambda: v["x"])
    assert tel.render() == "foo:bar,host=none bas=1.0\n"
    v["x"] = 2.0
    assert tel.render() == "foo:bar,host=none bas=2.0\n"
    tree, stats, tel = _influx()
    stats.add_gauge("abc", f=lambda: v["x"])
    stats.add_gauge("def", f=lambda: v["x"] * 2)
    assert tel.render() == "root,host=none abc=2.0,def=4.0\n"


def test_influx_stat_and_stats_no_scope():
    """:89-172 (P3)."""
    tree, stats, tel = _influx()
    s = stats.scope("foo", "bar").stat("bas")
    assert tel.render() == ""
    s._set_snapshot(ONE)
    assert tel.render() == ("foo:bar,host=none bas_avg=1.0,bas_count=1,bas_max=1,bas_min=1,bas_p50=1,bas_p90=1,"
                            "bas_p95=1,bas_p99=1,bas_p999=1,bas_p9999=1,bas_sum=1\n")
    s._set_snapshot(ONE_TWO)
    assert tel.render() == ("foo:bar,host=none bas_avg=1.5,bas_count=2,bas_max=2,bas_min=1,bas_p50=1,bas_p90=2,"
                            "bas_p95=2,bas_p99=2,bas_p999=2,bas_p9999=2,bas_sum=3\n")
    tree, stats, tel = _influx()
    a, d = stats.stat("abc"), stats.stat("def")
    a._set_snapshot(ONE_TWO)
    d._set_snapshot(TWO_FOUR)
    assert tel.render() == (
        "root,host=none abc_avg=1.5,abc_count=2,abc_max=2,abc_min=1,abc_p50=1,abc_p90=2,abc_p95=2,abc_p99=2,"
        "abc_p999=2,abc_p9999=2,abc_sum=3,def_avg=3.0,def_count=2,def_max=4,def_min=2,def_p50=2,def_p90=4,"
        "def_p95=4,def_p99=4,def_p999=4,def_p9999=4,def_sum=6\n")


def test_influx_labelled_paths():
    """:174-204."""
    cases = [(("rt", "incoming", "service", "/svc/foo"), "rt:service,host=none,rt=incoming,service=/svc/foo requests=1\n"),
             (("rt", "incoming", "client", "/#/bar"), "rt:client,client=/#/bar,host=none,rt=incoming requests=1\n"),
             (("rt", "incoming", "client", "/#/bar", "service", "/svc/foo"),
              "rt:client:service,client=/#/bar,host=none,rt=incoming,service=/svc/foo requests=1\n"),
             (("rt", "incoming", "server", "127.0.0.1/4141"),
              "rt:server,host=none,rt=incoming,server=127.0.0.1/4141 requests=1\n")]
    for scope, want in cases:
        tree, stats, tel = _influx()
        stats.scope(*scope).counter("requests").incr()
        assert tel.render() == want
