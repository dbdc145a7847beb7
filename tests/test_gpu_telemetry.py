"""The reference's telemetry tests, end to end through the GPU engine:
Stat.add -> (batched ingest) -> snapshot -> PrometheusTelemeter text.

P1/P2: PrometheusTelemeterTest.scala:41-86; P3: InfluxDbTelemeterTest.scala:141-172;
P4: AdminMetricsExportTelemeterTest.scala:47-85 (interval reset semantics);
C5: a tree of stats, counters and gauges exported as Prometheus text,
compared as a line multiset against the same export built from oracle summaries.
"""
import numpy as np
import pytest

from linkerd_amd.prometheus import PrometheusTelemeter, line_multiset
from linkerd_amd.telemetry import (HistogramSummary, MetricsTree, MetricsTreeStatsReceiver, StatEngine,
                                   snapshot_histograms)

pytestmark = pytest.mark.gpu


def _setup(capacity=64):
    eng = StatEngine(capacity=capacity, batch=1024)
    tree = MetricsTree(eng)
    return eng, tree, MetricsTreeStatsReceiver(tree), PrometheusTelemeter(tree)


def test_p1_p2_prometheus_through_gpu():
    eng, tree, stats, prom = _setup()
    stat = stats.scope("foo", "bar").stat("bas")
    mstat = tree.resolve(["foo", "bar", "bas"]).metric
    stat.add(1.0)
    assert prom.render() == ""
    mstat.snapshot()
    assert prom.render().startswith("foo:bar:bas_count 1\nfoo:bar:bas_sum 1\nfoo:bar:bas_avg 1.0\n")
    stat.add(2.0)
    mstat.snapshot()
    assert prom.render() == (
        "foo:bar:bas_count 2\nfoo:bar:bas_sum 3\nfoo:bar:bas_avg 1.5\n"
        'foo:bar:bas{quantile="0"} 1\nfoo:bar:bas{quantile="0.5"} 1\nfoo:bar:bas{quantile="0.9"} 2\n'
        'foo:bar:bas{quantile="0.95"} 2\nfoo:bar:bas{quantile="0.99"} 2\nfoo:bar:bas{quantile="0.999"} 2\n'
        'foo:bar:bas{quantile="0.9999"} 2\nfoo:bar:bas{quantile="1"} 2\n')


def test_p3_two_stats():
    eng, tree, stats, prom = _setup()
    a, d = stats.stat("abc"), stats.stat("def")
    a.add(1.0); d.add(2.0); a.add(2.0); d.add(4.0)
    assert a.summary == HistogramSummary(2, 1, 2, 3, 1, 2, 2, 2, 2, 2, 1.5)
    assert d.summary == HistogramSummary(2, 2, 4, 6, 2, 4, 4, 4, 4, 4, 3.0)


def test_p4_interval_reset_and_peek():
    eng, tree, stats, prom = _setup()
    stat = stats.scope("foo", "bar").stat("bas")
    mstat = tree.resolve(["foo", "bar", "bas"]).metric
    stat.add(1.0)
    assert snapshot_histograms(tree, eng) == 1
    assert mstat.snapshotted_summary == HistogramSummary(1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1.0)
    stat.add(2.0)
    assert mstat.snapshotted_summary.max == 1  # served from the previous snapshot
    assert [(b.lower, b.upper, b.count) for b in mstat.peek()] == [(2, 3, 1)]
    snapshot_histograms(tree, eng)
    assert mstat.snapshotted_summary == HistogramSummary(1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2.0)
    stat.add(3030.0)
    buckets, _ = mstat.reset()
    assert [(b.lower, b.upper, b.count) for b in buckets] == [(3011, 3042, 1)]
    assert mstat.summary.count == 0


def test_c5_prometheus_export_matches_oracle(oracle):
    """C5 at reduced size: 2000 stats (rt/<r>/client/<c>/service/<s>/request_latency_ms
    shape) + 2000 counters + 200 gauges -> Prometheus text == oracle-built text."""
    rng = np.random.default_rng(55)
    S = 2000
    eng, tree, stats, prom = _setup(capacity=S)
    otree = MetricsTree()
    ostats = MetricsTreeStatsReceiver(otree)
    paths = [("rt", f"r{i % 3}", "client", f"/#/c{i % 50}", "service", f"/svc/s{i}", "request_latency_ms")
             for i in range(S)]
    st = [stats.stat(*p) for p in paths]
    ost = [ostats.stat(*p) for p in paths]
    for i in range(2000):
        stats.scope("rt", f"r{i % 3}", "server", f"10.0.0.{i % 7}/4141").counter(f"c{i}").incr(i)
        ostats.scope("rt", f"r{i % 3}", "server", f"10.0.0.{i % 7}/4141").counter(f"c{i}").incr(i)
    for i in range(200):
        stats.scope("jvm").add_gauge(f"g{i}", f=lambda i=i: i * 1.5)
        ostats.scope("jvm").add_gauge(f"g{i}", f=lambda i=i: i * 1.5)
    ids = rng.integers(0, S, 200_000)
    vals = np.exp(rng.uniform(0, 8, S)[ids] + 0.8 * rng.standard_normal(ids.size)).astype(np.float32)
    for i, v in zip(ids[:5000], vals[:5000]):  # some through Stat.add (per-thread staging)
        st[i].add(float(v))
    eng.flush()
    eng.engine.ingest(np.array([st[i].series_id for i in ids[5000:]], np.uint32), vals[5000:])
    snapshot_histograms(tree, eng)
    # oracle side: same samples per series, summaries via the C oracle
    o = oracle.OracleHistograms(S)
    o.ingest(np.array([st[i].series_id for i in ids], np.uint32), vals)
    osumm = o.snapshot()
    for i in range(S):
        ost[i]._set_snapshot(HistogramSummary.from_record(osumm[st[i].series_id]))
    got, want = prom.render(), PrometheusTelemeter(otree).render()
    assert line_multiset(got) == line_multiset(want)
    assert len(got.splitlines()) == S * 11 + 2000 + 200


def test_p4_admin_metrics_json_through_gpu():
    """AdminMetricsExportTelemeterTest.scala:47-85 end to end: Stat.add -> GPU ->
    one fused snapshot+reset per interval (tick) -> /admin/metrics.json."""
    from linkerd_amd.admin_metrics import AdminMetricsExportTelemeter
    from tests.test_exporters_host import mk_histo_json
    eng, tree, stats, _ = _setup()
    tel = AdminMetricsExportTelemeter(tree, 60.0, eng)
    stat = stats.scope("foo", "bar").stat("bas")
    stat.add(1.0)
    assert tel.handle("/admin/metrics.json")[2] == "{}"
    assert tel.tick() == 1
    assert tel.handle("/admin/metrics.json")[2] == mk_histo_json("foo/bar/bas", 1)
    stat.add(2.0)
    assert tel.handle("/admin/metrics.json")[2] == mk_histo_json("foo/bar/bas", 1)
    tel.tick()
    assert tel.handle("/admin/metrics.json")[2] == mk_histo_json("foo/bar/bas", 2)


def test_p3_influx_line_through_gpu():
    """InfluxDbTelemeterTest.scala:141-172 end to end (cumulative Stat.snapshot())."""
    from linkerd_amd.influxdb import InfluxDbTelemeter
    eng, tree, stats, _ = _setup()
    tel = InfluxDbTelemeter(tree)
    a, d = stats.stat("abc"), stats.stat("def")
    ma, md = tree.resolve(["abc"]).metric, tree.resolve(["def"]).metric
    a.add(1.0)
    d.add(2.0)
    assert tel.render() == ""
    ma.snapshot()
    md.snapshot()
    assert tel.render() == (
        "root,host=none abc_avg=1.0,abc_count=1,abc_max=1,abc_min=1,abc_p50=1,abc_p90=1,abc_p95=1,abc_p99=1,"
        "abc_p999=1,abc_p9999=1,abc_sum=1,def_avg=2.0,def_count=1,def_max=2,def_min=2,def_p50=2,def_p90=2,"
        "def_p95=2,def_p99=2,def_p999=2,def_p9999=2,def_sum=2\n")
    a.add(2.0)
    d.add(4.0)
    ma.snapshot()
    md.snapshot()
    assert tel.render() == (
        "root,host=none abc_avg=1.5,abc_count=2,abc_max=2,abc_min=1,abc_p50=1,abc_p90=2,abc_p95=2,abc_p99=2,"
        "abc_p999=2,abc_p9999=2,abc_sum=3,def_avg=3.0,def_count=2,def_max=4,def_min=2,def_p50=2,def_p90=4,"
        "def_p95=4,def_p99=4,def_p999=4,def_p9999=4,def_sum=6\n")
