"""Every BASELINE config at its stated size on the GPU, against the oracle
(BASELINE.json configs).  C3 at full size is in test_gpu_fullsize.py.

* C1  1 series x 1e7 log-normal samples: bit-exact vs the 1-thread oracle.
* C2  100k series x 1k samples (1e8), permuted COO: counts + summaries bit-exact
      vs the oracle (16 threads).
* C4  fleet merge, 1M series, 1e9 Zipf samples sample-sharded 8 ways (sample i to
      engine i mod 8): each engine exports its dense partial state, the exports are
      summed on the GPU (the reduce-scatter's arithmetic) and summarized with
      l5dh_summarize_dense.  Checked against one engine holding all 1e9 samples
      (identical counts and summaries), through the C3 properties, and by a
      bit-exact oracle replay of sampled series.
* C5  100k stats (the C2 samples) + 100k counters + 10k gauges in one tree ->
      Prometheus text, compared as a line multiset with the same tree built from
      oracle summaries (PrometheusTelemeter.scala:61-135).
Inputs are generated on the GPU (l5dh_synth.hip) and the same bytes go to the
engine and the oracle.
"""
import ctypes

import numpy as np
import pytest

from linkerd_amd import _native as N
from linkerd_amd import synth

pytestmark = pytest.mark.gpu
THREADS = 16  # the GPU box's CPU share per GPU


def _synth():
    lib = ctypes.CDLL(N.SYNTH_PATH)
    for fn in ("l5ds_gen_c1", "l5ds_gen_c2", "l5ds_gen_zipf"):
        getattr(lib, fn).restype = ctypes.c_int
    return lib


def _eq(got, want, label):
    for f in N.SUMMARY_FIELDS:
        g, w = got[f], want[f]
        bad = g != w
        if bad.any():
            i = int(np.flatnonzero(bad)[0])
            raise AssertionError(f"{label} field {f}: {int(bad.sum())} mismatches, first series {i}: {g[i]} vs {w[i]}")


def test_c1_single_stat_1e7(oracle):
    import torch
    from linkerd_amd.engine import HistogramEngine
    n = 10_000_000
    dev = torch.device("cuda", 0)
    s = torch.empty(n, dtype=torch.int32, device=dev)
    v = torch.empty(n, dtype=torch.float32, device=dev)
    assert _synth().l5ds_gen_c1(ctypes.c_void_p(v.data_ptr()), ctypes.c_void_p(s.data_ptr()), ctypes.c_uint64(n),
                                ctypes.c_uint64(1), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
    torch.cuda.synchronize()
    eng = HistogramEngine(1)
    eng.ingest(s, v)
    got, counts = eng.snapshot(reset=True, with_counts=True)
    o = oracle.OracleHistograms(1)
    o.ingest(s.cpu().numpy().view(np.uint32), v.cpu().numpy(), threads=1)
    np.testing.assert_array_equal(counts, o.counts())
    _eq(got, o.snapshot(), "C1")
    assert int(got["count"][0]) == n
    eng.close()


@pytest.fixture(scope="module")
def c2(oracle):
    """The C2 batch (host copies) and the oracle's counts and summaries of it."""
    import torch
    S, K = 100_000, 1_000
    n = S * K
    dev = torch.device("cuda", 0)
    s = torch.empty(n, dtype=torch.int32, device=dev)
    v = torch.empty(n, dtype=torch.float32, device=dev)
    assert _synth().l5ds_gen_c2(ctypes.c_void_p(s.data_ptr()), ctypes.c_void_p(v.data_ptr()), ctypes.c_uint64(S),
                                ctypes.c_uint64(K), ctypes.c_uint64(2), ctypes.c_double(0.8), ctypes.c_uint32(0),
                                ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
    torch.cuda.synchronize()
    hs, hv = s.cpu().numpy().view(np.uint32), v.cpu().numpy()
    del s, v
    o = oracle.OracleHistograms(S)
    assert o.ingest(hs, hv, threads=THREADS) == 0
    counts = o.counts()
    return {"S": S, "series": hs, "values": hv, "counts": counts, "summaries": o.snapshot()}


def test_c2_100k_series_x_1k(c2):
    import torch
    from linkerd_amd.engine import HistogramEngine
    S = c2["S"]
    dev = torch.device("cuda", 0)
    eng = HistogramEngine(S)
    eng.ingest(torch.from_numpy(c2["series"].view(np.int32)).to(dev), torch.from_numpy(c2["values"]).to(dev))
    summ = torch.empty((S, 11), dtype=torch.int64, device=dev)
    rows = torch.empty((S, N.NBUCKETS), dtype=torch.int32, device=dev)
    eng.snapshot_into(summ, rows, reset=True)
    np.testing.assert_array_equal(rows.cpu().numpy(), c2["counts"])
    _eq(summ.cpu().numpy().view(N.SUMMARY_DTYPE).reshape(-1), c2["summaries"], "C2")
    eng.close()


def test_c5_prometheus_100k_stats_counters_10k_gauges(c2):
    """BASELINE C5 at full size: the C2 stats in the stats-tree shape of the fixture
    (rt/<r>/client/<c>/service/<s>/request_latency_ms), 100k counters, 10k gauges."""
    from linkerd_amd.prometheus import PrometheusTelemeter, line_multiset
    from linkerd_amd.telemetry import HistogramSummary, MetricsTree, MetricsTreeStatsReceiver, StatEngine, \
        snapshot_histograms
    S = c2["S"]
    eng = StatEngine(capacity=S)
    tree, otree = MetricsTree(eng), MetricsTree()
    stats, ostats = MetricsTreeStatsReceiver(tree), MetricsTreeStatsReceiver(otree)
    paths = [("rt", f"r{i % 4}", "client", f"/#/io.l5d.k8s/ns/http/c{i % 997}", "service", f"/svc/s{i}",
              "request_latency_ms") for i in range(S)]
    sid = np.empty(S, np.uint32)
    ost = []
    for i, p in enumerate(paths):
        sid[i] = stats.stat(*p).series_id
        ost.append(ostats.stat(*p))
    for i in range(100_000):
        for st in (stats, ostats):
            st.scope("rt", f"r{i % 4}", "server", f"10.1.{i % 250}.{i % 7}/4141").counter(f"requests_{i}").incr(i * 7)
    for i in range(10_000):
        for st in (stats, ostats):
            st.scope("jvm", f"pool{i % 10}").add_gauge(f"g{i}", f=lambda i=i: i * 1.37 + 0.1)
    # the C2 samples, C2 series k -> Stat k
    eng.engine.ingest(sid[c2["series"]], c2["values"])
    assert snapshot_histograms(tree, eng) == S
    want = c2["summaries"]
    for i in range(S):
        ost[i]._set_snapshot(HistogramSummary.from_record(want[i]))
    got_text = PrometheusTelemeter(tree).render()
    want_text = PrometheusTelemeter(otree).render()
    got, exp = line_multiset(got_text), line_multiset(want_text)
    assert sum(got.values()) == S * 11 + 100_000 + 10_000
    assert got == exp


def test_c4_fleet_merge_8_way_1m_series(oracle):
    import torch
    from linkerd_amd.engine import HistogramEngine
    S, n, W = 1_000_000, 1_000_000_000, 8
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    series = torch.empty(n, dtype=torch.int32, device=dev)
    values = torch.empty(n, dtype=torch.float32, device=dev)
    cdf = torch.from_numpy(synth.zipf_cdf(S)).to(dev)
    assert _synth().l5ds_gen_zipf(ctypes.c_void_p(series.data_ptr()), ctypes.c_void_p(values.data_ptr()),
                                  ctypes.c_uint64(n), ctypes.c_uint64(S), ctypes.c_void_p(cdf.data_ptr()),
                                  ctypes.c_uint64(3), ctypes.c_double(0.8), ctypes.c_uint64(0), ctypes.c_uint32(0),
                                  ctypes.c_void_p(stream)) == 0
    torch.cuda.synchronize()
    acc = torch.zeros((S, N.NBUCKETS), dtype=torch.int32, device=dev)
    acc_t = torch.zeros(S, dtype=torch.int64, device=dev)
    part = torch.empty_like(acc)
    part_t = torch.empty_like(acc_t)
    for r in range(W):  # sample i -> engine i mod 8 (one engine alive at a time: same arithmetic)
        eng = HistogramEngine(S)
        eng.ingest(series[r::W].contiguous(), values[r::W].contiguous())
        eng.export_state(counts=part, totals=part_t, reset=True)
        acc += part
        acc_t += part_t
        eng.close()
    merged = torch.empty((S, 11), dtype=torch.int64, device=dev)
    eng = HistogramEngine(S)
    eng.summarize_dense(acc, acc_t, out=merged)
    # one engine holding all samples: identical rows and summaries
    eng.ingest(series, values)
    one = torch.empty_like(merged)
    eng.snapshot_into(one, part, reset=True)
    assert torch.equal(part, acc), "merged rows differ from the single-engine rows"
    assert torch.equal(one, merged), "merged summaries differ from the single-engine summaries"
    eng.close()
    # C3 properties
    ids = series.long()
    want_count = torch.bincount(ids, minlength=S)
    assert torch.equal(acc.sum(dim=1, dtype=torch.int64), want_count)
    assert torch.equal(merged[:, 0], want_count)
    want_sum = torch.zeros(S, dtype=torch.int64, device=dev).index_add_(0, ids, values.to(torch.int64))
    del ids
    assert torch.equal(merged[:, 3], want_sum) and torch.equal(acc_t, want_sum)
    live = want_count > 0
    order = merged[live][:, [1, 4, 5, 6, 7, 8, 9, 2]]
    assert bool((order[:, 1:] >= order[:, :-1]).all())
    # sampled oracle replay
    rng = np.random.default_rng(44)
    chosen = np.unique(np.concatenate([[0, 1, 5, 31, 32, 600, 2047, 2048, 9000], rng.integers(10_000, S, 55)]))
    sel = torch.from_numpy(chosen.astype(np.int64)).to(dev)
    m = torch.isin(series, sel.to(torch.int32))
    s_sub = series[m].cpu().numpy().astype(np.int64)
    v_sub = values[m].cpu().numpy()
    o = oracle.OracleHistograms(chosen.size)
    o.ingest(np.searchsorted(chosen, s_sub).astype(np.uint32), v_sub, threads=THREADS)
    np.testing.assert_array_equal(acc[sel].cpu().numpy(), o.counts())
    got = merged[sel].cpu().numpy().view(N.SUMMARY_DTYPE).reshape(-1)
    _eq(got, o.snapshot(), "C4 sampled")
    del series, values, acc, part, m
    torch.cuda.empty_cache()
