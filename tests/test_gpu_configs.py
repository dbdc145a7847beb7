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

from .test_gpu_fullsize import _all_summaries_match_oracle

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


def test_c4_product_sparse_merge_8_way_1m_series(oracle):
    """C4 through the PRODUCT merge at full size: 8 loopback ranks (one device), 1M
    series, the 1e9-sample C3 batch sample-sharded (sample i -> rank i mod 8), merged
    by l5dh_merge_all(MERGE_REDUCE_SCATTER) -- the sparse export from the accumulate
    kernels (first-touch lists and whole-row encodes), the half-tile pack, the
    per-destination slices (~125K rows each), the exchange, the totals' reduce-scatter
    and the decode + summaries of every slice.  Two intervals through the same
    buffers (seeds 3, 4).  Every rank's slice is checked against a torch ground truth
    independent of the engine (bincount of series * 1798 + upper_bound(limits,
    (long)value), exact int64 sums), its summaries against one engine's snapshot of the
    whole batch, and a sample of series by a bit-exact oracle replay."""
    import torch
    from linkerd_amd.engine import HistogramEngine
    S, n, W = 1_000_000, 1_000_000_000, 8
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream().cuda_stream
    lib = N.load()
    series = torch.empty(n, dtype=torch.int32, device=dev)
    values = torch.empty(n, dtype=torch.float32, device=dev)
    cdf = torch.from_numpy(synth.zipf_cdf(S)).to(dev)
    lim = torch.from_numpy(oracle.limits().astype(np.int64)).to(dev)
    per = -(-S // W)
    engines = [HistogramEngine(S) for _ in range(W)]
    summ = [torch.empty((per, 11), dtype=torch.int64, device=dev) for _ in range(W)]
    rows = [torch.empty((per, N.NBUCKETS), dtype=torch.int32, device=dev) for _ in range(W)]
    tots = [torch.empty(per, dtype=torch.int64, device=dev) for _ in range(W)]
    ctxs = (ctypes.c_void_p * W)(*[e._ctx.value for e in engines])
    o_arr = (ctypes.c_void_p * W)(*[t.data_ptr() for t in summ])
    c_arr = (ctypes.c_void_p * W)(*[t.data_ptr() for t in rows])
    t_arr = (ctypes.c_void_p * W)(*[t.data_ptr() for t in tots])
    firsts, counts = (ctypes.c_uint32 * W)(), (ctypes.c_uint32 * W)()
    try:
        HistogramEngine.comm_init_loopback(engines)
        for seed in (3, 4):
            assert _synth().l5ds_gen_zipf(ctypes.c_void_p(series.data_ptr()), ctypes.c_void_p(values.data_ptr()),
                                          ctypes.c_uint64(n), ctypes.c_uint64(S), ctypes.c_void_p(cdf.data_ptr()),
                                          ctypes.c_uint64(seed), ctypes.c_double(0.8), ctypes.c_uint64(0),
                                          ctypes.c_uint32(0), ctypes.c_void_p(stream)) == 0
            torch.cuda.synchronize()
            # the single-engine summaries of the whole batch (the engine's own dense path)
            one = HistogramEngine(S)
            one_summ = torch.empty((S, 11), dtype=torch.int64, device=dev)
            one.ingest(series, values)
            one.snapshot_into(one_summ, None, reset=True)
            torch.cuda.synchronize()
            one.close()
            del one
            torch.cuda.empty_cache()
            for r, e in enumerate(engines):
                sr, vr = series[r::W].contiguous(), values[r::W].contiguous()
                torch.cuda.synchronize()
                e.ingest(sr, vr)
                torch.cuda.synchronize()
                del sr, vr
            rc = lib.l5dh_merge_all(ctxs, W, N.MERGE_REDUCE_SCATTER, o_arr, c_arr, t_arr, firsts, counts)
            if rc != 0:
                engines[0]._check(rc, "l5dh_merge_all")
            torch.cuda.synchronize()
            # the torch ground truth, independent of the engine's LUTs and kernels
            truth = torch.zeros(S * N.NBUCKETS, dtype=torch.int32, device=dev)
            sums = torch.zeros(S, dtype=torch.int64, device=dev)
            step = 100_000_000
            for o in range(0, n, step):
                ids = series[o:o + step].long()
                v = values[o:o + step].to(torch.int64)  # values in [0, 1e9]: (long)value
                b = torch.searchsorted(lim, v, right=True)
                truth.index_add_(0, ids * N.NBUCKETS + b, torch.ones_like(b, dtype=torch.int32))
                sums.index_add_(0, ids, v)
                del ids, v, b
            truth = truth.view(S, N.NBUCKETS)
            for r in range(W):
                f, c = firsts[r], counts[r]
                assert (f, c) == (min(r * per, S), max(0, min(per, S - r * per))), f"rank {r} slice"
                bad = (rows[r][:c] != truth[f:f + c]).any(dim=1)
                assert int(bad.sum()) == 0, \
                    f"seed {seed} rank {r}: {int(bad.sum())} rows differ, first {(torch.nonzero(bad)[:8].flatten() + f).tolist()}"
                assert torch.equal(tots[r][:c], sums[f:f + c]), f"seed {seed} rank {r}: totals"
                assert torch.equal(summ[r][:c], one_summ[f:f + c]), f"seed {seed} rank {r}: summaries vs one engine"
                assert torch.equal(summ[r][:c, 0], truth[f:f + c].sum(dim=1, dtype=torch.int64))
                assert torch.equal(summ[r][:c, 3], sums[f:f + c])
                # every field of every series of the slice against the oracle's summary of
                # the truth rows (Metric.scala:53-67), bytewise
                _all_summaries_match_oracle(oracle, truth[f:f + c], sums[f:f + c], summ[r][:c],
                                            f"seed {seed} rank {r}", first=f)
            del truth, sums, one_summ
            # bit-exact oracle replay of sampled series (head, direct/split, cold; every rank's slice)
            rng = np.random.default_rng(100 + seed)
            chosen = np.unique(np.concatenate([[0, 1, 2, 31, 32, 2047, 9000, per - 1, per, 3 * per + 7, S - 1],
                                               rng.integers(10_000, S, 53)])).astype(np.int64)
            sel = torch.from_numpy(chosen).to(dev)
            m = torch.isin(series, sel.to(torch.int32))
            s_sub = series[m].cpu().numpy().astype(np.int64)
            v_sub = values[m].cpu().numpy()
            del m
            o = oracle.OracleHistograms(chosen.size)
            o.ingest(np.searchsorted(chosen, s_sub).astype(np.uint32), v_sub, threads=THREADS)
            want_c, want_s = o.counts(), o.snapshot()
            for i, sid in enumerate(chosen):
                r = int(sid) // per
                k = int(sid) - firsts[r]
                np.testing.assert_array_equal(rows[r][k].cpu().numpy(), want_c[i], err_msg=f"series {sid} counts")
                got = summ[r][k].cpu().numpy().view(N.SUMMARY_DTYPE)
                for fld in N.SUMMARY_FIELDS:
                    assert got[fld][0] == want_s[fld][i], f"series {sid} field {fld}: {got[fld][0]} vs {want_s[fld][i]}"
    finally:
        for e in engines:
            e.close()
        del series, values, rows, summ, tots
        torch.cuda.empty_cache()
