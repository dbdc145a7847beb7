"""GPU side of the fleet merge (C4) on one device: two engines hold disjoint sample
shards of the same series space; their exported dense state is summed on the GPU
(what the RCCL reduce-scatter does across GPUs; the collective itself is covered by
tests/test_fleet_gloo.py) and summarized with l5dh_summarize_dense."""
import numpy as np
import pytest

from linkerd_amd import synth
from linkerd_amd import _native as N

pytestmark = pytest.mark.gpu


def test_sample_sharded_merge_on_gpu(oracle):
    import torch
    from linkerd_amd.engine import HistogramEngine
    S, n = 3000, 400_000
    series, vals = synth.c3(S=S, N=n, seed=21)
    dev = torch.device("cuda", 0)
    counts = torch.zeros((S, N.NBUCKETS), dtype=torch.int32, device=dev)
    totals = torch.zeros(S, dtype=torch.int64, device=dev)
    for r in range(2):
        eng = HistogramEngine(S)
        m = np.arange(n) % 2 == r
        eng.ingest(series[m], vals[m])
        c = torch.empty_like(counts)
        t = torch.empty_like(totals)
        eng.export_state(counts=c, totals=t, reset=True)
        torch.cuda.synchronize()
        counts += c
        totals += t
        eng.close()
    eng = HistogramEngine(S)
    summ = torch.empty((S, 11), dtype=torch.int64, device=dev)
    eng.summarize_dense(counts, totals, out=summ)
    torch.cuda.synchronize()
    o = oracle.OracleHistograms(S)
    o.ingest(series, vals)
    np.testing.assert_array_equal(counts.cpu().numpy(), o.counts())
    assert summ.cpu().numpy().tobytes() == o.snapshot().tobytes()


@pytest.mark.parametrize("dev_bufs", [True, False])
def test_export_reset_fused_matches_oracle(oracle, dev_bufs):
    """export_state(reset=True) over the whole series range runs as one aggregate
    pass into the caller's rows: kept state (dirty tiles), split/direct tiles of a
    Zipf head and pending segments must all land, and the state is clean after."""
    import torch
    from linkerd_amd.engine import HistogramEngine
    S = 5000
    o = oracle.OracleHistograms(S)
    eng = HistogramEngine(S)
    batches = [synth.c3(S=S, N=n, seed=31 + i) for i, n in enumerate((1_500_000, 1_200_000, 900_000))]
    eng.ingest(*batches[0])
    o.ingest(*batches[0])
    eng.snapshot(reset=False)  # folds into state: dirty tiles
    for b in batches[1:]:      # two pending segments, the second sized from the first
        eng.ingest(*b)
        o.ingest(*b)
    if dev_bufs:
        dev = torch.device("cuda", 0)
        c = torch.empty((S, N.NBUCKETS), dtype=torch.int32, device=dev)
        t = torch.empty(S, dtype=torch.int64, device=dev)
        eng.export_state(counts=c, totals=t, reset=True)
        torch.cuda.synchronize()
        counts, totals = c.cpu().numpy(), t.cpu().numpy()
    else:
        counts, totals = eng.export_state(reset=True)
    np.testing.assert_array_equal(counts, o.counts())
    np.testing.assert_array_equal(totals, o.totals())
    after = eng.snapshot(reset=False)
    assert not after["count"].any() and not after["sum"].any()
    # the engine keeps working from the clean state
    s2, v2 = synth.c3(S=S, N=300_000, seed=41)
    eng.ingest(s2, v2)
    o2 = oracle.OracleHistograms(S)
    o2.ingest(s2, v2)
    counts, totals = eng.export_state(reset=True)
    np.testing.assert_array_equal(counts, o2.counts())
    np.testing.assert_array_equal(totals, o2.totals())
    eng.close()


def _oracle_of(oracle, S, parts):
    o = oracle.OracleHistograms(S)
    for s, v in parts:
        o.ingest(s, v)
    return o


@pytest.mark.parametrize("mode", [N.MERGE_REDUCE_SCATTER, N.MERGE_ALL_REDUCE], ids=["reduce_scatter", "all_reduce"])
@pytest.mark.parametrize("W", [2, 3, 8])
def test_loopback_multirank_merge(oracle, W, mode):
    """The W > 1 merge code on one GPU (l5dh_comm_init_loopback): per-destination
    slices of the sparse encoding, the size all-gather, the payload exchange, the
    local slice decoded in place, the totals' reduce-scatter -- or the dense
    all-reduce -- with S not divisible by W, an escaped count (> 2^21 - 1 samples of
    one bucket on one rank), a cold row with more non-empty buckets than the export's
    per-row list (ENC_LIST) and two merge intervals through the same buffers, the
    second with kept state (dirty tiles) under new records."""
    from linkerd_amd.engine import HistogramEngine
    S = 4001
    engines = [HistogramEngine(S) for _ in range(W)]
    try:
        HistogramEngine.comm_init_loopback(engines)
        with pytest.raises(N.L5dhError):
            engines[0].merge(mode)  # a loopback group merges through l5dh_merge_all only
        for interval in range(2):
            series, vals = synth.c3(S=S, N=300_000 + 50_000 * interval, seed=60 + 7 * W + interval)
            parts = []
            for r, e in enumerate(engines):
                p = (series[r::W], vals[r::W])
                if interval == 1:  # kept state: half folded by a non-resetting snapshot (dirty tiles)
                    h = p[0].size // 2
                    e.ingest(p[0][:h], p[1][:h])
                    e.snapshot(reset=False)
                    e.ingest(p[0][h:], p[1][h:])
                else:
                    e.ingest(*p)
                parts.append(p)
            if interval == 0:  # series 17: one bucket past the encoding's count field, on the last rank
                heavy = (np.full(2_100_000, 17, np.uint32), np.full(2_100_000, 3.0, np.float32))
                engines[-1].ingest(*heavy)
                parts.append(heavy)
                # series 40 (a cold tile): more non-empty buckets than the export lists per row
                wide = (np.full(20_000, 40, np.uint32), np.arange(1, 20_001, dtype=np.float32))
                engines[0].ingest(*wide)
                parts.append(wide)
            o = _oracle_of(oracle, S, parts)
            want_c, want_t, want_s = o.counts(), o.totals(), o.snapshot()
            res = HistogramEngine.merge_all(engines, mode, with_counts=True)
            per = -(-S // W)
            for r, (first, count, summ, cnt, tot) in enumerate(res):
                if mode == N.MERGE_REDUCE_SCATTER:
                    assert (first, count) == (min(r * per, S), max(0, min(per, S - r * per)))
                else:
                    assert (first, count) == (0, S)
                sl = slice(first, first + count)
                np.testing.assert_array_equal(cnt, want_c[sl])
                np.testing.assert_array_equal(tot, want_t[sl])
                assert summ.tobytes() == want_s[sl].tobytes()
            if mode == N.MERGE_REDUCE_SCATTER:
                assert all(e.merge_bytes()["sent"] > 0 for e in engines)
            for e in engines:  # the export consumed every rank's interval
                after = e.snapshot(reset=False)
                assert not after["count"].any() and not after["sum"].any()
    finally:
        for e in engines:
            e.close()


def test_comm_rejects_more_than_64_ranks_before_any_state_is_consumed(oracle):
    """the sparse reduce-scatter holds <= 64 sources; a larger communicator
    is refused at init (not inside a merge, after the export consumed the interval)."""
    from linkerd_amd.engine import HistogramEngine
    S = 300
    series, vals = synth.c3(S=S, N=50_000, seed=71)
    eng = HistogramEngine(S)
    try:
        eng.ingest(series, vals)
        with pytest.raises(N.L5dhError):
            eng.comm_init_rank(HistogramEngine.comm_unique_id(), 65, 0)
        got = eng.snapshot(reset=True)
        o = _oracle_of(oracle, S, [(series, vals)])
        assert got.tobytes() == o.snapshot().tobytes()
    finally:
        eng.close()


@pytest.mark.parametrize("forced", [0, 1])
def test_one_rank_loopback_merge_ignores_the_rccl_forcing_param(oracle, forced):
    """a 1-rank loopback group has no transport that could send the slice to
    itself, so L5DH_PARAM_MERGE_RCCL_1RANK must not route it into the exchange (whose
    decode would read receive buffers nothing wrote): the merge is the identity."""
    from linkerd_amd.engine import HistogramEngine
    S = 2500
    eng = HistogramEngine(S)
    try:
        eng.set_param(N.PARAM_MERGE_RCCL_1RANK, forced)
        HistogramEngine.comm_init_loopback([eng])
        eng.set_param(N.PARAM_MERGE_RCCL_1RANK, forced)  # either order
        for rnd in range(2):  # stale buffers of a first merge must not leak into a second
            s, v = synth.c3(S=S, N=200_000 + 1000 * rnd, seed=83 + rnd)
            eng.ingest(s, v)
            o = _oracle_of(oracle, S, [(s, v)])
            (first, count, summ, cnt, tot), = HistogramEngine.merge_all([eng], N.MERGE_REDUCE_SCATTER, with_counts=True)
            assert (first, count) == (0, S)
            np.testing.assert_array_equal(cnt, o.counts())
            np.testing.assert_array_equal(tot, o.totals())
            assert summ.tobytes() == o.snapshot().tobytes()
    finally:
        eng.close()
