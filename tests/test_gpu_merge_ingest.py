"""GPU tests of the C-ABI additions of round 2, against the oracle:

* l5dh_merge (RCCL fleet merge) through both communicator forms
  (l5dh_comm_init_rank with a unique id, l5dh_comm_init_all for one process holding
  its GPUs).  One GPU here, so the communicator has one rank: the export, the RCCL
  reduce-scatter / all-reduce (a copy at one rank) and the slice summaries run for
  real; the multi-rank sum is covered by tests/test_gpu_configs.py (C4: eight
  engines summed) and tests/test_fleet_gloo.py.
* the staging ring: many small l5dh_ingest calls from pinned host memory
  (l5dh_pin_alloc, what the JNI side stages into) and from device memory.
* deferred invalid-id errors, stream ordering with torch, and 8
  threads calling Stat.add / ingest concurrently with a snapshot thread
  (Metric.scala:30: add is called from any Finagle thread).
"""
import ctypes
import threading

import numpy as np
import pytest

from linkerd_amd import _native as N
from linkerd_amd import synth

pytestmark = pytest.mark.gpu


def _eq_summaries(got, want):
    g, w = got.view(np.uint8).reshape(-1, 88), want.view(np.uint8).reshape(-1, 88)
    bad = np.flatnonzero((g != w).any(axis=1))
    assert bad.size == 0, f"{bad.size} summaries differ, first series {bad[0]}: {got[bad[0]]} vs {want[bad[0]]}"


@pytest.mark.parametrize("rccl", [True, False], ids=["rccl", "identity"])
@pytest.mark.parametrize("form", ["init_rank", "init_all"])
@pytest.mark.parametrize("mode", [N.MERGE_REDUCE_SCATTER, N.MERGE_ALL_REDUCE], ids=["reduce_scatter", "all_reduce"])
def test_merge_one_rank_matches_oracle(oracle, form, mode, rccl):
    """rccl: the 1-rank collective runs through RCCL (forced); identity: skipped."""
    from linkerd_amd.engine import HistogramEngine
    S = 3001
    s1, v1 = synth.c3(S=S, N=400_000, seed=61)
    s2, v2 = synth.c3(S=S, N=300_000, seed=62)
    eng = HistogramEngine(S)
    eng.set_param(N.PARAM_MERGE_RCCL_1RANK, int(rccl))
    if form == "init_rank":
        eng.comm_init_rank(HistogramEngine.comm_unique_id(), 1, 0)
    else:
        HistogramEngine.comm_init_all([eng])
    o = oracle.OracleHistograms(S)
    eng.ingest(s1, v1)
    o.ingest(s1, v1)
    eng.snapshot(reset=False)  # folded state (dirty tiles) + a pending segment
    eng.ingest(s2, v2)
    o.ingest(s2, v2)
    rows = eng.merge_rows(mode)
    assert rows == S
    counts = np.zeros((rows, N.NBUCKETS), np.int32)
    totals = np.zeros(rows, np.int64)
    first, count, summ = eng.merge(mode, counts=counts, totals=totals)
    assert (first, count) == (0, S)
    np.testing.assert_array_equal(counts, o.counts())
    np.testing.assert_array_equal(totals, o.totals())
    _eq_summaries(summ, o.snapshot())
    # the merge exported with reset: the engine is empty afterwards
    after = eng.snapshot(reset=False)
    assert not after["count"].any()
    eng.comm_destroy()
    eng.close()


@pytest.mark.parametrize("value", [7.0, 3e9], ids=["bucket", "overflow"])
def test_merge_sparse_escaped_counts(oracle, value):
    """The sparse exchange's escape: one bucket of one series holds 2.5M > 2^21 - 1
    samples, so its count takes a second word; the decoder must take that word as a
    count (whatever its low bits) -- through RCCL at one rank, against the oracle."""
    from linkerd_amd.engine import HistogramEngine
    S = 300
    rng = np.random.default_rng(7)
    hot = np.zeros(2_500_000, np.uint32)
    cold = rng.integers(0, S, 200_000).astype(np.uint32)
    series = np.concatenate([hot, cold])
    vals = np.concatenate([np.full(hot.size, value, np.float32),
                           np.exp(2 + rng.standard_normal(cold.size)).astype(np.float32)])
    perm = rng.permutation(series.size)
    series, vals = series[perm], vals[perm]
    eng = HistogramEngine(S)
    eng.set_param(N.PARAM_MERGE_RCCL_1RANK, 1)
    eng.comm_init_rank(HistogramEngine.comm_unique_id(), 1, 0)
    eng.ingest(series, vals)
    counts = np.zeros((S, N.NBUCKETS), np.int32)
    totals = np.zeros(S, np.int64)
    first, count, summ = eng.merge(N.MERGE_REDUCE_SCATTER, counts=counts, totals=totals)
    o = oracle.OracleHistograms(S)
    o.ingest(series, vals)
    np.testing.assert_array_equal(counts, o.counts())
    np.testing.assert_array_equal(totals, o.totals())
    _eq_summaries(summ, o.snapshot())
    mb = eng.merge_bytes()
    assert mb["dense"] == S * (N.NBUCKETS * 4 + 8) and 0 < mb["encoded"] < mb["dense"]
    eng.comm_destroy()
    eng.close()


def test_merge_without_communicator_is_einval():
    from linkerd_amd.engine import HistogramEngine
    eng = HistogramEngine(64)
    with pytest.raises(N.L5dhError, match="EINVAL"):
        eng.merge()
    eng.close()


def _pinned(lib, n, dtype):
    p = ctypes.c_void_p()
    assert lib.l5dh_pin_alloc(n * np.dtype(dtype).itemsize, ctypes.byref(p)) == 0
    arr = np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint8)), shape=(n * np.dtype(dtype).itemsize,))
    return p, arr.view(dtype)


@pytest.mark.parametrize("piece", [65536, 1 << 20, 777])
def test_streaming_small_batches_from_pinned_memory(oracle, piece):
    """The JNI staging shape: a batch delivered in `piece`-sample calls from one
    pinned buffer that is refilled after every call (the library must have copied
    it by then); the ring is flushed when full and at the snapshot."""
    from linkerd_amd.engine import HistogramEngine
    S, n = 20_000, 3_000_000
    series, vals = synth.c3(S=S, N=n, seed=71)
    lib = N.load()
    eng = HistogramEngine(S)
    eng.set_param(N.PARAM_STAGE_SAMPLES, 1 << 21)
    ps, hs = _pinned(lib, piece, np.uint32)
    pv, hv = _pinned(lib, piece, np.float32)
    for off in range(0, n, piece):
        m = min(piece, n - off)
        hs[:m] = series[off:off + m]
        hv[:m] = vals[off:off + m]
        eng._check(lib.l5dh_ingest(eng._ctx, ps, pv, m), "l5dh_ingest")
        hs[:m] = 0xFFFFFFFF  # overwrite right away: the call must not read it any more
        hv[:m] = np.nan
    got, counts = eng.snapshot(reset=True, with_counts=True)
    eng.sync()  # no invalid id was ever ingested
    o = oracle.OracleHistograms(S)
    o.ingest(series, vals, threads=8)
    np.testing.assert_array_equal(counts, o.counts())
    _eq_summaries(got, o.snapshot())
    lib.l5dh_pin_free(ps)
    lib.l5dh_pin_free(pv)
    eng.close()


@pytest.mark.parametrize("piece,stage", [(65536, None), (777, None), (1 << 20, 0)], ids=["64k", "777", "1m-unstaged"])
def test_async_double_buffered_ingest(oracle, piece, stage):
    """l5dh_ingest_async with two pinned staging pairs (the JNI thread's shape): a pair
    is refilled only after its ticket completed, and overwritten right after."""
    from linkerd_amd.engine import HistogramEngine
    S, n = 20_000, 3_000_000
    series, vals = synth.c3(S=S, N=n, seed=72)
    lib = N.load()
    eng = HistogramEngine(S)
    if stage is not None:
        eng.set_param(N.PARAM_STAGE_SAMPLES, stage)
    bufs = [(_pinned(lib, piece, np.uint32), _pinned(lib, piece, np.float32)) for _ in range(2)]
    tickets = [0, 0]
    import ctypes as C
    t = C.c_uint64(0)
    for i, off in enumerate(range(0, n, piece)):
        k = i & 1
        if tickets[k]:
            eng.ingest_wait(tickets[k])
        (ps, hs), (pv, hv) = bufs[k]
        hs[:] = 0xFFFFFFFF
        hv[:] = np.nan
        m = min(piece, n - off)
        hs[:m] = series[off:off + m]
        hv[:m] = vals[off:off + m]
        eng._check(lib.l5dh_ingest_async(eng._ctx, ps, pv, m, C.byref(t)), "l5dh_ingest_async")
        assert t.value > max(tickets)
        tickets[k] = t.value
    eng.ingest_wait(max(tickets))
    for (ps, hs), (pv, hv) in bufs:  # everything consumed: the buffers may go
        hs[:] = 0xFFFFFFFF
    got, counts = eng.snapshot(reset=True, with_counts=True)
    eng.sync()
    o = oracle.OracleHistograms(S)
    o.ingest(series, vals, threads=8)
    np.testing.assert_array_equal(counts, o.counts())
    _eq_summaries(got, o.snapshot())
    for (ps, _), (pv, _) in bufs:
        lib.l5dh_pin_free(ps)
        lib.l5dh_pin_free(pv)
    eng.close()


def test_staged_device_batches_and_deferred_errors(oracle):
    import torch
    from linkerd_amd.engine import HistogramEngine
    S = 500
    rng = np.random.default_rng(3)
    eng = HistogramEngine(S)
    o = oracle.OracleHistograms(S)
    bad_seen = 0
    for k in range(40):
        s = rng.integers(0, S, 5000).astype(np.uint32)
        v = np.exp(rng.uniform(0, 9, 5000)).astype(np.float32)
        if k == 17:
            s[::1000] = S + 5  # dropped, reported later
        ds = torch.from_numpy(s.view(np.int32)).cuda()
        dv = torch.from_numpy(v).cuda()
        try:
            eng.ingest(ds, dv)
        except N.L5dhError as e:
            assert "EINVAL" in str(e)
            bad_seen += 1
        ok = s < S
        o.ingest(s[ok], v[ok])
    try:
        eng.sync()
    except N.L5dhError:
        bad_seen += 1
    assert bad_seen == 1, "the invalid ids are reported exactly once"
    eng.sync()
    got, counts = eng.snapshot(with_counts=True)
    np.testing.assert_array_equal(counts, o.counts())
    _eq_summaries(got, o.snapshot())
    eng.close()


@pytest.mark.parametrize("side", [False, True], ids=["default_stream", "side_stream"])
def test_stream_ordered_with_torch_no_sync(oracle, side):
    """device inputs produced by torch work are read in stream order --
    `counts += c` then summarize_dense on an already open engine, no synchronize --
    on torch's default (legacy null) stream and on a torch side stream."""
    import contextlib
    import torch
    from linkerd_amd.engine import HistogramEngine
    ctx = torch.cuda.stream(torch.cuda.Stream()) if side else contextlib.nullcontext()
    with ctx:
        _stream_ordered_body(oracle, torch, HistogramEngine)


def _stream_ordered_body(oracle, torch, HistogramEngine):
    S = 4000
    series, vals = synth.c3(S=S, N=500_000, seed=81)
    o = oracle.OracleHistograms(S)
    o.ingest(series, vals)
    want = o.snapshot(reset=False)
    eng = HistogramEngine(S)
    dev = torch.device("cuda", 0)
    base = torch.from_numpy(o.counts()).to(dev)
    tot = torch.from_numpy(o.totals()).to(dev)
    torch.cuda.synchronize()
    for _ in range(3):
        counts = torch.zeros_like(base)
        totals = torch.zeros_like(tot)
        counts += base  # queued on torch's stream, not synchronized
        totals += tot
        summ = torch.empty((S, 11), dtype=torch.int64, device=dev)
        eng.summarize_dense(counts, totals, out=summ)
        got = summ.cpu().numpy().view(N.SUMMARY_DTYPE).reshape(-1)
        _eq_summaries(got, want)
    eng.close()


@pytest.mark.parametrize("pct", [100, 40], ids=["regions", "redo"])
def test_snapshot_stream_ordered_on_caller_stream(oracle, pct):
    """An engine on torch's stream (l5dh_set_stream) with device outputs returns from
    l5dh_snapshot without a host wait: batches generated, ingested and snapshotted
    back to back, each snapshot read by torch work queued behind it, no synchronize
    in between -- every interval bit-exact (reset: each holds only its own batch)."""
    import torch
    from linkerd_amd.engine import HistogramEngine
    S = 3000
    dev = torch.device("cuda", 0)
    with torch.cuda.stream(torch.cuda.Stream()):
        eng = HistogramEngine(S)
        eng.set_param(N.PARAM_REGION_PCT, pct)
        eng.set_stream(torch.cuda.current_stream().cuda_stream)
        batches = [synth.c3(S=S, N=400_000, seed=90 + k) for k in range(4)]
        dbat = [(torch.from_numpy(sr.astype(np.int32)).to(dev), torch.from_numpy(v).to(dev)) for sr, v in batches]
        torch.cuda.synchronize()
        outs = []
        for ds, dv in dbat:
            eng.ingest(ds, dv)
            summ = torch.empty((S, 11), dtype=torch.int64, device=dev)
            counts = torch.empty((S, N.NBUCKETS), dtype=torch.int32, device=dev)
            eng.snapshot_into(summ, counts, reset=True)
            outs.append((summ.clone(), counts.sum(dim=0)))  # torch work behind the snapshot
        torch.cuda.synchronize()
        for (sr, v), (summ, csum) in zip(batches, outs):
            o = oracle.OracleHistograms(S)
            o.ingest(sr, v)
            np.testing.assert_array_equal(csum.cpu().numpy(), o.counts().sum(axis=0))
            _eq_summaries(summ.cpu().numpy().view(N.SUMMARY_DTYPE).reshape(-1), o.snapshot())
        eng.close()


def test_concurrent_adds_and_snapshots_bitexact(oracle):
    """8 producer threads (Stat.add through per-thread staging, and direct batched
    ingest) while a timer thread snapshots with reset: the snapshots together hold
    every sample exactly once (snapshot + reset is atomic per call)."""
    from linkerd_amd.telemetry import MetricsTree, MetricsTreeStatsReceiver, StatEngine
    S = 256
    eng = StatEngine(capacity=S, batch=512)
    tree = MetricsTree(eng)
    stats = [MetricsTreeStatsReceiver(tree).scope("rt", "r", "client", f"c{i}").stat("request_latency_ms")
             for i in range(S)]
    ids = np.array([s.series_id for s in stats], np.uint32)
    rng = np.random.default_rng(12)
    per = [(rng.integers(0, S, 40_000), np.exp(rng.uniform(0, 10, 40_000)).astype(np.float32)) for _ in range(8)]
    acc = {"counts": np.zeros((S, N.NBUCKETS), np.int64), "sum": np.zeros(S, np.int64)}
    stop = threading.Event()
    errors = []

    def producer(k):
        try:
            which, vals = per[k]
            if k % 2:
                for w, v in zip(which[:4000], vals[:4000]):
                    stats[w].add(float(v))
                eng.engine.ingest(ids[which[4000:]], vals[4000:])
            else:
                for w, v in zip(which, vals):
                    stats[w].add(float(v))
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    def timer():
        while not stop.is_set():
            eng.flush()
            summ, counts = eng.engine.snapshot(reset=True, with_counts=True)
            acc["counts"] += counts
            acc["sum"] += summ["sum"]

    ts = [threading.Thread(target=producer, args=(k,)) for k in range(8)]
    tt = threading.Thread(target=timer)
    tt.start()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    stop.set()
    tt.join()
    assert not errors, errors
    eng.flush()
    summ, counts = eng.engine.snapshot(reset=True, with_counts=True)
    acc["counts"] += counts
    acc["sum"] += summ["sum"]
    o = oracle.OracleHistograms(S)
    for which, vals in per:
        o.ingest(ids[which], vals)
    np.testing.assert_array_equal(acc["counts"], o.counts())
    np.testing.assert_array_equal(acc["sum"], o.totals())
