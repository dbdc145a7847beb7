"""Full-size parity (BASELINE config C3: 1M series, Zipf(s=1) ids, log-normal values)
through size-independent properties, where the CPU oracle cannot replay the whole
batch in seconds.

The batch holds 1.1e9 samples, more than one binned piece (2^30 - 65536), so the
engine splits it into two segments: both pieces' split/direct/cold tile paths and
the multi-segment snapshot run at full width.  Checked on the GPU with plain torch
integer ops (independent of the engine's kernels):
  * dense row sums == bincount of the series ids (every sample in exactly one bucket),
  * summary count == row sum and summary sum == the exact integer sum of the
    truncated values ((long)value, Metric.scala:32; the values are in [0, 1e9]),
  * min <= p50 <= p90 <= p95 <= p99 <= p999 <= p9999 <= max for every non-empty series,
  * and a bit-exact oracle replay (counts + summaries) of a sample of series --
    direct-tile, split-tile and cold-tile ones -- with all their samples gathered
    from the full batch.
"""
import ctypes

import numpy as np
import pytest

from linkerd_amd import _native as N
from linkerd_amd import synth

pytestmark = pytest.mark.gpu


def test_c3_full_size_invariants_and_sampled_oracle(oracle):
    import torch
    from linkerd_amd.engine import HistogramEngine

    S, n = 1_000_000, 1_100_000_000
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream().cuda_stream
    lib = ctypes.CDLL(N.SYNTH_PATH)
    lib.l5ds_gen_zipf.restype = ctypes.c_int
    series = torch.empty(n, dtype=torch.int32, device=dev)
    values = torch.empty(n, dtype=torch.float32, device=dev)
    cdf = torch.from_numpy(synth.zipf_cdf(S)).to(dev)
    rc = lib.l5ds_gen_zipf(ctypes.c_void_p(series.data_ptr()), ctypes.c_void_p(values.data_ptr()),
                           ctypes.c_uint64(n), ctypes.c_uint64(S), ctypes.c_void_p(cdf.data_ptr()),
                           ctypes.c_uint64(3), ctypes.c_double(0.8), ctypes.c_uint64(0), ctypes.c_uint32(0),
                           ctypes.c_void_p(stream))
    assert rc == 0
    torch.cuda.synchronize()

    eng = HistogramEngine(S)
    summ = torch.empty((S, 11), dtype=torch.int64, device=dev)
    rows = torch.empty((S, N.NBUCKETS), dtype=torch.int32, device=dev)
    eng.ingest(series, values)  # > one binned piece: two segments
    eng.snapshot_into(summ, rows, reset=True)
    torch.cuda.synchronize()

    ids = series.long()
    want_count = torch.bincount(ids, minlength=S)
    row_sum = rows.sum(dim=1, dtype=torch.int64)
    assert torch.equal(row_sum, want_count), "dense rows do not hold every sample exactly once"
    assert torch.equal(summ[:, 0], want_count), "summary count != samples per series"
    want_sum = torch.zeros(S, dtype=torch.int64, device=dev).index_add_(0, ids, values.to(torch.int64))
    del ids
    assert torch.equal(summ[:, 3], want_sum), "summary sum != exact sum of (long)value"
    live = want_count > 0
    order = summ[live][:, [1, 4, 5, 6, 7, 8, 9, 2]]  # min p50 p90 p95 p99 p999 p9999 max
    assert bool((order[:, 1:] >= order[:, :-1]).all()), "percentiles out of order"

    # bit-exact oracle replay of sampled series: the Zipf head (series 0 alone holds
    # 6.95 % of the batch, 0-2 together 12.7 %), direct/split tiles (ids < 8192 are
    # the hottest tiles) and cold tiles
    rng = np.random.default_rng(5)
    chosen = np.unique(np.concatenate([[0, 1, 2, 3, 9, 17, 33, 100, 517, 1024, 1500, 4095, 8191],
                                       rng.integers(8192, S, size=54)])).astype(np.int64)
    sel = torch.from_numpy(chosen).to(dev)
    m = torch.isin(series, sel.to(torch.int32))
    s_sub = series[m].cpu().numpy().astype(np.int64)
    v_sub = values[m].cpu().numpy()
    remap = np.searchsorted(chosen, s_sub).astype(np.uint32)
    o = oracle.OracleHistograms(chosen.size)
    o.ingest(remap, v_sub, threads=8)
    np.testing.assert_array_equal(rows[sel].cpu().numpy(), o.counts())
    got = summ[sel].cpu().numpy()
    want = o.snapshot()
    for i, f in enumerate(N.SUMMARY_FIELDS):
        w = want[f].view(np.int64) if f == "avg" else want[f]
        np.testing.assert_array_equal(got[:, i], w, err_msg=f"field {f}")
    eng.close()
    del series, values, rows, summ, m
    torch.cuda.empty_cache()


THREADS = 16  # the GPU box's CPU share per GPU


def _all_summaries_match_oracle(oracle, truth, sums, summ, what, first=0):
    """All 11 HistogramSummary fields of every row of `summ` (device [n][11] int64, avg as
    its bits) == the oracle's summaries of the torch truth rows `truth` (device [n][1798])
    with the exact totals `sums`, compared as bytes; a mismatch names its first series and
    field (`first` offsets the series ids)."""
    want = oracle.summarize_counts(truth.cpu().numpy(), sums.cpu().numpy(), threads=THREADS)
    got = summ.cpu().numpy()
    assert got.shape[0] == want.shape[0]
    wb = want.view(np.int64).reshape(-1, 11)
    if not np.array_equal(got, wb):
        bad = np.nonzero((got != wb).any(axis=1))[0]
        i = int(bad[0])
        fld = [f for k, f in enumerate(N.SUMMARY_FIELDS) if got[i, k] != wb[i, k]]
        raise AssertionError(f"{what}: {bad.size} summaries differ from the oracle; first series "
                             f"{first + i} fields {fld}: {got[i].tolist()} vs {wb[i].tolist()}")


def _gen_c3(lib, series, values, S, seed, stream):
    import torch
    cdf = torch.from_numpy(synth.zipf_cdf(S)).to(series.device)
    rc = lib.l5ds_gen_zipf(ctypes.c_void_p(series.data_ptr()), ctypes.c_void_p(values.data_ptr()),
                           ctypes.c_uint64(series.numel()), ctypes.c_uint64(S), ctypes.c_void_p(cdf.data_ptr()),
                           ctypes.c_uint64(seed), ctypes.c_double(0.8), ctypes.c_uint64(0), ctypes.c_uint32(0),
                           ctypes.c_void_p(stream))
    assert rc == 0
    torch.cuda.synchronize()


def test_c3_whole_batches_bucket_exact(oracle):
    """Every bucket of whole C3 batches (1e9 samples each) against a torch ground truth:
    bincount of series * 1798 + upper_bound(limits, (long)value) -- the
    Arrays.binarySearch insertion rule of BucketedHistogram.add (Metric.scala:30-33),
    computed with torch.searchsorted, independent of the engine's LUTs and kernels --
    plus the exact per-series sums and counts of the summaries.  Three batches in a
    row through one engine (seeds 3, 4, 3: the bench's rotation), so the second and
    third are binned with regions planned from a different previous batch."""
    import torch
    from linkerd_amd.engine import HistogramEngine
    S, n = 1_000_000, 1_000_000_000
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream().cuda_stream
    lib = ctypes.CDLL(N.SYNTH_PATH)
    lib.l5ds_gen_zipf.restype = ctypes.c_int
    series = torch.empty(n, dtype=torch.int32, device=dev)
    values = torch.empty(n, dtype=torch.float32, device=dev)
    lim = torch.from_numpy(oracle.limits().astype(np.int64)).to(dev)  # the oracle's makeLimitsFor
    eng = HistogramEngine(S)
    rows = torch.empty((S, N.NBUCKETS), dtype=torch.int32, device=dev)
    summ = torch.empty((S, 11), dtype=torch.int64, device=dev)
    try:
        for seed in (3, 4, 3):
            _gen_c3(lib, series, values, S, seed, stream)
            eng.ingest(series, values)
            eng.snapshot_into(summ, rows, reset=True)
            torch.cuda.synchronize()
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
            bad = (rows != truth).any(dim=1)
            assert int(bad.sum()) == 0, f"seed {seed}: {int(bad.sum())} series differ, first {torch.nonzero(bad)[:8].flatten().tolist()}"
            assert torch.equal(summ[:, 0], truth.sum(dim=1, dtype=torch.int64)), f"seed {seed}: counts"
            assert torch.equal(summ[:, 3], sums), f"seed {seed}: sums"
            # every field of every series' summary against the oracle's summary of the truth
            # rows (Metric.scala:53-67, l5do_summary_of_counts per row), bytewise
            _all_summaries_match_oracle(oracle, truth, sums, summ, f"seed {seed}")
            del truth, sums, bad
    finally:
        eng.close()
        del series, values, rows, summ
        torch.cuda.empty_cache()
