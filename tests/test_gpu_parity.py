"""GPU parity: the HIP engine (through the C-ABI) against the CPU oracle.

Bucket counts, count/sum/min/max/percentiles are compared bit-exactly; avg is
compared bit-exactly as well (sum and count are exact integers on both sides, so
IEEE division gives the same double; BASELINE allows 1e-12 relative).
"""
import numpy as np
import pytest

from linkerd_amd import synth
from linkerd_amd import _native as N

pytestmark = pytest.mark.gpu

EDGE_VALUES = np.array([
    0.0, 0.25, 0.5, 0.999, 1.0, 1.5, 2.0, 99.9, 100.0, 112.0, 112.99, 113.0, 114.0, 115.0, 116.5,
    3030.0, 2323.0, 65535.0, 65536.0, 1e6, 6.5e6, 1.3e7, 1e9, 2137204090.0, 2137204091.0,
    2147483520.0, 2147483648.0, 3e9, 1e20, np.inf,
    -0.0, -0.5, -1.0, -113.0, -3e9, -5e9, -1e19, -np.inf, np.nan,
], dtype=np.float32)


# Partition regimes: region capacities as predicted; regions at 40 % of the
# prediction (every batch overflows and is redone with exact regions); no direct
# tiles (every record through level 2).
REGIME_PARAMS = {"default": {}, "redo": {N.PARAM_REGION_PCT: 40}, "nodirect": {N.PARAM_DIRECT_MAX: 0}}


def _engine(S, regime="default", stage=0):
    """stage=0: every ingest call is binned at once (one segment per call), so the
    multi-segment paths stay covered; stage=None keeps the default ring."""
    from linkerd_amd.engine import HistogramEngine
    e = HistogramEngine(S)
    for k, v in REGIME_PARAMS[regime].items():
        e.set_param(k, v)
    if stage is not None:
        e.set_param(N.PARAM_STAGE_SAMPLES, stage)
    return e


BIN_MODES = pytest.mark.parametrize("bin_mode", ["default", "redo", "nodirect"])
TWO_LEVEL = pytest.mark.parametrize("mode", ["default", "redo"])


def _assert_summaries_equal(got, want, label=""):
    for f in N.SUMMARY_FIELDS:
        g, w = got[f], want[f]
        if f == "avg":
            bad = ~((g == w) | (np.isnan(g) & np.isnan(w)))
        else:
            bad = g != w
        if bad.any():
            i = int(np.flatnonzero(bad)[0])
            raise AssertionError(f"{label} field {f}: {int(bad.sum())} mismatches; first series {i}: "
                                 f"got {g[i]!r} want {w[i]!r}\n got={got[i]}\nwant={want[i]}")


def _random_batch(rng, S, n, edge_frac=0.01):
    series = rng.integers(0, S, size=n, dtype=np.uint32)
    mu = np.log(rng.uniform(1, 1000, size=S))
    vals = np.exp(mu[series] + 0.8 * rng.standard_normal(n)).astype(np.float32)
    k = int(n * edge_frac)
    if k:
        pos = rng.choice(n, size=k, replace=False)
        vals[pos] = rng.choice(EDGE_VALUES, size=k)
    return series, vals


def test_limits_match_oracle(oracle):
    np.testing.assert_array_equal(N.limits(), oracle.limits())


@BIN_MODES
def test_small_random_bitexact(oracle, bin_mode):
    rng = np.random.default_rng(11)
    S, n = 1000, 300_000
    series, vals = _random_batch(rng, S, n)
    eng = _engine(S, bin_mode)
    eng.ingest(series, vals)
    got, counts = eng.snapshot(reset=True, with_counts=True)
    o = oracle.OracleHistograms(S)
    o.ingest(series, vals)
    np.testing.assert_array_equal(counts, o.counts())
    want = o.snapshot(reset=True)
    _assert_summaries_equal(got, want, "small")
    # after reset everything is empty
    got2 = eng.snapshot(reset=True)
    assert (got2["count"] == 0).all() and (got2["sum"] == 0).all() and (got2["avg"] == 0).all()


@BIN_MODES
def test_edge_values_every_series(oracle, bin_mode):
    S = 70  # not a multiple of the 32-series tile
    series = np.repeat(np.arange(S, dtype=np.uint32), EDGE_VALUES.size)
    vals = np.tile(EDGE_VALUES, S)
    rng = np.random.default_rng(3)
    perm = rng.permutation(series.size)
    series, vals = series[perm], vals[perm]
    eng = _engine(S, bin_mode)
    eng.ingest(series, vals)
    got, counts = eng.snapshot(with_counts=True)
    o = oracle.OracleHistograms(S)
    o.ingest(series, vals)
    np.testing.assert_array_equal(counts, o.counts())
    _assert_summaries_equal(got, o.snapshot(), "edge")


@TWO_LEVEL
@pytest.mark.parametrize("stage", [0, None, 50_000], ids=["unstaged", "ring", "smallring"])
@pytest.mark.parametrize("reset", [False, True])
def test_multi_batch_and_cumulative_snapshots(oracle, reset, stage, mode):
    """Several ingests (segments + folds, or the staging ring flushed when full and
    at the snapshot) and snapshots with / without reset (Prometheus P2 is
    cumulative: snapshot() without reset, PrometheusTelemeterTest.scala:70-86)."""
    rng = np.random.default_rng(5 + reset)
    S = 333
    eng = _engine(S, mode, stage=stage)
    eng.set_param(N.PARAM_MAX_SEGMENTS, 2)
    o = oracle.OracleHistograms(S)
    for it in range(3):
        for b in range(3):
            series, vals = _random_batch(rng, S, int(rng.integers(1, 20000)))
            eng.ingest(series, vals)
            o.ingest(series, vals)
        got, counts = eng.snapshot(reset=reset, with_counts=True)
        np.testing.assert_array_equal(counts, o.counts(), err_msg=f"iter {it}")
        _assert_summaries_equal(got, o.snapshot(reset=reset), f"iter {it}")


@BIN_MODES
def test_hot_tile_split_path(oracle, bin_mode):
    """Big tiles (> cold_limit records): (chunk, half-tile) items with u32 LDS bins;
    single-chunk tiles emit in place, bigger ones flush with global atomics and are
    summarized by k_hot_finish."""
    rng = np.random.default_rng(9)
    S = 100
    eng = _engine(S, bin_mode)
    eng.set_param(N.PARAM_COLD_LIMIT, 500)
    eng.set_param(N.PARAM_HOT_CHUNK, 20000)
    o = oracle.OracleHistograms(S)
    # series 0..3 (tile 0) hot: 3+ chunks; tiles 1..3 warm; a few cold-ish
    series = np.concatenate([rng.integers(0, 4, 200_000), rng.integers(32, S, 20_000)]).astype(np.uint32)
    vals = np.exp(3 + rng.standard_normal(series.size)).astype(np.float32)
    vals[::97] = rng.choice(EDGE_VALUES, size=vals[::97].size)
    eng.ingest(series, vals)
    o.ingest(series, vals)
    got, counts = eng.snapshot(reset=False, with_counts=True)
    np.testing.assert_array_equal(counts, o.counts())
    _assert_summaries_equal(got, o.snapshot(reset=False), "hot1")
    # second round on top of dirty state, then reset
    eng.ingest(series[:150_000], vals[:150_000])
    o.ingest(series[:150_000], vals[:150_000])
    got, counts = eng.snapshot(reset=True, with_counts=True)
    np.testing.assert_array_equal(counts, o.counts())
    _assert_summaries_equal(got, o.snapshot(reset=True), "hot2")
    # and a fold (range snapshot) through the hot path
    eng.ingest(series, vals)
    o.ingest(series, vals)
    got = eng.snapshot(first=0, count=40, reset=True)
    _assert_summaries_equal(got, o.snapshot(reset=False)[:40], "hot fold")


@TWO_LEVEL
@pytest.mark.parametrize("direct_max", [0, 2, 255])
def test_split_tiles_across_batches(oracle, direct_max, mode):
    """Hot sets that move between batches: a tile is direct (level-1 records) in some
    pending segments and level-2 (16-bit records) in others; big tiles are
    accumulated per half across all of them."""
    rng = np.random.default_rng(21 + direct_max)
    S = 4000
    eng = _engine(S, mode)
    eng.set_param(N.PARAM_COLD_LIMIT, 500)
    eng.set_param(N.PARAM_HOT_CHUNK, 5000)
    eng.set_param(N.PARAM_MAX_SEGMENTS, 3)
    eng.set_param(N.PARAM_DIRECT_MAX, direct_max)
    o = oracle.OracleHistograms(S)

    def batch(hot_lo, hot_hi, n_hot, n_cold):
        series = np.concatenate([rng.integers(hot_lo, hot_hi, n_hot), rng.integers(0, S, n_cold)]).astype(np.uint32)
        rng.shuffle(series)
        vals = np.exp(2 + 1.5 * rng.standard_normal(series.size)).astype(np.float32)
        vals[::89] = rng.choice(EDGE_VALUES, size=vals[::89].size)
        return series, vals

    plan = [[(0, 64, 30_000, 5_000)], [(32, 100, 40_000, 8_000), (0, 20, 12_000, 1_000)],
            [(0, 64, 25_000, 3_000), (0, 64, 25_000, 3_000), (2000, 2400, 60_000, 2_000)],
            [(3000, 3040, 9_000, 500)]]
    for it, batches in enumerate(plan):
        for b in batches:
            series, vals = batch(*b)
            eng.ingest(series, vals)
            o.ingest(series, vals)
        reset = it % 2 == 1
        got, counts = eng.snapshot(reset=reset, with_counts=True)
        np.testing.assert_array_equal(counts, o.counts(), err_msg=f"snapshot {it}")
        _assert_summaries_equal(got, o.snapshot(reset=reset), f"split {it}")


@pytest.mark.parametrize("value", [5.0, 2_000_000.0])
@TWO_LEVEL
def test_split_bins_one_bucket(oracle, value, mode):
    """A big half-tile whose 300k records per batch all fall in ONE bucket: one LDS
    bin of a 2^18-record item reaches 2^18 (u32 bins), the dense state row
    accumulates across batches.  At 2e6 (the largest payloads below the escape) one
    lane's value-sum slot of an item takes 4096 x 2e6 > 2^32 (u64 slots)."""
    rng = np.random.default_rng(5)
    S = 64
    eng = _engine(S, mode)
    o = oracle.OracleHistograms(S)
    for it in range(3):
        series = np.concatenate([np.zeros(300_000, np.uint32), rng.integers(0, S, 20_000).astype(np.uint32)])
        vals = np.concatenate([np.full(300_000, value, np.float32),
                               np.exp(2 + rng.standard_normal(20_000)).astype(np.float32)])
        perm = rng.permutation(series.size)
        eng.ingest(series[perm], vals[perm])
        o.ingest(series[perm], vals[perm])
        got, counts = eng.snapshot(reset=it == 1, with_counts=True)
        np.testing.assert_array_equal(counts, o.counts(), err_msg=f"batch {it}")
        _assert_summaries_equal(got, o.snapshot(reset=it == 1), f"capacity {it}")


@TWO_LEVEL
def test_unsplit_direct_tiles(oracle, mode):
    """Direct tiles come from THIS batch's sample: a hot set the previous batch did
    not have is binned straight into its half-tile regions by level 1, and the
    regions sized from the previous batch's counts are too small for it where the
    sample estimate is low (level-1 redo)."""
    rng = np.random.default_rng(31)
    S = 5000
    eng = _engine(S, mode)
    o = oracle.OracleHistograms(S)
    for it, (lo, hi) in enumerate([(0, 0), (320, 448), (3000, 3007), (320, 448)]):
        n_hot = 0 if hi == lo else 1_200_000
        series = np.concatenate([rng.integers(lo, max(hi, lo + 1), n_hot), rng.integers(0, S, 800_000)]).astype(np.uint32)
        rng.shuffle(series)
        vals = np.exp(3 + rng.standard_normal(series.size)).astype(np.float32)
        vals[::101] = rng.choice(EDGE_VALUES, size=vals[::101].size)
        eng.ingest(series, vals)
        o.ingest(series, vals)
        reset = it != 1
        got, counts = eng.snapshot(reset=reset, with_counts=True)
        np.testing.assert_array_equal(counts, o.counts(), err_msg=f"batch {it}")
        _assert_summaries_equal(got, o.snapshot(reset=reset), f"unsplit direct {it}")


@BIN_MODES
def test_reset_snapshot_mixed_clean_dirty_big_tiles(oracle, bin_mode):
    """A resetting full snapshot with dense counts counts the big tiles that were
    clean at the plan straight into the output rows and copies the dirty ones from
    state: tile A (series 0-31) big and clean (a range snapshot reset it), tile B
    (320-351) big and dirty (folded by that range snapshot), tile C (640-671) big
    and clean, several items each, cold tiles everywhere."""
    rng = np.random.default_rng(41)
    S = 2000
    eng = _engine(S, bin_mode)
    eng.set_param(N.PARAM_COLD_LIMIT, 500)
    eng.set_param(N.PARAM_HOT_CHUNK, 5000)
    o = oracle.OracleHistograms(S)

    def batch(hot, n_hot, n_cold):
        parts = [rng.integers(lo, lo + 32, n_hot) for lo in hot] + [rng.integers(0, S, n_cold)]
        series = np.concatenate(parts).astype(np.uint32)
        rng.shuffle(series)
        vals = np.exp(3 + 1.2 * rng.standard_normal(series.size)).astype(np.float32)
        vals[::97] = rng.choice(EDGE_VALUES, size=vals[::97].size)
        return series, vals

    s0, v0 = batch([0, 320], 30_000, 5_000)
    eng.ingest(s0, v0)
    o.ingest(s0, v0)
    got, counts = eng.snapshot(reset=True, with_counts=True)
    np.testing.assert_array_equal(counts, o.counts(), err_msg="b0")
    _assert_summaries_equal(got, o.snapshot(reset=True), "b0")
    s1, v1 = batch([0, 320], 20_000, 4_000)
    eng.ingest(s1, v1)
    a = s1 < 32
    oa = oracle.OracleHistograms(32)
    oa.ingest(s1[a], v1[a])
    o.ingest(s1[~a], v1[~a])
    _assert_summaries_equal(eng.snapshot(first=0, count=32, reset=True), oa.snapshot(reset=True), "range A")
    s2, v2 = batch([0, 320, 640], 25_000, 6_000)
    eng.ingest(s2, v2)
    o.ingest(s2, v2)
    got, counts = eng.snapshot(reset=True, with_counts=True)
    np.testing.assert_array_equal(counts, o.counts(), err_msg="b2")
    _assert_summaries_equal(got, o.snapshot(reset=True), "b2")
    s3, v3 = batch([640], 15_000, 3_000)  # after the reset: every tile clean again
    eng.ingest(s3, v3)
    o.ingest(s3, v3)
    got, counts = eng.snapshot(reset=True, with_counts=True)
    np.testing.assert_array_equal(counts, o.counts(), err_msg="b3")
    _assert_summaries_equal(got, o.snapshot(reset=True), "b3")


@TWO_LEVEL
def test_big_tile_bins_past_u16(oracle, mode):
    """One series with 70k-300k records of one value per batch: one u32 bin of a
    big half-tile item far past 2^16; a clean and a dirty tile, and a hot set that
    moves between batches."""
    rng = np.random.default_rng(17)
    S = 100
    eng = _engine(S, mode)
    o = oracle.OracleHistograms(S)
    plan = [(0, 7.0, 300_000, False), (40, 1_000_000.0, 200_000, False), (0, 113.0, 70_000, True),
            (70, 2_000_000.0, 280_000, True)]
    for it, (sid, value, n, reset) in enumerate(plan):
        series = np.concatenate([np.full(n, sid, np.uint32), rng.integers(0, S, 20_000).astype(np.uint32)])
        vals = np.concatenate([np.full(n, value, np.float32), np.exp(2 + rng.standard_normal(20_000)).astype(np.float32)])
        perm = rng.permutation(series.size)
        eng.ingest(series[perm], vals[perm])
        o.ingest(series[perm], vals[perm])
        got, counts = eng.snapshot(reset=reset, with_counts=True)
        np.testing.assert_array_equal(counts, o.counts(), err_msg=f"batch {it}")
        _assert_summaries_equal(got, o.snapshot(reset=reset), f"big tile {it}")


@TWO_LEVEL
@pytest.mark.parametrize("S", [500, 20], ids=["tiles", "one_tile"])
def test_range_snapshot_peek_export(oracle, mode, S):
    """Range snapshot (with its reset), peek, state export and summarize_dense against the
    oracle; the one-tile space folds every batch into its state rows at ingest, escaped
    samples' sums included (1 % edge values: negative, NaN, beyond 2^21)."""
    rng = np.random.default_rng(21)
    series, vals = _random_batch(rng, S, 100_000)
    eng = _engine(S, mode)
    eng.ingest(series, vals)
    o = oracle.OracleHistograms(S)
    o.ingest(series, vals)
    want_all = o.snapshot(reset=False)
    a, b = (100, 150) if S > 100 else (3, 10)
    got = eng.snapshot(first=a, count=b - a, reset=True)
    _assert_summaries_equal(got, want_all[a:b], "range")
    # reset only that range
    got_all = eng.snapshot(reset=False)
    want_after = want_all.copy()
    want_after[a:b] = np.zeros(b - a, dtype=want_after.dtype)
    _assert_summaries_equal(got_all, want_after, "after range reset")
    # peek == bucketAndCounts of the oracle
    L = oracle.limits()
    for s in (0, a - 1, S - 1):  # (outside the reset range)
        pk = eng.peek(s)
        c = o.counts()[s]
        nz = np.flatnonzero(c > 0)
        assert pk.size == nz.size
        np.testing.assert_array_equal(pk["count"], c[nz])
        np.testing.assert_array_equal(pk["lower"], np.where(nz == 0, 0, L[np.maximum(nz - 1, 0)]))
        np.testing.assert_array_equal(pk["upper"], np.where(nz < 1797, L[np.minimum(nz, 1796)], 2147483647))
    counts, totals = eng.export_state()
    want_counts = o.counts()
    want_counts[a:b] = 0
    np.testing.assert_array_equal(counts, want_counts)
    want_tot = o.totals()
    want_tot[a:b] = 0
    np.testing.assert_array_equal(totals, want_tot)
    summ = eng.summarize_dense(counts, totals)
    _assert_summaries_equal(summ, want_after, "summarize_dense")


@TWO_LEVEL
def test_invalid_series_reported(oracle, mode):
    S = 64
    eng = _engine(S, mode)
    series = np.array([1, 2, 64, 3, 1000], dtype=np.uint32)
    vals = np.array([1, 2, 3, 4, 5], dtype=np.float32)
    eng.ingest(series, vals)  # accepted: the invalid ids are found by the kernels
    with pytest.raises(N.L5dhError, match="EINVAL"):  # and reported by sync
        eng.sync()
    eng.sync()  # reported once
    got = eng.snapshot()
    o = oracle.OracleHistograms(S)
    o.ingest(series[[0, 1, 3]], vals[[0, 1, 3]])
    _assert_summaries_equal(got, o.snapshot(), "invalid dropped")


@pytest.mark.parametrize("stage", [0, None], ids=["unstaged", "ring"])
@pytest.mark.parametrize("variant", [0, 1], ids=["fold1", "fold1_u16"])
@pytest.mark.parametrize("S", [1, 9, 32])
def test_one_tile_series_space(oracle, S, variant, stage):
    """S <= 32 (one tile): each batch is folded into the tile's state rows at ingest
    (k_fold1: u32 bins up to 16 series, else -- and with variant bit 0 -- the u16 bins
    with the 2^15 hand-off).  Invalid ids are dropped and reported, edge values
    escape, a cold batch and hot multi-item batches, snapshots with and without reset."""
    rng = np.random.default_rng(60 + S)
    eng = _engine(S, stage=stage)
    eng.set_param(N.PARAM_VARIANT, variant)
    o = oracle.OracleHistograms(S)
    bad = np.array([S, S + 7, 0xFFFFFFFF], dtype=np.uint32)
    eng.ingest(bad, np.ones(3, np.float32))
    with pytest.raises(N.L5dhError):
        eng.sync()
    eng.sync()
    eng.set_param(N.PARAM_HOT_CHUNK, 100_000)  # several items per batch, a ragged last one
    for it, n in enumerate([1, 3_000, 400_001, 1_500_000, 262_147]):
        series = rng.integers(0, S, n).astype(np.uint32)
        vals = np.exp(3 + 1.5 * rng.standard_normal(n)).astype(np.float32)
        vals[::53] = rng.choice(EDGE_VALUES, size=vals[::53].size)
        eng.ingest(series, vals)
        o.ingest(series, vals)
        reset = it % 2 == 1
        got, counts = eng.snapshot(reset=reset, with_counts=True)
        np.testing.assert_array_equal(counts, o.counts(), err_msg=f"batch {it}")
        _assert_summaries_equal(got, o.snapshot(reset=reset), f"one tile {it}")


@BIN_MODES
def test_c2_slice_bitexact(oracle, bin_mode):
    """C2 recipe at 1/10 of the series: 10k series x 1k samples."""
    series, vals = synth.c2(S=10_000, K=1_000)
    eng = _engine(10_000, bin_mode)
    eng.ingest(series, vals)
    got, counts = eng.snapshot(with_counts=True)
    o = oracle.OracleHistograms(10_000)
    o.ingest(series, vals, threads=8)
    np.testing.assert_array_equal(counts, o.counts())
    _assert_summaries_equal(got, o.snapshot(), "c2 slice")


@TWO_LEVEL
def test_device_buffers_in_and_out(oracle, mode):
    import torch
    rng = np.random.default_rng(4)
    S = 2000
    series, vals = _random_batch(rng, S, 500_000)
    eng = _engine(S, mode)
    ds = torch.from_numpy(series.view(np.int32)).cuda()
    dv = torch.from_numpy(vals).cuda()
    eng.ingest(ds, dv)
    summ = torch.zeros(S * 11, dtype=torch.int64, device="cuda")
    cnt = torch.zeros((S, 1798), dtype=torch.int32, device="cuda")
    eng.snapshot_into(summ, cnt)
    torch.cuda.synchronize()
    got = summ.cpu().numpy().view(N.SUMMARY_DTYPE)
    o = oracle.OracleHistograms(S)
    o.ingest(series, vals)
    np.testing.assert_array_equal(cnt.cpu().numpy(), o.counts())
    _assert_summaries_equal(got, o.snapshot(), "device io")


@pytest.mark.parametrize("name", ["mixed64", "c1_100k", "c2_200x500", "c3_zipf1000"])
def test_golden_vectors(name):
    """Committed golden fixtures (tests/golden/make_golden.py) reproduced on the GPU."""
    import os
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", f"golden_{name}.npz"))
    S = int(g["nseries"])
    eng = _engine(S)
    eng.ingest(g["series"], g["values"])
    got, counts = eng.snapshot(with_counts=True)
    np.testing.assert_array_equal(counts, g["counts"])
    assert got.view(np.uint8).reshape(S, 88).tobytes() == g["summaries"].tobytes()


@BIN_MODES
def test_zipf_series_space_1m(oracle, bin_mode):
    """1M-series engine (F = 32768 tiles, 512 super-tiles) on a Zipf C3 slice."""
    S = 1_000_000
    series, vals = synth.c3(S=S, N=2_000_000)
    eng = _engine(S, bin_mode)
    eng.ingest(series, vals)
    got, counts = eng.snapshot(with_counts=True)
    o = oracle.OracleHistograms(S)
    o.ingest(series, vals, threads=8)
    want_counts = o.counts()
    want = o.snapshot()
    _assert_summaries_equal(got, want, "zipf 1M")
    touched = np.unique(series)
    np.testing.assert_array_equal(counts[touched], want_counts[touched])
    assert counts.sum() == series.size


@TWO_LEVEL
@pytest.mark.parametrize("gmax", [1, 3, 7, 512])
def test_slab_counts_bitexact(oracle, gmax, mode):
    """Ingest with G = min(max_slabs, n / 8192) slabs (default: one per CU): the
    level-1 run reservations must place every record exactly for any slab count,
    including one slab and odd counts.  Two Zipf batches (direct tiles; the second
    sized from the first's counts)."""
    rng = np.random.default_rng(100 + gmax)
    S, n = 5000, 1_500_000
    eng = _engine(S, mode)
    eng.set_param(N.PARAM_MAX_SLABS, gmax)
    o = oracle.OracleHistograms(S)
    for _ in range(2):
        series = ((rng.zipf(1.2, size=n) - 1) % S).astype(np.uint32)
        vals = np.exp(np.log(20.0) + rng.standard_normal(n)).astype(np.float32)
        eng.ingest(series, vals)
        o.ingest(series, vals)
    got, counts = eng.snapshot(reset=True, with_counts=True)
    np.testing.assert_array_equal(counts, o.counts())
    _assert_summaries_equal(got, o.snapshot(reset=True), f"gmax={gmax}")


@pytest.mark.parametrize("regime", ["default", "redo", "nodirect"])
def test_tile_totals_are_the_batch_load(regime):
    """l5dh_tile_totals (the load-derived shard plan's input) = records per 32-series
    tile of the last binned batch, exactly: invalid ids excluded, direct and level-2
    tiles alike, after a redo too."""
    rng = np.random.default_rng(11)
    S = 70_001
    F = (S + 31) // 32
    s, _ = synth.c3(S=S, N=2_000_000, seed=5)
    s = s.copy()
    s[:1000] = S + 7  # invalid ids: dropped, not counted
    v = rng.uniform(0, 5000, s.size).astype(np.float32)
    e = _engine(S, regime)
    try:
        for k in range(2):  # the second batch plans from the first's exact counts
            try:
                e.ingest(s, v)
            except Exception:
                pass  # the invalid ids are reported (the valid samples are ingested)
            want = np.bincount(s[s < S] // 32, minlength=F).astype(np.uint64)
            np.testing.assert_array_equal(e.tile_totals(), want)
    finally:
        e.close()


@pytest.mark.parametrize("n", [60_000, 150_000])
def test_direct_run_delta_at_region_start(oracle, n):
    """A direct half-bin whose region starts at rec16 index 0 while its run sits at
    stage offset 1 (one super-tile record before it) has the run delta 0 - 1 =
    0xFFFFFFFF: it must not read as a dropped run.  All tiles but the last are direct
    (S = 4001: tile 125 holds one series), one slab."""
    from linkerd_amd.engine import HistogramEngine
    S = 4001
    series, vals = synth.c3(S=S, N=2 * n, seed=74)
    s, v = series[0::2], vals[0::2]
    eng = HistogramEngine(S)
    try:
        eng.set_param(N.PARAM_MAX_SLABS, 1)
        eng.ingest(s, v)
        counts, totals = eng.export_state(reset=True)
        o = oracle.OracleHistograms(S)
        o.ingest(s, v)
        np.testing.assert_array_equal(counts, o.counts())
        np.testing.assert_array_equal(totals, o.totals())
    finally:
        eng.close()


def test_moving_load_counts_level2_first(oracle):
    """A first interval and a hot set that moves (C3's Zipf head rotated by a third of
    the series space between batches, as bench.py --hot-shift does): no level-1 redo
    (rcap's two-sided consistency test sizes a bin that lost its load from the
    sample, so the plan fits the buffer), and level 2 counts its keys first instead
    of writing a pass that overflows and is redone (k_rfix1 sees the super-tiles
    outgrow their previous loads); a steady batch of the same load does neither.
    Counts and summaries exact throughout."""
    S, n = 300_000, 3_000_000
    eng = _engine(S)
    o = oracle.OracleHistograms(S)
    hist = []
    for seed, shift in [(1, 0), (2, 0), (3, S // 3), (4, 2 * S // 3)]:
        s, v = synth.c3(S=S, N=n, seed=seed)
        s = ((s.astype(np.int64) + shift) % S).astype(np.uint32)
        eng.ingest(s, v)
        o.ingest(s, v, threads=8)
        hist.append(eng.partition_redos())
    got, counts = eng.snapshot(reset=True, with_counts=True)
    np.testing.assert_array_equal(counts, o.counts())
    _assert_summaries_equal(got, o.snapshot(reset=True), "moving load")
    # (level-1 redos, level-2 redos, level-2 counting first passes) after each batch
    assert hist == [(0, 0, 1), (0, 0, 1), (0, 0, 2), (0, 0, 3)], hist


def test_sparse_key_space_steady_state(oracle):
    """A sparse series space (1M series, each batch's 4M samples on 6000 of its 62.5 K
    keys, the others never seen): after the first interval, steady batches take no redo and no
    counting pass -- a never-sampled key's region stays small (4 samples per draw, round
    5's bound), so the plan of ~60 K empty keys does not outgrow the buffer."""
    rng = np.random.default_rng(77)
    S, n = 1_000_000, 4_000_000
    keys = rng.choice(S // 16, 6000, replace=False)  # the other ~56 K keys are never seen
    eng = _engine(S)
    o = oracle.OracleHistograms(S)
    hist = []
    for it in range(3):
        series = (keys[rng.integers(0, keys.size, n)] * 16 + rng.integers(0, 16, n)).astype(np.uint32)
        vals = np.exp(3 + rng.standard_normal(n)).astype(np.float32)
        eng.ingest(series, vals)
        o.ingest(series, vals, threads=8)
        hist.append(eng.partition_redos())
    got, counts = eng.snapshot(reset=True, with_counts=True)
    np.testing.assert_array_equal(counts.sum(), 3 * n)
    _assert_summaries_equal(got, o.snapshot(reset=True), "sparse")
    assert hist[2][:3] == hist[0][:3], hist  # (batches 2 and 3: nothing redone or counted)
