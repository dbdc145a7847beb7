"""bench.py's multi-rank harness on CPU: `--gpus N` spawns N ranks itself
(torch.distributed.run, gloo under --dry-run) and every rank derives its shard of
the BASELINE configs.  No GPU and no engine are involved (--dry-run)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _dry(*args):
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--dry-run", *args],
                       capture_output=True, text=True, timeout=240, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    return json.loads(line)


@pytest.mark.parametrize("gpus", [1, 2])
def test_c3_ranks_cover_the_series_space(gpus):
    d = _dry("--gpus", str(gpus))
    assert d["world"] == gpus and len(d["plans"]) == gpus
    plans = sorted(d["plans"], key=lambda p: p["rank"])
    assert plans[0]["first"] == 0
    for a, b in zip(plans, plans[1:]):
        assert b["first"] == a["first"] + a["count"]
        assert b["base_index"] == a["base_index"] + a["samples"]
    assert plans[-1]["first"] + plans[-1]["count"] == 1_000_000
    assert sum(p["samples"] for p in plans) == 1_000_000_000
    # equal modelled device time per rank (fleet.plan_shards over the expected tile load), within 3 %
    sys.path.insert(0, REPO)
    import bench
    from linkerd_amd import fleet, synth
    cdf = synth.zipf_cdf(1_000_000)
    load = bench.expected_tile_load(cdf, 1_000_000_000)
    shards = [fleet.Shard(p["rank"], p["first"], p["count"]) for p in plans]
    assert fleet.plan_spread(shards, load, 1_000_000, fleet.CostModel(**bench.C3_COST)) < 1.03


def test_c3_plan_is_load_derived_for_any_size():
    """One cost model for any (S, N): the plan comes from per-tile loads (no table tied
    to C3), and balances C3 and other sizes alike."""
    sys.path.insert(0, REPO)
    import bench
    import numpy as np
    from linkerd_amd import fleet, synth
    cost = fleet.CostModel(**bench.C3_COST)
    assert not [n for n in dir(bench) if n.startswith("COST_CALIBRATION")]
    for S, N, world in ((1_000_000, 1_000_000_000, 8), (1_000_000, 1_000_000_000, 4), (300_000, 200_000_000, 8),
                        (50_000, 10_000_000, 2)):
        cdf = synth.zipf_cdf(S)
        load = bench.expected_tile_load(cdf, N)
        sh = bench.shard_plan(S, N, world, cdf)
        assert sum(x.count for x in sh) == S and all(b.first == a.first + a.count for a, b in zip(sh, sh[1:]))
        assert fleet.plan_spread(sh, load, S, cost) < 1.03, (S, N, world)
    # a measured load (l5dh_tile_totals of the previous interval) plans the same way
    rng = np.random.default_rng(0)
    load = rng.poisson(bench.expected_tile_load(synth.zipf_cdf(100_000), 50_000_000)).astype(np.uint64)
    sh = fleet.plan_shards(load, 100_000, 4, cost)
    assert fleet.plan_spread(sh, load, 100_000, cost) < 1.03


def test_c4_ranks_split_the_samples():
    d = _dry("--gpus", "2", "--workload", "c4")
    plans = sorted(d["plans"], key=lambda p: p["rank"])
    assert all(p["count"] == 1_000_000 and p["first"] == 0 for p in plans)
    assert sum(p["samples"] for p in plans) == 1_000_000_000
    assert plans[1]["base_index"] == plans[0]["samples"]


def test_plan_keeps_the_last_partial_tiles_load():
    """with S % 32 != 0 the last tile's load is spread over its real series
    count (none of it dropped), and a zero-time rank gives an infinite spread rather
    than a ZeroDivisionError."""
    import numpy as np
    from linkerd_amd import fleet
    S = 32 * 10 + 7
    t = np.arange(1, 12, dtype=np.float64) * 1000.0
    cost = fleet.CostModel(per_sample=1e-6, per_series=1e-4, per_sample_fold=1e-6, fixed=0.0)
    per = fleet._per_series(t, S)
    assert per.size == S and abs(per.sum() - t.sum()) < 1e-6
    assert np.allclose(per[-7:], t[-1] / 7)
    shards = fleet.plan_shards(t, S, 3, cost)
    assert sum(x.count for x in shards) == S
    ms = fleet.plan_ms(shards, t, S, cost)
    assert abs(sum(ms) - sum(cost.range_ms(float(per[x.first:x.first + x.count].sum()), x.count)
                            for x in shards)) < 1e-9
    zero = fleet.CostModel(per_sample=0.0, per_series=0.0, per_sample_fold=0.0, fixed=0.0)
    assert fleet.plan_spread(shards, t, S, zero) == 1.0
    lopsided = [fleet.Shard(0, 0, 32), fleet.Shard(1, 32, S - 32), fleet.Shard(2, S, 0)]
    assert fleet.plan_spread(lopsided, t, S, cost) >= 1.0


def test_tile_features_choose_direct_tiles_as_rplan1():
    """fleet.tile_features restates k_rplan1's direct-tile rule (l5dh_ingest.hip): among
    the tiles with >= n / 8192 records, those at or above the smallest power of two that
    keeps <= 255 of them skip level 2; a big tile holds > 65535 records."""
    import numpy as np
    from linkerd_amd import fleet
    e = np.full(300, 2.0 ** 20)  # one power-of-two bucket holding > 255 tiles: none is direct
    n, l2, hot = fleet.tile_features(e)
    assert l2 == n == hot
    e = np.concatenate([np.full(10, 2.0 ** 21), np.full(300, 2.0 ** 16)])
    n, l2, hot = fleet.tile_features(e)
    assert l2 == 300 * 2.0 ** 16 and hot == n
    e = np.full(50, 60_000.0)  # few cold tiles: all direct, none big
    assert fleet.tile_features(e)[1:] == (0.0, 0.0)
    e = np.concatenate([np.full(5, 1e6), np.full(100, 10.0)])  # tiles below n / 8192 are never direct
    assert fleet.tile_features(e)[1] == 1000.0


def test_tiled_plan_minimizes_the_slowest_rank():
    """With the tiled model the plan's boundaries sit at tile boundaries and no single
    boundary moved by one tile lowers the slowest rank's modelled time."""
    sys.path.insert(0, REPO)
    import bench
    from linkerd_amd import fleet, synth
    S, N, world = 60_000, 50_000_000, 4
    cost = fleet.CostModel(**bench.C3_COST)
    assert cost.tiled
    load = bench.expected_tile_load(synth.zipf_cdf(S), N)
    sh = fleet.plan_shards(load, S, world, cost)
    assert sum(x.count for x in sh) == S
    worst = max(fleet.plan_ms(sh, load, S, cost))
    bounds = [x.first for x in sh] + [S]
    for r in range(1, world):
        for d in (-32, 32):
            b = list(bounds)
            b[r] += d
            if not (b[r - 1] <= b[r] <= b[r + 1]):
                continue
            alt = [fleet.Shard(k, b[k], b[k + 1] - b[k]) for k in range(world)]
            assert max(fleet.plan_ms(alt, load, S, cost)) >= worst * (1 - 1e-3)


def test_pmc_kernel_map_matches_the_committed_summary():
    """Every kernel that bench.load_pmc_traffic sums for a timed phase exists in the
    committed PMC summary of the default build (profiles/pmc_latest.json), so each
    priced phase of the bench line carries its measured traffic; the accumulate
    phase is the sum of its two side-by-side kernels and k_hot_finish (same timer)."""
    sys.path.insert(0, REPO)
    import bench
    path = os.path.join(REPO, "profiles", "pmc_latest.json")
    pm = json.load(open(path))
    ks = pm["kernels"]
    for phase, kernels in bench.PMC_KERNELS.items():
        for k in kernels:
            assert k in ks and "hbm_bytes_per_launch" in ks[k], f"{phase}: {k} not in {path}"
    assert set(bench.PMC_KERNELS["accum"]) == {"accum_cold_h", "accum_split", "hot_finish"}
    pl = {"workload": pm["workload"], "count": pm["series"], "samples": pm["samples"]}
    from linkerd_amd import _native
    real = _native.engine_source_hash
    try:
        _native.engine_source_hash = lambda: pm["src_hash"]  # (the committed summary's sources)
        out, note = bench.load_pmc_traffic(path, pl)
    finally:
        _native.engine_source_hash = real
    want = int(sum(ks[k]["hbm_bytes_per_launch"] for k in bench.PMC_KERNELS["accum"]))
    assert out["accum"] == want and set(out) == set(bench.PMC_KERNELS), (out, note)
