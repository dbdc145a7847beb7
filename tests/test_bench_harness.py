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
    # equal modelled device time per rank (bench.shard_cost), within 2 %
    sys.path.insert(0, REPO)
    import bench
    from linkerd_amd import synth
    w = bench.shard_cost(synth.zipf_cdf(1_000_000), 1_000_000_000, gpus)
    cost = [w[p["first"]:p["first"] + p["count"]].sum() for p in plans]
    assert max(cost) / min(cost) < 1.02


def test_c3_eight_way_plan_pins_the_folded_first_tile():
    """8 ranks: rank 0 holds exactly the first tile (one tile is folded at ingest,
    k_fold1), the other 7 split the rest with equal modelled device time; 2 and 4
    ranks keep a partitioned head shard."""
    sys.path.insert(0, REPO)
    import bench
    from linkerd_amd import synth
    cdf = synth.zipf_cdf(1_000_000)
    sh = bench.shard_plan(1_000_000, 1_000_000_000, 8, cdf)
    assert (sh[0].first, sh[0].count) == (0, bench.ONE_TILE)
    assert sum(x.count for x in sh) == 1_000_000 and all(b.first == a.first + a.count for a, b in zip(sh, sh[1:]))
    w = bench.shard_cost(cdf, 1_000_000_000, 8)
    cost = [w[x.first:x.first + x.count].sum() for x in sh[1:]]
    assert max(cost) / min(cost) < 1.02
    assert bench.COST_FIRST_TILE_FOLDED < min(cost)
    for world in (2, 4):
        assert bench.shard_plan(1_000_000, 1_000_000_000, world, cdf)[0].count > bench.ONE_TILE


def test_c4_ranks_split_the_samples():
    d = _dry("--gpus", "2", "--workload", "c4")
    plans = sorted(d["plans"], key=lambda p: p["rank"])
    assert all(p["count"] == 1_000_000 and p["first"] == 0 for p in plans)
    assert sum(p["samples"] for p in plans) == 1_000_000_000
    assert plans[1]["base_index"] == plans[0]["samples"]
