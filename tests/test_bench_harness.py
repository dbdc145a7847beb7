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
    w = bench.shard_cost(synth.zipf_cdf(1_000_000), 1_000_000_000)
    cost = [w[p["first"]:p["first"] + p["count"]].sum() for p in plans]
    assert max(cost) / min(cost) < 1.02


def test_c4_ranks_split_the_samples():
    d = _dry("--gpus", "2", "--workload", "c4")
    plans = sorted(d["plans"], key=lambda p: p["rank"])
    assert all(p["count"] == 1_000_000 and p["first"] == 0 for p in plans)
    assert sum(p["samples"] for p in plans) == 1_000_000_000
    assert plans[1]["base_index"] == plans[0]["samples"]
