"""Refit bench.py's C3 shard cost model (fleet.CostModel) to measured single-GPU lines:
the shards of a sweep (tools/shard_sweep.sh) and whole-workload C3 / C2 / C1 lines.
  python tools/fit_cost.py gpurun_out/sw_<tag> [more dirs or bench .json files ...]
Each line's features come from its workload's expected per-tile load (a shard: its own
range, tiled from its first series): samples, samples outside the direct tiles,
samples in big tiles, series (fleet.tile_features).  Prints the least-squares
constants (ranges of one tile set per_sample_fold), each line's measured vs modelled
time, and the measured spread of the sweep."""
import glob
import json
import os
import re
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def lines(paths):
    for p in paths:
        files = sorted(glob.glob(os.path.join(p, "*.json"))) if os.path.isdir(p) else [p]
        for f in files:
            try:
                d = json.loads(open(f).read().strip().splitlines()[-1])
            except (OSError, ValueError, IndexError):
                continue
            c = d.get("config", {})
            if "series_per_gpu" in c and "samples_per_gpu_per_step" in c:
                yield f, c, d["ms_per_step"]


def features(c):
    """(samples, level-2 samples, big-tile samples, series) of a bench line."""
    import bench
    from linkerd_amd import fleet, synth
    S, n = int(c["series_per_gpu"]), float(c["samples_per_gpu_per_step"])
    wl = c.get("workload", "")
    if wl.startswith("C2"):
        per = np.full(S, n / S)
        tiles = fleet._range_tiles(per, 0, S)
    elif wl.startswith("C3"):
        St = int(c.get("series_total", S))
        Nt = float(c.get("samples_per_step", n))
        per = fleet._per_series(bench.expected_tile_load(synth.zipf_cdf(St), Nt), St)
        first = 0
        m = re.search(r"series \[(\d+), (\d+)\)", c.get("shard", ""))
        if m:
            first = int(m.group(1))
        tiles = fleet._range_tiles(per, first, S) * (n / max(per[first:first + S].sum(), 1.0))
    else:  # one series: the fold
        tiles = np.array([n])
    tot, l2, hot = fleet.tile_features(tiles)
    return n, l2, hot, S


def main():
    rows = [(f, c, ms, features(c)) for f, c, ms in lines(sys.argv[1:])]
    if not rows:
        sys.exit("no bench lines found")
    big = [(x, ms) for _, _, ms, x in rows if x[3] > 32]
    A = np.array([[1.0, n, l2, hot, S] for (n, l2, hot, S), _ in big])
    y = np.array([ms for _, ms in big])
    (fixed, a, b, h, c), *_ = np.linalg.lstsq(A, y, rcond=None)
    fold = [(x, ms) for _, _, ms, x in rows if x[3] <= 32]  # folded ranges: their own fixed cost
    if len(fold) >= 2:
        (fixed_fold, per_fold), *_ = np.linalg.lstsq(np.array([[1.0, n] for (n, _, _, _), _ in fold]),
                                                     np.array([ms for _, ms in fold]), rcond=None)
    else:
        fixed_fold, per_fold = fixed, a
    print("C3_COST = dict(per_sample=%.3g, per_series=%.3g, per_sample_fold=%.3g, fixed=%.3g, per_sample_l2=%.3g, "
          "per_sample_hot=%.3g, fixed_fold=%.3g)" % (a, c, per_fold, fixed, b, h, fixed_fold))
    for f, _, ms, (n, l2, hot, S) in rows:
        m = (fixed_fold + per_fold * n) if S <= 32 else fixed + c * S + a * n + b * l2 + h * hot
        print(f"  {os.path.basename(f):12s} S={S:8d} n={n:11.0f} l2={l2:11.0f} hot={hot:11.0f} measured {ms:7.3f} ms"
              f"  model {m:7.3f} ms  ({(m / ms - 1) * 100:+.1f} %)")
    shards = [ms for f, _, ms, _ in rows if os.path.basename(f).startswith("s")]
    if shards:
        print(f"measured shard spread (max / min): {max(shards) / min(shards):.3f}; slowest {max(shards):.3f} ms")


if __name__ == "__main__":
    main()
