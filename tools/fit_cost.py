"""Refit bench.py's C3 shard cost model (fleet.CostModel) to measured single-GPU lines:
the shards of a sweep (tools/shard_sweep.sh) and optionally whole-workload lines.
  python tools/fit_cost.py gpurun_out/sw_<tag> [more dirs or bench .json files ...]
Prints the least-squares constants (ms = fixed + per_sample n + per_series S for ranges
of more than one tile; the one-tile fold range sets per_sample_fold), each line's
measured vs modelled time, and the plan's modelled spread with the refitted model."""
import glob
import json
import os
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
                yield f, c["series_per_gpu"], c["samples_per_gpu_per_step"], d["ms_per_step"]


def main():
    rows = list(lines(sys.argv[1:]))
    if not rows:
        sys.exit("no bench lines found")
    big = [(S, n, ms) for _, S, n, ms in rows if S > 32]
    A = np.array([[1.0, n, S] for S, n, _ in big])
    y = np.array([ms for _, _, ms in big])
    (fixed, per_sample_ms, per_series_ms), *_ = np.linalg.lstsq(A, y, rcond=None)
    fold = [(S, n, ms) for _, S, n, ms in rows if S <= 32]
    per_fold_ms = (np.mean([(ms - fixed - per_series_ms * S) / n for S, n, ms in fold]) if fold else per_sample_ms)
    # (fleet.CostModel's constants are ms per sample / per series / ms: bench.py C3_COST)
    print("C3_COST = dict(per_sample=%.3g, per_series=%.3g, per_sample_fold=%.3g, fixed=%.3g)" % (
        per_sample_ms, per_series_ms, per_fold_ms, fixed))
    for f, S, n, ms in rows:
        m = fixed + (per_fold_ms if S <= 32 else per_sample_ms) * n + per_series_ms * S
        print(f"  {os.path.basename(f):24s} S={S:8d} n={n:11d} measured {ms:7.3f} ms  model {m:7.3f} ms  "
              f"({(m / ms - 1) * 100:+.1f} %)")
    shards = [(S, n, ms) for f, S, n, ms in rows if os.path.basename(f).startswith("s")]
    if shards:
        t = [ms for _, _, ms in shards]
        print(f"measured shard spread (max / min): {max(t) / min(t):.3f}; slowest {max(t):.3f} ms")


if __name__ == "__main__":
    main()
