#!/bin/bash
# Per-kernel device times of a short bench run (rocprofv3 kernel trace + stats).
# Usage: tools/kstats.sh <tag> [ENV=val ...] [bench args...]
set -o pipefail
TAG=$1; shift
envs=(); args=()
for w in "$@"; do if [[ $w == *=* && $w != --* ]]; then envs+=("$w"); else args+=("$w"); fi; done
ROOT=$(pwd)
mkdir -p gpurun_out/ks_$TAG
export TMPDIR=/tmp
for e in "${envs[@]}"; do export "$e"; done
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/ks_$TAG" -o run -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --cpu-sample 0 "${args[@]}" > "$ROOT/gpurun_out/ks_$TAG/bench.log" 2>&1) || { echo "kstats $TAG failed"; tail -5 "$ROOT/gpurun_out/ks_$TAG/bench.log"; exit 1; }
f=$(find "$ROOT/gpurun_out/ks_$TAG" -name "*kernel_stats.csv" | head -1)
python3 - "$f" "$TAG" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
out = []
for r in rows:
    n = r["Name"]
    if not n.startswith("_ZN4l5dh") and "k_" not in n:
        continue
    import re
    m = re.search(r"k_[a-z0-9_]+", n)
    out.append((m.group(0) if m else n[:30], float(r["AverageNs"]) / 1e3, int(r["Calls"])))
print(sys.argv[2], " ".join(f"{k}={v:.0f}us" for k, v, c in sorted(out, key=lambda x: -x[1])))
PY
