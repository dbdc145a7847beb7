#!/bin/bash
# Development sweep on the GPU box: bench variants, one line each.
# Usage: tools/exp.sh "<env and bench args 1>" "<...2>" ...   e.g. "L5DH_DBG=1 --direct-max 0"
set -o pipefail
mkdir -p gpurun_out
i=0
for a in "$@"; do
  i=$((i+1))
  envs=(); args=()
  for w in $a; do if [[ $w == *=* && $w != --* ]]; then envs+=("$w"); else args+=("$w"); fi; done
  env "${envs[@]}" timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 2 --cpu-sample 0 "${args[@]}" > gpurun_out/exp_$i.json 2> gpurun_out/exp_$i.err || { echo "variant $i failed: $a"; tail -20 gpurun_out/exp_$i.err; exit 1; }
  python3 - "$a" gpurun_out/exp_$i.json <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith("{"):
        d = json.loads(l)
        print(f"[{sys.argv[1]}] {d['ms_per_step']:.3f} ms {d['value']:.3e}/s path {d['path_roofline']['frac']:.3f} |",
              " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in d["kernels"].items()))
PY
done
