#!/bin/bash
# GPU round trip used during development: parity tests, then C3 and C2 bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tcheck.log 2>&1 || { tail -30 gpurun_out/tcheck.log; exit 1; }
tail -2 gpurun_out/tcheck.log
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --cpu-sample 0 "$@" > gpurun_out/bcheck.json 2> gpurun_out/bcheck.err || { tail -20 gpurun_out/bcheck.err; exit 1; }
timeout -k 10 200 python3 -u bench.py --workload c2 --steps 10 --warmup 3 --cpu-sample 0 "$@" >> gpurun_out/bcheck.json 2>> gpurun_out/bcheck.err || { tail -20 gpurun_out/bcheck.err; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/bcheck.json"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["config"]["workload"][:3], d["ms_per_step"], "%.3e" % d["value"], d["path_roofline"]["frac"],
              {k: v["avg_ms"] for k, v in d["kernels"].items()})
PY
