#!/bin/bash
# Round-4 baseline on the GPU box: C3/C2 bench lines (no CPU baseline) and per-kernel
# device times of the current sources -> gpurun_out/<TAG>/
set -o pipefail
T=${TAG:-r04base}
OUT=gpurun_out/$T
mkdir -p $OUT
for w in c3 c2; do
  timeout -k 10 300 python3 -u bench.py --workload $w --cpu-sample 0 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail -20 $OUT/bench_$w.err; exit 1; }
  echo "bench $w: $(python3 -c "import json; d=json.loads(open('$OUT/bench_$w.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['path_roofline']['frac'], json.dumps(d['kernels']))")"
done
echo done
