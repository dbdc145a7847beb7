#!/bin/bash
# One-tile series spaces: k_fold1 (variant 0), k_encode1 (variant bit 3) and the partition pipeline
# (variant bit 2) on C1 and the 8-way C3 head shard, interleaved in one box.
set -o pipefail
mkdir -p gpurun_out/e1
for r in 1 2; do for v in 0 1 8 4; do
  for w in "--workload c1" "--shard 0/8"; do
    tag=$(echo "$w" | tr -dc 'a-z0-9')_v${v}_$r
    timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --cpu-sample 0 --variant $v $w > gpurun_out/e1/$tag.json 2> gpurun_out/e1/$tag.err || exit 1
    python3 -c "
import json;d=json.loads(open('gpurun_out/e1/$tag.json').read().strip().splitlines()[-1]);print('$tag',d['ms_per_step'],{k:v['avg_ms'] for k,v in d['kernels'].items()})"
  done
done; done
