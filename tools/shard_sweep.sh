#!/bin/bash
# One C3 shard sweep: each rank's shard of a W-way split (bench.py --shard r/W) on
# this one GPU (the load-derived plan of fleet.plan_shards).  tools/shard_sweep.sh <tag> [W]
set -o pipefail
TAG=$1; W=${2:-8}
mkdir -p gpurun_out/sw_$TAG
for ((r = 0; r < W; r++)); do
  timeout -k 10 200 python3 -u bench.py --shard $r/$W --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/sw_$TAG/s$r.json 2> gpurun_out/sw_$TAG/s$r.err || { tail -5 gpurun_out/sw_$TAG/s$r.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/sw_$TAG/s$r.json').read().strip().splitlines()[-1]);print(d['config']['shard'] if 'shard' in d['config'] else '', d['ms_per_step'])"
done
