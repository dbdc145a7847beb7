#!/bin/bash
# Round-2 GPU round trip: all GPU tests, then bench lines for C3 (default), the C3
# shards of an 8-way split (first and last rank), C4 at one rank (RCCL merge) and
# the streaming ingest shape.  Every GPU step has its own time limit; stop at the
# first failure.
set -o pipefail
mkdir -p gpurun_out/r02
O=gpurun_out/r02
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for a in ${BENCHES:-"" "--shard 0/8" "--shard 4/8" "--shard 7/8" "--workload c4" "--piece 65536 --steps 2 --warmup 1" "--piece 1048576 --steps 2 --warmup 1"}; do
  echo "== bench $a"
  timeout -k 10 300 python3 -u bench.py --cpu-sample 0 $a > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  cat $O/b.json >> $O/bench_all.jsonl
  python3 -c "
import json,sys
d=json.loads(open('$O/b.json').read().strip().splitlines()[-1])
print(d['ms_per_step'], '%.3e'%d['value'], d['path_roofline']['frac'], (d['roofline'] or {}).get('frac'), {k:v['avg_ms'] for k,v in d['kernels'].items()}, d.get('merge'))
"
done
