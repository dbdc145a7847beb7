#!/bin/bash
# Round-2 GPU round trip: all GPU tests (skip with NOTESTS=1), then bench lines for
# C3 (default), C3 shards of an 8-way split, C4 at one rank (RCCL merge) and the
# streaming ingest shape.  Every GPU step has its own time limit; stop at the first
# failure.  BENCH_ARGS='a;b;c' overrides the bench list (';' between runs).
set -o pipefail
O=gpurun_out/r02
mkdir -p $O
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
if [ -n "$BENCH_ARGS" ]; then
  IFS=';' read -r -a runs <<< "$BENCH_ARGS"
else
  runs=("" "--shard 0/8" "--shard 4/8" "--shard 7/8" "--workload c4" "--piece 65536 --steps 2 --warmup 1" "--piece 1048576 --steps 2 --warmup 1")
fi
for a in "${runs[@]}"; do
  echo "== bench $a"
  timeout -k 10 300 python3 -u bench.py --cpu-sample 0 $a > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  cat $O/b.json >> $O/bench_all.jsonl
  python3 -c "
import json
d=json.loads(open('$O/b.json').read().strip().splitlines()[-1])
print(d['ms_per_step'], '%.3e'%d['value'], d['path_roofline']['frac'], (d['roofline'] or {}).get('frac'), {k:v['avg_ms'] for k,v in d['kernels'].items()}, d.get('merge'))
"
done
