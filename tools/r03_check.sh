#!/bin/bash
# Round-3 GPU round trip: GPU tests (skip with NOTESTS=1; TESTS=<pytest args> for a subset),
# then bench lines (BENCH_ARGS='a;b;c', ';' between runs).  Every GPU step has its own
# time limit; the script stops at the first failure.
set -o pipefail
O=gpurun_out/${TAG:-r03}
mkdir -p $O
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests -m gpu} -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
IFS=';' read -r -a runs <<< "${BENCH_ARGS:-}"
for a in "${runs[@]}"; do
  echo "== bench $a"
  timeout -k 10 300 python3 -u bench.py --cpu-sample 0 $a > $O/b.json 2> $O/b.err || { tail -30 $O/b.err; exit 1; }
  cat $O/b.json >> $O/bench_all.jsonl
  python3 -c "
import json
d=json.loads(open('$O/b.json').read().strip().splitlines()[-1])
print(d['ms_per_step'], '%.3e'%d['value'], d['path_roofline']['frac'], (d['roofline'] or {}).get('frac'), {k:v['avg_ms'] for k,v in d['kernels'].items()}, d.get('merge'))
"
done
