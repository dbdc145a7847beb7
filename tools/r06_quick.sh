#!/bin/bash
# Quick check on the GPU box: the selected GPU tests (TESTS, pytest args), then bench
# lines (WORKLOADS: c3 c2 c1 c4 c3hot c3first) without the CPU baseline -> gpurun_out/<TAG>/.
set -o pipefail
T=${TAG:-r06quick}
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
  tail -1 $OUT/gpu_tests.log
fi
for w in ${WORKLOADS:-c3 c3hot c3first c2}; do
  extra=""; wl=$w
  [ $w = c3hot ] && { wl=c3; extra="--hot-shift"; }
  [ $w = c3first ] && { wl=c3; extra="--first-interval"; }
  timeout -k 10 400 python3 -u bench.py --workload $wl --cpu-sample 0 $extra $BENCH_ARGS > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail -20 $OUT/bench_$w.err; exit 1; }
  echo "bench $w: $(python3 -c "import json; d=json.loads(open('$OUT/bench_$w.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['path_roofline']['frac'], d.get('redos'), {k: v['avg_ms'] for k, v in d['kernels'].items()})")"
done
echo done
