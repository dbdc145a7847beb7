#!/bin/bash
# Round-5 GPU call: (1) GPU tests (all, or $TESTS), (2) interleaved A/B of library builds
# on C3 ($ABLIBS), (3) the C3 bench line -> gpurun_out/<TAG>/.  Each GPU step under its
# own time limit; the script stops at the first failure.
set -o pipefail
T=${TAG:-r05run}
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest $TESTS -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
  tail -1 $OUT/gpu_tests.log
fi
if [ -n "$ABLIBS" ]; then
  for wl in ${ABWL:-c3}; do
    bash tools/ab_libs.sh ${ROUNDS:-2} $wl $ABLIBS > $OUT/ab_$wl.log 2>&1 || { tail -30 $OUT/ab_$wl.log; exit 1; }
    grep "ms/step" $OUT/ab_$wl.log
  done
fi
if [ -n "$BENCH" ]; then
  for wl in $BENCH; do
    timeout -k 10 400 python3 -u bench.py --workload $wl --cpu-sample 0 > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || { tail -20 $OUT/bench_$wl.err; exit 1; }
    echo "bench $wl: $(python3 -c "import json; d=json.loads(open('$OUT/bench_$wl.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['path_roofline']['frac'], {k: v['avg_ms'] for k, v in d['kernels'].items()})")"
  done
fi
if [ -n "$PMC" ]; then  # HBM traffic per launch of the level-1 / level-2 / accumulate kernels
  PMC_PASSES="FETCH_SIZE;WRITE_SIZE" PMC_KERNELS="rbin|accum" bash tools/profile_pmc.sh $OUT/pmc --steps 2 --warmup 1 --cpu-sample 0 || exit 1
  python3 tools/pmc_summary.py $OUT/pmc $OUT/pmc.json '{"workload": "c3", "series": 1000000, "samples": 1000000000}' > $OUT/pmc_summary.txt && grep -E "rbin|accum" $OUT/pmc_summary.txt | cut -c1-220
fi
echo done
