#!/bin/bash
# Round-4 check on the GPU box: GPU tests, C3/C2 bench lines, and interleaved per-kernel
# timings of the default library against development builds in linkerd_amd/lib_ab
# (ABLIBS="name ...") -> gpurun_out/<TAG>/
set -o pipefail
T=${TAG:-r04check}
OUT=gpurun_out/$T
mkdir -p $OUT
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
  tail -3 $OUT/gpu_tests.log
fi
for w in ${WLS:-c3 c2}; do
  timeout -k 10 300 python3 -u bench.py --workload $w --cpu-sample 0 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail -20 $OUT/bench_$w.err; exit 1; }
  echo "bench $w: $(python3 -c "import json; d=json.loads(open('$OUT/bench_$w.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['path_roofline']['frac'], ' '.join(k+'='+str(v['avg_ms']) for k,v in d['kernels'].items()))")"
done
if [ -n "$C4LB" ]; then
  timeout -k 10 400 python3 -u bench.py --workload c4 --loopback $C4LB --steps 5 --warmup 2 > $OUT/bench_c4lb.json 2> $OUT/bench_c4lb.err || { tail -20 $OUT/bench_c4lb.err; exit 1; }
  echo "bench c4 loopback $C4LB: $(python3 -c "import json; d=json.loads(open('$OUT/bench_c4lb.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['config']['per_rank_ms'], d['path_roofline']['frac'], d['per_rank_kernels_ms'][0])")"
fi
for r in $(seq 1 ${ABREPS:-2}); do
  for L in default $ABLIBS; do
    if [ $L = default ]; then lib=""; else lib=linkerd_amd/lib_ab/lib$L.so; fi
    L5DH_LIB=$lib timeout -k 10 200 python3 -u tools/time_lib.py --workload ${ABWL:-c3} >> $OUT/ab.txt 2>> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
  done
done
cat $OUT/ab.txt
echo done
