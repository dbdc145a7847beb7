#!/bin/bash
# Round-6 development run on the GPU box (every GPU step under its own time limit; stops
# at the first failure): the GPU tests named in TESTS (default: the parity and merge/ingest
# files) against the working-tree library, then interleaved A/B timing of the libraries
# given as arguments (tools/time_lib.py) on C3 and C2, then (PMC=1) one instruction-mix
# PMC pass of level 1 for each library -> gpurun_out/<TAG>/.  Development tool.
#   TAG=r06b tools/r06_ab.sh linkerd_amd/lib_ab/libA.so linkerd_amd/lib_ab/libB.so
set -o pipefail
OUT=gpurun_out/${TAG:-r06ab}
ROOT=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
TESTS=${TESTS:-tests/test_gpu_parity.py tests/test_gpu_merge_ingest.py}
if [ "$TESTS" != none ]; then
  timeout -k 10 ${TEST_LIMIT:-600} python3 -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
for wl in ${WORKLOADS:-c3 c2}; do
  tools/ab_libs.sh ${ROUNDS:-3} $wl "$@" > $OUT/ab_$wl.txt 2>&1 || { tail -20 $OUT/ab_$wl.txt; exit 1; }
  cat $OUT/ab_$wl.txt
done
if [ -n "$PMC" ]; then
  i=0
  for lib in "$@"; do
    i=$((i+1))
    (cd /tmp && L5DH_LIB=$(realpath $ROOT/$lib) timeout -s KILL 120 rocprofv3 --pmc ${PMC_SET:-SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY} --kernel-include-regex "${PMC_KERNELS:-rbin1w|rbin2}" --output-format csv -d $ROOT/$OUT/pmc$i/p1 -o run -- python3 $ROOT/bench.py --steps 2 --warmup 1 --cpu-sample 0 > $ROOT/$OUT/pmc$i.log 2>&1) || { echo "pmc $lib failed"; tail -5 $OUT/pmc$i.log; exit 1; }
    echo "pmc $i: $lib"
    python3 tools/pmc_summary.py $OUT/pmc$i > $OUT/pmc$i.txt 2>&1 && grep -E "^(rbin1w|rbin2)" $OUT/pmc$i.txt
  done
fi
echo done
