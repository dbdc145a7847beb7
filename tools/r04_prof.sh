#!/bin/bash
# rocprofv3 kernel trace + stats of the default C3 bench command -> gpurun_out/<TAG>/trace
set -o pipefail
T=${TAG:-r04prof}
OUT=gpurun_out/$T
ROOT=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/trace -o run -- python3 $ROOT/bench.py --steps 10 --warmup 3 --cpu-sample 0 ${BENCHARGS} > $ROOT/$OUT/trace_bench.json 2> $ROOT/$OUT/trace.log) || { tail -20 $OUT/trace.log; exit 1; }
f=$(find $OUT/trace -name '*kernel_stats.csv' | head -n 1)
python3 tools/prof_summary.py "$f" $OUT/kernel_stats.md
t=$(find $OUT/trace -name '*kernel_trace.csv' | head -n 1)
cp "$t" $OUT/kernel_trace.csv
