#!/bin/bash
# Round-5 A/B on one GPU box: interleaved per-kernel times of library builds
# (tools/ab_libs.sh) -> gpurun_out/<TAG>/ab.log.  Every GPU step has its own limit.
set -o pipefail
T=${TAG:-r05ab}
OUT=gpurun_out/$T
mkdir -p $OUT
R=${ROUNDS:-2}
WL=${WL:-c3}
bash tools/ab_libs.sh $R $WL "$@" > $OUT/ab_$WL.log 2>&1 || { tail -30 $OUT/ab_$WL.log; exit 1; }
grep "ms/step" $OUT/ab_$WL.log
