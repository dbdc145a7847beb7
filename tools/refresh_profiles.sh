#!/bin/bash
# Round artefacts on the GPU box: parity tests, the default bench line (with the
# CPU baseline), a rocprofv3 kernel-trace summary of the same command, and the
# HBM-traffic PMC passes (FETCH_SIZE / WRITE_SIZE in separate runs).
#   tools/refresh_profiles.sh <tag>      -> gpurun_out/prof_<tag>/
set -o pipefail
TAG=${1:-latest}
OUT=gpurun_out/prof_$TAG
ROOT=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 400 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/trace -o run -- python3 $ROOT/bench.py --steps 10 --warmup 3 --cpu-sample 0 > $ROOT/$OUT/trace.log 2>&1) || { tail -20 $OUT/trace.log; exit 1; }
PMC_PASSES="FETCH_SIZE;WRITE_SIZE" bash tools/profile_pmc.sh $OUT/pmc --steps 2 --warmup 1 --cpu-sample 0 || exit 1
python3 tools/pmc_summary.py $OUT/pmc $OUT/pmc.json '{"workload": "c3", "series": 1000000, "samples": 1000000000}' > $OUT/pmc_summary.txt
echo done
