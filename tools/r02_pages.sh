#!/bin/bash
# Page-pool level-1 prototype (tools/mb_pages.hip) on the GPU box, beside the
# engine's own C3 bench line (same box): timing, correctness check, HBM PMC.
set -o pipefail
O=gpurun_out/pages
ROOT=$(pwd)
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py --cpu-sample 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
timeout -k 10 120 ./tools/mb_pages 1e9 5 ${PAGE:-4096} > $O/mb.log 2>&1 || { cat $O/mb.log; exit 1; }
cat $O/mb.log
for c in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex k_bin1p --output-format csv -d $ROOT/$O/$c -o run -- $ROOT/tools/mb_pages 1e9 1 ${PAGE:-4096} > $ROOT/$O/$c.log 2>&1) || { tail -5 $O/$c.log; exit 1; }
done
echo done
