#!/bin/bash
# Page-pool level-1 prototype (tools/mb_pages.hip) on the GPU box: timing of the
# page layout against exact-placement layouts (same kernel, same process), the
# correctness check, and HBM PMC passes (FETCH_SIZE / WRITE_SIZE, separate runs).
set -o pipefail
O=gpurun_out/pages
ROOT=$(pwd)
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 ./tools/mb_pages 1e9 5 > $O/mb.log 2>&1 || { cat $O/mb.log; exit 1; }
cat $O/mb.log
for c in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && timeout -s KILL 180 rocprofv3 --pmc $c --kernel-include-regex k_bin1p --output-format csv -d $ROOT/$O/$c -o run -- $ROOT/tools/mb_pages 1e9 1 > $ROOT/$O/$c.log 2>&1) || { tail -5 $O/$c.log; exit 1; }
done
echo done
