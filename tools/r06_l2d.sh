#!/bin/bash
# Round-6 A/B of level 2 without its stage (k_rbin2<.., true>, variant bit 8): the parity
# tests through each direct build, then interleaved timing against the staged build.
set -o pipefail
OUT=gpurun_out/${TAG:-r06l2d}
mkdir -p $OUT
for v in d2 d3; do
  L5DH_LIB=$(pwd)/linkerd_amd/lib_ab/lib$v.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $OUT/tests_$v.log 2>&1 || { tail -30 $OUT/tests_$v.log; exit 1; }
  echo "tests $v: $(tail -1 $OUT/tests_$v.log)"
done
for wl in c3 c2; do
  tools/ab_libs.sh ${ROUNDS:-3} $wl linkerd_amd/lib_ab/libst.so linkerd_amd/lib_ab/libd2.so linkerd_amd/lib_ab/libd3.so > $OUT/ab_$wl.txt 2>&1 || { tail -20 $OUT/ab_$wl.txt; exit 1; }
  cat $OUT/ab_$wl.txt
done
echo done
