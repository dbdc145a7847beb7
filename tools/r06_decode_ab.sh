#!/bin/bash
# Round-6 A/B of k_mdecode with the next row's first words prefetched (libpf5: 5 waves per
# SIMD, libpf4: 4) against HEAD (libm0): the fleet tests through each build, then the C4
# loopback-8 step and the 1-rank C4 step interleaved.  Development tool.
set -o pipefail
for v in pf5 pf4; do
  L5DH_LIB=$(pwd)/linkerd_amd/lib_ab/lib$v.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fleet.py -x -q --timeout 300 --timeout-method thread > gpurun_out/dec_tests_$v.log 2>&1 || { tail -20 gpurun_out/dec_tests_$v.log; exit 1; }
  echo "tests $v: $(tail -1 gpurun_out/dec_tests_$v.log)"
done
tools/ab_c4.sh 2 linkerd_amd/lib_ab/libm0.so linkerd_amd/lib_ab/libpf5.so linkerd_amd/lib_ab/libpf4.so 2>/dev/null | grep -v amdgpu.ids || exit 1
tools/ab_libs.sh 2 c4 linkerd_amd/lib_ab/libm0.so linkerd_amd/lib_ab/libpf5.so linkerd_amd/lib_ab/libpf4.so 2>/dev/null | grep -v amdgpu.ids || exit 1
