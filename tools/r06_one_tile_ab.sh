#!/bin/bash
# Round-6 A/B of the one-tile snapshot through k_rows (libr1) against the plan + accumulate
# kernels (libr0): the one-tile and C1 tests through libr1, then C1 interleaved.
set -o pipefail
L5DH_LIB=$(pwd)/linkerd_amd/lib_ab/libr1.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_merge_ingest.py -k "one_tile or c1 or C1 or range" -x -q --timeout 300 --timeout-method thread > gpurun_out/r1_tests.log 2>&1 || { tail -20 gpurun_out/r1_tests.log; exit 1; }
echo "tests r1: $(tail -1 gpurun_out/r1_tests.log)"
tools/ab_libs.sh 4 c1 linkerd_amd/lib_ab/libr0.so linkerd_amd/lib_ab/libr1.so 2>/dev/null | grep -v amdgpu.ids
