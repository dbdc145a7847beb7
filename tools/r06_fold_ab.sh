#!/bin/bash
# Round-6 A/B of k_fold1 variants (libf1) against HEAD
# (libf0): the one-tile parity tests and the C1 config test through libf1, then the C1
# step interleaved.  Development tool.
set -o pipefail
L5DH_LIB=$(pwd)/linkerd_amd/lib_ab/libf1.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -k "one_tile or c1 or C1" -x -q --timeout 300 --timeout-method thread > gpurun_out/f1_tests.log 2>&1 || { tail -20 gpurun_out/f1_tests.log; exit 1; }
echo "tests f1: $(tail -1 gpurun_out/f1_tests.log)"
tools/ab_libs.sh 4 c1 linkerd_amd/lib_ab/libf0.so linkerd_amd/lib_ab/libf1.so 2>/dev/null | grep -v amdgpu.ids
