#!/bin/bash
# Round-6 A/B of level 2 with one stage and three workgroups per CU (libsg, variant bit 8)
# against the double-buffered two-workgroup kernel (libcur): the parity tests through libsg,
# then interleaved timing on C3 and C2.  Development tool.
set -o pipefail
L5DH_LIB=$(pwd)/linkerd_amd/lib_ab/libsg.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/sg_tests.log 2>&1 || { tail -20 gpurun_out/sg_tests.log; exit 1; }
echo "tests sg: $(tail -1 gpurun_out/sg_tests.log)"
for wl in c3 c2; do tools/ab_libs.sh 3 $wl linkerd_amd/lib_ab/libcur.so linkerd_amd/lib_ab/libsg.so 2>/dev/null | grep -v amdgpu.ids || exit 1; done
