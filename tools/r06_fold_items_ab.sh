#!/bin/bash
# Round-6 A/B of the one-tile fold's items per CU (chunk = n / (k CUs)): libi1, libi2 (HEAD's
# rule), libi4, interleaved on C1.  Development tool.
set -o pipefail
tools/ab_libs.sh 4 c1 linkerd_amd/lib_ab/libi2.so linkerd_amd/lib_ab/libi1.so linkerd_amd/lib_ab/libi4.so 2>/dev/null | grep -v amdgpu.ids
