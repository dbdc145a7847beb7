#!/bin/bash
# Round-6 A/B of k_mdecode fetching a header's count by LDS permute only in chunks that hold a header
# (libnsh) against HEAD (libm1): the fleet tests through libnsh, then the C4 loopback-8 step
# interleaved (every rank's merge time).  Development tool.
set -o pipefail
L5DH_LIB=$(pwd)/linkerd_amd/lib_ab/libnsh.so timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fleet.py -x -q --timeout 600 --timeout-method thread > gpurun_out/ah4_tests.log 2>&1 || { tail -20 gpurun_out/ah4_tests.log; exit 1; }
echo "tests nsh: $(tail -1 gpurun_out/ah4_tests.log)"
for i in 1 2; do
  for v in m1 nsh; do
    L5DH_LIB=$(pwd)/linkerd_amd/lib_ab/lib$v.so timeout -k 10 300 python3 -u bench.py --workload c4 --loopback 8 --cpu-sample 0 --steps 5 --warmup 2 > /tmp/ab_c4.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open('/tmp/ab_c4.json').read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['config']['per_rank_ms_loopback'], [k['merge'] for k in d['per_rank_kernels_ms']])" $v
  done
done
