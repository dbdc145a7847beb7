#!/bin/bash
# Interleaved A/B of library builds on the C4 fleet step (8 ranks over the loopback
# transport on one GPU): bench.py's line per build, round after round.  Development tool.
#   tools/ab_c4.sh <rounds> <lib.so>...
set -o pipefail
R=$1; shift
for i in $(seq 1 "$R"); do
  for lib in "$@"; do
    L5DH_LIB=$(realpath "$lib") timeout -k 10 300 python3 -u bench.py --workload c4 --loopback 8 --cpu-sample 0 --steps 5 --warmup 2 > /tmp/ab_c4.json || exit 1
    python3 -c "import json,sys; d=json.loads(open('/tmp/ab_c4.json').read().strip().splitlines()[-1]); k=d['per_rank_kernels_ms'][0]; print(sys.argv[1], d['ms_per_step'], d['config']['per_rank_ms_loopback'], k)" "$(basename $lib)"
  done
done
