#!/bin/bash
# Round-6 A/B of the big-tile accumulate grid: libcur (all CUs when k_accum_split runs alone
# on its stream) against libs38 (3/8 of the CUs in either mode, round 5), interleaved, on
# C3 shards 1-3 of the 8-way plan, C3 and C2.  Development tool.
set -o pipefail
for a in "--shard 2/8" "--shard 1/8" "--shard 3/8" "--workload c3" "--workload c2"; do
  for i in 1 2; do
    for v in cur s38; do
      echo -n "$a $v: "
      L5DH_LIB=$(pwd)/linkerd_amd/lib_ab/lib$v.so timeout -k 10 180 python3 -u tools/time_lib.py $a --steps 4 2>/dev/null | tail -1 || exit 1
    done
  done
done
