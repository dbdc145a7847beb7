#!/bin/bash
# Round-6 bisection of the split-heavy shards' accumulate time: libraries built at
# 19c26f8 (round 5), caac027 (split grid per stream mode), ebf9e2e (lean level 2) and the
# working tree, interleaved on C3 shards 2 and 3 of the 8-way plan.  Development tool.
set -o pipefail
for a in "--shard 2/8" "--shard 3/8"; do
  for i in 1 2; do
    for v in r05 grid lean cur; do
      echo -n "$a $v: "
      L5DH_LIB=$(pwd)/linkerd_amd/lib_ab/lib$v.so timeout -k 10 180 python3 -u tools/time_lib.py $a --steps 4 2>/dev/null | tail -1 || exit 1
    done
  done
done
