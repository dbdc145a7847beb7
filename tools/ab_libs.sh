#!/bin/bash
# Interleaved A/B of library builds on one GPU box: per-kernel device times (HIP events)
# of each build on the same workload, round after round (A B C A B C ...).  Every run is
# under its own time limit; the script stops at the first failure.  Development tool.
#   tools/ab_libs.sh <rounds> <workload> <lib.so>...
set -o pipefail
R=$1; WL=$2; shift 2
for i in $(seq 1 "$R"); do
  for lib in "$@"; do
    L5DH_LIB=$(realpath "$lib") timeout -k 10 180 python3 -u tools/time_lib.py --workload "$WL" --steps 4 || exit 1
  done
done
