#!/bin/bash
# A/B timing of two builds of libl5dhist.so on the same box, interleaved
# (A B A B ...), per-kernel device times from rocprofv3 kernel stats.
#   tools/ab.sh <libA.so> <libB.so> [rounds=3] [bench args...]
set -o pipefail
A=$1; B=$2; R=${3:-3}; shift 3
for i in $(seq 1 $R); do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    L5DH_LIB=$(realpath $lib) bash tools/kstats.sh "${v}$i" "$@" | sed 's/k_gen_[a-z0-9]*=[0-9]*us //' || exit 1
  done
done
