#!/bin/bash
# Per-kernel times of several lib_ab variants (tools/mk_var.sh), one kstats run each.
#   tools/kvar.sh "<name> [ENV=val ...]" ...
set -o pipefail
for spec in "$@"; do
  set -- $spec
  n=$1; shift
  L5DH_LIB=$(realpath linkerd_amd/lib_ab/lib$n.so) bash tools/kstats.sh "$n" "$@" | sed 's/k_gen_[a-z0-9]*=[0-9]*us //' || exit 1
done
