#!/bin/bash
# Build linkerd_amd/lib_ab/lib<name>.so from the working tree with extra compile
# flags (e.g. -DL5DH_PHASES for per-workgroup phase stamps).  Development tool.
#   tools/mk_var.sh <name> [hipcc flags...]
set -e
cd "$(dirname "$0")/../linkerd_amd/csrc"
N=$1; shift
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math -w -DL5DH_DEV $*"
T=$(mktemp -d)
mkdir -p ../lib_ab
/opt/rocm/bin/hipcc $F -c l5dh_ingest.hip -o $T/i.o &
/opt/rocm/bin/hipcc $F -c l5dh_snapshot.hip -o $T/s.o &
/opt/rocm/bin/hipcc $F -x hip -c l5dh_engine.cpp -o $T/e.o &
/opt/rocm/bin/hipcc $F -c l5dh_merge.hip -o $T/m.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib_ab/lib$N.so $T/i.o $T/s.o $T/m.o $T/e.o -L/opt/rocm/lib -lrccl
rm -rf $T
