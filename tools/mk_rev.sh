#!/bin/bash
# Build linkerd_amd/lib_ab/lib<name>.so from a git revision (default HEAD), for
# interleaved A/B timing of the working tree against it (tools/r04_check.sh ABLIBS).
# Development tool.   tools/mk_rev.sh <name> [rev] [hipcc flags...]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
N=$1; REV=${2:-HEAD}; shift; shift || true
W=$(mktemp -d)
git -C "$ROOT" worktree add -f "$W/wt" "$REV" -q
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math -w $*"
T=$(mktemp -d)
cd "$W/wt/linkerd_amd/csrc"
/opt/rocm/bin/hipcc $F -c l5dh_ingest.hip -o $T/i.o &
/opt/rocm/bin/hipcc $F -c l5dh_snapshot.hip -o $T/s.o &
/opt/rocm/bin/hipcc $F -x hip -c l5dh_engine.cpp -o $T/e.o &
/opt/rocm/bin/hipcc $F -c l5dh_merge.hip -o $T/m.o &
wait
mkdir -p "$ROOT/linkerd_amd/lib_ab"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/linkerd_amd/lib_ab/lib$N.so" $T/i.o $T/s.o $T/m.o $T/e.o -L/opt/rocm/lib -lrccl
cd "$ROOT"
git worktree remove --force "$W/wt"
rm -rf "$T" "$W"
