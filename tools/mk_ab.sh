#!/bin/bash
# Build linkerd_amd/lib_ab/libA.so from HEAD and libB.so from the working tree
# (for tools/ab.sh on the GPU box).  Development tool.
set -e
cd "$(dirname "$0")/.."
mkdir -p linkerd_amd/lib_ab
make -s -C linkerd_amd/csrc
cp linkerd_amd/lib/libl5dhist.so linkerd_amd/lib_ab/libB.so
git stash -q
trap 'git stash pop -q' EXIT
make -s -C linkerd_amd/csrc
cp linkerd_amd/lib/libl5dhist.so linkerd_amd/lib_ab/libA.so
git stash pop -q
trap - EXIT
make -s -C linkerd_amd/csrc
