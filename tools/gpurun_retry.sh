#!/bin/bash
# Run one gpurun call, re-submitting it (up to TRIES times, WAIT seconds apart) only while
# the pool reports no free box or slot (nothing ran, nothing charged).  Any call that
# ran -- whatever its result -- is not repeated.  Development tool (this container).
#   tools/gpurun_retry.sh <timeout-seconds> '<command>'
TRIES=${TRIES:-8}; WAIT=${WAIT:-150}
T=$1; shift
for i in $(seq 1 $TRIES); do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1); rc=$?
  if echo "$out" | grep -q "status=transient\|no free box\|slot(s) on this pod are busy"; then
    echo "[retry $i: pool busy]"; sleep "$WAIT"; continue
  fi
  echo "$out"; exit $rc
done
echo "pool busy after $TRIES tries"; exit 3
