#!/bin/bash
# Wall-clock A/B of library builds (tools/mk_var.sh) with bench.py, interleaved.
#   TAG=... tools/ab_wall.sh "<lib>[:variant] ..." [rounds=3] [bench args...]
set -o pipefail
O=gpurun_out/${TAG:-ab}
mkdir -p $O
LIBS=$1; R=${2:-3}; shift 2
for i in $(seq 1 $R); do
  for v in $LIBS; do
    lib=${v%%:*}; var=0; [ "$lib" != "$v" ] && var=${v#*:}
    L5DH_LIB=$PWD/linkerd_amd/lib_ab/lib$lib.so timeout -k 10 240 python3 -u bench.py --cpu-sample 0 --variant $var "$@" > $O/ab_$v$i.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/ab_$v$i.json').read().strip().splitlines()[-1])
print('$v$i', d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})
"
  done
done
