#!/bin/bash
# Round-6 evidence on the GPU box (every GPU step under its own time limit; stops at
# the first failure): the GPU tests and smoke(), a rocprofv3 kernel trace + stats of
# the default C3 command, its PMC passes (HBM FETCH_SIZE / WRITE_SIZE, LDS and wait
# counters) -> profiles/pmc_latest.json, then the bench lines: C3 (with the CPU
# baseline), C2, C1, C4 at one rank through RCCL, the 8-rank fleet on this GPU over the
# loopback transport, and C3 off its capacity plan's best case (a moving hot set; every
# batch planned as a first interval) -> gpurun_out/<TAG>/.  NOTEST=1 skips the tests.
set -o pipefail
T=${TAG:-r06final}
OUT=gpurun_out/$T
ROOT=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
  timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
  tail -1 $OUT/gpu_tests.log
  timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/trace -o run -- python3 $ROOT/bench.py --steps 10 --warmup 3 --cpu-sample 0 > $ROOT/$OUT/trace_bench.json 2> $ROOT/$OUT/trace.log) || { tail -20 $OUT/trace.log; exit 1; }
echo trace done
PMC_PASSES="FETCH_SIZE;WRITE_SIZE;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES;SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY" bash tools/profile_pmc.sh $OUT/pmc --steps 2 --warmup 1 --cpu-sample 0 || exit 1
python3 tools/pmc_summary.py $OUT/pmc $OUT/pmc.json '{"workload": "c3", "series": 1000000, "samples": 1000000000}' > $OUT/pmc_summary.txt
cp $OUT/pmc.json profiles/pmc_latest.json  # (the bench lines below read their traffic from it)
for w in c3 c2 c1 c4 c4s c3hot c3first; do
  extra=""; wl=$w
  [ $w = c4 ] && extra="--cpu-sample 0"
  [ $w = c4s ] && { wl=c4; extra="--cpu-sample 0 --loopback 8"; }
  [ $w = c3hot ] && { wl=c3; extra="--cpu-sample 0 --hot-shift"; }
  [ $w = c3first ] && { wl=c3; extra="--cpu-sample 0 --first-interval"; }
  timeout -k 10 400 python3 -u bench.py --workload $wl $extra > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail -20 $OUT/bench_$w.err; exit 1; }
  echo "bench $w: $(python3 -c "import json; d=json.loads(open('$OUT/bench_$w.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['path_roofline']['frac'], (d.get('cpu_baseline') or {}).get('value'), d.get('redos'))")"
done
echo done
