#!/bin/bash
# Round-2 profiles of the default bench command (C3): rocprofv3 kernel trace, then
# PMC passes (one rocprofv3 run per counter group): HBM FETCH_SIZE / WRITE_SIZE and
# two SQ groups (LDS bank conflicts, LDS / VMEM instruction mix).
#   tools/r02_prof.sh <tag> [bench args]   -> gpurun_out/prof_<tag>/
set -o pipefail
TAG=${1:-r02}; shift
OUT=gpurun_out/prof_$TAG
ROOT=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="$@"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/trace -o run -- python3 $ROOT/bench.py --steps 10 --warmup 3 --cpu-sample 0 $ARGS > $ROOT/$OUT/trace.log 2>&1) || { tail -20 $OUT/trace.log; exit 1; }
echo trace done
PMC_PASSES="FETCH_SIZE;WRITE_SIZE;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE;SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS_ATOMIC SQ_LDS_ADDR_CONFLICT" bash tools/profile_pmc.sh $OUT/pmc --steps 2 --warmup 1 --cpu-sample 0 $ARGS || exit 1
python3 tools/pmc_summary.py $OUT/pmc $OUT/pmc.json '{"workload": "c3", "series": 1000000, "samples": 1000000000}' > $OUT/pmc_summary.txt
python3 -c "
import glob, shutil, sys
sys.path.insert(0, 'tools')
import prof_summary
f = sorted(glob.glob('$OUT/trace/**/*kernel_stats.csv', recursive=True))
if f:
    shutil.copy(f[0], '$OUT/kernel_stats.csv')
    prof_summary.main(f[0], '$OUT/kernel_stats.md')
"
echo done
