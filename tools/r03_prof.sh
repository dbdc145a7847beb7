#!/bin/bash
# Round-3 profile pass: kernel stats of C3 and C2, then HBM + LDS PMC passes of C3.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
T=${TAG:-r03p}
bash tools/kstats.sh ${T}_c3 || exit 1
bash tools/kstats.sh ${T}_c2 --workload c2 || exit 1
if [ -z "$NOPMC" ]; then
  PMC_PASSES="FETCH_SIZE;WRITE_SIZE;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
    bash tools/profile_pmc.sh gpurun_out/${T}_pmc_c3 --steps 2 --warmup 1 --cpu-sample 0 || exit 1
  python3 tools/pmc_summary.py gpurun_out/${T}_pmc_c3 gpurun_out/${T}_pmc_c3.json '{"workload": "c3", "series": 1000000, "samples": 1000000000}'
fi
