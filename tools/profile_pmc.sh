#!/bin/bash
# PMC passes over a short bench run (one rocprofv3 run per counter group, as the
# MI355X guide requires).  Usage (on the GPU box, from the repo root):
#   tools/profile_pmc.sh <outdir> [bench args...]
# PMC_PASSES='A B C;D E' overrides the counter groups (';' between passes);
# PMC_KERNELS=<regex> restricts collection to matching kernels.
set -o pipefail
OUT=${1:-gpurun_out/pmc}; shift
ARGS=${@:---steps 2 --warmup 1 --cpu-sample 0}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
if [ -n "$PMC_PASSES" ]; then
  IFS=';' read -r -a passes <<< "$PMC_PASSES"
else
  passes=(
    "FETCH_SIZE"
    "WRITE_SIZE"
    "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS"
    "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS_ATOMIC SQ_LDS_ATOMIC_RETURN SQ_LDS_ADDR_CONFLICT GRBM_GUI_ACTIVE"
    "TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
  )
fi
KF=()
[ -n "$PMC_KERNELS" ] && KF=(--kernel-include-regex "$PMC_KERNELS")
i=0
for p in "${passes[@]}"; do
  i=$((i+1))
  echo "pass $i: $p"
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $p "${KF[@]}" --output-format csv -d "$ROOT/$OUT/p$i" -o run -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/p$i.log" 2>&1) || { echo "pass $i failed rc=$?"; tail -5 "$ROOT/$OUT/p$i.log"; exit 1; }
done
echo ok
