# WRITE_SIZE of the level-1/2 kernels in timing-only builds: default, no write-out stores
# (EXP 32), no direct value sums (EXP 1) -> gpurun_out/r04v/
set -o pipefail
mkdir -p gpurun_out/r04v
ROOT=$(pwd)
for n in default w32 w1; do
  L=""; [ $n != default ] && L=$ROOT/linkerd_amd/lib_ab/lib$n.so
  L5DH_LIB=$L PMC_KERNELS="rbin1w|rbin2" PMC_PASSES="WRITE_SIZE;FETCH_SIZE" bash tools/profile_pmc.sh gpurun_out/r04v/pmc_$n --steps 2 --warmup 1 --cpu-sample 0 > /dev/null || exit 1
  python3 tools/pmc_summary.py gpurun_out/r04v/pmc_$n | sed "s/^/$n /" | cut -c1-220 >> gpurun_out/r04v/summary.txt
done
cat gpurun_out/r04v/summary.txt
