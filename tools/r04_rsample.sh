# Sample-size A/B (k_rsample draws 2^20 / 2^19 / 2^18) on C3, C2 and the smallest C3 shard
set -o pipefail
mkdir -p gpurun_out/r04z
for wl in "--workload c3" "--workload c2" "--workload c3 --shard 7/8"; do
  for r in 1 2; do for L in "" linkerd_amd/lib_ab/librs19.so linkerd_amd/lib_ab/librs18.so; do
    L5DH_LIB=$L timeout -k 10 200 python3 -u tools/time_lib.py $wl 2>/dev/null | sed "s|^|$wl |" >> gpurun_out/r04z/ab.txt || exit 1
  done; done
done
cat gpurun_out/r04z/ab.txt
