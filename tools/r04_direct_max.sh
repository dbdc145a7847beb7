set -o pipefail
mkdir -p gpurun_out/r04t
for r in 1 2; do for dm in 255 128 64 32; do timeout -k 10 200 python3 -u tools/time_lib.py --workload c3 --direct-max $dm 2>/dev/null | sed "s/^/dm=$dm /" >> gpurun_out/r04t/dm.txt || exit 1; done; done
cat gpurun_out/r04t/dm.txt
for dm in 64 255; do PMC_KERNELS="rbin1w|rbin2|accum" PMC_PASSES="WRITE_SIZE" bash tools/profile_pmc.sh gpurun_out/r04t/pmc_dm$dm --steps 2 --warmup 1 --cpu-sample 0 --direct-max $dm > /dev/null && python3 tools/pmc_summary.py gpurun_out/r04t/pmc_dm$dm | sed "s/^/dm=$dm /" | cut -c1-60 >> gpurun_out/r04t/pmc.txt || exit 1; done
cat gpurun_out/r04t/pmc.txt
