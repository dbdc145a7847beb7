for d in 0 1 2 3 4; do
  echo "dbg=$d"
  L5DH_DBG=$d timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/exp_$d.json 2>&1 || exit 1
done
