mkdir -p gpurun_out/hc
for r in 1 2; do for h in 262144 65536 131072; do
timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 3 --cpu-sample 0 --hot-chunk $h > gpurun_out/hc/b_${h}_$r.json 2> gpurun_out/hc/e_${h}_$r.log || exit 1
python3 -c "
import json,sys;d=json.loads(open('gpurun_out/hc/b_${h}_$r.json').read().strip().splitlines()[-1]);print($h,d['ms_per_step'],{k:v['avg_ms'] for k,v in d['kernels'].items()})"
done; done
