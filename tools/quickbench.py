"""Quick perf probe: C2 (100k series x 1k samples) ingest + snapshot, per-kernel times.
  python tools/quickbench.py [S] [K] [region_pct] [zipf]"""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from linkerd_amd import synth, _native as N
from linkerd_amd.engine import HistogramEngine

S = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
K = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000
PCT = int(sys.argv[3]) if len(sys.argv) > 3 else 100  # L5DH_PARAM_REGION_PCT (< 100: the redo path)
t0 = time.time()
if len(sys.argv) > 4 and sys.argv[4] == "zipf":
    series, vals = synth.c3(S=S, N=S * K)
else:
    series, vals = synth.c2(S=S, K=K)
print(f"gen {time.time()-t0:.1f}s", flush=True)
ds = torch.from_numpy(series.view(np.int32)).cuda()
dv = torch.from_numpy(vals).cuda()
eng = HistogramEngine(S)
summ = torch.zeros(S * 11, dtype=torch.int64, device="cuda")
cnt = torch.zeros((S, 1798), dtype=torch.int32, device="cuda")
eng.set_param(N.PARAM_TIMING, 1)
eng.set_param(N.PARAM_REGION_PCT, PCT)
print("region pct", PCT)
for it in range(5):
    torch.cuda.synchronize()
    t = time.perf_counter()
    eng.ingest(ds, dv)
    eng.snapshot_into(summ, cnt)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    kt = eng.kernel_times(reset=True)
    n = S * K
    balg = 8 * n + 7280 * S
    print(f"iter {it}: {dt*1e3:.3f} ms  {n/dt:.3e} samples/s  alg {balg/dt/1e12:.2f} TB/s  " +
          " ".join(f"{k}={v[0]:.3f}ms/{v[1]}" for k, v in kt.items()), flush=True)
