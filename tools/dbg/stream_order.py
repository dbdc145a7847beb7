import faulthandler, sys
faulthandler.dump_traceback_later(60, exit=True)
sys.path.insert(0, ".")
import numpy as np
import torch
from linkerd_amd.engine import HistogramEngine
from linkerd_amd import synth, _native as N
from oracle import oracle as O
S = 4000
series, vals = synth.c3(S=S, N=500_000, seed=81)
o = O.OracleHistograms(S); o.ingest(series, vals)
want = o.snapshot()
dev = torch.device("cuda", 0)
for variant in ("sync", "nosync", "nosync", "sync"):
    eng = HistogramEngine(S)
    base = torch.from_numpy(o.counts()).to(dev)
    tot = torch.from_numpy(o.totals()).to(dev)
    torch.cuda.synchronize()
    for it in range(3):
        counts = torch.zeros_like(base); totals = torch.zeros_like(tot)
        counts += base; totals += tot
        if variant == "sync":
            torch.cuda.synchronize()
        summ = torch.empty((S, 11), dtype=torch.int64, device=dev)
        eng.summarize_dense(counts, totals, out=summ)
        got = summ.cpu().numpy().view(N.SUMMARY_DTYPE).reshape(-1)
        print(variant, it, "ok" if got.tobytes() == want.tobytes() else f"BAD {got[0]} counts.sum={int(counts.sum())} totals.sum={int(totals.sum())} base.sum={int(base.sum())}", flush=True)
    eng.close()
# summarize_dense with numpy inputs
eng = HistogramEngine(S)
got = eng.summarize_dense(o.counts(), o.totals())
print("numpy", "ok" if got.tobytes() == want.tobytes() else f"BAD {got[0]}")
