"""Repeat a small export many times per engine setting; count wrong exports (GPU box)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

from linkerd_amd import _native as N, synth  # noqa: E402
from linkerd_amd.engine import HistogramEngine  # noqa: E402
from oracle import oracle as O  # noqa: E402

S = 4001
series, vals = synth.c3(S=S, N=300_000, seed=74)
p = (series[0::2], vals[0::2])
o = O.OracleHistograms(S)
o.ingest(*p)
want = o.counts()
settings = [("default", {}), ("direct_max=0", {N.PARAM_DIRECT_MAX: 0}), ("stage=0", {N.PARAM_STAGE_SAMPLES: 0}),
            ("cold_limit=65535,hot_chunk=2^20", {N.PARAM_HOT_CHUNK: 1 << 20}), ("slabs=1", {N.PARAM_MAX_SLABS: 1}),
            ("slabs=8", {N.PARAM_MAX_SLABS: 8})]
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 12
for name, prm in settings:
    fails = []
    for rep in range(reps):
        e = HistogramEngine(S)
        for k, v in prm.items():
            e.set_param(k, v)
        e.ingest(*p)
        c, t = e.export_state(reset=True)
        bad = np.nonzero((c != want).any(axis=1))[0]
        if bad.size:
            d = c[bad[0]].astype(np.int64) - want[bad[0]]
            fails.append((rep, bad.size, int(bad[0]), int(d.sum()), int(d[0])))
        e.close()
    print(f"{name}: {len(fails)}/{reps} wrong {fails[:4]}", flush=True)
