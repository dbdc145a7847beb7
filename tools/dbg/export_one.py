"""One-slab export of a small Zipf batch: where the direct path goes wrong (GPU box)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

from linkerd_amd import _native as N, synth  # noqa: E402
from linkerd_amd.engine import HistogramEngine  # noqa: E402
from oracle import oracle as O  # noqa: E402

S = 4001
for n, prm in ((150_000, {}), (60_000, {}), (150_000, {N.PARAM_REGION_PCT: 50}), (30_000, {}),
               (150_000, {N.PARAM_DIRECT_MAX: 1})):
    series, vals = synth.c3(S=S, N=2 * n, seed=74)
    p = (series[0::2], vals[0::2])
    o = O.OracleHistograms(S)
    o.ingest(*p)
    want = o.counts()
    e = HistogramEngine(S)
    e.set_param(N.PARAM_MAX_SLABS, 1)
    for k, v in prm.items():
        e.set_param(k, v)
    e.ingest(*p)
    c, t = e.export_state(reset=True)
    bad = np.nonzero((c != want).any(axis=1))[0]
    print(f"n={n} {prm}: {bad.size} rows differ {bad[:20]}; totals differ {np.nonzero(t != o.totals())[0][:8]}")
    for r in bad[:4]:
        d = c[r].astype(np.int64) - want[r]
        b = np.nonzero(d)[0]
        print(f"   row {r}: sum diff {int(d.sum())}, {b.size} buckets: {list(zip(b[:10].tolist(), d[b[:10]].tolist()))}")
    e.close()
