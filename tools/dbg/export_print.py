"""One small one-slab export with the debug-print build (L5DH_LIB=.../libdbg.so)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

from linkerd_amd import _native as N, synth  # noqa: E402
from linkerd_amd.engine import HistogramEngine  # noqa: E402
from oracle import oracle as O  # noqa: E402

S = 4001
n = int(sys.argv[1]) if len(sys.argv) > 1 else 60_000
series, vals = synth.c3(S=S, N=2 * n, seed=74)
p = (series[0::2], vals[0::2])
o = O.OracleHistograms(S)
o.ingest(*p)
want = o.counts()
e = HistogramEngine(S)
e.set_param(N.PARAM_MAX_SLABS, 1)
e.ingest(*p)
e.sync()
print("---- export", flush=True)
c, t = e.export_state(reset=True)
bad = np.nonzero((c != want).any(axis=1))[0]
print(f"n={n}: {bad.size} rows differ {bad[:20]}; want tile0 halves {want[:16].sum()} {want[16:32].sum()}", flush=True)
e.close()
