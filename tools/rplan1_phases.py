"""k_rplan1 phase times (wall_clock64 stamps of thread 0; a -DL5DH_PHASES build given
by L5DH_LIB): a C3-shaped engine (1M series) ingesting Zipf batches.  Development tool.
  L5DH_LIB=linkerd_amd/lib_ab/libph.so python tools/rplan1_phases.py"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from linkerd_amd import _native as N  # noqa: E402
from linkerd_amd import synth  # noqa: E402
from linkerd_amd.engine import HistogramEngine  # noqa: E402

for S, n in ((1_000_000, 4_000_000), (100_000, 4_000_000)):
    eng = HistogramEngine(S)
    eng.set_param(N.PARAM_STAGE_SAMPLES, 0)
    s, v = synth.c3(S=S, N=n) if S == 1_000_000 else synth.c2(S=S, K=n // S)
    lib = N.load()
    out = (ctypes.c_ulonglong * 16)()
    rows, rs = [], []
    for it in range(4):
        eng.ingest(s, v)
        eng.sync()
        assert lib.l5dh_dev_phases_plan(out) == 0
        t = [out[k] for k in range(7)]
        rows.append([(t[k + 1] - t[k]) / 100.0 for k in range(6)])  # 100 MHz wall clock -> us
        u = [out[k] for k in range(8, 12)]
        rs.append([(u[k + 1] - u[k]) / 100.0 for k in range(3)])
    eng.close()
    r = np.array(rows[1:]).mean(0)
    print(f"S={S}: loads+clear {r[0]:.1f} us, histogram+thr {r[1]:.1f}, bitmap/sums {r[2]:.1f}, "
          f"scan+dlist {r[3]:.1f}, super-tile caps {r[4]:.1f}, rest {r[5]:.1f}, total {r.sum():.1f}")
    q = np.array(rs[1:]).mean(0)
    print(f"  k_rsample workgroup 0: LDS clear {q[0]:.1f} us, draws {q[1]:.1f}, flush {q[2]:.1f}")
