"""Debug the loopback multi-rank merge (GPU box): which rank / rows / buckets differ."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

from linkerd_amd import _native as N, synth  # noqa: E402
from linkerd_amd.engine import HistogramEngine  # noqa: E402
from oracle import oracle as O  # noqa: E402


def run(W, heavy, mode=N.MERGE_REDUCE_SCATTER, S=4001):
    series, vals = synth.c3(S=S, N=300_000, seed=60 + 7 * W)
    parts = [(series[r::W], vals[r::W]) for r in range(W)]
    if heavy:
        parts[-1] = (np.concatenate([parts[-1][0], np.full(2_100_000, 17, np.uint32)]),
                     np.concatenate([parts[-1][1], np.full(2_100_000, 3.0, np.float32)]))
    # each rank's export alone
    for r, p in enumerate(parts):
        e = HistogramEngine(S)
        e.ingest(*p)
        c, t = e.export_state(reset=True)
        o = O.OracleHistograms(S)
        o.ingest(*p)
        bad = np.nonzero((c != o.counts()).any(axis=1))[0]
        print(f"W={W} heavy={heavy} rank {r} export: {bad.size} rows differ {bad[:8]}", flush=True)
        e.close()
    engines = [HistogramEngine(S) for _ in range(W)]
    HistogramEngine.comm_init_loopback(engines)
    for e, p in zip(engines, parts):
        e.ingest(*p)
    o = O.OracleHistograms(S)
    for p in parts:
        o.ingest(*p)
    wc = o.counts()
    res = HistogramEngine.merge_all(engines, mode, with_counts=True)
    for r, (f, cnt, summ, cc, tt) in enumerate(res):
        d = (cc != wc[f:f + cnt])
        rows = np.nonzero(d.any(axis=1))[0]
        print(f"  rank {r} slice [{f}, {f + cnt}): {rows.size} rows differ, first {rows[:10] + f}", flush=True)
        for row in rows[:3]:
            b = np.nonzero(d[row])[0]
            print(f"    series {row + f}: buckets {b[:8]} got {cc[row, b[:8]]} want {wc[f + row, b[:8]]}", flush=True)
        print("   merge bytes", engines[r].merge_bytes(), flush=True)
    for e in engines:
        e.close()


if __name__ == "__main__":
    for W in (2, 3):
        for heavy in (False, True):
            run(W, heavy)
