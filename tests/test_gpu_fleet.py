"""GPU side of the fleet merge (C4) on one device: two engines hold disjoint sample
shards of the same series space; their exported dense state is summed on the GPU
(what the RCCL reduce-scatter does across GPUs; the collective itself is covered by
tests/test_fleet_gloo.py) and summarized with l5dh_summarize_dense."""
import numpy as np
import pytest

from linkerd_amd import synth
from linkerd_amd import _native as N

pytestmark = pytest.mark.gpu


def test_sample_sharded_merge_on_gpu(oracle):
    import torch
    from linkerd_amd.engine import HistogramEngine
    S, n = 3000, 400_000
    series, vals = synth.c3(S=S, N=n, seed=21)
    dev = torch.device("cuda", 0)
    counts = torch.zeros((S, N.NBUCKETS), dtype=torch.int32, device=dev)
    totals = torch.zeros(S, dtype=torch.int64, device=dev)
    for r in range(2):
        eng = HistogramEngine(S)
        m = np.arange(n) % 2 == r
        eng.ingest(series[m], vals[m])
        c = torch.empty_like(counts)
        t = torch.empty_like(totals)
        eng.export_state(counts=c, totals=t, reset=True)
        torch.cuda.synchronize()
        counts += c
        totals += t
        eng.close()
    eng = HistogramEngine(S)
    summ = torch.empty((S, 11), dtype=torch.int64, device=dev)
    eng.summarize_dense(counts, totals, out=summ)
    torch.cuda.synchronize()
    o = oracle.OracleHistograms(S)
    o.ingest(series, vals)
    np.testing.assert_array_equal(counts.cpu().numpy(), o.counts())
    assert summ.cpu().numpy().tobytes() == o.snapshot().tobytes()
