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


@pytest.mark.parametrize("dev_bufs", [True, False])
def test_export_reset_fused_matches_oracle(oracle, dev_bufs):
    """export_state(reset=True) over the whole series range runs as one aggregate
    pass into the caller's rows: kept state (dirty tiles), split/direct tiles of a
    Zipf head and pending segments must all land, and the state is clean after."""
    import torch
    from linkerd_amd.engine import HistogramEngine
    S = 5000
    o = oracle.OracleHistograms(S)
    eng = HistogramEngine(S)
    batches = [synth.c3(S=S, N=n, seed=31 + i) for i, n in enumerate((1_500_000, 1_200_000, 900_000))]
    eng.ingest(*batches[0])
    o.ingest(*batches[0])
    eng.snapshot(reset=False)  # folds into state: dirty tiles
    for b in batches[1:]:      # two pending segments, the second sized from the first
        eng.ingest(*b)
        o.ingest(*b)
    if dev_bufs:
        dev = torch.device("cuda", 0)
        c = torch.empty((S, N.NBUCKETS), dtype=torch.int32, device=dev)
        t = torch.empty(S, dtype=torch.int64, device=dev)
        eng.export_state(counts=c, totals=t, reset=True)
        torch.cuda.synchronize()
        counts, totals = c.cpu().numpy(), t.cpu().numpy()
    else:
        counts, totals = eng.export_state(reset=True)
    np.testing.assert_array_equal(counts, o.counts())
    np.testing.assert_array_equal(totals, o.totals())
    after = eng.snapshot(reset=False)
    assert not after["count"].any() and not after["sum"].any()
    # the engine keeps working from the clean state
    s2, v2 = synth.c3(S=S, N=300_000, seed=41)
    eng.ingest(s2, v2)
    o2 = oracle.OracleHistograms(S)
    o2.ingest(s2, v2)
    counts, totals = eng.export_state(reset=True)
    np.testing.assert_array_equal(counts, o2.counts())
    np.testing.assert_array_equal(totals, o2.totals())
    eng.close()
