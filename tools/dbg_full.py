"""Full-size C3 check of the engine's dense rows against a torch ground truth
(bincount of series * 1798 + bucket, bucket = upper_bound(limits, (long)value)),
for several engine parameter settings.  Development tool (GPU box):
  python tools/dbg_full.py [N]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from linkerd_amd import _native as N, synth  # noqa: E402
from linkerd_amd.engine import HistogramEngine  # noqa: E402


def main():
    S = 1_000_000
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream().cuda_stream
    lib = ctypes.CDLL(N.SYNTH_PATH)
    lib.l5ds_gen_zipf.restype = ctypes.c_int
    series = torch.empty(n, dtype=torch.int32, device=dev)
    values = torch.empty(n, dtype=torch.float32, device=dev)
    cdf = torch.from_numpy(synth.zipf_cdf(S)).to(dev)
    assert lib.l5ds_gen_zipf(ctypes.c_void_p(series.data_ptr()), ctypes.c_void_p(values.data_ptr()),
                             ctypes.c_uint64(n), ctypes.c_uint64(S), ctypes.c_void_p(cdf.data_ptr()),
                             ctypes.c_uint64(3), ctypes.c_double(0.8), ctypes.c_uint64(0), ctypes.c_uint32(0),
                             ctypes.c_void_p(stream)) == 0
    torch.cuda.synchronize()
    lim = torch.from_numpy(N.limits().astype(np.int64)).to(dev)
    truth = torch.zeros(S * N.NBUCKETS, dtype=torch.int64, device=dev)
    step = 100_000_000
    for o in range(0, n, step):
        v = values[o:o + step].to(torch.int64)  # values in [0, 1e9]: (long)value
        b = torch.searchsorted(lim, v, right=True)
        truth += torch.bincount(series[o:o + step].long() * N.NBUCKETS + b, minlength=S * N.NBUCKETS)
    truth = truth.view(S, N.NBUCKETS).to(torch.int32)
    print("truth ready", int(truth.sum()), flush=True)
    rows = torch.empty((S, N.NBUCKETS), dtype=torch.int32, device=dev)
    summ = torch.empty((S, 11), dtype=torch.int64, device=dev)
    settings = [("default", {}), ("hot_chunk=16384", {N.PARAM_HOT_CHUNK: 16384}),
                ("direct_max=0", {N.PARAM_DIRECT_MAX: 0}), ("region_pct=40", {N.PARAM_REGION_PCT: 40}),
                ("variant=4", {N.PARAM_VARIANT: 4}), ("variant=8", {N.PARAM_VARIANT: 8}),
                ("variant=12", {N.PARAM_VARIANT: 12}), ("variant=12,region_pct=40", {N.PARAM_VARIANT: 12, N.PARAM_REGION_PCT: 40}), ("variant=8,region_pct=40", {N.PARAM_VARIANT: 8, N.PARAM_REGION_PCT: 40})]
    if len(sys.argv) > 2:
        settings = [x for x in settings if x[0] in sys.argv[2].split(";")]
    for name, prm in settings:
        eng = HistogramEngine(S)
        for k, v in prm.items():
            eng.set_param(k, v)
        for rep in range(2):  # the second batch plans from the first's exact counts
            eng.ingest(series, values)
            eng.snapshot_into(summ, rows, reset=True)
            torch.cuda.synchronize()
            bad = (rows != truth).any(dim=1)
            nb = int(bad.sum())
            msg = f"{name} rep {rep}: {nb} series differ"
            if nb:
                idx = torch.nonzero(bad).flatten()[:8].tolist()
                tiles = sorted(set(i // 32 for i in idx))
                d = (rows[idx[0]].long() - truth[idx[0]].long())
                msg += f"; first {idx}; tiles {tiles}; row {idx[0]}: got {int(rows[idx[0]].sum())} want " \
                       f"{int(truth[idx[0]].sum())}, diff buckets {torch.nonzero(d).flatten()[:6].tolist()}"
            print(msg, flush=True)
        eng.close()


if __name__ == "__main__":
    main()
