"""Interleaved A/B of engine variants inside one process (development tool).

Each variant is an L5DH_DBG value (read by l5dh_open) -- or "param=value,..."
engine parameters -- applied to its own context; the variants run the same C3
step (ingest + snapshot with reset) in turn, R rounds, and per-kernel-group
times (HIP events, the engine's timing mode) are reported as medians.

  python tools/ab_ctx.py --rounds 8 "0" "4194304" ["0;direct_max=64" ...]
"""
import argparse
import ctypes
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--samples", type=int, default=1_000_000_000)
    ap.add_argument("--series", type=int, default=1_000_000)
    a = ap.parse_args()
    import torch
    import bench
    from linkerd_amd import _native as N_
    from linkerd_amd.engine import HistogramEngine

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    synth_lib = ctypes.CDLL(os.path.join(REPO, "linkerd_amd", "lib", "libl5dsynth.so"))
    stream = torch.cuda.current_stream().cuda_stream
    S, N = a.series, a.samples
    series, values = bench.gen_inputs(torch, synth_lib, "c3", S, N, 0, stream)
    summ = torch.empty((S, 11), dtype=torch.int64, device=dev)
    counts = torch.empty((S, N_.NBUCKETS), dtype=torch.int32, device=dev)
    engines = []
    for v in a.variants:
        dbg, _, params = v.partition(";")
        os.environ["L5DH_DBG"] = dbg
        e = HistogramEngine(S, device=0)
        for kv in filter(None, params.split(",")):
            k, val = kv.split("=")
            e.set_param(getattr(N_, "PARAM_" + k.upper()), int(val))
        e.set_param(N_.PARAM_TIMING, 1)
        engines.append(e)
    os.environ.pop("L5DH_DBG", None)
    res = [dict() for _ in engines]
    for r in range(a.rounds + 1):
        for i, e in enumerate(engines):
            e.kernel_times(reset=True)
            e.ingest(series, values)
            e.snapshot_into(summ, counts, reset=True)
            torch.cuda.synchronize()
            kt = e.kernel_times(reset=True)
            if r == 0:
                continue  # warm-up round (first batch has no split set)
            tot = 0.0
            for name, (ms, launches) in kt.items():
                if launches:
                    res[i].setdefault(name, []).append(ms)
                    tot += ms
            res[i].setdefault("sum", []).append(tot)
    for v, rr in zip(a.variants, res):
        print(f"[{v}] " + " ".join(f"{k}={statistics.median(x):.3f}" for k, x in rr.items()), flush=True)


if __name__ == "__main__":
    main()
