"""Streaming ceilings of one MI355X for the byte counts of a C3 step (development tool).

Times, with HIP events on torch's stream, the plain streams the engine's phases are
compared with in DESIGN.md §4/§6:
  * write-only: a 7.19 GB int32 fill (the dense rows of 1 M series x 1798 buckets);
  * read-only:  an 8 GB int32 sum (the batch: 1e9 x (u32 id + f32 value));
  * copy:       8 GB read + 8 GB written.
Prints one JSON line.  Usage: python tools/hbm_ceiling.py [--reps 10]
"""
import argparse
import json

import torch


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    tot = 0.0
    for _ in range(reps):
        a.record()
        fn()
        b.record()
        b.synchronize()
        t = a.elapsed_time(b)
        best = min(best, t)
        tot += t
    return best, tot / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    out = {}
    rows = torch.empty(1_000_000 * 1798, dtype=torch.int32, device=dev)
    wb = rows.numel() * 4
    best, avg = timed(lambda: rows.fill_(1), args.reps)
    out["write_fill"] = {"bytes": wb, "best_ms": best, "avg_ms": avg, "TBps_best": wb / best / 1e9}
    del rows
    batch = torch.ones(2_000_000_000, dtype=torch.int32, device=dev)
    rb = batch.numel() * 4
    best, avg = timed(lambda: batch.sum(), args.reps)
    out["read_sum"] = {"bytes": rb, "best_ms": best, "avg_ms": avg, "TBps_best": rb / best / 1e9}
    dst = torch.empty_like(batch)
    best, avg = timed(lambda: dst.copy_(batch), args.reps)
    out["copy"] = {"bytes": 2 * rb, "best_ms": best, "avg_ms": avg, "TBps_best": 2 * rb / best / 1e9}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
