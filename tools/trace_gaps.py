"""Timeline of the engine's kernels in one bench step from a rocprofv3 kernel trace CSV:
start offset, duration and the idle gap before each dispatch, plus per-step totals of
busy time and gaps (development tool).  A step is taken to begin at each k_rsample (or
k_fold1) dispatch.  Usage: python tools/trace_gaps.py <run_kernel_trace.csv> [step]"""
import csv
import re
import sys


def main():
    path = sys.argv[1]
    rows = []
    for r in csv.DictReader(open(path)):
        m = re.search(r"k_[a-z0-9_]+", r["Kernel_Name"])
        name = m.group(0) if m else r["Kernel_Name"][:24]
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if r[2] in ("k_rsample", "k_fold1_init", "k_fold1")]
    steps = []
    for j, i in enumerate(starts):
        end = starts[j + 1] if j + 1 < len(starts) else len(rows)
        steps.append(rows[i:end])
    # engine kernels only (the bench's generator and torch kernels run outside the step)
    steps = [[r for r in s if r[2].startswith("k_") and r[2] != "k_gen_zipf"] for s in steps]
    pick = int(sys.argv[2]) if len(sys.argv) > 2 else len(steps) - 1
    s = steps[pick]
    t0 = s[0][0]
    prev = t0
    print(f"step {pick} of {len(steps)}: {len(s)} dispatches")
    for a, b, n in s:
        print(f"  {n:16s} start {(a - t0) / 1e3:9.1f} us  dur {(b - a) / 1e3:8.1f}  gap {(a - prev) / 1e3:6.1f}")
        prev = max(prev, b)
    for k, st in enumerate(steps):
        if not st:
            continue
        busy, cur_a, cur_b = 0, None, None  # union of the dispatches' intervals
        for a, b, _ in sorted(st):
            if cur_b is None or a > cur_b:
                if cur_b is not None:
                    busy += cur_b - cur_a
                cur_a, cur_b = a, b
            else:
                cur_b = max(cur_b, b)
        busy = (busy + cur_b - cur_a) / 1e3
        span = (max(b for _, b, _ in st) - st[0][0]) / 1e3
        print(f"step {k}: span {span:8.1f} us  busy {busy:8.1f}  idle {span - busy:6.1f}  dispatches {len(st)}")


if __name__ == "__main__":
    main()
