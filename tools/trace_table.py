"""Per-dispatch kernel durations (us) from a rocprofv3 kernel trace CSV, grouped by
kernel, in dispatch order.  Usage: python tools/trace_table.py <run_kernel_trace.csv>..."""
import collections
import csv
import re
import sys

for path in sys.argv[1:]:
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        m = re.search(r"k_[a-z0-9_]+", r["Kernel_Name"])
        if m:
            d[m.group(0)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(path)
    for k, v in sorted(d.items(), key=lambda x: -sum(x[1])):
        print(f"  {k:16s} n={len(v):3d} " + " ".join(f"{x:.0f}" for x in v[:16]))
