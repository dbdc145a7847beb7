"""Aggregate rocprofv3 --pmc CSVs (tools/profile_pmc.sh) per kernel: average value
of each counter per dispatch, HBM bytes per launch with the gfx950 corrections of
MI355X_MICROARCH.md (FETCH_SIZE counts half the bytes of wide streaming reads:
doubled; WRITE_SIZE taken as is; both in KB).  The first dispatch of each kernel
(no split set yet) is excluded when a kernel has >= 3 dispatches."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"k_[a-z0-9_]+", name)
    return m.group(0)[2:] if m else name[:40]


def main(d, out_json=None, meta=None):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r.get("Kernel_Name", ""))
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, cs in sorted(acc.items()):
        # steady state: the first dispatch of a kernel runs before the engine has
        # a split set (the previous batch's big tiles), so it is dropped when
        # there are >= 3 dispatches
        # dispatches that did (almost) nothing -- a redo pass that exits at once -- are
        # not launches of the work being measured: drop those under 2 % of the max
        def steady(v):
            v = v[1:] if len(v) >= 3 else v
            top = max(v) if v else 0.0
            w = [x for x in v if x >= 0.02 * top] or v
            return sum(w) / len(w)
        row = {c: steady(v) for c, v in cs.items()}
        if "FETCH_SIZE" in row or "WRITE_SIZE" in row:
            rd = 2 * 1024 * row.get("FETCH_SIZE", 0.0)
            wr = 1024 * row.get("WRITE_SIZE", 0.0)
            row["hbm_read_bytes_per_launch"] = rd
            row["hbm_write_bytes_per_launch"] = wr
            row["hbm_bytes_per_launch"] = rd + wr
        res[k] = row
    for k, row in res.items():
        print(k, json.dumps({c: (round(v / 1e6, 2) if "bytes" in c else round(v)) for c, v in row.items()}))
    if out_json:
        doc = dict(meta or {})
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
        from linkerd_amd._native import engine_source_hash
        doc["src_hash"] = engine_source_hash()  # bench.py marks the traffic stale when the sources change
        doc["kernels"] = res
        json.dump(doc, open(out_json, "w"), indent=1)


if __name__ == "__main__":
    meta = json.loads(sys.argv[3]) if len(sys.argv) > 3 else None
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None, meta)
