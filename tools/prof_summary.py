"""Condense a rocprofv3 --kernel-trace --stats kernel_stats.csv into a short table
(kernel, calls, avg/min/max us, % of GPU time) for profiles/."""
import csv
import re
import sys


def short(name):
    m = re.search(r"\bk_[a-z0-9_]+", name)
    if m:
        return m.group(0)
    return name.split("(")[0].split("<")[0][:48]


def main(src, dst=None):
    rows = list(csv.DictReader(open(src)))
    lines = ["| kernel | calls | avg us | min us | max us | % time |", "|---|---:|---:|---:|---:|---:|"]
    for r in rows:
        lines.append(f"| {short(r['Name'])} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                     f"{float(r['MinNs']) / 1e3:.1f} | {float(r['MaxNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |")
    text = "\n".join(lines) + "\n"
    if dst:
        open(dst, "w").write(text)
    print(text, end="")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
