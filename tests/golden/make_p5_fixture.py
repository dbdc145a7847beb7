"""Extract the P5 pin from the reference's own admin-dashboard
fixture: every histogram summary recorded in tree-mode /admin/metrics.json
output (admin/src/main/resources/io/buoyant/admin/js/spec/fixtures/metrics.js).

The fixture holds only summaries (raw samples are unknown), so it pins the
summary *invariants*: min/max/percentiles are bucket midpoints, avg == sum/count
as a Java double, count/sum consistency.  Run here (the reference is not on the
GPU box); output: tests/golden/p5_fixture_summaries.json (data only).
"""
import json
import os
import re
import sys

SRC = "/root/reference/admin/src/main/resources/io/buoyant/admin/js/spec/fixtures/metrics.js"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "p5_fixture_summaries.json")
OUT_TEXTS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "p5_number_texts.json")
# every non-integral number literal of the fixture, as the JVM printed it (JDK 8
# Double.toString for stat.avg, Float.toString for gauges; the fixture spells the
# exponent "E+12" where the JVM wrote "E12")
NUM_RE = re.compile(r'"([^"]*)"\s*:\s*(-?[0-9][0-9.]*(?:E[-+]?[0-9]+)?)\s*[,}\n]')


def main(src=SRC, out=OUT):
    text = open(src).read()
    body = text[text.index("return") + len("return"):]
    body = body[:body.rindex("}")]  # drop trailing ");" of define(...)
    tree = json.loads(body[: body.rindex("}") + 1])
    rows = []

    def walk(node, path):
        if isinstance(node, dict):
            if "stat.count" in node:
                rows.append({"path": "/".join(path), **{k[5:]: node[k] for k in node if k.startswith("stat.")}})
            for k, v in node.items():
                if isinstance(v, dict):
                    walk(v, path + [k])

    walk(tree, [])
    with open(out, "w") as f:
        json.dump({"source": "admin/src/main/resources/io/buoyant/admin/js/spec/fixtures/metrics.js",
                   "summaries": rows}, f, indent=1, sort_keys=True)
    print(f"wrote {len(rows)} summaries to {out}")
    texts = [{"key": k, "text": v} for k, v in NUM_RE.findall(text) if "." in v or "E" in v]
    with open(OUT_TEXTS, "w") as f:
        json.dump({"source": "admin/src/main/resources/io/buoyant/admin/js/spec/fixtures/metrics.js",
                   "note": "raw number texts (JDK 8 output) of stat.avg and gauge entries",
                   "texts": texts}, f, indent=0)
    print(f"wrote {len(texts)} number texts to {OUT_TEXTS}")


if __name__ == "__main__":
    main(*sys.argv[1:])
