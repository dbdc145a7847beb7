"""Extract the child-key order of every node of the reference's tree-mode
/admin/metrics.json fixture (admin/src/main/resources/io/buoyant/admin/js/spec/
fixtures/metrics.js) -- the order the reference's MetricsTree.children produced.
Pins linkerd_amd.javamap.reference_child_order.  Run here (the reference is not on
the GPU box); output: tests/golden/metrics_key_order.json (key lists only).
"""
import json
import os

SRC = "/root/reference/admin/src/main/resources/io/buoyant/admin/js/spec/fixtures/metrics.js"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "metrics_key_order.json")


def main(src=SRC, out=OUT):
    text = open(src).read()
    body = text[text.index("return") + len("return"):]
    body = body[:body.rindex("}")]
    nodes = []

    def hook(pairs):
        kids = [k for k, v in pairs if isinstance(v, list) and v and v[0] == "__node__"]
        if len(kids) >= 2:
            nodes.append(kids)
        return ["__node__"]

    json.loads(body[: body.rindex("}") + 1], object_pairs_hook=hook)
    with open(out, "w") as f:
        json.dump({"source": "admin/src/main/resources/io/buoyant/admin/js/spec/fixtures/metrics.js",
                   "child_key_orders": nodes}, f, indent=0)
    print(f"wrote {len(nodes)} nodes to {out}")


if __name__ == "__main__":
    main()
