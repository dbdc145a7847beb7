"""Same-context A/B of kernel variants (L5DH_PARAM_VARIANT): one engine, the same
input buffers and scratch placement, variants interleaved step by step; per-kernel
device times (HIP events) per variant.  Development tool (GPU box).
  python tools/ab_var.py <variant bits B> [--workload c3] [--rounds 6] [--shard r/W]
Variant A is 0 (the default kernels)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("variant", type=int)
    p.add_argument("--workload", default="c3")
    p.add_argument("--shard", default=None)
    p.add_argument("--rounds", type=int, default=6)
    p.add_argument("--steps", type=int, default=3)
    a = p.parse_args()
    sys.argv = ["bench.py", "--workload", a.workload] + (["--shard", a.shard] if a.shard else [])
    args = bench.parse()
    import ctypes
    import torch
    from linkerd_amd import _native as N
    from linkerd_amd.engine import HistogramEngine
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    pl = bench.plan(args, 1, 0)
    lib = ctypes.CDLL(N.SYNTH_PATH)
    for fn in ("l5ds_gen_c1", "l5ds_gen_c2", "l5ds_gen_zipf"):
        getattr(lib, fn).restype = ctypes.c_int
    stream = torch.cuda.current_stream().cuda_stream
    batches = [bench.gen_batch(torch, lib, pl, k, stream) for k in range(2)]
    S = pl["count"]
    eng = HistogramEngine(S)
    eng.set_stream(stream)
    summ = torch.empty((S, 11), dtype=torch.int64, device="cuda")
    counts = torch.empty((S, N.NBUCKETS), dtype=torch.int32, device="cuda")
    k = 0

    def step():
        nonlocal k
        eng.ingest(*batches[k % 2])
        k += 1
        eng.snapshot_into(summ, counts, reset=True)

    for _ in range(3):
        step()
    eng.set_param(N.PARAM_TIMING, 1)
    acc = {0: {}, a.variant: {}}
    for r in range(a.rounds):
        for v in (0, a.variant) if r % 2 == 0 else (a.variant, 0):
            eng.set_param(N.PARAM_VARIANT, v)
            step()  # settle: the split set follows the previous batch
            eng.kernel_times(reset=True)
            for _ in range(a.steps):
                step()
            for name, (ms, n) in eng.kernel_times(reset=True).items():
                if n:
                    acc[v].setdefault(name, []).append(ms / a.steps)
    for v, d in acc.items():
        tot = sum(sum(x) / len(x) for x in d.values())
        print(f"variant {v}: total {tot:.4f} ms/step  " +
              "  ".join(f"{n} {sum(x) / len(x):.4f}" for n, x in sorted(d.items())), flush=True)


if __name__ == "__main__":
    main()
