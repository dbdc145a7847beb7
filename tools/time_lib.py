"""Per-kernel device times (HIP events, L5DH_PARAM_TIMING) of one library build on a
bench workload, without result checks -- for timing-only development builds
(tools/mk_var.sh, L5DH_LIB=<lib>).  Development tool (GPU box).
  L5DH_LIB=... python tools/time_lib.py [--workload c3] [--steps 4]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    steps = 4
    argv = sys.argv[1:]
    if "--steps" in argv:
        i = argv.index("--steps")
        steps = int(argv[i + 1])
        del argv[i:i + 2]
    sys.argv = ["bench.py"] + argv
    args = bench.parse()
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
    for prm, v in ((N.PARAM_DIRECT_MAX, args.direct_max), (N.PARAM_DIRECT_DIV, args.direct_div)):
        if v is not None:
            eng.set_param(prm, v)
    summ = torch.empty((S, 11), dtype=torch.int64, device="cuda")
    counts = torch.empty((S, N.NBUCKETS), dtype=torch.int32, device="cuda")
    for k in range(3):
        eng.ingest(*batches[k % 2])
        eng.snapshot_into(summ, counts, reset=True)
    eng.set_param(N.PARAM_TIMING, 1)
    eng.kernel_times(reset=True)
    core = N.load()
    phases = [getattr(core, f"l5dh_dev_phases{i}", None) for i in (1, 2, 3)]  # (L5DH_PHASES builds)
    before = [snap_phases(f) for f in phases]
    for k in range(steps):
        eng.ingest(*batches[k % 2])
        eng.snapshot_into(summ, counts, reset=True)
    kt = eng.kernel_times(reset=True)
    tot = sum(ms for ms, n in kt.values() if n) / steps
    print(f"{os.path.basename(N.LIB_PATH)}: {tot:.4f} ms/step  " +
          "  ".join(f"{k} {ms / steps:.4f}" for k, (ms, n) in kt.items() if n), flush=True)
    for name, f, b in zip(("level1", "cold", "level2"), phases, before):
        if f is None:
            continue
        a = snap_phases(f)
        d = [[a[w][k] - b[w][k] for k in range(8)] for w in range(1024)]
        act = [x for x in d if x[7] > 0]
        if not act:
            continue
        # wall_clock64 runs at 100 MHz: ticks * 0.01 us; per launch, averaged over workgroups
        per = [sum(x[k] for x in act) / sum(x[7] for x in act) * 0.01 for k in range(7)]
        per = [v for v in per if v > 0] if name != "level1" else per
        print(f"  phases {name} ({len(act)} wgs, us per launch per wg): " +
              " ".join(f"p{k}={v:.1f}" for k, v in enumerate(per)), flush=True)


def snap_phases(f):
    if f is None:
        return None
    buf = (ctypes.c_ulonglong * (1024 * 8))()
    f(buf)
    return [[buf[w * 8 + k] for k in range(8)] for w in range(1024)]


if __name__ == "__main__":
    main()
