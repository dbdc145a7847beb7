"""The C4 loopback step of one library build (L5DH_LIB=linkerd_amd/lib_ab/lib<name>.so): step
time, rank 0's kernel times and -- for an L5DH_PHASES build (tools/mk_var.sh <name>
-DL5DH_PHASES) -- per-phase device times.  Development tool (GPU box).
  L5DH_LIB=... python tools/phases_c4.py [--loopback 8] [--steps 3]"""
import ctypes
import io
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def snap(f):
    buf = (ctypes.c_ulonglong * (1024 * 8))()
    f(buf)
    return [[buf[w * 8 + k] for k in range(8)] for w in range(1024)]


def main():
    argv = sys.argv[1:]
    if "--loopback" not in argv:
        argv += ["--loopback", "8"]
    sys.argv = ["bench.py", "--workload", "c4", "--steps", "3", "--warmup", "1"] + argv
    args = bench.parse()
    from linkerd_amd import _native as N
    core = N.load()
    fns = [getattr(core, f"l5dh_dev_phases{i}", None) for i in (1, 2)]
    out = io.StringIO()
    bench.run_c4_loopback(args, out, check=False)
    import json
    d = json.loads(out.getvalue().strip().splitlines()[-1])
    print(f"{os.path.basename(N.LIB_PATH)}: C4 loopback {d['ms_per_step']} ms/step, per rank {d['config']['per_rank_ms']}: "
          f"{d['per_rank_kernels_ms'][0]}", flush=True)
    for name, f in zip(("level1", "cold"), fns):
        if f is None:
            continue
        d = snap(f)
        act = [x for x in d if x[7] > 0]
        if not act:
            continue
        per = [sum(x[k] for x in act) / sum(x[7] for x in act) * 0.01 for k in range(4)]
        print(f"  phases {name} ({len(act)} wgs, us per launch per wg): " +
              " ".join(f"p{k}={v:.1f}" for k, v in enumerate(per)), flush=True)


if __name__ == "__main__":
    main()
