"""Benchmark of the histogram hot path (BASELINE.json metric).

One step = one snapshot interval of the reference's Metric.Stat path: ingest a
batch of (series u32, value f32) samples already resident in HBM (Metric.Stat.add,
batched) and snapshot + reset every series into dense int32 bucket counts and
88-byte HistogramSummary records (snapshotHistograms,
AdminMetricsExportTelemeter.scala:154-162).  Steps rotate over --rotate batches
drawn with different seeds, so the engine's split/direct-tile choice (made from
the previous batch) is tested on a batch it has not seen.

Workloads (synthetic inputs generated on the GPU):
  c3 (default)  1M series, 1e9 samples per step in total, Zipf(s=1) series ids,
                log-normal values.  With N ranks the series space is split into
                contiguous ranges of equal modelled device time (fleet.plan_shards:
                a per-sample + per-series cost model over the per-tile load) and
                each rank ingests the samples of its range: series-sharded, no
                collective, strong scaling.
  c4            fleet merge: the same 1M series, the 1e9 samples sample-sharded
                over the ranks; each rank ingests its share and calls l5dh_merge
                (sparse export + RCCL exchange + dense rows and summaries of its
                slice).  `--loopback W` runs the whole W-rank merge on this one GPU: W
                contexts, each ingesting its share, merged through l5dh_merge_all over
                the loopback transport (device copies instead of xGMI) -- every rank's
                work; ms_per_step / W is a one-GPU per-rank estimate WITHOUT the
                interconnect (a modelled xGMI term is reported beside it).
  c2            100k series x 1k samples on one GPU (replicas when N > 1).
  c1            1 series x 1e7 samples (replicas when N > 1).
--piece P streams the batch from pinned host memory in P-sample l5dh_ingest
calls (the JNI staging shape; PCIe-inclusive), instead of HBM-resident batches.

Launch: `python bench.py --gpus N` spawns N ranks itself (torch.distributed.run,
before any GPU call); under torchrun (WORLD_SIZE set) it is one rank.  Rank 0
prints ONE JSON line: `value` = samples/s over all ranks (max-over-ranks time);
`roofline` = the dominant kernel's algorithmic bytes / its
average duration (HIP events on the engine's stream); `path_roofline` = B_alg
(8 B/sample + 7280 B/series) / ms_per_step -- the headline fraction;
`cpu_baseline` = the C oracle (restatement of the JVM path) on host cores.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import platform
import shutil
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
XGMI_LINK_GBS = 153.0  # one MI355X xGMI link (7 per GPU, a full mesh on an 8-GPU node); C4 loopback model only
S_C3, N_C3 = 1_000_000, 1_000_000_000
# algorithmic bytes per launch: 8 B per sample read once, 7192 B of
# final counts + 88 B of summary written once per series; partition / sort passes,
# zeroing and re-reads of records are not credited
KERNEL_ALG_BYTES = {
    "bin1": lambda n, s, fleet: 8 * n,                         # reads (series, value) once
    "accum": lambda n, s, fleet: (7192 if fleet else 7280) * s,  # writes counts (+ summary)
}
# the engine's timed phases (l5dh_kernel_time ids) -> the default build's kernels in the PMC
# summary whose per-launch bytes add up to the phase (the two accumulate kernels run
# side by side: one launch of each per snapshot)
# (the accumulate phase's timer spans k_hot_finish too: it runs under the cold kernel)
PMC_KERNELS = {"bin1": ["rbin1w"], "bin2": ["rbin2"], "accum": ["accum_cold_h", "accum_split", "hot_finish"]}
METRIC = "histogram samples ingested+summarized/sec (1M series) and % HBM peak"
# device cost model of one step on MI355X for the C3 shard plan (fleet.CostModel): one
# per-sample, per-series and fold cost for any series / sample count, fitted to the
# measured single-GPU steps; the plan is derived from per-tile loads
# (fleet.plan_shards) -- here the workload's expected load, in a fleet the previous
# interval's l5dh_tile_totals
# fleet.CostModel fitted by tools/fit_cost.py to the round-5 8-way shard sweep + the C3/C2/C1
# lines at the same sources (profiles/r05_shard_sweep_fit.txt: 11 lines, every one within 3.1 %)
C3_COST = dict(per_sample=3.11e-09, per_series=1.13e-06, per_sample_fold=2.55e-09, fixed=0.168,
               per_sample_l2=2.51e-09, per_sample_hot=5.3e-10, fixed_fold=0.0368)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--workload", choices=["c3", "c2", "c1", "c4"], default="c3")
    p.add_argument("--rotate", type=int, default=3, help="distinct batches (seeds) cycled over the steps")
    p.add_argument("--hot-shift", action="store_true",
                   help="c3/c4: batch k's series ids rotated by k/rotate of the range, so the hot set moves every step")
    p.add_argument("--piece", type=int, default=0, help="stream from pinned host memory in calls of this many samples")
    p.add_argument("--shard", default=None, help="r/W: run rank r's C3 shard of a W-way split on this one GPU")
    p.add_argument("--series", type=int, default=None, help="series (default: workload's)")
    p.add_argument("--samples", type=int, default=None, help="samples per step in total (default: workload's)")
    p.add_argument("--region-pct", type=int, default=None, help="engine param: region capacity percent (redo path below 100)")
    p.add_argument("--direct-max", type=int, default=None, help="engine param: direct tiles (0..255)")
    p.add_argument("--direct-div", type=int, default=None, help="engine param: direct-tile run divisor")
    p.add_argument("--variant", type=int, default=0, help="engine param L5DH_PARAM_VARIANT (A/B timing; 0: default)")
    p.add_argument("--first-interval", action="store_true",
                   help="plan every batch's partition regions as a first interval does (from its sample alone: "
                        "variant bit 2)")
    p.add_argument("--hot-chunk", type=int, default=None, help="engine param L5DH_PARAM_HOT_CHUNK (records per big-tile item)")
    p.add_argument("--cpu-sample", type=int, default=None, help="samples in the CPU baseline sample (0: skip)")
    p.add_argument("--cpu-threads", type=int, default=None, help="oracle threads (default: c1 1, else the host's)")
    p.add_argument("--pmc-json", default=os.path.join(REPO, "profiles", "pmc_latest.json"))
    p.add_argument("--dry-run", action="store_true", help="ranks + shard plan only (gloo, no GPU, no engine)")
    p.add_argument("--loopback", type=int, default=0,
                   help="c4: the whole W-rank fleet merge on this GPU (W contexts, loopback transport)")
    return p.parse_args()


# ---------------------------------------------------------------- launch
def spawn(args) -> int:
    """--gpus N without torchrun: start N ranks as children of this process (which
    never touches the GPU) and exit with their status."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


# ---------------------------------------------------------------- workload plan
def plan(args, world: int, rank: int) -> dict:
    """What this rank ingests per step: series range / count, samples, generator
    parameters.  Pure host arithmetic (no GPU)."""
    import numpy as np
    from linkerd_amd import fleet, synth
    wl = args.workload
    if args.shard:
        rank, world = (int(x) for x in args.shard.split("/"))
    if wl in ("c3", "c4"):
        S = args.series or S_C3
        N = args.samples or N_C3
        cdf = synth.zipf_cdf(S)
        if wl == "c4":  # sample-sharded: every rank the whole series space
            n = N // world + (1 if rank < N % world else 0)
            base = rank * (N // world) + min(rank, N % world)
            return dict(workload=wl, S_total=S, N_total=N, first=0, count=S, samples=n, base_index=base,
                        world=world, rank=rank, scaling="strong")
        # balanced by modelled device time over the per-tile load (balancing by samples
        # alone would leave the last rank most of the dense series rows)
        shards = shard_plan(S, N, world, cdf)
        sh = shards[rank]
        mass = [float(cdf[x.first + x.count - 1] - (cdf[x.first - 1] if x.first else 0.0)) if x.count else 0.0
                for x in shards]
        ns = [int(round(N * m)) for m in mass]
        ns[-1] = N - sum(ns[:-1])
        base = sum(ns[:rank])
        return dict(workload=wl, S_total=S, N_total=N, first=sh.first, count=sh.count, samples=ns[rank],
                    base_index=base, world=world, rank=rank, scaling="strong",
                    shard_samples=ns, shard_series=[x.count for x in shards])
    if wl == "c2":
        S, N = args.series or 100_000, args.samples or 100_000_000
    else:
        S, N = args.series or 1, args.samples or 10_000_000
    return dict(workload=wl, S_total=S * world, N_total=N * world, first=rank * S, count=S, samples=N,
                base_index=0, world=world, rank=rank, scaling="weak")


def expected_tile_load(cdf, N):
    """Samples per 32-series tile the Zipf workload puts on each tile (its expected
    load: what l5dh_tile_totals reports for a batch, up to sampling noise)."""
    import numpy as np
    S = cdf.size
    c = np.concatenate([[0.0], cdf])
    edges = np.minimum(np.arange(0, S + 32, 32), S)
    edges = np.unique(edges)
    return N * np.diff(c[edges])


def shard_plan(S, N, world, cdf):
    """C3 series ranges of equal modelled device time (fleet.plan_shards over the
    expected per-tile load, fleet.CostModel C3_COST)."""
    from linkerd_amd import fleet
    return fleet.plan_shards(expected_tile_load(cdf, N), S, world, fleet.CostModel(**C3_COST))


def gen_batch(torch, synth_lib, pl, seed_off, stream):
    """One batch of this rank's samples in HBM (l5dh_synth.hip, the synth.py recipe)."""
    import numpy as np
    from linkerd_amd import synth
    dev = torch.device("cuda", torch.cuda.current_device())
    n = pl["samples"]
    series = torch.empty(max(n, 1), dtype=torch.int32, device=dev)[:n]
    values = torch.empty(max(n, 1), dtype=torch.float32, device=dev)[:n]
    sp, vp = ctypes.c_void_p(series.data_ptr()), ctypes.c_void_p(values.data_ptr())
    wl = pl["workload"]
    if wl in ("c3", "c4"):
        cdf = synth.zipf_cdf(pl["S_total"])
        f, c = pl["first"], pl["count"]
        lo = cdf[f - 1] if f else 0.0
        sub = (cdf[f:f + c] - lo) / (cdf[f + c - 1] - lo)  # Zipf restricted to this rank's range
        sub[-1] = 1.0
        dcdf = torch.from_numpy(np.ascontiguousarray(sub)).to(dev)
        rc = synth_lib.l5ds_gen_zipf(sp, vp, ctypes.c_uint64(n), ctypes.c_uint64(c), ctypes.c_void_p(dcdf.data_ptr()),
                                     ctypes.c_uint64(3 + seed_off), ctypes.c_double(0.8),
                                     ctypes.c_uint64(pl["base_index"]), ctypes.c_uint32(f), ctypes.c_void_p(stream))
    elif wl == "c2":
        S = pl["count"]
        rc = synth_lib.l5ds_gen_c2(sp, vp, ctypes.c_uint64(S), ctypes.c_uint64(n // S), ctypes.c_uint64(2 + 16 * seed_off),
                                   ctypes.c_double(0.8), ctypes.c_uint32(pl["first"]), ctypes.c_void_p(stream))
    else:
        rc = synth_lib.l5ds_gen_c1(vp, sp, ctypes.c_uint64(n), ctypes.c_uint64(1 + pl["rank"] + 16 * seed_off),
                                   ctypes.c_void_p(stream))
    assert rc == 0, "synthetic generator launch failed"
    torch.cuda.synchronize()
    return series, values


# ---------------------------------------------------------------- baselines / profiles
def host_cpu():
    model = platform.processor() or ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    nproc = os.cpu_count() or 1
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = nproc
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)  # the GPU box's CPU share per GPU
    return model, nproc, avail, (min(avail, share) if share > 0 else avail)


def java_probe() -> str:
    j = shutil.which("java")
    if not j:
        return "absent (no `java` on PATH): the JVM reference path cannot run; the C restatement is timed instead"
    try:
        r = subprocess.run([j, "-version"], capture_output=True, text=True, timeout=20)
        return (r.stderr or r.stdout).strip().splitlines()[0]
    except Exception as e:  # noqa: BLE001
        return f"java present but -version failed: {e}"


def cpu_baseline(pl, sample, thread_counts):
    """C oracle (restatement of the JVM Metric.Stat path: per-series mutex, binary
    search, int32[1798] per series, 8-scan summary) on the same recipe: `sample`
    samples ingested with each thread count of `thread_counts` (a thread takes a
    contiguous slice of the COO stream and locks the series of each sample, as the
    Finagle worker threads lock each Stat, Metric.scala:30-33), then all series
    snapshot on ONE thread (the timer thread, AdminMetricsExportTelemeter.scala:154-162).
    A sample smaller than the step is extrapolated to one full step (said so in
    `sample`).  The fastest thread count is the headline `value` (with every core, the
    per-series locks contend on the Zipf head series: C3 is 10x slower at 256 threads
    than at 16); every count is listed in `by_threads`."""
    from linkerd_amd import synth
    from oracle import oracle as O
    wl, S, N = pl["workload"], pl["count"], pl["samples"]
    n = min(sample, N)
    if wl in ("c3", "c4"):
        s, v = synth.c3(S=S, N=n)
    elif wl == "c2":
        s, v = synth.c2(S=S, K=max(1, n // S))
        n = s.size
    else:
        s, v = synth.c1(n=n)
    runs = []
    for threads in thread_counts:
        h = O.OracleHistograms(S)
        h.ingest(s[: min(n, 100_000)], v[: min(n, 100_000)], threads=threads)  # first-touch warmup
        h = O.OracleHistograms(S)
        t0 = time.perf_counter()
        assert h.ingest(s, v, threads=threads) == 0
        t_ing = time.perf_counter() - t0
        t0 = time.perf_counter()
        h.snapshot(reset=True)
        t_snap = time.perf_counter() - t0
        full = t_ing * (N / n) + t_snap
        del h
        runs.append({"threads": threads, "value": N / full, "ingest_s": round(t_ing, 3), "snapshot_s": round(t_snap, 3)})
    best = max(runs, key=lambda r: r["value"])  # the fastest thread count (per-series locks contend on Zipf heads)
    model, nproc, avail, share = host_cpu()
    extra = "" if n == N else f", extrapolated to {N} samples/step"
    return {"value": best["value"], "unit": "samples/s", "cores": best["threads"], "kind": "port",
            "sample": (f"{wl} recipe, {n} samples ingested with " + " / ".join(f"{r['threads']}" for r in runs) +
                       f" thread(s) + snapshot of all {S} series on 1 thread{extra}"),
            "by_threads": runs, "cpu_model": model, "nproc": nproc, "cpus_available": avail, "cpu_share": share,
            "java": java_probe(),
            "note": "C restatement of the JVM path (oracle/hist_oracle.c); no JDK/finagle-stats jar on the box"}


def load_pmc_traffic(path, pl):
    """HBM bytes per launch from a committed PMC summary (tools/profile_pmc.sh +
    tools/pmc_summary.py) of the same workload and the same engine sources."""
    from linkerd_amd._native import engine_source_hash
    try:
        pm = json.load(open(path))
    except (OSError, ValueError):
        return {}, "no PMC summary"
    if pm.get("workload") != pl["workload"] or pm.get("series") != pl["count"] or pm.get("samples") != pl["samples"]:
        return {}, "PMC summary is of another workload"
    if pm.get("src_hash") != engine_source_hash():
        return {}, "stale: PMC summary measured other engine sources (re-run tools/profile_pmc.sh)"
    ks = pm.get("kernels", {})
    out = {name: int(sum(ks[p]["hbm_bytes_per_launch"] for p in ps)) for name, ps in PMC_KERNELS.items()
           if all(p in ks and "hbm_bytes_per_launch" in ks[p] for p in ps)}
    return out, f"PMC {os.path.basename(path)} (src {pm['src_hash']})"


# ---------------------------------------------------------------- main
def result_stream():
    """The result line's stream: a duplicate of stdout, while fd 1 itself is pointed at
    stderr, so that library banners (RCCL prints its version block on stdout when a
    communicator is created) never mix with the ONE JSON line."""
    out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    return out


def run_c4_loopback(args, result_out, check=True):
    """C4 on one GPU: the W ranks of a sample-sharded fleet as W contexts of this
    device, each ingesting its share of the 1e9 samples, merged by l5dh_merge_all over
    the loopback transport (l5dh_comm_init_loopback: the same encode / size / payload /
    decode steps as RCCL, the exchange by device copies).  A step is the whole fleet's
    work: every rank's ingest, sparse export, exchange, and the dense rows + summaries
    of every slice (device outputs).  Per-rank time = ms_per_step / W (the ranks' work
    is serialized on this GPU); B_alg = 8 N + 7280 S for the fleet, once."""
    import torch
    from linkerd_amd import _native as N_
    from linkerd_amd.engine import HistogramEngine
    W = args.loopback
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    synth_lib = ctypes.CDLL(N_.SYNTH_PATH)
    synth_lib.l5ds_gen_zipf.restype = ctypes.c_int
    plans = [plan(args, W, r) for r in range(W)]
    S, Ntot = plans[0]["count"], plans[0]["N_total"]
    batches = [gen_batch(torch, synth_lib, p, 0, stream) for p in plans]
    engines = [HistogramEngine(S, device=0) for _ in range(W)]
    for e in engines:
        e.set_stream(stream)
    HistogramEngine.comm_init_loopback(engines)
    rows = engines[0].merge_rows(N_.MERGE_REDUCE_SCATTER)
    summ = [torch.empty((rows, 11), dtype=torch.int64, device=dev) for _ in range(W)]
    cnts = [torch.empty((rows, N_.NBUCKETS), dtype=torch.int32, device=dev) for _ in range(W)]
    lib = N_.load()
    ctxs = (ctypes.c_void_p * W)(*[e._ctx.value for e in engines])
    o_arr = (ctypes.c_void_p * W)(*[t.data_ptr() for t in summ])
    c_arr = (ctypes.c_void_p * W)(*[t.data_ptr() for t in cnts])
    firsts, counts = (ctypes.c_uint32 * W)(), (ctypes.c_uint32 * W)()

    def step():
        for e, b in zip(engines, batches):
            e.ingest(*b)
        rc = lib.l5dh_merge_all(ctxs, W, N_.MERGE_REDUCE_SCATTER, o_arr, c_arr, None, firsts, counts)
        if rc != 0:
            engines[0]._check(rc, "l5dh_merge_all")

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if check:  # (tools/phases_c4.py times development builds whose results are not checked)
        got = sum(int(summ[r][:counts[r], 0].sum()) for r in range(W))
        assert got == Ntot, f"summary counts sum {got} != {Ntot}"
        assert sum(int(cnts[r][:counts[r]].sum(dtype=torch.int64)) for r in range(W)) == Ntot
    for e in engines:
        e.set_param(N_.PARAM_TIMING, 1)
        e.kernel_times(reset=True)
    tsteps = 3
    for _ in range(tsteps):
        step()
    per_rank = []
    for e in engines:
        kt = e.kernel_times(reset=True)
        per_rank.append({k: round(ms / tsteps, 4) for k, (ms, n) in kt.items() if n})
        e.set_param(N_.PARAM_TIMING, 0)
    mb = [e.merge_bytes() for e in engines]
    ms = elapsed / args.steps * 1e3
    # what the device copies stand in for: each rank's slices to the W-1 others over its
    # own xGMI links in parallel (a full mesh: one link per peer), at XGMI_LINK_GBS each
    xgmi_ms = max(m["sent"] for m in mb) / max(1, W - 1) / (XGMI_LINK_GBS * 1e9) * 1e3
    balg = 8 * Ntot + 7280 * S
    path_gbs = balg / (ms * 1e-3) / 1e9
    line = {
        "metric": METRIC, "value": Ntot * args.steps / elapsed, "unit": "samples/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": "C4: fleet merge, 1M series, 1e9 Zipf(s=1) samples per step sample-sharded over "
                               f"{W} ranks, all {W} ranks on this one GPU (l5dh_comm_init_loopback)",
                   "series_total": S, "samples_per_step": Ntot, "ranks": W,
                   "step": "every rank: ingest + sparse export; exchange (device copies); every slice's dense rows "
                           "+ summaries",
                   "per_rank_ms_loopback": round(ms / W, 4),
                   "per_rank_ms_note": "ms_per_step / W with the ranks serialized on one GPU and the exchange done "
                                       "by same-device copies: a one-GPU estimate of a rank's device time that "
                                       "EXCLUDES the interconnect; modelled_xgmi_ms is a model of that term, not "
                                       "a measurement",
                   "modelled_xgmi_ms": round(xgmi_ms, 4),
                   "modelled_xgmi": f"largest per-rank sent bytes / (W-1) links / {XGMI_LINK_GBS} GB/s per link "
                                    "(ideal links, no receive-side contention)",
                   # the explicit sum: measured one-GPU rank time + the modelled interconnect term
                   # (a model: not a fleet measurement)
                   "per_rank_ms_loopback_plus_modelled_xgmi": round(ms / W + xgmi_ms, 4)},
        "path_roofline": {"bound": "hbm", "achieved": round(path_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": round(path_gbs / HBM_PEAK_GBS, 4), "alg_bytes_per_step": balg,
                          "formula": "8 B/sample + 7280 B/series for the fleet, once (SURVEY.md §8d)"},
        "per_rank_kernels_ms": per_rank,
        "merge": {"encoded_bytes": [m["encoded"] for m in mb], "sent_bytes": [m["sent"] for m in mb],
                  "dense_bytes_per_rank": mb[0]["dense"] * (W - 1) // W,
                  "note": "sent = what a rank sends the other W-1 ranks (sparse); dense = the dense rows + totals "
                          "a dense reduce-scatter would send"},
        "roofline": None, "cpu_baseline": None,
    }
    print(json.dumps(line), file=result_out, flush=True)
    for e in engines:
        e.close()


def run(args):
    result_out = result_stream()
    if args.workload == "c4" and args.shard:
        sys.exit("bench.py: --shard is a C3 series shard; for the W-rank C4 fleet on one GPU use --loopback W")
    if args.workload == "c4" and args.loopback:
        return run_c4_loopback(args, result_out)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    import torch
    import torch.distributed as dist

    pl = plan(args, world, rank)
    if args.dry_run:  # the rank harness without a device (CPU tests)
        if distributed:
            dist.init_process_group("gloo")
            plans = [None] * world
            dist.all_gather_object(plans, pl)
        else:
            plans = [pl]
        if rank == 0:
            print(json.dumps({"dry_run": True, "world": world, "plans": plans}), file=result_out, flush=True)
        if distributed:
            dist.destroy_process_group()
        return

    # L5DH_BENCH_BACKEND=gloo: the rank harness over gloo with ranks sharing the GPUs
    # there are (a 1-GPU rehearsal of the multi-rank C3 path; the driver's runs use RCCL)
    backend = os.environ.get("L5DH_BENCH_BACKEND", "nccl")
    if distributed:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        gpu = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(gpu)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    coll_dev = dev if backend == "nccl" else torch.device("cpu")  # where reductions run
    # one non-default stream for the generator, torch and the engine (l5dh_set_stream):
    # device inputs and outputs are then stream ordered, no host wait per ingest
    torch.cuda.set_stream(torch.cuda.Stream())

    from linkerd_amd import _native as N_
    from linkerd_amd.engine import HistogramEngine
    synth_lib = ctypes.CDLL(N_.SYNTH_PATH)
    for fn in ("l5ds_gen_c1", "l5ds_gen_c2", "l5ds_gen_zipf"):
        getattr(synth_lib, fn).restype = ctypes.c_int

    stream = torch.cuda.current_stream().cuda_stream
    fleet = pl["workload"] == "c4"
    streaming = args.piece > 0
    R = 1 if streaming else max(1, args.rotate)
    batches = [gen_batch(torch, synth_lib, pl, k, stream) for k in range(R)]
    if args.hot_shift and pl["workload"] in ("c3", "c4"):
        # a moving hot set: the split / direct tiles chosen from the previous batch are
        # the wrong ones (untimed: ids rotated within the rank's range before the run)
        f, c = pl["first"], pl["count"]
        for k, (sr, _) in enumerate(batches):
            if k:
                sr.copy_(((sr.long() - f + k * c // R) % c + f).to(torch.int32))
        torch.cuda.synchronize()
    S = pl["count"]
    n = pl["samples"]

    eng = HistogramEngine(S, device=torch.cuda.current_device())
    for prm, v in ((N_.PARAM_DIRECT_MAX, args.direct_max), (N_.PARAM_DIRECT_DIV, args.direct_div),
                   (N_.PARAM_REGION_PCT, args.region_pct),
                   (N_.PARAM_VARIANT, (args.variant | (4 if args.first_interval else 0)) or None),
                   (N_.PARAM_HOT_CHUNK, args.hot_chunk)):
        if v is not None:
            eng.set_param(prm, v)
    if fleet:
        if distributed:
            obj = [HistogramEngine.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            eng.comm_init_rank(obj[0], world, rank)
        else:
            eng.comm_init_rank(HistogramEngine.comm_unique_id(), 1, 0)
            # one rank: run the sparse exchange (encode, RCCL send/recv to itself, decode)
            # instead of skipping it, so its bytes and time are measured
            eng.set_param(N_.PARAM_MERGE_RCCL_1RANK, 1)
    rows = eng.merge_rows() if fleet else S
    summ = torch.empty((max(rows, 1), 11), dtype=torch.int64, device=dev)
    counts = None if fleet else torch.empty((max(S, 1), N_.NBUCKETS), dtype=torch.int32, device=dev)
    eng.set_stream(stream)

    host = None
    if streaming:  # the batch in pinned host memory (l5dh_pin_alloc, what the JNI side stages into)
        lib = N_.load()
        hs, hv = ctypes.c_void_p(), ctypes.c_void_p()
        assert lib.l5dh_pin_alloc(max(n, 1) * 4, ctypes.byref(hs)) == 0
        assert lib.l5dh_pin_alloc(max(n, 1) * 4, ctypes.byref(hv)) == 0
        for dst, src in zip((hs, hv), batches[0]):
            h = src.cpu().numpy()  # keep the host copy alive across the memmove
            ctypes.memmove(dst, h.ctypes.data, n * 4)
            del h
        host = (lib, hs.value, hv.value)
        batches = [None]

    state = {"k": 0, "merged": None}

    def step():
        b = batches[state["k"] % R]
        state["k"] += 1
        if host:
            # the JNI staging shape: piece after piece of pinned host memory through
            # l5dh_ingest_async, double-buffered (the call two back is waited for
            # before the next one, as a thread refilling two staging buffers does)
            lib, hs, hv = host
            tk = ctypes.c_uint64(0)
            tickets = []
            for off in range(0, n, args.piece):
                m = min(args.piece, n - off)
                if len(tickets) >= 2:
                    eng._check(lib.l5dh_ingest_wait(eng._ctx, tickets[-2]), "l5dh_ingest_wait")
                eng._check(lib.l5dh_ingest_async(eng._ctx, hs + 4 * off, hv + 4 * off, m, ctypes.byref(tk)),
                           "l5dh_ingest_async")
                tickets.append(tk.value)
        else:
            eng.ingest(*b)
        if fleet:
            state["merged"] = eng.merge(N_.MERGE_REDUCE_SCATTER, out=summ)
        else:
            eng.snapshot_into(summ, counts, reset=True)

    def barrier():
        if distributed:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    redo0 = eng.partition_redos()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    redo1 = eng.partition_redos()
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # sanity: every sample of the last step landed in exactly one bucket
    if fleet:
        first, cnt = state["merged"]
        tot = torch.stack([summ[:cnt, 0].sum(), torch.tensor(0, device=dev)])
        want = pl["N_total"]
    else:
        tot = torch.stack([counts[:S].sum(dtype=torch.int64), summ[:S, 0].sum()])
        want = n
    if distributed and fleet:
        tot = tot.to(coll_dev)
        dist.all_reduce(tot)
    assert int(tot[0].item()) == want, f"summary counts sum {int(tot[0].item())} != {want}"
    if not fleet:
        assert int(tot[1].item()) == want

    # per-kernel device time (HIP events on the engine's stream), separate steps
    eng.set_param(N_.PARAM_TIMING, 1)
    eng.kernel_times(reset=True)
    tsteps = max(3, min(args.steps, 5))
    for _ in range(tsteps):
        step()
    kt = eng.kernel_times(reset=True)
    eng.set_param(N_.PARAM_TIMING, 0)
    barrier()

    ms_per_step = elapsed / args.steps * 1e3
    total_samples = pl["N_total"] if pl["scaling"] == "strong" and not args.shard else n * world
    value = total_samples * args.steps / elapsed
    kernels = {}
    for name, (ms, launches) in kt.items():
        if launches == 0:
            continue
        avg = ms / launches
        entry = {"avg_ms": round(avg, 4), "launches_per_step": round(launches / tsteps, 2)}
        if name in KERNEL_ALG_BYTES:
            ab = KERNEL_ALG_BYTES[name](n, S, fleet) / (launches / tsteps)
            entry["alg_GBs"] = round(ab / (avg * 1e-3) / 1e9, 1)
            entry["alg_bytes"] = int(ab)
        kernels[name] = entry
    pmc, pmc_note = load_pmc_traffic(args.pmc_json, pl)
    for name, entry in kernels.items():
        if name in pmc:
            entry["traffic"] = pmc[name]
    priced = [k for k in kernels if k in KERNEL_ALG_BYTES]
    roofline = None
    if priced:
        dom = max(priced, key=lambda k: kernels[k]["avg_ms"])
        d = kernels[dom]
        roofline = {"bound": "hbm", "kernel": dom, "achieved": d["alg_GBs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(d["alg_GBs"] / HBM_PEAK_GBS, 4), "traffic": pmc.get(dom), "traffic_source": pmc_note,
                    "alg_bytes_per_launch": d["alg_bytes"], "avg_launch_ms": d["avg_ms"],
                    "pricing": "SURVEY.md §8d: bin1 8 B/sample, accum 7280 B/series (7192 for the c4 export)"}
    # path: B_alg of everything this step processed, over the step time and all GPUs' peak
    rows_summarized = pl["S_total"] if not args.shard else S
    world_c4 = pl["world"] if fleet else 1
    balg = 8 * (total_samples if not args.shard else n) + 7280 * rows_summarized
    gpus = 1 if args.shard else world
    path_gbs = balg / (ms_per_step * 1e-3) / 1e9
    merge = None
    if fleet:
        mb = eng.merge_bytes()
        cms = kt["merge"][0] / kt["merge"][1] if "merge" in kt and kt["merge"][1] else None
        merge = {"collective": "sparse reduce-scatter over RCCL send/recv + int64 reduce-scatter of the totals (l5dh_merge)",
                 "collective_ms": round(cms, 4) if cms else None,
                 "bytes_per_rank": mb["sent"] if world > 1 else mb["encoded"] * (world_c4 - 1) // world_c4,
                 "dense_bytes_per_rank": mb["dense"] * (world_c4 - 1) // world_c4,
                 "encoded_bytes": mb["encoded"], "dense_bytes": mb["dense"],
                 "encoded_over_dense": round(mb["encoded"] / mb["dense"], 4) if mb["dense"] else None,
                 "note": (f"bytes per rank of a {world_c4}-rank merge: (W-1)/W of this rank's sparse encoding "
                          "(entries + words per row + totals) against (W-1)/W of the dense rows + totals; at one "
                          "rank the exchange runs through RCCL to itself (L5DH_PARAM_MERGE_RCCL_1RANK)")}
    cpu = None
    # C1 and C2: the whole step (no extrapolation); C3: a bounded sample of the step
    default_sample = {"c1": n, "c2": n}.get(pl["workload"], 50_000_000)
    sample = args.cpu_sample if args.cpu_sample is not None else default_sample
    if rank == 0 and world == 1 and sample > 0 and not streaming:
        _, nproc, avail, share = host_cpu()
        if args.cpu_threads:
            tcounts = [args.cpu_threads]
        elif pl["workload"] == "c1":
            tcounts = [1]  # one Stat: every add serializes on its monitor (Metric.scala:30-33)
        else:
            tcounts = sorted({share, avail})  # the GPU's CPU share and every core of the box
        cpu = cpu_baseline(pl, sample, tcounts)
    if rank == 0:
        wl_names = {"c3": "C3: 1M series, 1e9 Zipf(s=1) samples per step, log-normal values",
                    "c2": "C2: 100k series x 1k samples, permuted COO",
                    "c1": "C1: 1 series x 1e7 log-normal samples",
                    "c4": "C4: fleet merge, 1M series, 1e9 Zipf(s=1) samples per step sample-sharded over the "
                          "ranks, RCCL reduce-scatter of dense counts, summaries of each rank's slice"}
        cfg = {"workload": wl_names[pl["workload"]], "series_total": pl["S_total"], "samples_per_step": total_samples,
               "series_per_gpu": S, "samples_per_gpu_per_step": n, "rotating_batches": R,
               **({"hot_shift": True} if args.hot_shift else {}),
               **({"first_interval": True} if args.first_interval else {}),
               "parallelism": (f"sample-sharded x{world}" if fleet else
                               f"series-sharded x{world} (weighted ranges)" if pl["workload"] == "c3" else
                               f"replicas x{world}"),
               "step": ("ingest + l5dh_merge (export, reduce-scatter, slice summaries)" if fleet else
                        "ingest (sample+plan+bin1+bin2) + snapshot(reset, dense counts + summaries)")}
        if distributed and backend != "nccl":
            cfg["rehearsal"] = (f"{backend} rank harness, {world} ranks on {torch.cuda.device_count()} GPU(s): "
                                "not a scaling number")
        if args.shard:
            cfg["shard"] = f"rank {pl['rank']} of {pl['world']}: series [{pl['first']}, {pl['first'] + S}), {n} samples"
        if streaming:
            cfg["ingest"] = (f"pinned host memory (l5dh_pin_alloc), {args.piece}-sample l5dh_ingest_async calls, "
                             "double-buffered: PCIe-inclusive, not the HBM-resident headline")
        line = {
            "metric": METRIC, "value": value, "unit": "samples/s", "n_gpus": gpus, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": pl["scaling"], "vs_baseline": None, "dtype": "u32", "data": "synthetic", "config": cfg,
            "path_roofline": {"bound": "hbm", "achieved": round(path_gbs, 1), "peak": HBM_PEAK_GBS * gpus,
                              "unit": "GB/s", "frac": round(path_gbs / (HBM_PEAK_GBS * gpus), 4),
                              "alg_bytes_per_step": balg, "formula": "8 B/sample + 7280 B/series (SURVEY.md §8d)"},
            "roofline": roofline, "kernels": kernels, "cpu_baseline": cpu,
            # partition passes redone in the timed steps (a capacity-planned region overflowed)
            # (level2_counted: batches whose level-2 regions were known not to fit after
            # level 1 -- the first level-2 pass only counted, the second wrote exact regions)
            "redos": {"level1": redo1[0] - redo0[0], "level2": redo1[1] - redo0[1],
                      "level2_counted": redo1[2] - redo0[2], "steps": args.steps},
        }
        if merge:
            line["merge"] = merge
        print(json.dumps(line), file=result_out, flush=True)
    if host:
        host[0].l5dh_pin_free(ctypes.c_void_p(host[1]))
        host[0].l5dh_pin_free(ctypes.c_void_p(host[2]))
    eng.close()
    if distributed:
        dist.destroy_process_group()


def main():
    args = parse()
    if os.environ.get("L5DH_DBG"):
        sys.exit("bench.py: L5DH_DBG is set -- it selects timing-only kernel variants (results invalid) in "
                 "development builds; unset it for a bench line")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn(args))
    run(args)


if __name__ == "__main__":
    main()
