"""Benchmark of the histogram hot path (BASELINE.json metric).

One step = one snapshot interval of the reference's Metric.Stat path: ingest the
whole batch of (series u32, value f32) samples already resident in HBM
(Metric.Stat.add, batched) and snapshot + reset every series into dense int32
bucket counts and 88-byte HistogramSummary records (snapshotHistograms,
AdminMetricsExportTelemeter.scala:154-162).

Default workload (N=1): BASELINE config C3 on one GPU -- 1,000,000 series,
1e9 samples, Zipf(s=1) series ids, log-normal values (synthetic; BASELINE.md
§C3).  With --gpus N (torchrun, one rank per GPU) every rank owns its own
1M-series shard (series-sharded, no collective on the data path): weak scaling.
--workload c4 (BASELINE config C4, fleet merge): the same 1M series are
sample-sharded over the ranks (1e9 samples per step in total); each rank ingests
its shard, exports dense state, the ranks reduce-scatter it over RCCL and each
summarizes its series slice (strong scaling; collective time and bus GB/s are
reported under "merge").

Prints ONE JSON line (rank 0).  `value` = samples/s over all ranks;
`roofline` = the dominant kernel's algorithmic bytes / its average duration
(HIP events on the engine's stream); `path_roofline` = BASELINE's B_alg
(8 B/sample + 7280 B/series) / ms_per_step; `cpu_baseline` = the C oracle
(restatement of the JVM path, per-series mutex) on host cores.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
KERNEL_ALG_BYTES = {
    # algorithmic bytes per launch, per unit
    "count": lambda n, s: 4 * n,                  # reads series ids
    "bin1": lambda n, s: 8 * n + 4 * n,           # reads (series, value), writes 4-B level-1 record
    # bin2 moves only the records of non-direct tiles (a data-dependent share of n):
    # it is timed but not priced
    "accum": lambda n, s: 4 * n + 7280 * s,       # reads final record, writes counts + summary
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--workload", choices=["c3", "c2", "c1", "c4"], default="c3")
    p.add_argument("--series", type=int, default=None, help="series per rank (default: workload's)")
    p.add_argument("--samples", type=int, default=None, help="samples per rank per step (default: workload's)")
    p.add_argument("--bin-mode", type=int, default=0)
    p.add_argument("--direct-max", type=int, default=None, help="engine param: direct tiles (0..512)")
    p.add_argument("--direct-div", type=int, default=None, help="engine param: direct-tile run divisor")
    p.add_argument("--split-min", type=int, default=None, help="engine param: min records of a split tile")
    p.add_argument("--cpu-sample", type=int, default=20_000_000, help="samples in the CPU baseline sample (0: skip)")
    p.add_argument("--cpu-threads", type=int, default=16)
    p.add_argument("--pmc-json", default=os.path.join(REPO, "profiles", "pmc_latest.json"))
    return p.parse_args()


def workload_defaults(args):
    if args.workload == "c3":
        S, N = 1_000_000, 1_000_000_000
    elif args.workload == "c4":  # N = this rank's share of the 1e9 samples
        S, N = 1_000_000, 1_000_000_000 // int(os.environ.get("WORLD_SIZE", "1"))
    elif args.workload == "c2":
        S, N = 100_000, 100_000_000
    else:
        S, N = 1, 10_000_000
    return args.series or S, args.samples or N


def gen_inputs(torch, synth_lib, workload, S, N, rank, stream):
    dev = torch.device("cuda", torch.cuda.current_device())
    series = torch.empty(N, dtype=torch.int32, device=dev)
    values = torch.empty(N, dtype=torch.float32, device=dev)
    sp = ctypes.c_void_p(series.data_ptr())
    vp = ctypes.c_void_p(values.data_ptr())
    if workload in ("c3", "c4"):
        from linkerd_amd import synth
        cdf = torch.from_numpy(synth.zipf_cdf(S)).to(dev)
        # c3: every rank its own series shard; c4: one series space, rank r draws samples [r N, (r+1) N)
        rc = synth_lib.l5ds_gen_zipf(sp, vp, ctypes.c_uint64(N), ctypes.c_uint64(S), ctypes.c_void_p(cdf.data_ptr()),
                                     ctypes.c_uint64(3), ctypes.c_double(0.8), ctypes.c_uint64(rank * N),
                                     ctypes.c_uint32(rank * S if workload == "c3" else 0), ctypes.c_void_p(stream))
    elif workload == "c2":
        K = N // S
        rc = synth_lib.l5ds_gen_c2(sp, vp, ctypes.c_uint64(S), ctypes.c_uint64(K), ctypes.c_uint64(2),
                                   ctypes.c_double(0.8), ctypes.c_uint32(rank * S), ctypes.c_void_p(stream))
    else:
        rc = synth_lib.l5ds_gen_c1(vp, sp, ctypes.c_uint64(N), ctypes.c_uint64(1 + rank), ctypes.c_void_p(stream))
    assert rc == 0, "synthetic generator launch failed"
    torch.cuda.synchronize()
    return series, values


# engine timer -> the kernels it brackets (names as in tools/pmc_summary.py)
# (steady state: the accumulate timer brackets the persistent cold kernel and the split kernel)
PMC_PARTS = {"count": ["count"], "bin1": ["bin1"], "bin2": ["bin2"], "accum": ["accum_cold_p", "accum_split"]}


def load_pmc_traffic(path, workload, S, N):
    """HBM bytes per launch from a committed PMC summary (tools/profile_pmc.sh +
    tools/pmc_summary.py) of the same workload; {} if absent or for another one."""
    try:
        pm = json.load(open(path))
    except (OSError, ValueError):
        return {}
    if pm.get("workload") != workload or pm.get("series") != S or pm.get("samples") != N:
        return {}
    ks = pm.get("kernels", {})
    out = {}
    for name, parts in PMC_PARTS.items():
        if all(p in ks and "hbm_bytes_per_launch" in ks[p] for p in parts):
            out[name] = int(sum(ks[p]["hbm_bytes_per_launch"] for p in parts))
    return out


def cpu_baseline(workload, S, N, sample, threads):
    """C oracle (restatement of the JVM Metric.Stat path) on a bounded sample:
    ingest `sample` samples of the same recipe with `threads` workers (per-series
    mutex, Metric.scala:30) and snapshot all S series on one thread (the timer
    thread, AdminMetricsExportTelemeter.scala:154-162); extrapolate to one full
    step (N samples + S summaries)."""
    import numpy as np
    from linkerd_amd import synth
    from oracle import oracle as O
    n = min(sample, N)
    if workload in ("c3", "c4"):
        s, v = synth.c3(S=S, N=n)
    elif workload == "c2":
        s, v = synth.c2(S=S, K=max(1, n // S))
        n = s.size
    else:
        s, v = synth.c1(n=n)
    h = O.OracleHistograms(S)
    h.ingest(s[: min(n, 100_000)], v[: min(n, 100_000)], threads=threads)  # first-touch warmup
    h = O.OracleHistograms(S)
    t0 = time.perf_counter()
    rc = h.ingest(s, v, threads=threads)
    t_ing = time.perf_counter() - t0
    assert rc == 0
    t0 = time.perf_counter()
    h.snapshot(reset=True)
    t_snap = time.perf_counter() - t0
    full = t_ing * (N / n) + t_snap
    return {"value": N / full, "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"{workload} recipe, {n} samples ingested with {threads} threads ({t_ing:.2f} s) + snapshot "
                      f"of all {S} series on 1 thread ({t_snap:.2f} s), extrapolated to {N} samples/step; "
                      "C restatement of the JVM path (no JDK/finagle jar on the box), per-series mutex"}


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    if distributed:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from linkerd_amd import _native as N_
    from linkerd_amd.engine import HistogramEngine
    synth_lib = ctypes.CDLL(N_.SYNTH_PATH)
    for fn in ("l5ds_gen_c1", "l5ds_gen_c2", "l5ds_gen_zipf"):
        getattr(synth_lib, fn).restype = ctypes.c_int

    S, N = workload_defaults(args)
    stream = torch.cuda.current_stream().cuda_stream
    series, values = gen_inputs(torch, synth_lib, args.workload, S, N, rank, stream)

    eng = HistogramEngine(S, device=torch.cuda.current_device())
    eng.set_param(N_.PARAM_BIN_MODE, args.bin_mode)
    if args.direct_max is not None:
        eng.set_param(N_.PARAM_DIRECT_MAX, args.direct_max)
    if args.direct_div is not None:
        eng.set_param(N_.PARAM_DIRECT_DIV, args.direct_div)
    if args.split_min is not None:
        eng.set_param(N_.PARAM_SPLIT_MIN, args.split_min)
    fleet = args.workload == "c4"
    summ = torch.empty((S, 11), dtype=torch.int64, device=dev)
    counts = torch.empty((S, N_.NBUCKETS), dtype=torch.int32, device=dev)
    totals = torch.empty(S, dtype=torch.int64, device=dev)
    merged = {}
    merge_ev = []

    def step():
        eng.ingest(series, values)
        if not fleet:
            eng.snapshot_into(summ, counts, reset=True)
            return
        # C4: dense partial state -> reduce-scatter (RCCL) -> summaries of this rank's slice
        eng.export_state(counts=counts, totals=totals, reset=True)
        if merge_ev:
            merge_ev[0].record()
        if distributed:
            from linkerd_amd.fleet import fleet_merge
            c, t, first = fleet_merge(counts, totals, mode="reduce_scatter")
        else:
            c, t, first = counts, totals, 0
        if merge_ev:
            merge_ev[1].record()
        eng.summarize_dense(c, t, out=summ[:c.shape[0]])
        merged.update(c=c, n=c.shape[0])

    def barrier():
        if distributed:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # sanity: every sample landed in exactly one bucket of the last snapshot
    if fleet:
        tot = torch.stack([merged["c"].sum(dtype=torch.int64), summ[:merged["n"], 0].sum()])
        if distributed:
            dist.all_reduce(tot)
        want = N * world
    else:
        tot = torch.stack([counts.sum(dtype=torch.int64), summ[:, 0].sum()])
        want = N
    if not os.environ.get("L5DH_DBG"):  # L5DH_DBG selects timing-only kernel variants
        assert int(tot[0].item()) == want, f"bucket counts sum {int(tot[0].item())} != {want}"
        assert int(tot[1].item()) == want

    merge = None
    if fleet:  # collective time alone (events around the reduce-scatter, separate steps)
        merge_ev[:] = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)]
        ms = []
        for _ in range(3):
            step()
            torch.cuda.synchronize()
            ms.append(merge_ev[0].elapsed_time(merge_ev[1]))
        merge_ev.clear()
        cms = sorted(ms)[1]
        nbytes = S * (N_.NBUCKETS * 4 + 8)  # int32 counts + int64 total per series, per rank
        merge = {"collective": "reduce_scatter (RCCL)" if distributed else "none (1 rank)",
                 "collective_ms": round(cms, 4), "bytes_per_rank": nbytes,
                 "bus_GBs": round(nbytes * (world - 1) / world / (cms * 1e-3) / 1e9, 1) if world > 1 else None}

    # per-kernel device time (HIP events on the engine's stream), separate steps
    eng.set_param(N_.PARAM_TIMING, 1)
    eng.kernel_times(reset=True)
    tsteps = max(3, min(args.steps, 5))
    for _ in range(tsteps):
        step()
    kt = eng.kernel_times(reset=True)
    eng.set_param(N_.PARAM_TIMING, 0)

    ms_per_step = elapsed / args.steps * 1e3
    total_samples = N * world
    value = total_samples * args.steps / elapsed
    balg = 8 * N + 7280 * S if not fleet else 8 * N + 7280 * S // world  # c4: a rank writes its slice
    kernels = {}
    for name, (ms, launches) in kt.items():
        if launches == 0:
            continue
        avg = ms / launches
        entry = {"avg_ms": round(avg, 4), "launches_per_step": round(launches / tsteps, 2)}
        if name in KERNEL_ALG_BYTES:
            ab = KERNEL_ALG_BYTES[name](N, S) / (launches / tsteps)
            entry["alg_GBs"] = round(ab / (avg * 1e-3) / 1e9, 1)
            entry["alg_bytes"] = int(ab)
        kernels[name] = entry
    dom = max((k for k in kernels if k in KERNEL_ALG_BYTES), key=lambda k: kernels[k]["avg_ms"])
    d = kernels[dom]
    pmc = load_pmc_traffic(args.pmc_json, args.workload, S, N)
    for name, entry in kernels.items():
        if name in pmc:
            entry["traffic"] = pmc[name]
    traffic = pmc.get(dom)
    roofline = {"bound": "hbm", "kernel": dom, "achieved": d["alg_GBs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(d["alg_GBs"] / HBM_PEAK_GBS, 4), "traffic": traffic,
                "alg_bytes_per_launch": d["alg_bytes"], "avg_launch_ms": d["avg_ms"]}
    path_gbs = balg / (ms_per_step * 1e-3) / 1e9
    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        cpu = cpu_baseline(args.workload, S, N, args.cpu_sample, args.cpu_threads)
    if rank == 0:
        line = {
            "metric": "histogram samples ingested+summarized/sec (1M series) and % HBM peak",
            "value": value, "unit": "samples/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "strong" if fleet else "weak", "vs_baseline": None,
            "dtype": "u32", "data": "synthetic",
            "config": {"workload": {"c3": "C3: 1M series x 1e9 samples, Zipf(s=1) ids, log-normal values",
                                    "c2": "C2: 100k series x 1k samples, permuted COO",
                                    "c1": "C1: 1 series x 1e7 log-normal samples",
                                    "c4": "C4: fleet merge, 1M series, 1e9 Zipf(s=1) samples per step "
                                          "sample-sharded over the ranks, reduce-scatter of dense counts"}[args.workload],
                       "series_per_gpu": S, "samples_per_gpu_per_step": N, "parallelism": f"{'sample-sharded' if fleet else 'series-sharded'} x{world}",
                       "step": "ingest (count+scan+bin1+bin2) + snapshot(reset, dense counts + summaries)"},
            "roofline": roofline,
            "path_roofline": {"bound": "hbm", "achieved": round(path_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": round(path_gbs / HBM_PEAK_GBS, 4), "alg_bytes_per_step": balg,
                              "formula": "8 B/sample + 7280 B/series (BASELINE.md)"},
            "kernels": kernels,
            "cpu_baseline": cpu,
        }
        if merge:
            line["merge"] = merge
        print(json.dumps(line), flush=True)
    eng.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
