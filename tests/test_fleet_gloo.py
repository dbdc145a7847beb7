"""Multi-rank paths on CPU with gloo (world_size 2): the series-sharded layout (C3)
and the sample-sharded fleet merge (C4).  Per-rank histogram state comes from the
CPU oracle here (no GPU); the GPU side of the same flow is tests/test_gpu_fleet.py.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from linkerd_amd import fleet, synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, S, N, mode, out_dir, padded=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    series, vals = synth.c3(S=S, N=N, seed=7)
    # sample-sharded: sample i -> rank i mod world
    mine = np.arange(N) % world == rank
    h = O.OracleHistograms(S)
    h.ingest(series[mine], vals[mine])
    counts = torch.from_numpy(h.counts())
    totals = torch.from_numpy(h.totals())
    if mode == "sparse":  # l5dh_merge's exchange: sparse slices over send/recv, dense totals
        c, t, first, sent = fleet.sparse_reduce_scatter(counts, totals)
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), counts=c.numpy(), totals=t.numpy(), first=first, sent=sent)
        dist.barrier()
        dist.destroy_process_group()
        return
    if padded:  # alloc_dense buffers: merged without a padded copy
        cb, tb = fleet.alloc_dense(S, world)
        cb[:S] = counts
        tb[:S] = totals
        c, t, first = fleet.fleet_merge(cb, tb, mode=mode, S=S)
    else:
        c, t, first = fleet.fleet_merge(counts, totals, mode=mode)
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), counts=c.numpy(), totals=t.numpy(), first=first)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("padded", [False, True], ids=["copy", "alloc_dense"])
@pytest.mark.parametrize("mode", ["reduce_scatter", "all_reduce", "sparse"])
def test_fleet_merge_gloo_bitexact(tmp_path, mode, padded):
    if mode == "sparse" and padded:
        pytest.skip("the sparse exchange pads internally")
    S, N, world = 301, 60_000, 2  # S not divisible by world: padded reduce-scatter
    mp.start_processes(_worker, args=(world, _free_port(), S, N, mode, str(tmp_path), padded), nprocs=world,
                       start_method="spawn")
    from oracle import oracle as O
    series, vals = synth.c3(S=S, N=N, seed=7)
    h = O.OracleHistograms(S)
    h.ingest(series, vals)
    want_c, want_t = h.counts(), h.totals()
    got_c = np.zeros_like(want_c)
    got_t = np.zeros_like(want_t)
    for r in range(world):
        d = np.load(tmp_path / f"r{r}.npz")
        f = int(d["first"])
        k = min(d["counts"].shape[0], S - f)  # all_reduce of padded buffers returns the pad rows too
        got_c[f:f + k] = d["counts"][:k]
        got_t[f:f + k] = d["totals"][:k]
    np.testing.assert_array_equal(got_c, want_c)
    np.testing.assert_array_equal(got_t, want_t)
    # the merged rows summarize exactly like the single-process histograms
    assert O.summarize_counts(got_c, got_t).tobytes() == h.snapshot().tobytes()
    if mode == "sparse":  # what went over the wire: well under the dense rows' (W-1)/W
        dense = (S + 1) // 2 * (fleet.NB * 4 + 8)
        sent = [int(np.load(tmp_path / f"r{r}.npz")["sent"]) for r in range(world)]
        assert all(0 < b < dense // 4 for b in sent), (sent, dense)


def test_shard_ranges_balanced_and_router():
    w = np.array([1.0 / (r + 1) for r in range(1000)])  # Zipf weights
    sh = fleet.shard_ranges(1000, 4, weights=w)
    assert sh[0].first == 0 and sh[-1].first + sh[-1].count == 1000
    loads = [w[s.first:s.first + s.count].sum() for s in sh]
    assert max(loads) < 1.6 * (w.sum() / 4) or sh[0].count == 1
    eq = fleet.shard_ranges(10, 3)
    assert [s.count for s in eq] == [3, 3, 4]
    router = fleet.SeriesRouter(eq)
    series = np.array([0, 3, 9, 5, 2, 6], dtype=np.uint32)
    vals = np.arange(6, dtype=np.float32)
    parts = router.route(series, vals)
    assert parts[0][0].tolist() == [0, 2] and parts[0][1].tolist() == [0.0, 4.0]
    assert parts[1][0].tolist() == [0, 2] and parts[1][1].tolist() == [1.0, 3.0]
    assert parts[2][0].tolist() == [3, 0] and parts[2][1].tolist() == [2.0, 5.0]


def test_router_torch_tensors_match_numpy():
    """The tensor path (batches resident in HBM are routed there) gives the numpy
    path's parts, in the same order, including ids stored as int32 bit patterns."""
    import torch
    rng = np.random.default_rng(3)
    S = 5000
    shards = fleet.shard_ranges(S, 4, weights=1.0 / (np.arange(S) + 1.0))
    series = rng.integers(0, S, 20_000).astype(np.uint32)
    vals = rng.random(20_000).astype(np.float32)
    want = fleet.SeriesRouter(shards).route(series, vals)
    got = fleet.SeriesRouter(shards).route(torch.from_numpy(series.view(np.int32)), torch.from_numpy(vals))
    for (ws, wv), (gs, gv) in zip(want, got):
        assert np.array_equal(gs.numpy().view(np.uint32), ws) and np.array_equal(gv.numpy(), wv)


def _sharded_worker(rank, world, port, S, N, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    series, vals = synth.c3(S=S, N=N, seed=11)
    shards = fleet.shard_ranges(S, world, weights=np.bincount(series, minlength=S))
    local_s, local_v = fleet.SeriesRouter(shards).route(series, vals)[rank]
    h = O.OracleHistograms(max(1, shards[rank].count))
    h.ingest(local_s, local_v)
    summ = h.snapshot()[: shards[rank].count]
    # gather summaries on rank 0 (the host concatenates 88-B records)
    buf = [None] * world
    dist.all_gather_object(buf, (shards[rank].first, summ.tobytes()))
    if rank == 0:
        np.save(os.path.join(out_dir, "summ.npy"), np.frombuffer(b"".join(b for _, b in sorted(buf)), np.uint8))
    dist.barrier()
    dist.destroy_process_group()


def test_series_sharded_gloo_matches_single_process(tmp_path):
    S, N, world = 500, 50_000, 2
    mp.start_processes(_sharded_worker, args=(world, _free_port(), S, N, str(tmp_path)), nprocs=world,
                       start_method="spawn")
    from oracle import oracle as O
    series, vals = synth.c3(S=S, N=N, seed=11)
    h = O.OracleHistograms(S)
    h.ingest(series, vals)
    assert np.load(tmp_path / "summ.npy").tobytes() == h.snapshot().tobytes()


def test_sparse_decode_takes_a_rows_entries_in_any_order():
    """The sparse export writes a clean cold row's entries in first-touch order (not
    bucket order); the decoder's sum does not depend on the order of a source's entries,
    an escaped count staying right after its header."""
    rng = np.random.default_rng(3)
    rows = np.zeros((5, fleet.NB), np.int32)
    for r in range(5):
        b = rng.choice(fleet.NB, size=40, replace=False)
        rows[r, b] = rng.integers(1, 1000, size=40)
    rows[2, 17] = fleet.CMAX + 5  # an escaped count: header + count word
    enc, words = fleet.sparse_encode(rows)
    offs = np.concatenate([[0], np.cumsum(words.astype(np.int64))])
    shuffled = enc.copy()
    for r in range(5):  # permute each row's entries, moving escape pairs as units
        seg = enc[offs[r]:offs[r + 1]]
        units, i = [], 0
        while i < seg.size:
            n = 2 if (int(seg[i]) & fleet.CMAX) == fleet.CMAX else 1
            units.append(seg[i:i + n])
            i += n
        order = rng.permutation(len(units))
        shuffled[offs[r]:offs[r + 1]] = np.concatenate([units[k] for k in order])
    np.testing.assert_array_equal(fleet.sparse_decode([(shuffled, words)], 5), rows)
    np.testing.assert_array_equal(fleet.sparse_decode([(enc, words), (shuffled, words)], 5), 2 * rows)
