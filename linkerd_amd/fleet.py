"""Multi-GPU layer: one process per GPU, torch.distributed
(backend "nccl" = RCCL over xGMI on MI355X; "gloo" for CPU tests).

* Series sharding (config C3): series are independent, so each rank owns a
  contiguous range of global series ids, balanced by (expected) sample counts;
  ingest is routed by series and no collective touches the data path.
* Fleet merge (config C4): samples of the same series space are spread over
  ranks; each rank exports its dense int32 counts [S][1798] + int64 totals [S]
  (l5dh_export_state), a reduce-scatter sums them (integer sums: bit-exact and
  order independent) so rank r owns series slice r, which it summarizes with
  l5dh_summarize_dense.  min/max are midpoints derived from counts, so they need
  no separate min/max reduction.  The library's own exchange (l5dh_merge) moves the
  rows sparse: sparse_encode / sparse_decode below restate its format, and
  fleet_merge(mode="sparse") runs the same exchange over torch.distributed.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

NB = 1798


@dataclass(frozen=True)
class Shard:
    rank: int
    first: int   # first global series id owned
    count: int   # number of series owned


def shard_ranges(total_series: int, world: int, weights: Optional[np.ndarray] = None) -> List[Shard]:
    """Contiguous series ranges, balanced by weights (e.g. last interval's per-series
    sample counts) when given, else by series count."""
    if world < 1:
        raise ValueError("world must be >= 1")
    if weights is None:
        bounds = [(total_series * r) // world for r in range(world + 1)]
    else:
        w = np.asarray(weights, dtype=np.float64)
        if w.size != total_series:
            raise ValueError("weights must have one entry per series")
        c = np.concatenate([[0.0], np.cumsum(w)])
        targets = c[-1] * np.arange(world + 1) / world
        bounds = np.searchsorted(c, targets, side="left").tolist()
        for r in range(1, world):  # the nearer of the two boundaries around the target
            b = bounds[r]
            if 0 < b <= total_series and targets[r] - c[b - 1] < c[b] - targets[r]:
                bounds[r] = b - 1
        bounds[0], bounds[-1] = 0, total_series
        for r in range(1, world + 1):  # monotone, every rank may own zero or more
            bounds[r] = max(bounds[r], bounds[r - 1])
    return [Shard(r, bounds[r], bounds[r + 1] - bounds[r]) for r in range(world)]


def tile_features(tile_loads, direct_max: int = 255, cold_limit: int = 65535) -> Tuple[float, float, float]:
    """(samples, samples outside the direct tiles, samples in big tiles) of one
    engine's batch with this per-tile load.  The direct tiles are chosen as k_rplan1
    does (l5dh_ingest.hip): among the tiles with >= n / 8192 records, those at or
    above the smallest power of two that keeps <= direct_max of them; their samples
    skip level 2.  A big tile holds > cold_limit records (accumulated by
    k_accum_split instead of the cold kernel)."""
    e = np.asarray(tile_loads, dtype=np.float64)
    n = float(e.sum())
    if e.size == 0 or n <= 0:
        return 0.0, 0.0, 0.0
    thr_min = max(1.0, float(int(n) // 8192))
    cand = e[e >= thr_min]
    direct = np.zeros(e.size, dtype=bool)
    if direct_max > 0 and cand.size:
        lg = np.floor(np.log2(np.maximum(cand, 1.0))).astype(np.int64)
        cnt = np.bincount(lg, minlength=64)
        kbest, cum = 64, 0
        for k in range(63, -1, -1):
            cum += int(cnt[k])
            if cum > direct_max:
                break
            kbest = k
        if kbest < 64:
            direct = e >= max(thr_min, 2.0 ** kbest)
    return n, float(e[~direct].sum()), float(e[e > cold_limit].sum())


@dataclass(frozen=True)
class CostModel:
    """Modelled device time (ms) of one snapshot interval of a series range on one
    MI355X: `per_sample` for a sample partitioned at ingest (level 1) and accumulated
    at the snapshot, `per_sample_l2` more for one outside the batch's direct tiles
    (level 2), `per_sample_hot` more for one in a big tile (> 65535 records: the split
    accumulate), `per_series` for a series' dense row + summary (7.2 KB written), and
    `per_sample_fold` for a range of at most one tile (32 series), which is folded
    into its state rows at ingest (k_fold1); `fixed` (`fixed_fold` for a folded
    range) = launches and plans.  One model for any series count and load
    (tools/fit_cost.py fits it to a measured shard sweep and the C3 / C2 / C1 steps)."""
    per_sample: float
    per_series: float
    per_sample_fold: float
    fixed: float
    per_sample_l2: float = 0.0
    per_sample_hot: float = 0.0
    fixed_fold: Optional[float] = None  # (a folded range's launches; None: `fixed`)

    @property
    def tiled(self) -> bool:
        """Whether the model needs a range's per-tile load (not only its totals)."""
        return bool(self.per_sample_l2 or self.per_sample_hot)

    def range_ms(self, samples: float, series: int, tile_loads=None) -> float:
        if series <= 32:
            f = self.fixed if self.fixed_fold is None else self.fixed_fold
            return f + self.per_sample_fold * samples + self.per_series * series
        t = self.fixed + self.per_sample * samples + self.per_series * series
        if self.tiled and tile_loads is not None:
            _, l2, hot = tile_features(tile_loads)
            t += self.per_sample_l2 * l2 + self.per_sample_hot * hot
        return t


def _per_series(tile_samples, S: int) -> np.ndarray:
    """A per-tile load spread evenly over each tile's series (the last tile holds
    S - 32 (F - 1) of them)."""
    t = np.asarray(tile_samples, dtype=np.float64)
    F = (S + 31) // 32
    if t.size != F:
        raise ValueError(f"tile_samples must hold {F} tiles")
    n = np.full(F, 32, dtype=np.int64)
    n[-1] = S - 32 * (F - 1)
    return np.repeat(t / n, n)


def _range_tiles(per_series: np.ndarray, first: int, count: int) -> np.ndarray:
    """The per-tile load of the engine that owns series [first, first + count): its
    tiles are 32 consecutive series from `first`."""
    if count <= 0:
        return np.zeros(0)
    return np.add.reduceat(per_series[first:first + count], np.arange(0, count, 32))


def _shard_ms(x: Shard, per_series: np.ndarray, cost: CostModel) -> float:
    if not x.count:
        return 0.0
    r = per_series[x.first:x.first + x.count]
    return cost.range_ms(float(r.sum()), x.count, _range_tiles(per_series, x.first, x.count) if cost.tiled else None)


def _plan_tiled(per_series: np.ndarray, first: int, S: int, world: int, cost: CostModel) -> List[Shard]:
    """Contiguous ranges of [first, S) at tile boundaries (multiples of 32 from
    `first`) minimizing the largest modelled time (bisection on that time; each
    candidate is checked by filling the ranks greedily, the range cost being
    monotone in its end)."""
    T = (S - first + 31) // 32  # tiles
    ends = [min(first + 32 * k, S) for k in range(T + 1)]

    def ms(t0: int, t1: int) -> float:
        return _shard_ms(Shard(0, ends[t0], ends[t1] - ends[t0]), per_series, cost) if t1 > t0 else 0.0

    def fill(limit: float) -> Optional[List[int]]:
        bounds, t = [0], 0
        for _ in range(world):
            lo, hi = t, T  # the largest end with ms(t, end) <= limit
            while lo < hi:
                mid = (lo + hi + 1) // 2
                if ms(t, mid) <= limit:
                    lo = mid
                else:
                    hi = mid - 1
            t = lo
            bounds.append(t)
        return bounds if t == T else None

    lo, hi = 0.0, ms(0, T)
    best = fill(hi)
    for _ in range(40):
        if hi - lo <= 1e-4 * hi:
            break
        mid = 0.5 * (lo + hi)
        b = fill(mid)
        if b is not None:
            hi, best = mid, b
        else:
            lo = mid
    return [Shard(r, ends[best[r]], ends[best[r + 1]] - ends[best[r]]) for r in range(world)]


def plan_shards(tile_samples, S: int, world: int, cost: CostModel) -> List[Shard]:
    """Contiguous series ranges of equal modelled device time, from a per-tile load:
    the records per 32-series tile of the last binned batch (l5dh_tile_totals of the
    rank that held them -- the previous interval's last batch -- or an expected
    load); a tile's records are spread evenly over its series for the boundaries.
    With a tiled model (level-2 and big-tile terms, which depend on a range's own
    tiles) the ranges split at tile boundaries and minimize the slowest rank's
    modelled time.  When the first tile alone, folded at ingest, costs less than
    the slowest rank of the plain split, rank 0 takes exactly that tile and the other
    ranks split the rest (a Zipf head concentrates there)."""
    per_series = _per_series(tile_samples, S)
    if cost.tiled:
        plain = _plan_tiled(per_series, 0, S, world, cost)
    else:
        w = cost.per_sample * per_series + cost.per_series
        plain = shard_ranges(S, world, weights=w)
    if world == 1 or S <= 32:
        return plain
    if cost.tiled:
        rest = _plan_tiled(per_series, 32, S, world - 1, cost)
        pinned = [Shard(0, 0, 32)] + [Shard(x.rank + 1, x.first, x.count) for x in rest]
    else:
        rest = shard_ranges(S - 32, world - 1, weights=w[32:])
        pinned = [Shard(0, 0, 32)] + [Shard(x.rank + 1, x.first + 32, x.count) for x in rest]
    if max(_shard_ms(x, per_series, cost) for x in pinned) < max(_shard_ms(x, per_series, cost) for x in plain):
        return pinned
    return plain


def plan_ms(shards: Sequence[Shard], tile_samples, S: int, cost: CostModel) -> List[float]:
    """Modelled device time (ms) of every rank of a plan."""
    per_series = _per_series(tile_samples, S)
    return [_shard_ms(x, per_series, cost) for x in shards]


def plan_spread(shards: Sequence[Shard], tile_samples, S: int, cost: CostModel) -> float:
    """max / min modelled rank time of a plan (1.0 = perfectly balanced).  A pinned
    one-tile rank 0 (plan_shards) cannot take more work without losing its fold, so
    it only has to stay at or below the others' maximum; the spread is of the rest."""
    ms = plan_ms(shards, tile_samples, S, cost)

    def ratio(hi: float, lo: float) -> float:
        return hi / lo if lo > 0 else float("inf")  # (a rank with no modelled time: unbalanced)

    if len(shards) > 1 and shards[0].count <= 32 < S:
        if ms[0] > max(ms[1:]):
            return ratio(ms[0], min(ms[1:]))
        ms = ms[1:]
    ms = [m for m in ms if m > 0]
    return ratio(max(ms), min(ms)) if ms else 1.0


class SeriesRouter:
    """Routes a COO batch of global series ids to the owning ranks (local ids)."""

    def __init__(self, shards: Sequence[Shard]):
        self.shards = list(shards)
        self.starts = np.array([s.first for s in self.shards] + [self.shards[-1].first + self.shards[-1].count],
                               dtype=np.int64)

    def route(self, series, values) -> List[Tuple]:
        """Per rank: (local ids, values).  numpy in, numpy out; torch tensors (device or
        host) in, tensors of the same device out -- a batch resident in HBM is routed
        in HBM (one stable sort by owner, one host read of the W counts)."""
        if not isinstance(series, np.ndarray) and hasattr(series, "device"):
            return self._route_torch(series, values)
        series = np.asarray(series, dtype=np.int64)
        owner = np.searchsorted(self.starts, series, side="right") - 1
        out = []
        for sh in self.shards:
            m = owner == sh.rank
            out.append(((series[m] - sh.first).astype(np.uint32), np.asarray(values)[m].astype(np.float32)))
        return out

    def _route_torch(self, series, values):
        import torch
        s = series.to(torch.int64)
        if series.dtype == torch.int32:  # uint32 ids arrive as int32 bit patterns
            s = s & 0xFFFFFFFF
        starts = torch.as_tensor(self.starts, dtype=torch.int64, device=series.device)
        owner = torch.searchsorted(starts, s, right=True) - 1  # ids past the last shard: owner W
        order = torch.sort(owner, stable=True).indices
        counts = torch.bincount(owner.clamp(0, len(self.shards)), minlength=len(self.shards) + 1)
        parts_s = torch.split(s[order], counts.tolist())
        parts_v = torch.split(values.to(torch.float32)[order], counts.tolist())
        return [((parts_s[r] - sh.first).to(torch.int32), parts_v[r]) for r, sh in enumerate(self.shards)]


def padded_rows(S: int, world: int) -> int:
    return ((S + world - 1) // world) * world


def alloc_dense(S: int, world: int, device=None):
    """Dense merge buffers with padded_rows(S, world) rows (pad rows zero): export
    into counts[:S] / totals[:S] and pass the padded tensors to fleet_merge, which
    then reduces them in place of a padded copy."""
    import torch
    Sp = padded_rows(S, world)
    return (torch.zeros((Sp, NB), dtype=torch.int32, device=device),
            torch.zeros(Sp, dtype=torch.int64, device=device))


def fleet_merge(counts, totals, group=None, mode: str = "reduce_scatter", S: Optional[int] = None):
    """Sum per-rank dense state across ranks.

    counts: torch int32 [S][1798], totals: torch int64 [S] (same S on every rank;
    device tensors with RCCL, CPU tensors with gloo), or the padded buffers of
    alloc_dense (pass the series count as S; no copy is made then).  Returns
    (counts_slice, totals_slice, first): the rows this rank owns after the merge
    (all rows for mode="all_reduce").  The engine's own merge is l5dh_merge
    (HistogramEngine.merge): RCCL inside the library; this is the same exchange
    over torch.distributed, kept for the gloo tests."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    S = counts.shape[0] if S is None else int(S)
    if mode == "all_reduce":
        dist.all_reduce(counts, op=dist.ReduceOp.SUM, group=group)
        dist.all_reduce(totals, op=dist.ReduceOp.SUM, group=group)
        return counts, totals, 0
    if mode != "reduce_scatter":
        raise ValueError(f"unknown merge mode {mode!r}")
    Sp = padded_rows(S, world)
    per = Sp // world
    if counts.shape[0] != Sp:  # not alloc_dense buffers: one padded copy
        counts = torch.cat([counts, counts.new_zeros((Sp - counts.shape[0], NB))])
        totals = torch.cat([totals, totals.new_zeros(Sp - totals.shape[0])])
    if dist.get_backend(group) == "gloo":
        # gloo has no reduce_scatter: all_reduce and keep this rank's slice
        dist.all_reduce(counts, op=dist.ReduceOp.SUM, group=group)
        dist.all_reduce(totals, op=dist.ReduceOp.SUM, group=group)
        c_out = counts[rank * per:(rank + 1) * per].clone()
        t_out = totals[rank * per:(rank + 1) * per].clone()
    else:
        c_out = counts.new_empty((per, NB))
        t_out = totals.new_empty(per)
        dist.reduce_scatter_tensor(c_out, counts.contiguous(), op=dist.ReduceOp.SUM, group=group)
        dist.reduce_scatter_tensor(t_out, totals.contiguous(), op=dist.ReduceOp.SUM, group=group)
    first = rank * per
    keep = max(0, min(per, S - first))
    return c_out[:keep], t_out[:keep], first


# ---- the sparse row exchange of l5dh_merge (linkerd_amd/csrc/l5dh_merge.hip) ----
CMAX = 0x1FFFFF  # count field of an entry; CMAX marks a count in the next word


def sparse_encode(rows: np.ndarray):
    """Rows int32 [n][1798] -> (entries u32, words per row u32): per row its non-empty
    buckets, bucket << 21 | count, or bucket << 21 | CMAX followed by the count's 32 bits
    when count >= CMAX.  Written here in bucket order (as k_menc writes dense rows); the
    library's sparse export writes a clean cold row's entries in first-touch order, and
    the decoder adds a source's entries in any order."""
    rows = np.ascontiguousarray(rows, dtype=np.int32).view(np.uint32)
    r, b = np.nonzero(rows)
    c = rows[r, b]
    esc = c >= CMAX
    head = (b.astype(np.uint32) << 21) | np.where(esc, CMAX, c).astype(np.uint32)
    enc = np.empty(head.size + int(esc.sum()), np.uint32)
    pos = np.arange(head.size) + np.concatenate([[0], np.cumsum(esc)[:-1]]).astype(np.int64) if head.size else \
        np.zeros(0, np.int64)
    enc[pos] = head
    enc[pos[esc] + 1] = c[esc]
    words = np.bincount(r, minlength=rows.shape[0]).astype(np.uint32) + \
        np.bincount(r[esc], minlength=rows.shape[0]).astype(np.uint32)
    return enc, words


def sparse_decode(sources, nrows: int) -> np.ndarray:
    """Sum of the rows encoded by several ranks: sources = [(entries, words per row)]
    of the same nrows rows (k_mdecode's arithmetic, one row at a time)."""
    out = np.zeros((nrows, NB), np.int64)
    for enc, words in sources:
        offs = np.concatenate([[0], np.cumsum(words.astype(np.int64))])
        for r in range(nrows):
            i, e = int(offs[r]), int(offs[r + 1])
            while i < e:
                x = int(enc[i])
                c = x & CMAX
                if c == CMAX:
                    c = int(enc[i + 1])
                    i += 1
                out[r, x >> 21] += c
                i += 1
    return out.astype(np.int32)


def sparse_reduce_scatter(counts, totals, group=None, S: Optional[int] = None):
    """l5dh_merge's reduce-scatter over torch.distributed (gloo tests): rank q sends
    each rank r the sparse encoding of r's row slice and the words per row (an
    all-gather of the slice sizes first, as the library sizes its receive buffers),
    the totals are summed densely.  Returns (counts_slice, totals_slice, first,
    bytes_sent)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    S = counts.shape[0] if S is None else int(S)
    Sp = padded_rows(S, world)
    per = Sp // world
    rows = np.zeros((Sp, NB), np.int32)
    rows[:S] = counts[:S].cpu().numpy()
    parts = [sparse_encode(rows[q * per:(q + 1) * per]) for q in range(world)]
    sizes = torch.tensor([p[0].size for p in parts], dtype=torch.int64)
    mat = [torch.zeros(world, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(mat, sizes, group=group)
    sent = 0
    recv = [None] * world
    reqs = []
    for q in range(world):
        if q == rank:
            recv[q] = parts[q]
            continue
        enc, words = parts[q]
        sent += 4 * enc.size + 4 * per + 8 * per
        reqs.append(dist.isend(torch.from_numpy(enc.view(np.int32).copy()), q, group=group))
        reqs.append(dist.isend(torch.from_numpy(words.view(np.int32).copy()), q, group=group))
    for q in range(world):
        if q == rank:
            continue
        e = torch.empty(int(mat[q][rank]), dtype=torch.int32)
        w = torch.empty(per, dtype=torch.int32)
        dist.recv(e, q, group=group)
        dist.recv(w, q, group=group)
        recv[q] = (e.numpy().view(np.uint32), w.numpy().view(np.uint32))
    for rq in reqs:
        rq.wait()
    c_out = torch.from_numpy(sparse_decode(recv, per))
    tt = torch.zeros(Sp, dtype=torch.int64)
    tt[:S] = totals[:S].cpu()
    dist.all_reduce(tt, op=dist.ReduceOp.SUM, group=group)
    first = rank * per
    keep = max(0, min(per, S - first))
    return c_out[:keep], tt[first:first + per][:keep].clone(), first, sent
