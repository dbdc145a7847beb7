// l5dh_ingest.hip -- ingest-side kernels (Metric.Stat.add, batched).
//
//   k_count    LDS tile histogram of each slab of the COO batch -> table[g][t]
//   k_colscan  per tile, exclusive prefix over slabs (in place) + tile totals
//   k_tilescan exclusive prefix over tiles -> tile_base[F+1] (final layout)
//   k_bin1     level 1: slab -> super-tiles (64 tiles) and direct tiles, LDS
//              counting sort of 16K-sample sub-chunks, run writes
//   k_bin2     level 2: (super-tile, slab block) -> per-(slab, tile) segments
//   k_bin      single-level alternative (direct scatter)
//
// Records (l5dh_kernels.hpp): [31:26] tile in super-tile | [25:21] series in
//   tile | [20:0] payload = v (0 <= v < V_ESC) or V_ESC + bucket (escaped: the
//   exact sum difference went to sumfix[series], integer atomics, order free).
#include <algorithm>

#include "l5dh_device.hpp"
// L5DH_EXP (compile time, tools/mk_var.sh): timing-only variants, results invalid.
//   4 k_count without hot-column aggregation, 8 k_count loads only,
//   16 k_bin1 loads + ranking only (no scan, scatter or run writes),
//   1024 k_bin1 run writes replaced by the same number of sequential stores,
//   2048 ... by whole 64-B segments in 1024 interleaved sequential streams
#ifndef L5DH_EXP
#define L5DH_EXP 0
#endif
// hot count columns aggregated by ballot in k_count (2 or 4; the plan holds 4 hints)
#ifndef L5DH_HK
#define L5DH_HK 2
#endif
static_assert(L5DH_HK >= 2 && L5DH_HK <= 4, "k_count's tail path uses two hot columns; the plan holds four");

namespace l5dh {
namespace {

constexpr int ST_TILES = 64;
constexpr int ST_SHIFT = 11;  // 64 tiles x 32 series
constexpr uint32_t NOKEY = 0xFFFFFFFFu;
constexpr int NHOT = 8;       // k_bin1 bins counted in lane-private slots
#ifndef L5DH_B2_ITEM
#define L5DH_B2_ITEM 32768
#endif
constexpr uint32_t B2_ITEM = L5DH_B2_ITEM;  // target level-1 records per k_bin2 item
static_assert(B2_ITEM >= 16384, "the plan's item map holds (2^30 / 16384 + 1024) items");

// ------------------------------------------------------------------------
// Count key of a valid sample: its tile, or for a split tile the column of its
// half (F + 2 s + half).  sw[w] = {split bits of word w, split tiles before it}.
__device__ __forceinline__ uint32_t count_key(uint32_t s, uint32_t F, uint2 sw) {
  const uint32_t t = s >> TILE_SHIFT;
  const uint32_t bit = 1u << (t & 31u);
  const uint32_t sk = F + 2u * (sw.y + (uint32_t)__popc(sw.x & (bit - 1u))) + ((s >> 4) & 1u);
  return (sw.x & bit) ? sk : t;
}

__global__ __launch_bounds__(WG) void k_count(const uint32_t* __restrict__ series, size_t n, size_t per, uint32_t S,
                                              uint32_t F, uint32_t* __restrict__ table, uint32_t* __restrict__ err,
                                              const uint32_t* __restrict__ hint, const uint32_t* __restrict__ split,
                                              int vec) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t C = F + COLS;
  uint2* sw = reinterpret_cast<uint2*>(smem);  // [1024] split words
  uint32_t* cnt = smem + 2048;                  // [C]
  const uint32_t NW = (F + 31) / 32;
  for (uint32_t t = threadIdx.x; t < C; t += WG) cnt[t] = 0;
  for (uint32_t w = threadIdx.x; w < NW; w += WG) sw[w] = make_uint2(split[SPLIT_BITS + w], split[SPLIT_PRE + w]);
  __syncthreads();
  const size_t lo = (size_t)blockIdx.x * per;
  const size_t hi = lo + per < n ? lo + per : n;
  uint32_t hk[L5DH_HK];  // hot columns of the previous batch (aggregation only)
#pragma unroll
  for (int h = 0; h < L5DH_HK; ++h) hk[h] = hint[h] < C && !(L5DH_EXP & 4) ? hint[h] : 0xFFFFFFFFu;
  bool bad = false;
  if (lo < hi) {
    size_t done = lo;
    if (vec) {  // lo and the base pointer are 16-B aligned
      const size_t nv = (hi - lo) >> 2;
      const uint4* __restrict__ p = reinterpret_cast<const uint4*>(series + lo);
      size_t i = threadIdx.x;
      const size_t wlast = threadIdx.x | 63;  // last lane of this wave: uniform loop bound
      // software-pipelined: the next two groups of 4 x 16 B per thread are in flight
      // during this one's LDS counting, so the HBM stream does not pause behind it
      auto full = [&](size_t j) { return wlast - threadIdx.x + j + 3 * WG < nv; };
      auto load4 = [&](size_t j, uint4 (&x)[4]) {
        if (full(j)) {
#pragma unroll
          for (int q = 0; q < 4; ++q) x[q] = p[j + q * WG];
        }
      };
      uint4 n0[4], n1[4];
      load4(i, n0);
      if (!(L5DH_EXP & 128)) load4(i + 4 * WG, n1);
      for (; full(i); i += 4 * WG) {
        const uint4 a = n0[0], b = n0[1], c = n0[2], d = n0[3];
        if (!(L5DH_EXP & 128)) {
#pragma unroll
          for (int q = 0; q < 4; ++q) n0[q] = n1[q];
          load4(i + 8 * WG, n1);
        } else {
          load4(i + 4 * WG, n0);
        }
        if (L5DH_EXP & 8) {  // timing: loads only
          asm volatile("" ::"v"(a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w));
          continue;
        }
        const uint32_t sv[16] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w};
        uint2 wv[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) wv[k] = sw[(sv[k] >> (TILE_SHIFT + 5)) & 1023u];  // (any word when s >= S)
        uint32_t key[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const bool ok = sv[k] < S;
          bad |= !ok;
          key[k] = ok ? count_key(sv[k], F, wv[k]) : 0xFFFFFFFFu;
        }
        hot_inc_batch<L5DH_HK, 16>(cnt, key, hk);
      }
      for (; i - threadIdx.x < nv; i += WG) {  // convergent: out-of-range lanes pass invalid ids
        uint4 a = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
        if (i < nv) a = p[i];
        const bool in = i < nv;
        auto one_in = [&](uint32_t s) {
          const bool ok = in && s < S;
          bad |= in && !ok;
          hot_inc(cnt, ok ? count_key(s, F, sw[s >> (TILE_SHIFT + 5)]) : 0u, ok, hk[0], hk[1]);
        };
        one_in(a.x); one_in(a.y); one_in(a.z); one_in(a.w);
      }
      done = lo + (nv << 2);
    }
    for (size_t i0 = done; i0 < hi; i0 += WG) {  // convergent tail (the aggregation needs whole waves)
      const size_t i = i0 + threadIdx.x;
      const uint32_t s = i < hi ? series[i] : 0xFFFFFFFFu;
      const bool ok = s < S;
      bad |= i < hi && !ok;
      hot_inc(cnt, ok ? count_key(s, F, sw[s >> (TILE_SHIFT + 5)]) : 0u, ok, hk[0], hk[1]);
    }
  }
  if (bad) atomicAdd(err, 1u);  // monotonic: the host compares it with the count it already reported
  __syncthreads();
  uint32_t* row = table + (size_t)blockIdx.x * C;
  for (uint32_t t = threadIdx.x; t < C; t += WG) row[t] = cnt[t];
}

// WG = 64 tiles x 16 slab groups.
__global__ __launch_bounds__(1024) void k_colscan(uint32_t* __restrict__ table, int G, uint32_t C,
                                                  uint32_t* __restrict__ tile_tot) {
  __shared__ uint32_t part[16][64];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const uint32_t t = blockIdx.x * 64 + lane;
  const int gper = (G + 15) / 16;
  const int g0 = w * gper;
  const int g1 = min(G, g0 + gper);
  // G <= 512: a wave's <= 32 slabs are loaded at once (one memory latency, not one
  // per slab: the in-place prefix stores would otherwise order every load)
  constexpr int GW = 32;
  uint32_t v[GW];
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < GW; ++k) {
    v[k] = (t < C && g0 + k < g1) ? table[(size_t)(g0 + k) * C + t] : 0u;
    s += v[k];
  }
  part[w][lane] = s;
  __syncthreads();
  if (w == 0) {
    uint32_t acc = 0;
    for (int k = 0; k < 16; ++k) {
      const uint32_t x = part[k][lane];
      part[k][lane] = acc;
      acc += x;
    }
    if (t < C) tile_tot[t] = acc;
  }
  __syncthreads();
  if (t < C) {
    uint32_t acc = part[w][lane];
#pragma unroll
    for (int k = 0; k < GW; ++k)
      if (g0 + k < g1) {
        table[(size_t)(g0 + k) * C + t] = acc;
        acc += v[k];
      }
  }
}
__global__ __launch_bounds__(1024) void k_tilescan(uint32_t* __restrict__ coltot, uint32_t F,
                                                   const uint32_t* __restrict__ split, uint32_t* __restrict__ tile_base) {
  __shared__ uint32_t lds[17];
  const uint32_t per = (F + 1023) / 1024;
  const uint32_t t0 = threadIdx.x * per;
  // a thread's tiles: totals of split tiles are the sums of their halves
  auto tile_total = [&](uint32_t t, uint32_t v) {
    const uint32_t wd = split[SPLIT_BITS + (t >> 5)];
    const uint32_t bit = 1u << (t & 31u);
    if (wd & bit) {
      const uint32_t si = split[SPLIT_PRE + (t >> 5)] + (uint32_t)__popc(wd & (bit - 1u));
      v += coltot[F + 2 * si] + coltot[F + 2 * si + 1];
      coltot[t] = v;
    }
    return v;
  };
  constexpr int PT = 32;  // F <= 32 K tiles: all of a thread's loads issued at once
  uint32_t v[PT];
  uint32_t s = 0, tot;
  if (per <= PT) {
    // a thread's <= 32 consecutive tiles span <= 2 split words; every load (totals,
    // split words, half totals) is issued before any store (the split tiles' sums
    // are written back to coltot[t] after the loads)
    const uint32_t wb = t0 >> 5;
    const uint32_t sw0 = t0 < F ? split[SPLIT_BITS + wb] : 0u, sp0 = t0 < F ? split[SPLIT_PRE + wb] : 0u;
    const uint32_t sw1 = (wb + 1) * 32 < F ? split[SPLIT_BITS + wb + 1] : 0u;
    const uint32_t sp1 = (wb + 1) * 32 < F ? split[SPLIT_PRE + wb + 1] : 0u;
    uint32_t h[PT];
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      const uint32_t t = t0 + k;
      const bool in = (uint32_t)k < per && t < F;
      v[k] = in ? coltot[t] : 0u;
      const bool hi = (t >> 5) != wb;
      const uint32_t wd = hi ? sw1 : sw0, bit = 1u << (t & 31u);
      h[k] = 0u;
      if (in && (wd & bit)) {
        const uint32_t si = (hi ? sp1 : sp0) + (uint32_t)__popc(wd & (bit - 1u));
        h[k] = 1u + coltot[F + 2 * si] + coltot[F + 2 * si + 1];  // +1: split (a split tile may be empty)
      }
    }
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      if (h[k]) {
        v[k] += h[k] - 1u;
        coltot[t0 + k] = v[k];
      }
      s += v[k];
    }
    uint32_t acc = block_excl_scan<1024>(s, lds, &tot);
#pragma unroll
    for (int k = 0; k < PT; ++k)
      if ((uint32_t)k < per && t0 + k < F) {
        tile_base[t0 + k] = acc;
        acc += v[k];
      }
  } else {
    for (uint32_t k = 0; k < per && t0 + k < F; ++k) s += tile_total(t0 + k, coltot[t0 + k]);
    uint32_t acc = block_excl_scan<1024>(s, lds, &tot);
    for (uint32_t k = 0; k < per && t0 + k < F; ++k) {
      tile_base[t0 + k] = acc;
      acc += coltot[t0 + k];
    }
  }
  if (threadIdx.x == 0) tile_base[F] = tot;
}
// k_tilescan + k_seginfo in one workgroup, through LDS: the column totals are loaded
// coalesced (a thread's 32 consecutive tiles read strided from global memory were
// ~30 us on C3), split tiles add their halves, every thread scans its 32 consecutive
// tiles from LDS (one pad word per 32: no bank conflicts), and tile_base goes out
// coalesced.  F <= 32768.
constexpr uint32_t tpad(uint32_t t) { return t + (t >> 5); }
__global__ __launch_bounds__(1024) void k_tilescan_seg(uint32_t* __restrict__ coltot, uint32_t F,
                                                       const uint32_t* __restrict__ split,
                                                       uint32_t* __restrict__ tile_base, uint32_t* __restrict__ sinfo) {
  extern __shared__ uint32_t tl[];  // [tpad(F) + 1]
  __shared__ uint32_t lds[17];
  const uint32_t NS = split[0];
  uint16_t* map = reinterpret_cast<uint16_t*>(sinfo + SINFO_MAP);
  for (uint32_t t = threadIdx.x; t < F; t += 1024) {
    tl[tpad(t)] = coltot[t];
    map[t] = NO_SPLIT;
  }
  __syncthreads();
  // split tiles: their samples were counted in the two half columns
  for (uint32_t si = threadIdx.x; si < NS; si += 1024) {
    const uint32_t t = split[SPLIT_LIST + si];
    const uint32_t h0 = coltot[F + 2 * si], h1 = coltot[F + 2 * si + 1];
    const uint32_t v = tl[tpad(t)] + h0 + h1;
    tl[tpad(t)] = v;
    coltot[t] = v;  // read as the tile's total by k_stplan
    sinfo[1 + si] = t;
    sinfo[SINFO_H0 + si] = h0;
    map[t] = (uint16_t)si;
  }
  if (threadIdx.x == 0) sinfo[0] = NS;
  __syncthreads();
  constexpr int PT = 32;
  const uint32_t t0 = threadIdx.x * PT;
  uint32_t v[PT], sum = 0, tot;
#pragma unroll
  for (int k = 0; k < PT; ++k) {
    v[k] = t0 + k < F ? tl[tpad(t0 + k)] : 0u;
    sum += v[k];
  }
  uint32_t acc = block_excl_scan<1024>(sum, lds, &tot);
#pragma unroll
  for (int k = 0; k < PT; ++k)
    if (t0 + k < F) {
      tl[tpad(t0 + k)] = acc;
      acc += v[k];
    }
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < F; t += 1024) tile_base[t] = tl[tpad(t)];
  if (threadIdx.x == 0) tile_base[F] = tot;
}

__global__ __launch_bounds__(1024) void k_seginfo(const uint32_t* __restrict__ split, const uint32_t* __restrict__ coltot,
                                                  uint32_t F, uint32_t* __restrict__ sinfo) {
  const uint32_t NS = split[0];
  uint16_t* map = reinterpret_cast<uint16_t*>(sinfo + SINFO_MAP);
  for (uint32_t t = threadIdx.x; t < F; t += 1024) map[t] = NO_SPLIT;
  __syncthreads();
  if (threadIdx.x == 0) sinfo[0] = NS;
  for (uint32_t si = threadIdx.x; si < NS; si += 1024) {
    const uint32_t t = split[SPLIT_LIST + si];
    sinfo[1 + si] = t;
    sinfo[SINFO_H0 + si] = coltot[F + 2 * si];
    map[t] = (uint16_t)si;
  }
}

// One-tile series spaces (S <= 32: C1, the head shard of a many-way C3): the
// tile's records are the samples in input order -- no counting pass, no partition.
// An invalid id becomes 0xFFFFFFFF, which no valid record equals (its bucket field
// would be 2047) and the accumulate kernels skip; the tile's range is the batch.
__global__ __launch_bounds__(256) void k_encode1(const uint32_t* __restrict__ series, const float* __restrict__ values,
                                                 size_t n, uint32_t S, Tables tb, uint32_t* __restrict__ records,
                                                 int64_t* __restrict__ sumfix, uint32_t* __restrict__ tile_base,
                                                 uint32_t* __restrict__ err, int vec) {
  bool bad = false;
  auto enc = [&](uint32_t s, float f) -> uint32_t {
    if (s >= S) {
      bad = true;
      return 0xFFFFFFFFu;
    }
    return ((s & (TILE - 1)) << 21) | payload1(s, f, tb, sumfix);
  };
  const size_t tid = (size_t)blockIdx.x * 256 + threadIdx.x, nth = (size_t)gridDim.x * 256;
  size_t done = 0;
  if (vec) {  // 16-B loads and stores
    const size_t nv = n >> 2;
    for (size_t i = tid; i < nv; i += nth) {
      const uint4 a = reinterpret_cast<const uint4*>(series)[i];
      const float4 v = reinterpret_cast<const float4*>(values)[i];
      reinterpret_cast<uint4*>(records)[i] = make_uint4(enc(a.x, v.x), enc(a.y, v.y), enc(a.z, v.z), enc(a.w, v.w));
    }
    done = nv << 2;
  }
  for (size_t i = done + tid; i < n; i += nth) records[i] = enc(series[i], values[i]);
  if (bad) atomicAdd(err, 1u);  // monotonic, like k_count's
  if (tid == 0) {
    tile_base[0] = 0u;
    tile_base[1] = (uint32_t)n;
  }
}

// Single-level: scatter records to the slab's exclusive (slab, tile) segment.
__global__ __launch_bounds__(WG) void k_bin(const uint32_t* __restrict__ series, const float* __restrict__ values,
                                            size_t n, size_t per, uint32_t S, uint32_t F,
                                            const uint32_t* __restrict__ table, const uint32_t* __restrict__ tile_base,
                                            Tables tb, uint32_t* __restrict__ records, int64_t* __restrict__ sumfix,
                                            int vec) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint32_t* cur = smem;
  const uint32_t* row = table + (size_t)blockIdx.x * (F + COLS);  // counted without split tiles
  for (uint32_t t = threadIdx.x; t < F; t += WG) cur[t] = tile_base[t] + row[t];
  __syncthreads();
  const size_t lo = (size_t)blockIdx.x * per;
  const size_t hi = lo + per < n ? lo + per : n;
  if (lo >= hi) return;
  auto one = [&](uint32_t s, float f) {
    if (s >= S) return;
    const uint32_t rec = (((s >> TILE_SHIFT) & 63u) << 26) | ((s & (TILE - 1)) << 21) | payload1(s, f, tb, sumfix);
    records[atomicAdd(&cur[s >> TILE_SHIFT], 1u)] = rec;
  };
  size_t done = lo;
  if (vec) {
    const size_t nv = (hi - lo) >> 2;
    const uint4* ps = reinterpret_cast<const uint4*>(series + lo);
    const float4* pv = reinterpret_cast<const float4*>(values + lo);
    for (size_t i = threadIdx.x; i < nv; i += WG) {
      const uint4 s = ps[i];
      const float4 f = pv[i];
      one(s.x, f.x); one(s.y, f.y); one(s.z, f.z); one(s.w, f.w);
    }
    done = lo + (nv << 2);
  }
  for (size_t i = done + threadIdx.x; i < hi; i += WG) one(series[i], values[i]);
}

// ------------------------------------------------------------------------
// Level 1.  LDS: stage[CH1] u32, stage_st[CH1] u16, stcnt/stoff/stcur[FS_MAX].

// Level 1.  Bins = the FS super-tiles (records of their non-direct tiles, into
// scratch1) and two bins per direct tile (records straight into the final layout;
// a split tile's half 0 from the tile's start, half 1 after all half-0 records; an
// unsplit tile's bins share one range, the even bin's run first), plus a trash bin for sample slots with no sample (batch
// tail, ids >= S: counted as errors by k_count) written to scratch1[n ..).  Both
// arrays share the final layout's index space: slab g's records of direct tile t
// start at tile_base[t] + pre[g][t]; its level-1 records of super-tile j at
// tile_base[j*64] + sum of pre[g][t] over the non-direct t of j.
// Per CH1-slot sub-chunk (every slot lands in exactly one bin, so the body has
// no per-sample branches): one LDS atomic ranks each slot in its bin (the NHOT
// hottest bins count in lane-private slots: no same-address serialization), a
// scan gives bin offsets, each slot is staged at its sorted position WITH its
// destination ({record, dst | direct << 31}), and all CH1 stage entries are
// written in order.  Batches are < 2^30 samples.
// LDS: stage[CH1] uint2, cnt[BINS], oc[BINS] {off, cur | direct << 31}, direct
// words {bits, prefix}, hot slots, lane-private hot counters (+1 zero row).
template <int CH1, int NT, int WPS, bool HS_ALWAYS>
__global__ __launch_bounds__(NT, WPS) void k_bin1(const uint32_t* __restrict__ series, const float* __restrict__ values,
                                                size_t n, size_t per, uint32_t S, uint32_t F,
                                                const uint32_t* __restrict__ pre,
                                                const uint32_t* __restrict__ tile_base, Tables tb,
                                                const uint32_t* __restrict__ plan, const uint32_t* __restrict__ coltot,
                                                const uint32_t* __restrict__ split, uint32_t* __restrict__ out1, uint32_t* __restrict__ records,
                                                int64_t* __restrict__ sumfix, int vec, int dbg) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint2* stage = reinterpret_cast<uint2*>(smem);                   // [CH1]
  uint32_t* cnt = smem + 2 * CH1;                                  // [BIN1_BINS]
  uint2* oc = reinterpret_cast<uint2*>(cnt + BIN1_BINS);           // [BIN1_BINS] {stage offset, cursor | direct << 31}
  uint2* dw = oc + BIN1_BINS;                                      // [1024] {direct bits, direct tiles before}
  uint8_t* hslot = reinterpret_cast<uint8_t*>(dw + 1024);          // [BIN1_BINS] hot slot of a bin (NHOT: none)
  uint32_t* hcnt = reinterpret_cast<uint32_t*>(hslot + BIN1_BINS); // [NHOT + 1][64] lane-private hot counters
  uint32_t* dun = hcnt + (NHOT + 1) * 64;                          // [8] unsplit direct tiles (bit d)
  const uint32_t FS = (F + ST_TILES - 1) / ST_TILES;
  const uint32_t NW = (F + 31) / 32;
  const uint32_t ND = plan[PLAN_ND];
  // lane-private counters for the hottest bins (development variant, HS_ALWAYS)
  const bool HS = HS_ALWAYS;
  // When one bin holds >= half the batch (a single-series or few-series shard: every
  // lane of a wave would otherwise serialize on its LDS counter), the batch's two
  // hottest bins are ranked by wave ballots; measured (tools/ab_var.py, same context):
  // 41 % faster on C3's first 8-way shard, 2 % slower on C3 (hottest bin 23 %), 17 %
  // slower on C2 (no hot bin) -- so only past that share.  Variant bit 0: never.
  const bool hotrank = !HS && plan[PLAN_HS] != 0u && !((dbg >> 27) & 1);
  const uint32_t hb0 = plan[3 * FS + 1], hb1 = plan[3 * FS + 2];  // NOKEY: none
  const int lane = lane_id();
  const int wv = threadIdx.x >> 6;
  const uint32_t TB = FS + 2 * ND;  // trash bin (TB + 1 <= BIN1_BINS bins)
  const uint32_t trash = (uint32_t)n;  // scratch1 has n + CH1 + 16 entries
  const uint32_t* prow = pre + (size_t)blockIdx.x * (F + COLS);
  for (uint32_t w = threadIdx.x; w < NW; w += NT) dw[w] = make_uint2(plan[PLAN_DBITS + w], plan[PLAN_DPRE + w]);
  for (uint32_t b = threadIdx.x; b < BIN1_BINS; b += NT) {
    uint32_t sl = NHOT;
#pragma unroll
    for (int q = 0; q < NHOT; ++q)
      if (plan[3 * FS + 1 + q] == b) sl = (uint32_t)q;
    hslot[b] = (uint8_t)sl;
    cnt[b] = 0;
  }
  for (uint32_t i = threadIdx.x; i < (NHOT + 1) * 64; i += NT) hcnt[i] = 0;
  // super-tile cursors: level-1 records of this slab before super-tile j; one
  // wave per super-tile, a lane per tile (independent, coalesced loads)
  for (uint32_t t = threadIdx.x; t < FS * ST_TILES; t += NT) {
    uint32_t v = 0;
    if (t < F && !((plan[PLAN_DBITS + (t >> 5)] >> (t & 31u)) & 1u)) {  // direct tiles have no level-1 records
      const uint32_t wd = split[SPLIT_BITS + (t >> 5)];
      const uint32_t bit = 1u << (t & 31u);
      if (wd & bit) {  // split: its count is in the two half columns
        const uint32_t si = split[SPLIT_PRE + (t >> 5)] + (uint32_t)__popc(wd & (bit - 1u));
        v = prow[F + 2 * si] + prow[F + 2 * si + 1];
      } else {
        v = prow[t];
      }
    }
    v = wave_sum(v);
    if (lane == 0) oc[t >> 6] = make_uint2(0u, tile_base[t] + v);
  }
  if (threadIdx.x < 8) dun[threadIdx.x] = 0u;
  __syncthreads();
  for (uint32_t h = threadIdx.x; h < 2 * ND; h += NT) {  // direct tile h/2: half 0 from its start, half 1 after it
    const uint32_t si = plan[PLAN_DSI + (h >> 1)];
    const uint32_t t = plan[PLAN_DLIST + (h >> 1)];
    uint32_t at;
    if (si == NOKEY) {
      // unsplit direct tile (counted per tile): both bins share the slab's one range,
      // the odd bin's cursor is canonical (the bin scan places the even bin's run first)
      at = tile_base[t] + prow[t];
      if (h & 1u) atomicOr(&dun[h >> 6], 1u << ((h >> 1) & 31u));
    } else {
      at = tile_base[t] + ((h & 1u) ? coltot[F + 2 * si] : 0u) + prow[F + 2 * si + (h & 1u)];
    }
    oc[FS + h] = make_uint2(0u, at | 0x80000000u);
  }
  if (threadIdx.x == 0) oc[TB] = make_uint2(0u, trash);
  __syncthreads();
  const size_t lo = (size_t)blockIdx.x * per;
  const size_t hi = lo + per < n ? lo + per : n;
  constexpr int PT = CH1 / NT;  // slots per thread: PT/4 groups of 4 consecutive
  for (size_t c0 = lo; c0 < hi; c0 += CH1) {
    uint32_t sv[PT];
    float fv[PT];
    if (vec && c0 + CH1 <= hi) {
#pragma unroll
      for (int k = 0; k < PT / 4; ++k) {
        const size_t base = c0 + 4 * ((size_t)k * NT + threadIdx.x);
        const uint4 s4 = *reinterpret_cast<const uint4*>(series + base);
        const float4 f4 = *reinterpret_cast<const float4*>(values + base);
        sv[4 * k] = s4.x; sv[4 * k + 1] = s4.y; sv[4 * k + 2] = s4.z; sv[4 * k + 3] = s4.w;
        fv[4 * k] = f4.x; fv[4 * k + 1] = f4.y; fv[4 * k + 2] = f4.z; fv[4 * k + 3] = f4.w;
      }
    } else {
#pragma unroll
      for (int k = 0; k < PT; ++k) {
        const size_t i = c0 + 4 * ((size_t)(k >> 2) * NT + threadIdx.x) + (k & 3);
        const bool in = i < hi;
        sv[k] = in ? series[i] : 0xFFFFFFFFu;
        fv[k] = in ? values[i] : 0.0f;
      }
    }
    if (dbg & 8) {  // timing: loads only
      uint32_t x = 0;
#pragma unroll
      for (int k = 0; k < PT; ++k) x ^= sv[k] ^ __float_as_uint(fv[k]);
      if (x == 0x12345678u) out1[threadIdx.x] = x;
      continue;
    }
    // Per group of 4 slots: payloads (samples outside [0, V_ESC) take a rare
    // path through this thread's still free stage slots), batched LDS reads of the
    // direct words, branch-free bin selection, then one rank atomic per slot; hot
    // bins count in lane-private counters.
    uint32_t rec[PT];
    uint32_t pk[PT];  // [13:0] local rank | [24:14] bin | [28:25] hot slot (NHOT: none)
#pragma unroll
    for (int g = 0; g < PT; g += 4) {
      uint32_t pl[4];
      uint32_t escm = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        // fast: +0 <= f < V_ESC, one integer compare of the bit pattern (-0, NaN and
        // (-1, 0) take the exact slow path, which also truncates them to 0)
        const float f = fv[g + q];
        const bool fast = __float_as_uint(f) < 0x49FFC000u;  // bits of (float)V_ESC
        pl[q] = fast ? (uint32_t)f : 0u;
        escm |= (!fast && sv[g + q] < S) ? (1u << q) : 0u;
      }
      if (__ballot(escm != 0u)) {
        uint32_t* tmp = reinterpret_cast<uint32_t*>(stage) + threadIdx.x * 8;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          tmp[2 * q] = sv[g + q];
          tmp[2 * q + 1] = __float_as_uint(fv[g + q]);
        }
#pragma unroll 1
        for (int q = 0; q < 4; ++q)
          if ((escm >> q) & 1u) tmp[2 * q] = payload1_slow(tmp[2 * q], __uint_as_float(tmp[2 * q + 1]), tb, sumfix);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if ((escm >> q) & 1u) pl[q] = tmp[2 * q];
      }
      uint2 dv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) dv[q] = dw[(sv[g + q] >> (TILE_SHIFT + 5)) & 1023u];  // (any word when s >= S)
      uint32_t bn[4], sl[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t s = sv[g + q];
        const uint32_t tw = __builtin_amdgcn_ubfe(s, TILE_SHIFT, 5);  // tile within its direct word
        const bool direct = __builtin_amdgcn_ubfe(dv[q].x, tw, 1) != 0u;
        rec[g + q] = ((s & (ST_TILES * TILE - 1)) << 21) | pl[q];  // tile in ST | series in tile | payload
        const uint32_t dbin =
            FS + 2u * (dv[q].y + (uint32_t)__popc(__builtin_amdgcn_ubfe(dv[q].x, 0, tw))) + ((s >> 4) & 1u);
        bn[q] = sel_u32(s < S, sel_u32(direct, dbin, s >> ST_SHIFT), TB);
      }
      if (HS) {
#pragma unroll
        for (int q = 0; q < 4; ++q) sl[q] = hslot[bn[q]];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const bool hot = sl[q] < (uint32_t)NHOT;
          uint32_t* ctr = hot ? hcnt + sl[q] * 64u + (uint32_t)lane : cnt + bn[q];
          pk[g + q] = atomicAdd(ctr, 1u) | (bn[q] << 14) | (sl[q] << 25);
        }
      } else {
        if (!hotrank) {
#pragma unroll
          for (int q = 0; q < 4; ++q) pk[g + q] = atomicAdd(cnt + bn[q], 1u) | (bn[q] << 14);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) pk[g + q] = bn[q] << 14;  // ranked below, all PT slots at once
        }
      }
      asm volatile("" ::: "memory");  // keep the groups apart (bounded register pressure)
    }
    if (hotrank) {
      // ranks: the batch's two hottest bins (k_stplan; e.g. a Zipf head's direct tile,
      // ~1/4 of C3) by wave ballots -- one LDS atomic per wave and bin for all PT
      // slots, and consecutive stage slots for a wave's hot samples -- the other bins
      // by one LDS atomic per slot.  Same-address atomics on a hot counter otherwise
      // serialize (SQ_LDS_ADDR_CONFLICT) and their scattered stage slots conflict.
      uint32_t wc0 = 0, wc1 = 0;
#pragma unroll
      for (int k = 0; k < PT; ++k) {
        const uint32_t b = pk[k] >> 14;
        const bool m0 = b == hb0, m1 = b == hb1;
        wc0 += (uint32_t)__popcll(__ballot(m0));
        wc1 += (uint32_t)__popcll(__ballot(m1));
        if (!m0 && !m1) pk[k] |= atomicAdd(cnt + b, 1u);
      }
      uint32_t base = 0;
      if (lane == 0 && wc0) base = atomicAdd(cnt + hb0, wc0);
      if (lane == 1 && wc1) base = atomicAdd(cnt + hb1, wc1);
      uint32_t r0 = __builtin_amdgcn_readlane(base, 0), r1 = __builtin_amdgcn_readlane(base, 1);
#pragma unroll
      for (int k = 0; k < PT; ++k) {
        const uint32_t b = pk[k] >> 14;
        const bool m0 = b == hb0, m1 = b == hb1;
        const unsigned long long x0 = __ballot(m0), x1 = __ballot(m1);
        if (m0) pk[k] |= r0 + mask_below(x0);
        if (m1) pk[k] |= r1 + mask_below(x1);
        r0 += (uint32_t)__popcll(x0);
        r1 += (uint32_t)__popcll(x1);
      }
    }
    if (L5DH_EXP & 16) {  // timing: loads + ranking only (no scan, scatter or run writes)
      uint32_t x = 0;
#pragma unroll
      for (int k = 0; k < PT; ++k) x ^= pk[k] ^ rec[k];
      if (x == 0x12345678u) out1[threadIdx.x] = x;
      __syncthreads();
      for (uint32_t j = threadIdx.x; j <= TB; j += NT) cnt[j] = 0;
      __syncthreads();
      continue;
    }
    __syncthreads();
    if (wv == 0) {  // one wave: hot-slot lane prefixes and totals, then the bin scan (DPP, no barriers)
      if (HS) {
        uint32_t hv[NHOT];
#pragma unroll
        for (int h = 0; h < NHOT; ++h) hv[h] = hcnt[h * 64 + lane];  // rows of unused slots are zero
#pragma unroll
        for (int h = 0; h < NHOT; ++h) {
          const uint32_t x = wave_incl_scan32(hv[h]);
          hcnt[h * 64 + lane] = x - hv[h];
          const uint32_t hk = plan[3 * FS + 1 + h];
          if (lane == 63 && hk != NOKEY) cnt[hk] = x;
        }
      }
      uint32_t c[16];  // lane l scans bins [16 l, 16 l + 16)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint4 v = *reinterpret_cast<const uint4*>(cnt + 16 * lane + 4 * q);
        c[4 * q] = v.x; c[4 * q + 1] = v.y; c[4 * q + 2] = v.z; c[4 * q + 3] = v.w;
      }
      uint32_t tl = 0;
#pragma unroll
      for (int q = 0; q < 16; ++q) tl += c[q];
      uint32_t e = wave_incl_scan32(tl) - tl;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        oc[16 * lane + q].x = e;
        e += c[q];
      }
      // unsplit direct tiles: this sub-chunk's run of the even bin, then the odd bin's,
      // from the shared cursor (held by the odd bin: the advance below adds both counts)
      for (uint32_t d = (uint32_t)lane; d < ND; d += 64)
        if ((dun[d >> 5] >> (d & 31u)) & 1u) {
          const uint32_t b0 = FS + 2 * d;
          const uint32_t base = oc[b0 + 1].y;
          oc[b0].y = base;
          oc[b0 + 1].y = base + cnt[b0];
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      const uint32_t bin = (pk[k] >> 14) & 2047u;
      const uint32_t r = (pk[k] & 16383u) + (HS ? hcnt[(pk[k] >> 25) * 64 + lane] : 0u);  // row NHOT is zero
      const uint2 x = oc[bin];
      stage[x.x + r] = make_uint2(rec[k], x.y + r);
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < TB; j += NT) {  // cursors advance; the stage carries the destinations
      oc[j].y += cnt[j];
      cnt[j] = 0;
    }
    if (threadIdx.x == 0) cnt[TB] = 0;
    if (HS)
      for (uint32_t i = threadIdx.x; i < NHOT * 64; i += NT) hcnt[i] = 0;
#pragma unroll
    for (int k = 0; k < PT; ++k) {  // all CH1 entries, in sorted order (trash entries land past scratch1[n])
      const uint2 e = stage[(uint32_t)wv * (PT * 64) + (uint32_t)k * 64 + (uint32_t)lane];  // each wave: a contiguous PT x 64 range
      if (L5DH_EXP & 1024)  // timing: the same stores, sequential (where the slots were read)
        out1[c0 + threadIdx.x + k * NT] = e.x;
      else if (L5DH_EXP & 2048) {  // timing: whole 64-B segments, 1024 interleaved sequential streams
        const size_t idx = c0 + threadIdx.x + k * NT;
        const size_t seg = idx >> 4, nseg = n >> 4;
        out1[((seg & 1023) * (nseg >> 10) + (seg >> 10)) * 16 + (idx & 15)] = e.x;
      }
      else if (!(dbg & 1))
        ((e.y >> 31) ? records : out1)[e.y & 0x7FFFFFFFu] = e.x;
    }
    __syncthreads();
  }
}

// Ingest plan (one workgroup, after the tile totals are known):
//   plan[0..FS]          level-2 item_start per super-tile (nb_j items of equal
//                        slab ranges, ~B2_ITEM level-1 records each: skew-balanced;
//                        0 items for a super-tile whose tiles are all split/empty)
//   plan[FS+1 .. 2FS]    slab-range size per super-tile
//   plan[2FS+1 .. 3FS]   hot non-split tiles of the super-tile (tile-in-ST, byte 0
//                        and 1; 0xFF = none): >= 1/8 of its level-1 records
//   plan[3FS+1 .. +NHOT] hot k_bin1 bins (>= 1/128 of all records, or ~0u)
//   plan[PLAN_DBITS..]   this batch's direct tiles (bitmap, prefixes, list, split index)
//   nxt                  the next batch's split set
//   plan[PLAN_HINT..+1]  hot count columns for the next batch's k_count
__global__ __launch_bounds__(1024) void k_stplan(uint32_t F, int G, const uint32_t* __restrict__ coltot,
                                                 uint32_t* __restrict__ plan, const uint32_t* __restrict__ cur,
                                                 uint32_t* __restrict__ nxt, uint32_t thr_min, uint32_t dmax,
                                                 uint32_t split_min, int hot_bins, const uint32_t* __restrict__ err,
                                                 uint32_t* __restrict__ err_host) {
  // the invalid-id count of k_count, to the host's mapped pinned word (no copy launch)
  if (threadIdx.x == 0) *reinterpret_cast<volatile uint32_t*>(err_host) = *err;
  __shared__ uint4 lds4[17];
  __shared__ unsigned long long best[16];
  __shared__ uint32_t lhd[33], lhs[33];
  __shared__ uint32_t sthr[2];
  const uint32_t FS = (F + ST_TILES - 1) / ST_TILES;
  const uint32_t j = threadIdx.x;
  const uint32_t NS = cur[0];
  if (j < 33) lhd[j] = lhs[j] = 0;
  __syncthreads();
  // direct tiles: tiles of this batch (split or not: the exact totals of k_count)
  // with >= max(thr_min, 2^k) records; next split set: tiles with >= max(split_min,
  // 2^k) records
  (void)NS;
  {  // F <= 32768 tiles: a thread's <= 32 totals are loaded at once (one latency, not 32)
    constexpr int PF = 32;
    uint32_t tv[PF];
#pragma unroll
    for (int k = 0; k < PF; ++k) tv[k] = j + 1024u * k < F ? coltot[j + 1024u * k] : 0u;
#pragma unroll
    for (int k = 0; k < PF; ++k) {
      if (tv[k] >= split_min && tv[k] > 0) atomicAdd(&lhs[31 - __clz((int)tv[k])], 1u);
      if (dmax > 0 && tv[k] >= thr_min && tv[k] > 0) atomicAdd(&lhd[31 - __clz((int)tv[k])], 1u);
    }
  }
  __syncthreads();
  if (j < 2) {
    // cum_k = tiles with floor(log2 v) >= k (non-increasing in k): the smallest k
    // with cum_k <= cap gives thr = max(lo, 2^k)
    const uint32_t* lh = j ? lhs : lhd;
    const uint32_t cap = j ? (uint32_t)SPLIT_MAX : dmax;
    const uint32_t lo = max(j ? split_min : thr_min, 1u);
    uint32_t thr = NOKEY;
    if (cap > 0) {
      uint32_t cum = 0;
      int kbest = 32;
      for (int k = 31; k >= 0; --k) {
        cum += lh[k];
        if (cum > cap) break;
        kbest = k;
      }
      if (kbest < 32) thr = max(lo, 1u << kbest);
    }
    sthr[j] = thr;
  }
  __syncthreads();
  const uint32_t thr_d = sthr[0], thr_s = sthr[1];
  uint32_t nb = 0, gsz = 0, hot = 0xFFFFu, nn = 0, ndt = 0, n0 = 0, n1 = 0, d0 = 0, d1 = 0;
  uint32_t c0 = 0, c1 = 0;  // this batch's split words of the super-tile
  uint64_t ctot = 0, tot = 0;
  unsigned long long tkA = 0, tkB = 0;  // (records << 16 | tile): this thread's two biggest tiles
  if (j < FS) {
    c0 = cur[SPLIT_BITS + 2 * j];
    c1 = 2 * j + 1 < 1024 ? cur[SPLIT_BITS + 2 * j + 1] : 0u;
    const uint32_t t1 = min(F, (j + 1) * ST_TILES);
    uint32_t b0 = 0, b1 = 0, i0 = 0xFF, i1 = 0xFF;  // two biggest level-1 tiles of this super-tile
    uint32_t a0 = 0, a1 = 0, k0 = 0xFF, k1 = 0xFF;  // two biggest tiles
    // the super-tile's 64 totals in 16 loads issued at once (coltot holds F + COLS
    // words, so the reads past F stay in bounds; those tiles are skipped)
    uint32_t cv[ST_TILES];
    const uint4* c4 = reinterpret_cast<const uint4*>(coltot + j * ST_TILES);
#pragma unroll
    for (int q = 0; q < ST_TILES / 4; ++q) {
      const uint4 x = c4[q];
      cv[4 * q] = x.x;
      cv[4 * q + 1] = x.y;
      cv[4 * q + 2] = x.z;
      cv[4 * q + 3] = x.w;
    }
#pragma unroll
    for (uint32_t tl = 0; tl < (uint32_t)ST_TILES; ++tl) {
      if (j * ST_TILES + tl < t1) {
        const uint32_t v = cv[tl];
        tot += v;
        if (v > a0) { a1 = a0; k1 = k0; a0 = v; k0 = tl; }
        else if (v > a1) { a1 = v; k1 = tl; }
        if (v >= thr_s) {
          if (tl < 32) n0 |= 1u << tl; else n1 |= 1u << (tl - 32);
        }
        if (v >= thr_d) {  // direct: no level-1 records
          if (tl < 32) d0 |= 1u << tl; else d1 |= 1u << (tl - 32);
        } else {
          ctot += v;
          if (v > b0) { b1 = b0; i1 = i0; b0 = v; i0 = tl; }
          else if (v > b1) { b1 = v; i1 = tl; }
        }
      }
    }
    nn = (uint32_t)(__popc(n0) + __popc(n1));
    ndt = (uint32_t)(__popc(d0) + __popc(d1));
    tkA = k0 != 0xFF ? (((unsigned long long)a0 << 16) | (j * ST_TILES + k0)) : 0ull;
    tkB = k1 != 0xFF ? (((unsigned long long)a1 << 16) | (j * ST_TILES + k1)) : 0ull;
    if ((uint64_t)b0 * 8 < ctot || b0 == 0) i0 = 0xFF;
    if ((uint64_t)b1 * 8 < ctot || b1 == 0) i1 = 0xFF;
    hot = (i0 == 0xFF ? 0xFFu : 2 * i0) | ((i1 == 0xFF ? 0xFFu : 2 * i1) << 8);  // k_bin2 keys (half 0)
    if (ctot > 0) {
      uint32_t want = (uint32_t)((ctot + B2_ITEM - 1) / B2_ITEM);
      want = max(1u, min(want, (uint32_t)G));
      gsz = ((uint32_t)G + want - 1) / want;
      nb = ((uint32_t)G + gsz - 1) / gsz;
    } else {
      gsz = (uint32_t)G;
    }
  }
  uint32_t sv3[4] = {nb, nn, ndt, 0u}, st3[4];
  block_excl_scan4<1024>(sv3, lds4, st3);
  const uint32_t e = sv3[0], ne = sv3[1], de = sv3[2];
  const uint32_t total = st3[0], nnt = st3[1], ndtot = st3[2];
  // this thread's NHOT biggest k_bin1 bins, descending: (records << 11 | bin)
  unsigned long long bk[NHOT] = {};
  auto push = [&](unsigned long long k) {
#pragma unroll
    for (int q = 0; q < NHOT; ++q)
      if (k > bk[q]) {
        const unsigned long long x = bk[q];
        bk[q] = k;
        k = x;
      }
  };
  if (j < FS) {
    plan[j] = e;
    plan[FS + 1 + j] = gsz;
    uint16_t* imap = reinterpret_cast<uint16_t*>(plan + PLAN_ITEMS);  // k_bin2: item -> super-tile, one load
    for (uint32_t k = 0; k < nb; ++k) imap[e + k] = (uint16_t)j;
    plan[2 * FS + 1 + j] = hot;
    // this batch's direct tiles, their split index and half bins
    plan[PLAN_DBITS + 2 * j] = d0;
    plan[PLAN_DPRE + 2 * j] = de;
    if (2 * j + 1 < 1024) {
      plan[PLAN_DBITS + 2 * j + 1] = d1;
      plan[PLAN_DPRE + 2 * j + 1] = de + (uint32_t)__popc(d0);
    }
    // (stores only: the half totals of the direct tiles are read below, one direct tile
    // per thread, instead of as a chain of dependent loads in this loop)
    uint32_t di = de;
    for (int q = 0; q < 2; ++q) {
      uint32_t w = q ? d1 : d0;
      const uint32_t cw = q ? c1 : c0;
      const uint32_t sp = cur[SPLIT_PRE + 2 * j + q];
      while (w) {
        const uint32_t b = (uint32_t)(__ffs((int)w) - 1);
        w &= w - 1u;
        plan[PLAN_DLIST + di] = j * ST_TILES + 32u * q + b;
        // split index, or NOKEY: an unsplit direct tile (its two bins share its range)
        plan[PLAN_DSI + di] = ((cw >> b) & 1u) ? sp + (uint32_t)__popc(cw & ((1u << b) - 1u)) : NOKEY;
        ++di;
      }
    }
    if (ctot && hot_bins) push((ctot << 11) | j);
    // the next batch's split set
    nxt[SPLIT_BITS + 2 * j] = n0;
    nxt[SPLIT_PRE + 2 * j] = ne;
    if (2 * j + 1 < 1024) {
      nxt[SPLIT_BITS + 2 * j + 1] = n1;
      nxt[SPLIT_PRE + 2 * j + 1] = ne + (uint32_t)__popc(n0);
    }
    uint32_t h = ne;
    for (int q = 0; q < 2; ++q) {
      uint32_t w = q ? n1 : n0;
      while (w) {
        const uint32_t tl = (uint32_t)(__ffs((int)w) - 1) + 32u * q;
        w &= w - 1u;
        nxt[SPLIT_LIST + h++] = j * ST_TILES + tl;
      }
    }
  }
  if (threadIdx.x == 0) {
    plan[FS] = total;
    plan[PLAN_ND] = ndtot;
    nxt[0] = nnt;
  }
  __syncthreads();  // the direct list is written
  for (uint32_t d = threadIdx.x; hot_bins && d < ndtot; d += 1024) {  // the direct tiles' half bins as hot-bin candidates
    const uint32_t si = plan[PLAN_DSI + d];
    if (si == NOKEY) {  // an unsplit direct tile: its records split between both bins by series bit 4
      const unsigned long long h = coltot[plan[PLAN_DLIST + d]] / 2;
      push((h << 11) | (FS + 2 * d));
      push((h << 11) | (FS + 2 * d + 1));
    } else {
      push(((unsigned long long)coltot[F + 2 * si] << 11) | (FS + 2 * d));
      push(((unsigned long long)coltot[F + 2 * si + 1] << 11) | (FS + 2 * d + 1));
    }
  }
  // grand total, the hot bins and the two biggest tiles (block reductions)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  auto block_reduce = [&](unsigned long long v, bool is_max) -> unsigned long long {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
      const unsigned long long o = __shfl_xor(v, d, 64);
      v = is_max ? (o > v ? o : v) : v + o;
    }
    __syncthreads();
    if (lane == 0) best[w] = v;
    __syncthreads();
    unsigned long long r = 0;
    for (int q = 0; q < 16; ++q) r = is_max ? (best[q] > r ? best[q] : r) : r + best[q];
    return r;
  };
  const unsigned long long grand = block_reduce(tot, false);
  // (only the lane-private hot-slot variants of k_bin1 use them: 16 barriers saved otherwise)
  unsigned long long ks[NHOT] = {};
  int head = 0;  // this thread's first bin not yet selected
  // the hottest bins: 2 for the ballot ranking; all NHOT for the lane-private-slot
  // development variant (hot_bins bit 2) -- each is a block reduction
  const int nh = (hot_bins & 4) ? NHOT : 2;
  if (hot_bins) {
#pragma unroll
    for (int q = 0; q < NHOT; ++q) {
      if (q >= nh) break;
      unsigned long long mine = 0;
#pragma unroll
      for (int r = 0; r < NHOT; ++r)
        if (r == head) mine = bk[r];
      ks[q] = block_reduce(mine, true);
      if (mine != 0 && mine == ks[q]) ++head;
    }
  }
  const unsigned long long t1 = block_reduce(tkA, true);
  const unsigned long long t2 = block_reduce(tkA == t1 ? tkB : tkA, true);
  if (threadIdx.x == 0) {
    // bins with >= 1/128 of the records: k_bin1 counts them in lane-private slots
    // when the hottest one holds >= half of all records
    for (int h = 0; h < NHOT; ++h) {
      const uint64_t v = ks[h] >> 11;
      plan[3 * FS + 1 + h] = (v > 0 && v * 128 >= grand) ? (uint32_t)(ks[h] & 2047u) : NOKEY;
    }
    plan[PLAN_HS] = grand > 0 && (ks[0] >> 11) * 2 >= grand ? 1u : 0u;  // k_bin1: ballot ranks
    // next batch's k_count hints: the count columns of the two biggest tiles
    // (both halves of a tile that will be split); aggregation only
    uint32_t hkey[4] = {NOKEY, NOKEY, NOKEY, NOKEY};
    int nh = 0;
    const unsigned long long ts[2] = {t1, t2};
    for (int q = 0; q < 2 && nh < 4; ++q) {
      const uint64_t v = ts[q] >> 16;
      if (v == 0 || v * 64 < grand) continue;
      const uint32_t t = (uint32_t)(ts[q] & 0xFFFFu);
      const uint32_t wd = nxt[SPLIT_BITS + (t >> 5)];  // written above by this workgroup
      const uint32_t bit = 1u << (t & 31u);
      if (wd & bit) {
        const uint32_t si = nxt[SPLIT_PRE + (t >> 5)] + (uint32_t)__popc(wd & (bit - 1u));
        hkey[nh++] = F + 2 * si;
        hkey[nh++] = F + 2 * si + 1;
      } else {
        hkey[nh++] = t;
      }
    }
    for (int h = 0; h < 4; ++h) plan[PLAN_HINT + h] = hkey[h];
  }
}

// Level 2.  Item = (super-tile j, slab range [g0, g1)).  Its level-1 records are
// one contiguous range; the records of tile t (of half h of t, for a split tile)
// in that range go, in any order, to [tile_base[t] (+ half-0 total) + pre[g0][col],
// ...) -- exactly where the per-(slab, tile) segments g0..g1-1 of the final
// layout lie.  Keys: 2 x tile-in-ST + half (half 0 for an unsplit tile).
constexpr int B2_KEYS = 2 * ST_TILES;
constexpr size_t bin2_lds(int ch) { return (size_t)ch * 8 + 3 * B2_KEYS * 4 + 16; }
template <int CH2, int B2_NT>
__global__ __launch_bounds__(B2_NT) void k_bin2(const uint32_t* __restrict__ out1, uint32_t F, int G,
                                                const uint32_t* __restrict__ pre,
                                                const uint32_t* __restrict__ tile_base,
                                                const uint32_t* __restrict__ coltot,
                                                const uint32_t* __restrict__ split,
                                                const uint32_t* __restrict__ plan, Tables tb,
                                                uint32_t* __restrict__ records) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint2* stage = reinterpret_cast<uint2*>(smem);  // [CH2] sub-chunk sorted by key: {record, global index - stage index}
  uint32_t* cur = smem + 2 * CH2;                 // [B2_KEYS] global write position of each key
  uint32_t* cnt = cur + B2_KEYS;                  // [B2_KEYS] records of each key in this sub-chunk
  uint32_t* off = cnt + B2_KEYS;                  // [B2_KEYS] their exclusive offsets in stage
  uint32_t* seg = off + B2_KEYS;                  // [2]
  const uint32_t FS = (F + ST_TILES - 1) / ST_TILES;
  const uint32_t C = F + COLS;
  const uint32_t item = blockIdx.x;
  // (both loads at once: entries past the batch's items are stale, never used)
  const uint32_t nitems = plan[FS];
  const uint32_t j = reinterpret_cast<const uint16_t*>(plan + PLAN_ITEMS)[item];
  if (item >= nitems) return;
  const uint32_t gsz = plan[FS + 1 + j];
  const int g0 = (int)((item - plan[j]) * gsz);
  const int g1 = min(G, g0 + (int)gsz);
  const uint32_t hp = plan[2 * FS + 1 + j];
  const uint32_t hot0 = (hp & 0xFFu) == 0xFFu ? NOKEY : (hp & 0xFFu);
  const uint32_t hot1 = ((hp >> 8) & 0xFFu) == 0xFFu ? NOKEY : ((hp >> 8) & 0xFFu);
  const uint32_t hk[2] = {hot0, hot1};
  const uint32_t t0 = j * ST_TILES;
  const uint32_t nt = min((uint32_t)ST_TILES, F - t0);
  // split (and not direct) tiles of the super-tile: records keyed by half
  const uint32_t sw0 = split[SPLIT_BITS + 2 * j] & ~plan[PLAN_DBITS + 2 * j];
  const uint32_t sw1 = 2 * j + 1 < 1024 ? split[SPLIT_BITS + 2 * j + 1] & ~plan[PLAN_DBITS + 2 * j + 1] : 0u;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    uint32_t q0 = 0, q1 = 0, r0 = 0, r1 = 0;  // keys 2 lane, 2 lane + 1: pre[g0], pre[g1]
    if ((uint32_t)lane < nt) {
      const uint32_t t = t0 + lane;
      const uint32_t bit = 1u << (t & 31u);
      const bool direct = plan[PLAN_DBITS + (t >> 5)] & bit;
      const uint32_t wd = split[SPLIT_BITS + (t >> 5)];
      const uint32_t tb0 = tile_base[t];
      if (direct) {  // its records never reach level 1
        cur[2 * lane] = cur[2 * lane + 1] = tb0;
      } else if (wd & bit) {
        const uint32_t si = split[SPLIT_PRE + (t >> 5)] + (uint32_t)__popc(wd & (bit - 1u));
        const uint32_t c0 = F + 2 * si;
        q0 = pre[(size_t)g0 * C + c0];
        q1 = pre[(size_t)g0 * C + c0 + 1];
        r0 = g1 < G ? pre[(size_t)g1 * C + c0] : coltot[c0];
        r1 = g1 < G ? pre[(size_t)g1 * C + c0 + 1] : coltot[c0 + 1];
        cur[2 * lane] = tb0 + q0;
        cur[2 * lane + 1] = tb0 + coltot[c0] + q1;
      } else {
        q0 = pre[(size_t)g0 * C + t];
        r0 = g1 < G ? pre[(size_t)g1 * C + t] : (tile_base[t + 1] - tb0);
        cur[2 * lane] = tb0 + q0;
        cur[2 * lane + 1] = 0;
      }
    }
    cnt[2 * lane] = cnt[2 * lane + 1] = 0;
    uint32_t p0 = q0 + q1, p1 = r0 + r1;
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
      p0 += __shfl_xor(p0, d, 64);
      p1 += __shfl_xor(p1, d, 64);
    }
    if (lane == 0) {
      seg[0] = tile_base[t0] + p0;
      seg[1] = tile_base[t0] + p1;
    }
  }
  __syncthreads();
  const uint32_t A = seg[0], B = seg[1];
  const uint32_t A16 = A & ~3u;  // 16-B aligned start; lanes below A are masked off
  constexpr int PT = CH2 / B2_NT;  // records per thread (groups of 4)
  uint4 xn[PT / 4];                 // next sub-chunk, prefetched while this one is sorted and written
#pragma unroll
  for (int k = 0; k < PT / 4; ++k) {
    const uint32_t base = A16 + 4 * (k * B2_NT + threadIdx.x);
    xn[k] = base < B ? *reinterpret_cast<const uint4*>(out1 + base) : make_uint4(0u, 0u, 0u, 0u);
  }
  for (uint32_t c0 = A16; c0 < B; c0 += CH2) {
    uint32_t rec[PT], kv[PT], rank[PT];
    uint4 xc[PT / 4];
#pragma unroll
    for (int k = 0; k < PT / 4; ++k) {
      xc[k] = xn[k];
      const uint32_t nbase = c0 + CH2 + 4 * (k * B2_NT + threadIdx.x);  // out1 padded to a multiple of 4
      xn[k] = nbase < B ? *reinterpret_cast<const uint4*>(out1 + nbase) : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int k = 0; k < PT / 4; ++k) {
      const uint32_t base = c0 + 4 * (k * B2_NT + threadIdx.x);
      const uint4 x = xc[k];
      const uint32_t xv[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t idx = base + e;
        const bool valid = idx >= A && idx < B;
        const uint32_t r = xv[e];
        const uint32_t tl = r >> 26;
        const uint32_t sp = ((tl < 32 ? sw0 : sw1) >> (tl & 31u)) & 1u;
        rec[4 * k + e] = r;  // records pass through unchanged (key order is all that changes)
        kv[4 * k + e] = valid ? 2u * tl + (sp & (r >> 25)) : 0xFFFFFFFFu;
      }
    }
    hot_rank_batch<2, PT>(cnt, kv, hk, rank);
    __syncthreads();
    if (threadIdx.x < 64) {  // exclusive scan of the 128 key counts (one wave, two per lane)
      const uint32_t a = cnt[2 * threadIdx.x], b = cnt[2 * threadIdx.x + 1];
      const uint32_t x = wave_incl_scan32(a + b) - (a + b);
      off[2 * threadIdx.x] = x;
      off[2 * threadIdx.x + 1] = x + a;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      if (kv[k] != 0xFFFFFFFFu) {
        const uint32_t o = off[kv[k]];
        const uint32_t pos = o + rank[k];
        stage[pos] = make_uint2(rec[k], cur[kv[k]] - o);
      }
    }
    const uint32_t total = off[B2_KEYS - 1] + cnt[B2_KEYS - 1];
    __syncthreads();
    {
      uint2 ev[PT];
      const uint32_t w0 = (threadIdx.x >> 6) * (PT * 64) + (threadIdx.x & 63u);  // each wave: a contiguous PT x 64 range
#pragma unroll
      for (int k = 0; k < PT; ++k) ev[k] = stage[w0 + k * 64];
#pragma unroll
      for (int k = 0; k < PT; ++k) {
        const uint32_t i = w0 + k * 64;
        if (i < total) records[ev[k].y + i] = ev[k].x;
      }
    }
    if (threadIdx.x < B2_KEYS) {
      cur[threadIdx.x] += cnt[threadIdx.x];
      cnt[threadIdx.x] = 0;
    }
    __syncthreads();
  }
}

// Small host batches into the staging ring: the GPU reads pinned host memory
// directly (zero-copy over PCIe) -- one kernel for both arrays, instead of two
// DMA copies whose setup dominates at 64K samples (35 us per pair measured).
__global__ __launch_bounds__(256) void k_fetch_host(const uint32_t* __restrict__ hs, const uint32_t* __restrict__ hv,
                                                    uint32_t* __restrict__ ds, uint32_t* __restrict__ dv, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t s = hs[i], v = hv[i];
    ds[i] = s;
    dv[i] = v;
  }
}

}  // namespace

hipError_t launch_fetch_host(const uint32_t* hs, const uint32_t* hv, uint32_t* ds, uint32_t* dv, size_t n,
                             hipStream_t st) {
  if (n == 0) return hipSuccess;
  const size_t blocks = std::min<size_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(k_fetch_host, dim3((unsigned)blocks), dim3(256), 0, st, hs, hv, ds, dv, n);
  return hipGetLastError();
}

// ------------------------------------------------------------------------
hipError_t set_ingest_attributes() {
  hipError_t e;
  const int big = 160 * 1024;
  if ((e = hipFuncSetAttribute((const void*)k_count, hipFuncAttributeMaxDynamicSharedMemorySize, big))) return e;
  if ((e = hipFuncSetAttribute((const void*)k_bin, hipFuncAttributeMaxDynamicSharedMemorySize, big))) return e;
  if ((e = hipFuncSetAttribute((const void*)k_tilescan_seg, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)((tpad(32768) + 1) * 4))))
    return e;
  if ((e = hipFuncSetAttribute((const void*)k_bin1<16384, 1024, 4, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)bin1_lds(16384))))
    return e;
  if ((e = hipFuncSetAttribute((const void*)k_bin1<6144, 512, 4, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)bin1_lds(6144))))
    return e;
  if ((e = hipFuncSetAttribute((const void*)k_bin1<16384, 1024, 4, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)bin1_lds(16384))))
    return e;
  if ((e = hipFuncSetAttribute((const void*)k_bin2<8192, 512>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)bin2_lds(8192))))
    return e;
  if ((e = hipFuncSetAttribute((const void*)k_bin2<16384, 1024>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)bin2_lds(16384))))
    return e;


  return hipSuccess;
}

hipError_t launch_count(const uint32_t* series, size_t n, size_t per, int G, uint32_t S, uint32_t F,
                        uint32_t* table, uint32_t* err, const uint32_t* hint, const uint32_t* split, bool vec,
                        hipStream_t st) {
  hipLaunchKernelGGL(k_count, dim3(G), dim3(WG), ((size_t)F + COLS + 2048) * 4, st, series, n, per, S, F, table, err,
                     hint, split, vec ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_colscan(uint32_t* table, int G, uint32_t F, uint32_t* coltot, hipStream_t st) {
  hipLaunchKernelGGL(k_colscan, dim3((F + COLS + 63) / 64), dim3(1024), 0, st, table, G, F + COLS, coltot);
  return hipGetLastError();
}

hipError_t launch_tilescan(uint32_t* coltot, uint32_t F, const uint32_t* split, uint32_t* tile_base, hipStream_t st) {
  hipLaunchKernelGGL(k_tilescan, dim3(1), dim3(1024), 0, st, coltot, F, split, tile_base);
  return hipGetLastError();
}

hipError_t launch_tilescan_seg(uint32_t* coltot, uint32_t F, const uint32_t* split, uint32_t* tile_base,
                               uint32_t* sinfo, hipStream_t st) {
  hipLaunchKernelGGL(k_tilescan_seg, dim3(1), dim3(1024), (tpad(F) + 1) * 4, st, coltot, F, split, tile_base, sinfo);
  return hipGetLastError();
}

hipError_t launch_seginfo(const uint32_t* split, const uint32_t* coltot, uint32_t F, uint32_t* sinfo, hipStream_t st) {
  hipLaunchKernelGGL(k_seginfo, dim3(1), dim3(1024), 0, st, split, coltot, F, sinfo);
  return hipGetLastError();
}

hipError_t launch_encode1(const uint32_t* series, const float* values, size_t n, uint32_t S, Tables tb,
                          uint32_t* records, int64_t* sumfix, uint32_t* tile_base, uint32_t* err, bool vec, int num_cu,
                          hipStream_t st) {
  const size_t groups = (n + 4 * 256 - 1) / (4 * 256);
  const uint32_t grid = (uint32_t)std::max<size_t>(1, std::min<size_t>(groups, (size_t)num_cu * 8));
  hipLaunchKernelGGL(k_encode1, dim3(grid), dim3(256), 0, st, series, values, n, S, tb, records, sumfix, tile_base, err,
                     vec ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_bin(const uint32_t* series, const float* values, size_t n, size_t per, int G, uint32_t S,
                      uint32_t F, const uint32_t* table, const uint32_t* tile_base, Tables tb, uint32_t* records,
                      int64_t* sumfix, bool vec, hipStream_t st) {
  const size_t lds = (size_t)F * 4;  // the batch was counted without split tiles (tile columns only)
  hipLaunchKernelGGL(k_bin, dim3(G), dim3(WG), lds, st, series, values, n, per, S, F, table, tile_base, tb, records,
                     sumfix, vec ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_stplan(uint32_t F, int G, const uint32_t* coltot, uint32_t* stplan, const uint32_t* cur,
                         uint32_t* nxt, uint32_t thr_min, uint32_t dmax, uint32_t split_min, int hot_bins,
                         const uint32_t* err, uint32_t* err_host, hipStream_t st) {
  const uint32_t FS = (F + 63) / 64;
  const uint32_t cap = std::min<uint32_t>((uint32_t)DIRECT_MAX, ((uint32_t)BIN1_BINS - 1 - FS) / 2);  // + trash bin
  hipLaunchKernelGGL(k_stplan, dim3(1), dim3(1024), 0, st, F, G, coltot, stplan, cur, nxt, thr_min, std::min(dmax, cap),
                     split_min, hot_bins, err, err_host);
  return hipGetLastError();
}

hipError_t launch_bin1(const uint32_t* series, const float* values, size_t n, size_t per, int G, uint32_t S,
                       uint32_t F, const uint32_t* pre, const uint32_t* tile_base, Tables tb, const uint32_t* stplan,
                       const uint32_t* coltot, const uint32_t* split, uint32_t* scratch1, uint32_t* records,
                       int64_t* sumfix, bool vec, int dbg, hipStream_t st) {
  // sub-chunk size x workgroup: (16384 slots, 1024 threads, 1 workgroup/CU) by
  // default -- longer runs per bin beat the second workgroup's overlap (measured);
  // L5DH_DBG bit 20 selects (6144, 512, 2 workgroups/CU)
  if ((dbg >> 20) & 1)
    hipLaunchKernelGGL((k_bin1<6144, 512, 4, true>), dim3(G), dim3(512), bin1_lds(6144), st, series, values, n, per, S, F,
                       pre, tile_base, tb, stplan, coltot, split, scratch1, records, sumfix, vec ? 1 : 0, dbg);
  else if ((dbg >> 22) & 1)  // bit 22: lane-private slots for the hottest bins (measured 5-8 % slower)
    hipLaunchKernelGGL((k_bin1<16384, 1024, 4, true>), dim3(G), dim3(1024), bin1_lds(16384), st, series, values, n, per, S,
                       F, pre, tile_base, tb, stplan, coltot, split, scratch1, records, sumfix, vec ? 1 : 0, dbg);
  else
    hipLaunchKernelGGL((k_bin1<16384, 1024, 4, false>), dim3(G), dim3(1024), bin1_lds(16384), st, series, values, n, per, S,
                       F, pre, tile_base, tb, stplan, coltot, split, scratch1, records, sumfix, vec ? 1 : 0, dbg);
  return hipGetLastError();
}

hipError_t launch_bin2(const uint32_t* scratch1, size_t n, int G, uint32_t F, const uint32_t* pre,
                       const uint32_t* tile_base, const uint32_t* coltot, const uint32_t* split, Tables tb,
                       const uint32_t* stplan, uint32_t* records, int dbg, hipStream_t st) {
  const uint32_t FS = (F + ST_TILES - 1) / ST_TILES;
  const size_t max_items = n / B2_ITEM + FS + 1;  // sum_j ceil(tot_j / B2_ITEM)
  // sub-chunk x workgroup: (8192, 512) by default (measured: longer runs per key
  // than (4096, 256)); L5DH_DBG bit 21: (16384, 1024)
  if ((dbg >> 21) & 1)
    hipLaunchKernelGGL((k_bin2<16384, 1024>), dim3((unsigned)max_items), dim3(1024), bin2_lds(16384), st, scratch1, F,
                       G, pre, tile_base, coltot, split, stplan, tb, records);
  else
    hipLaunchKernelGGL((k_bin2<8192, 512>), dim3((unsigned)max_items), dim3(512), bin2_lds(8192), st, scratch1, F, G,
                       pre, tile_base, coltot, split, stplan, tb, records);
  return hipGetLastError();
}

}  // namespace l5dh
