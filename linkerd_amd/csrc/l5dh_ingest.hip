// l5dh_ingest.hip -- ingest-side kernels (Metric.Stat.add, batched).
//
//   k_count    LDS tile histogram of each slab of the COO batch -> table[g][t]
//   k_colscan  per tile, exclusive prefix over slabs (in place) + tile totals
//   k_tilescan exclusive prefix over tiles -> tile_base[F+1] (final layout)
//   k_bin1     level 1: slab -> super-tiles (64 tiles), LDS counting sort of
//              8K-sample sub-chunks, run writes; payload = truncated sample
//   k_bin2     level 2: (super-tile, slab block) -> per-(slab, tile) segments,
//              bucket by LUT-bracketed search, final 4-byte records
//   k_bin      single-level alternative (bucketize + direct scatter)
//
// Final record (u32): [31:27] series in tile | [26:16] bucket | [15:0] off,
//   off = contribution - base[bucket] when < 0xFFFF, else 0xFFFF and the exact
//   difference went to sumfix[series] (integer atomics, order free).
// Level-1 record: [31:26] tile in super-tile | [25:21] series in tile |
//   [20:0] payload = v (0 <= v < V_ESC) or V_ESC + bucket (escaped).
#include "l5dh_device.hpp"

namespace l5dh {
namespace {

constexpr int ST_TILES = 64;
constexpr int ST_SHIFT = 11;  // 64 tiles x 32 series
constexpr uint32_t V_ESC = (1u << 21) - 2048u;
constexpr int B1_NT = 512;    // k_bin1 threads (2 workgroups per CU)
constexpr int CH1 = 8192;     // samples per level-1 sub-chunk (16 per thread)
constexpr int FS_MAX = 512;
constexpr int B2_NT = 256;
constexpr uint32_t B2_ITEM = 32768;  // target level-1 records per k_bin2 item
constexpr int CH2 = 4096;            // k_bin2 sub-chunk (LDS counting sort by tile)

// ------------------------------------------------------------------------
__global__ __launch_bounds__(WG) void k_count(const uint32_t* __restrict__ series, size_t n, size_t per, uint32_t S,
                                              uint32_t F, uint32_t* __restrict__ table, uint32_t* __restrict__ err,
                                              const uint32_t* __restrict__ hint, int vec) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint32_t* cnt = smem;
  for (uint32_t t = threadIdx.x; t < F; t += WG) cnt[t] = 0;
  __syncthreads();
  const size_t lo = (size_t)blockIdx.x * per;
  const size_t hi = lo + per < n ? lo + per : n;
  const uint32_t hot0 = hint[0], hot1 = hint[1];  // hot tiles of the previous batch (aggregation only)
  bool bad = false;
  auto one = [&](uint32_t s) {
    const bool ok = s < S;
    bad |= !ok;
    hot_inc(cnt, s >> TILE_SHIFT, ok, hot0, hot1);
  };
  if (lo < hi) {
    size_t done = lo;
    if (vec) {  // lo and the base pointer are 16-B aligned
      const size_t nv = (hi - lo) >> 2;
      const uint4* __restrict__ p = reinterpret_cast<const uint4*>(series + lo);
      size_t i = threadIdx.x;
      const size_t wlast = threadIdx.x | 63;  // last lane of this wave: uniform loop bound
      for (; wlast - threadIdx.x + i + 3 * WG < nv; i += 4 * WG) {
        const uint4 a = p[i], b = p[i + WG], c = p[i + 2 * WG], d = p[i + 3 * WG];
        one(a.x); one(a.y); one(a.z); one(a.w);
        one(b.x); one(b.y); one(b.z); one(b.w);
        one(c.x); one(c.y); one(c.z); one(c.w);
        one(d.x); one(d.y); one(d.z); one(d.w);
      }
      for (; i - threadIdx.x < nv; i += WG) {  // convergent: out-of-range lanes pass invalid ids
        uint4 a = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
        if (i < nv) a = p[i];
        const bool in = i < nv;
        auto one_in = [&](uint32_t s) {
          const bool ok = in && s < S;
          bad |= in && !ok;
          hot_inc(cnt, s >> TILE_SHIFT, ok, hot0, hot1);
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
      hot_inc(cnt, s >> TILE_SHIFT, ok, hot0, hot1);
    }
  }
  if (bad) atomicOr(err, 1u);
  __syncthreads();
  uint32_t* row = table + (size_t)blockIdx.x * F;
  for (uint32_t t = threadIdx.x; t < F; t += WG) row[t] = cnt[t];
}

// WG = 64 tiles x 16 slab groups.
__global__ __launch_bounds__(1024) void k_colscan(uint32_t* __restrict__ table, int G, uint32_t F,
                                                  uint32_t* __restrict__ tile_tot) {
  __shared__ uint32_t part[16][64];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const uint32_t t = blockIdx.x * 64 + lane;
  const int gper = (G + 15) / 16;
  const int g0 = w * gper;
  const int g1 = min(G, g0 + gper);
  uint32_t s = 0;
  if (t < F)
    for (int g = g0; g < g1; ++g) s += table[(size_t)g * F + t];
  part[w][lane] = s;
  __syncthreads();
  if (w == 0) {
    uint32_t acc = 0;
    for (int k = 0; k < 16; ++k) {
      const uint32_t v = part[k][lane];
      part[k][lane] = acc;
      acc += v;
    }
    if (t < F) tile_tot[t] = acc;
  }
  __syncthreads();
  if (t < F) {
    uint32_t acc = part[w][lane];
    for (int g = g0; g < g1; ++g) {
      const size_t i = (size_t)g * F + t;
      const uint32_t v = table[i];
      table[i] = acc;
      acc += v;
    }
  }
}

__global__ __launch_bounds__(1024) void k_tilescan(const uint32_t* __restrict__ tile_tot, uint32_t F,
                                                   uint32_t* __restrict__ tile_base) {
  __shared__ uint32_t lds[17];
  const uint32_t per = (F + 1023) / 1024;
  const uint32_t t0 = threadIdx.x * per;
  uint32_t s = 0;
  for (uint32_t k = 0; k < per; ++k)
    if (t0 + k < F) s += tile_tot[t0 + k];
  uint32_t tot;
  uint32_t acc = block_excl_scan<1024>(s, lds, &tot);
  for (uint32_t k = 0; k < per; ++k)
    if (t0 + k < F) {
      tile_base[t0 + k] = acc;
      acc += tile_tot[t0 + k];
    }
  if (threadIdx.x == 0) tile_base[F] = tot;
}

// Final record of one sample; escapes add their exact sum difference to sumfix.
__device__ __forceinline__ uint32_t final_record(uint32_t s, float f, const uint32_t* __restrict__ lut,
                                                 const int32_t* __restrict__ lim, int64_t* __restrict__ sumfix) {
  int64_t c;
  const uint32_t b = bucketize(f, lut, lim, c);
  const int64_t off = c - (b ? (int64_t)lim[b - 1] : 0);
  uint32_t o;
  if ((uint64_t)off < (uint64_t)OFF_ESC) {
    o = (uint32_t)off;
  } else {
    atomicAdd(reinterpret_cast<unsigned long long*>(&sumfix[s]), (unsigned long long)off);
    o = OFF_ESC;
  }
  return ((s & (TILE - 1)) << 27) | (b << 16) | o;
}

// Single-level: bucketize + scatter to the slab's exclusive (slab, tile) segment.
__global__ __launch_bounds__(WG) void k_bin(const uint32_t* __restrict__ series, const float* __restrict__ values,
                                            size_t n, size_t per, uint32_t S, uint32_t F,
                                            const uint32_t* __restrict__ table, const uint32_t* __restrict__ tile_base,
                                            Tables tb, uint32_t* __restrict__ records, int64_t* __restrict__ sumfix,
                                            int vec) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  int32_t* lim = reinterpret_cast<int32_t*>(smem);
  uint32_t* lut = smem + LIM_PAD;
  uint32_t* cur = smem + LIM_PAD + LUT_N;
  for (int i = threadIdx.x; i < LIM_PAD; i += WG) lim[i] = tb.lim_pad[i];
  for (int i = threadIdx.x; i < LUT_N; i += WG) lut[i] = tb.lut[i];
  const uint32_t* row = table + (size_t)blockIdx.x * F;
  for (uint32_t t = threadIdx.x; t < F; t += WG) cur[t] = tile_base[t] + row[t];
  __syncthreads();
  const size_t lo = (size_t)blockIdx.x * per;
  const size_t hi = lo + per < n ? lo + per : n;
  if (lo >= hi) return;
  auto one = [&](uint32_t s, float f) {
    if (s >= S) return;
    const uint32_t rec = final_record(s, f, lut, lim, sumfix);
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
__device__ __forceinline__ uint32_t payload1(uint32_t s, float f, Tables tb, int64_t* __restrict__ sumfix) {
  if (f >= 0.0f && f < (float)V_ESC) return (uint32_t)f;
  int64_t c;
  const uint32_t b = bucketize(f, tb.lut, tb.lim_pad, c);
  if (c >= 0 && c < (int64_t)V_ESC) return (uint32_t)c;  // e.g. f in (-1, 0) truncates to 0
  const int64_t off = c - (b ? (int64_t)tb.lim_pad[b - 1] : 0);
  atomicAdd(reinterpret_cast<unsigned long long*>(&sumfix[s]), (unsigned long long)off);
  return V_ESC + b;
}

__global__ __launch_bounds__(B1_NT, 4) void k_bin1(const uint32_t* __restrict__ series, const float* __restrict__ values,
                                                size_t n, size_t per, uint32_t S, uint32_t F,
                                                const uint32_t* __restrict__ pre,
                                                const uint32_t* __restrict__ tile_base, Tables tb,
                                                const uint32_t* __restrict__ stplan, uint32_t* __restrict__ out1,
                                                int64_t* __restrict__ sumfix, int vec) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  __shared__ uint32_t lds9[B1_NT / 64 + 1];
  uint32_t* stage = smem;                                         // [CH1]
  uint16_t* stage_st = reinterpret_cast<uint16_t*>(smem + CH1);   // [CH1]
  uint32_t* stcnt = smem + CH1 + CH1 / 2;                         // [FS_MAX]
  uint32_t* stoff = stcnt + FS_MAX;
  uint32_t* stcur = stoff + FS_MAX;
  const uint32_t FS = (F + ST_TILES - 1) / ST_TILES;
  const uint32_t hot0 = stplan[3 * FS + 1], hot1 = stplan[3 * FS + 2];
  const uint32_t* prow = pre + (size_t)blockIdx.x * F;
  for (uint32_t j = threadIdx.x; j < FS; j += B1_NT) {
    const uint32_t t0 = j * ST_TILES;
    const uint32_t t1 = min(F, t0 + ST_TILES);
    uint32_t acc = tile_base[t0];
    for (uint32_t t = t0; t < t1; ++t) acc += prow[t];
    stcur[j] = acc;
    stcnt[j] = 0;
  }
  __syncthreads();
  const size_t lo = (size_t)blockIdx.x * per;
  const size_t hi = lo + per < n ? lo + per : n;
  constexpr int PT = CH1 / B1_NT;  // 16 samples per thread: 4 groups of 4 consecutive
  for (size_t c0 = lo; c0 < hi; c0 += CH1) {
    uint32_t rec[PT], rank[PT];
    uint32_t stv[PT];
    uint32_t sv[PT];
    float fv[PT];
#pragma unroll
    for (int k = 0; k < PT / 4; ++k) {
      const size_t base = c0 + 4 * ((size_t)k * B1_NT + threadIdx.x);
      if (vec && base + 3 < hi) {
        const uint4 s4 = *reinterpret_cast<const uint4*>(series + base);
        const float4 f4 = *reinterpret_cast<const float4*>(values + base);
        sv[4 * k] = s4.x; sv[4 * k + 1] = s4.y; sv[4 * k + 2] = s4.z; sv[4 * k + 3] = s4.w;
        fv[4 * k] = f4.x; fv[4 * k + 1] = f4.y; fv[4 * k + 2] = f4.z; fv[4 * k + 3] = f4.w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool in = base + e < hi;
          sv[4 * k + e] = in ? series[base + e] : 0xFFFFFFFFu;
          fv[4 * k + e] = in ? values[base + e] : 0.0f;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      const uint32_t s = sv[k];
      stv[k] = 0xFFFFFFFFu;
      const bool ok = s < S;
      if (ok) {
        const uint32_t pl = payload1(s, fv[k], tb, sumfix);
        rec[k] = (((s >> TILE_SHIFT) & (ST_TILES - 1)) << 26) | ((s & (TILE - 1)) << 21) | pl;
        stv[k] = s >> ST_SHIFT;
      }
      rank[k] = hot_rank(stcnt, ok ? stv[k] : 0u, ok, hot0, hot1);
    }
    __syncthreads();
    uint32_t tot;
    {
      const uint32_t v = threadIdx.x < FS ? stcnt[threadIdx.x] : 0u;
      const uint32_t e = block_excl_scan<B1_NT>(v, lds9, &tot);
      if (threadIdx.x < FS) stoff[threadIdx.x] = e;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      if (stv[k] != 0xFFFFFFFFu) {
        const uint32_t pos = stoff[stv[k]] + rank[k];
        stage[pos] = rec[k];
        stage_st[pos] = (uint16_t)stv[k];
      }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < tot; i += B1_NT) {
      const uint32_t j = stage_st[i];
      out1[stcur[j] + (i - stoff[j])] = stage[i];
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < FS; j += B1_NT) {
      stcur[j] += stcnt[j];
      stcnt[j] = 0;
    }
    __syncthreads();
  }
}

// Super-tile plan (one workgroup, after the tile totals are known):
//   plan[0..FS]          level-2 item_start per super-tile (nb_j items of equal
//                        slab ranges, ~B2_ITEM records each: skew-balanced)
//   plan[FS+1 .. 2FS]    slab-range size per super-tile
//   plan[2FS+1 .. 3FS]   hot tiles of the super-tile (tile-in-ST, byte 0 and 1;
//                        0xFF = none): tiles holding >= 1/8 of its records
//   plan[3FS+1], [3FS+2] hot super-tiles: >= 1/8 of all records (or ~0u)
constexpr uint32_t NOKEY = 0xFFFFFFFFu;
constexpr int HINT_OFF = 2040;  // plan[2040..2041]: hot-tile hints (fixed slot, survives across batches)
__global__ __launch_bounds__(1024) void k_stplan(uint32_t F, int G, const uint32_t* __restrict__ tile_tot,
                                                 uint32_t* __restrict__ plan) {
  __shared__ uint32_t lds[17];
  __shared__ unsigned long long best[16];
  const uint32_t FS = (F + ST_TILES - 1) / ST_TILES;
  uint32_t nb = 0, gsz = 0, hot = 0xFFFFu;
  uint64_t tot = 0;
  unsigned long long tkA = 0, tkB = 0;  // (records << 16 | tile) of this thread's two biggest tiles
  const uint32_t j = threadIdx.x;
  if (j < FS) {
    const uint32_t t1 = min(F, (j + 1) * ST_TILES);
    uint32_t b0 = 0, b1 = 0, i0 = 0xFF, i1 = 0xFF;  // two biggest tiles of this super-tile
    for (uint32_t t = j * ST_TILES; t < t1; ++t) {
      const uint32_t v = tile_tot[t];
      tot += v;
      if (v > b0) { b1 = b0; i1 = i0; b0 = v; i0 = t - j * ST_TILES; }
      else if (v > b1) { b1 = v; i1 = t - j * ST_TILES; }
    }
    tkA = i0 != 0xFF ? (((unsigned long long)b0 << 16) | (j * ST_TILES + i0)) : 0ull;
    tkB = i1 != 0xFF ? (((unsigned long long)b1 << 16) | (j * ST_TILES + i1)) : 0ull;
    if ((uint64_t)b0 * 8 < tot || b0 == 0) i0 = 0xFF;
    if ((uint64_t)b1 * 8 < tot || b1 == 0) i1 = 0xFF;
    hot = i0 | (i1 << 8);
    uint32_t want = (uint32_t)((tot + B2_ITEM - 1) / B2_ITEM);
    want = max(1u, min(want, (uint32_t)G));
    gsz = ((uint32_t)G + want - 1) / want;
    nb = ((uint32_t)G + gsz - 1) / gsz;
  }
  uint32_t total;
  const uint32_t e = block_excl_scan<1024>(nb, lds, &total);
  if (j < FS) {
    plan[j] = e;
    plan[FS + 1 + j] = gsz;
    plan[2 * FS + 1 + j] = hot;
  }
  if (threadIdx.x == 0) plan[FS] = total;
  // grand total and the two biggest super-tiles (key = tot << 10 | j), block reductions
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
  const unsigned long long key = j < FS ? ((tot << 10) | j) : 0ull;
  const unsigned long long k1 = block_reduce(key, true);
  const unsigned long long k2 = block_reduce(key == k1 ? 0ull : key, true);
  const unsigned long long t1 = block_reduce(tkA, true);
  const unsigned long long t2 = block_reduce(tkA == t1 ? tkB : tkA, true);
  if (threadIdx.x == 0) {
    const unsigned long long ks[2] = {k1, k2};
    for (int h = 0; h < 2; ++h) {
      const uint64_t v = ks[h] >> 10;
      plan[3 * FS + 1 + h] = (v > 0 && v * 8 >= grand) ? (uint32_t)(ks[h] & 1023u) : NOKEY;
    }
    // hot-tile hints for the next batch's k_count (tiles with >= 1/64 of the records)
    const unsigned long long ts[2] = {t1, t2};
    for (int h = 0; h < 2; ++h) {
      const uint64_t v = ts[h] >> 16;
      plan[HINT_OFF + h] = (v > 0 && v * 64 >= grand) ? (uint32_t)(ts[h] & 0xFFFFu) : NOKEY;
    }
  }
}

// Level 2.  Item = (super-tile j, slab range [g0, g1)).  Its level-1 records are
// one contiguous range; tile t's records of that range go, in any order, to
// [tile_base[t] + pre[g0][t], ...) -- exactly where the per-(slab, tile)
// segments g0..g1-1 of the final layout lie.
__global__ __launch_bounds__(B2_NT) void k_bin2(const uint32_t* __restrict__ out1, uint32_t F, int G,
                                                const uint32_t* __restrict__ pre,
                                                const uint32_t* __restrict__ tile_base,
                                                const uint32_t* __restrict__ plan, Tables tb,
                                                uint32_t* __restrict__ records) {
  __shared__ uint2 lut2[LUT2_N];
  __shared__ uint32_t cur[ST_TILES];      // global write position of each tile
  __shared__ uint32_t cnt[ST_TILES];      // records of each tile in this sub-chunk
  __shared__ uint32_t off[ST_TILES];      // their exclusive offsets in stage
  __shared__ uint2 stage[CH2];            // sub-chunk sorted by tile: {record, global index - stage index}
  __shared__ uint32_t seg[2];
  const uint32_t FS = (F + ST_TILES - 1) / ST_TILES;
  const uint32_t item = blockIdx.x;
  if (item >= plan[FS]) return;
  uint32_t lo = 0, hi = FS;  // last j with plan[j] <= item
  while (hi - lo > 1) {
    const uint32_t m = (lo + hi) >> 1;
    if (plan[m] <= item) lo = m; else hi = m;
  }
  const uint32_t j = lo;
  const uint32_t gsz = plan[FS + 1 + j];
  const int g0 = (int)((item - plan[j]) * gsz);
  const int g1 = min(G, g0 + (int)gsz);
  const uint32_t hp = plan[2 * FS + 1 + j];
  const uint32_t hot0 = (hp & 0xFFu) == 0xFFu ? NOKEY : (hp & 0xFFu);
  const uint32_t hot1 = ((hp >> 8) & 0xFFu) == 0xFFu ? NOKEY : ((hp >> 8) & 0xFFu);
  for (int i = threadIdx.x; i < LUT2_N; i += B2_NT) lut2[i] = tb.lut2[i];
  const uint32_t t0 = j * ST_TILES;
  const uint32_t nt = min((uint32_t)ST_TILES, F - t0);
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    uint32_t p0 = 0, p1 = 0;
    if ((uint32_t)lane < nt) {
      const uint32_t t = t0 + lane;
      p0 = pre[(size_t)g0 * F + t];
      p1 = g1 < G ? pre[(size_t)g1 * F + t] : (tile_base[t + 1] - tile_base[t]);
      cur[lane] = tile_base[t] + p0;
    }
    cnt[lane] = 0;
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
  constexpr int PT = CH2 / B2_NT;  // 16 records per thread: 4 x uint4
  uint4 xn[PT / 4];                 // next sub-chunk, prefetched while this one is sorted and written
#pragma unroll
  for (int k = 0; k < PT / 4; ++k) {
    const uint32_t base = A16 + 4 * (k * B2_NT + threadIdx.x);
    xn[k] = base < B ? *reinterpret_cast<const uint4*>(out1 + base) : make_uint4(0u, 0u, 0u, 0u);
  }
  for (uint32_t c0 = A16; c0 < B; c0 += CH2) {
    uint32_t rec[PT], tlv[PT], rank[PT];
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
        const uint32_t loc = (r >> 21) & 31u;
        const uint32_t pl = r & 0x1FFFFFu;
        uint32_t b, o;
        if (pl < V_ESC) {
          b = bucket_lut2(pl, lut2, o);
        } else {
          b = pl - V_ESC;
          o = OFF_ESC;
        }
        rec[4 * k + e] = (loc << 27) | (b << 16) | o;
        tlv[4 * k + e] = valid ? tl : 0xFFu;
        rank[4 * k + e] = hot_rank(cnt, tl, valid, hot0, hot1);
      }
    }
    __syncthreads();
    if (threadIdx.x < 64) {  // exclusive scan of the 64 tile counts (one wave)
      const uint32_t v = cnt[threadIdx.x];
      uint32_t x = v;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if ((int)threadIdx.x >= d) x += y;
      }
      off[threadIdx.x] = x - v;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      if (tlv[k] != 0xFFu) {
        const uint32_t o = off[tlv[k]];
        const uint32_t pos = o + rank[k];
        stage[pos] = make_uint2(rec[k], cur[tlv[k]] - o);
      }
    }
    const uint32_t total = off[ST_TILES - 1] + cnt[ST_TILES - 1];
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < total; i += B2_NT) {
      const uint2 e = stage[i];
      records[e.y + i] = e.x;
    }
    if (threadIdx.x < 64) {
      cur[threadIdx.x] += cnt[threadIdx.x];
      cnt[threadIdx.x] = 0;
    }
    __syncthreads();
  }
}

}  // namespace

// ------------------------------------------------------------------------
hipError_t set_ingest_attributes() {
  hipError_t e;
  const int big = 160 * 1024;
  if ((e = hipFuncSetAttribute((const void*)k_count, hipFuncAttributeMaxDynamicSharedMemorySize, big))) return e;
  if ((e = hipFuncSetAttribute((const void*)k_bin, hipFuncAttributeMaxDynamicSharedMemorySize, big))) return e;
  if ((e = hipFuncSetAttribute((const void*)k_bin1, hipFuncAttributeMaxDynamicSharedMemorySize, (int)BIN1_LDS)))
    return e;
  return hipSuccess;
}

hipError_t launch_count(const uint32_t* series, size_t n, size_t per, int G, uint32_t S, uint32_t F,
                        uint32_t* table, uint32_t* err, const uint32_t* hint, bool vec, hipStream_t st) {
  hipLaunchKernelGGL(k_count, dim3(G), dim3(WG), (size_t)F * 4, st, series, n, per, S, F, table, err, hint,
                     vec ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_colscan(uint32_t* table, int G, uint32_t F, uint32_t* tile_tot, hipStream_t st) {
  hipLaunchKernelGGL(k_colscan, dim3((F + 63) / 64), dim3(1024), 0, st, table, G, F, tile_tot);
  return hipGetLastError();
}

hipError_t launch_tilescan(const uint32_t* tile_tot, uint32_t F, uint32_t* tile_base, hipStream_t st) {
  hipLaunchKernelGGL(k_tilescan, dim3(1), dim3(1024), 0, st, tile_tot, F, tile_base);
  return hipGetLastError();
}

hipError_t launch_bin(const uint32_t* series, const float* values, size_t n, size_t per, int G, uint32_t S,
                      uint32_t F, const uint32_t* table, const uint32_t* tile_base, Tables tb, uint32_t* records,
                      int64_t* sumfix, bool vec, hipStream_t st) {
  const size_t lds = (size_t)LIM_PAD * 4 + LUT_N * 4 + (size_t)F * 4;
  hipLaunchKernelGGL(k_bin, dim3(G), dim3(WG), lds, st, series, values, n, per, S, F, table, tile_base, tb, records,
                     sumfix, vec ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_stplan(uint32_t F, int G, const uint32_t* tile_tot, uint32_t* stplan, hipStream_t st) {
  hipLaunchKernelGGL(k_stplan, dim3(1), dim3(1024), 0, st, F, G, tile_tot, stplan);
  return hipGetLastError();
}

hipError_t launch_bin1(const uint32_t* series, const float* values, size_t n, size_t per, int G, uint32_t S,
                       uint32_t F, const uint32_t* pre, const uint32_t* tile_base, Tables tb, const uint32_t* stplan,
                       uint32_t* scratch1, int64_t* sumfix, bool vec, hipStream_t st) {
  hipLaunchKernelGGL(k_bin1, dim3(G), dim3(B1_NT), BIN1_LDS, st, series, values, n, per, S, F, pre, tile_base, tb,
                     stplan, scratch1, sumfix, vec ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_bin2(const uint32_t* scratch1, size_t n, int G, uint32_t F, const uint32_t* pre,
                       const uint32_t* tile_base, Tables tb, const uint32_t* stplan, uint32_t* records,
                       hipStream_t st) {
  const uint32_t FS = (F + ST_TILES - 1) / ST_TILES;
  const size_t max_items = n / B2_ITEM + FS + 1;  // sum_j ceil(tot_j / B2_ITEM)
  hipLaunchKernelGGL(k_bin2, dim3((unsigned)max_items), dim3(B2_NT), 0, st, scratch1, F, G, pre, tile_base, stplan,
                     tb, records);
  return hipGetLastError();
}

}  // namespace l5dh
