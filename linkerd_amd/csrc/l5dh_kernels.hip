// l5dh_kernels.hip -- CDNA4 (gfx950) kernels of the latency-histogram engine.
//
// Pipeline:
//   ingest:   k_count (LDS tile histogram per slab) -> k_colscan/k_tilescan
//             (exclusive offsets per (slab, tile)) -> k_bin (LDS binary search
//             over the 1797 limits + 4-byte record scatter by tile)
//   snapshot: k_plan (work items per tile) -> k_hot_init -> k_accum (LDS-private
//             tile histograms, fused summary + dense flush) -> k_hot_finish
//
// Semantics restated (reference paths relative to the linkerd checkout):
//   Metric.Stat.add(Float) -> BucketedHistogram.add(Long)   Metric.scala:30-33
//   Metric.Stat.summary / HistogramSummary                  Metric.scala:53-67,76-88
//   limits                                                  BucketedHistogram.scala:25-46
// and finagle-stats 6.45.0 BucketedHistogram (percentile/min/max/average), as
// written out in SURVEY.md §8a.
//
// Record format (u32): [31:27] series within tile | [26:16] bucket | [15:0] off
//   off = contribution - base[bucket] when 0 <= off < 0xFFFF, else 0xFFFF and
//   the exact difference goes to sumfix[series] (integer atomics: order free).
#include "l5dh_kernels.hpp"

namespace l5dh {

namespace {

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Java (long) float conversion (JLS 5.1.3), Metric.scala:32 `value.toLong`.
__device__ __forceinline__ int64_t java_f2l(float f) {
  if (f != f) return 0;
  if (f >= 9.223372036854775808e18f) return INT64_MAX;
  if (f <= -9.223372036854775808e18f) return INT64_MIN;
  return (int64_t)f;
}

// java.lang.Math.round for 0 <= x < 2^52: floor(x) + (frac >= 0.5), exact.
__device__ __forceinline__ int64_t java_round_nonneg(double x) {
  double fl = floor(x);
  double fr = __dsub_rn(x, fl);
  return (int64_t)fl + (fr >= 0.5 ? 1 : 0);
}

// upstream BucketedHistogram.add(Long): returns bucket, sets contribution to total.
// Bucket = number of limits <= key (== Arrays.binarySearch insertion rule),
// found with an 11-step branch-free search over the LDS-staged padded limits.
__device__ __forceinline__ uint32_t bucketize(float f, const int32_t* __restrict__ lim, int64_t& contrib) {
  int64_t v;
  if (f >= 0.0f && f < 2147483648.0f) {
    v = (int64_t)(uint32_t)f;  // common case: truncation of a non-negative float
  } else {
    v = java_f2l(f);
    if (v >= (int64_t)INT_MAXV) {
      contrib = INT_MAXV;
      return NL;
    }
  }
  contrib = v;
  const int32_t key = (int32_t)(uint32_t)(uint64_t)v;  // Long.toInt: low 32 bits
  int idx = 0;
#pragma unroll
  for (int step = 1024; step > 0; step >>= 1)
    if (lim[idx + step - 1] <= key) idx += step;
  return (uint32_t)(idx < NL ? idx : NL);
}

__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t x) {
  const int lane = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint64_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t x) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) x += __shfl_xor(x, d, 64);
  return x;
}

// ---- bin groups ----------------------------------------------------------
// Lane l of a wave owns bins [28l, 28l+28) = groups q = 0..6 of 4 bins; lane 63
// also owns 1792..1797 (groups 7 and 8; group 8 = bins 1796, 1797 + padding).
__device__ __forceinline__ int lane_groups(int lane) { return lane == 63 ? 9 : 7; }

// Count sources: get4(b0) returns bins b0..b0+3 (b0 % 4 == 0); bins >= 1798 read 0.
struct SrcLds16 {  // u16-packed row in LDS (cold tile: counts of the new records)
  const uint32_t* row;
  __device__ __forceinline__ uint4 get4(int b0) const {
    const uint2 w = *reinterpret_cast<const uint2*>(row + (b0 >> 1));  // word 899 is zero padding
    return make_uint4(w.x & 0xFFFFu, w.x >> 16, w.y & 0xFFFFu, w.y >> 16);
  }
};
struct SrcRow32 {  // state row, stride ROW = 1800 u32, 16-B aligned
  const uint32_t* row;
  __device__ __forceinline__ uint4 get4(int b0) const {
    uint4 v = *reinterpret_cast<const uint4*>(row + b0);
    if (b0 == 1796) v.z = v.w = 0u;
    return v;
  }
};
struct SrcExt {  // external dense rows, stride 1798 int32 (8-B aligned)
  const int32_t* row;
  __device__ __forceinline__ uint4 get4(int b0) const {
    const uint2 a = *reinterpret_cast<const uint2*>(row + b0);
    uint2 b = make_uint2(0u, 0u);
    if (b0 != 1796) b = *reinterpret_cast<const uint2*>(row + b0 + 2);
    return make_uint4(a.x, a.y, b.x, b.y);
  }
};

__device__ __forceinline__ uint32_t sum4(uint4 v) { return v.x + v.y + v.z + v.w; }

__device__ __forceinline__ uint64_t dot4(uint4 v, const int32_t* __restrict__ base, int b0) {
  const uint4 bb = *reinterpret_cast<const uint4*>(base + b0);  // base table padded to 1800 with 0
  return (uint64_t)v.x * bb.x + (uint64_t)v.y * bb.y + (uint64_t)v.z * bb.z + (uint64_t)v.w * bb.w;
}

__device__ __forceinline__ void store4_1798(int32_t* __restrict__ row, int b0, uint4 v) {
  *reinterpret_cast<uint2*>(row + b0) = make_uint2(v.x, v.y);
  if (b0 != 1796) *reinterpret_cast<uint2*>(row + b0 + 2) = make_uint2(v.z, v.w);
}

__device__ __forceinline__ void store4_state(uint32_t* __restrict__ row, int b0, uint4 v) {
  *reinterpret_cast<uint4*>(row + b0) = v;
}

// Wave-cooperative summary of one series (Metric.Stat.summary, Metric.scala:53-67;
// upstream percentile/minimum/maximum/average).  g[q] = sum of the lane's group q.
//   min  = first bucket whose running count >= 1
//   pXX  = first bucket whose running count >= Math.round(p * num)
//   max  = first bucket whose running count >= num (= last non-empty bucket)
// each reported as the bucket midpoint (mid[0] = 0, mid[1797] = Int.MaxValue).
// The owner lane of each of the 8 targets is found by ballot over the lane
// prefix; lanes 0..7 then locate the group (shuffles) and the bin (one get4).
template <class Src>
__device__ __forceinline__ void wave_summary(const uint32_t (&g)[9], const Src& src, int64_t total,
                                             const int32_t* __restrict__ mid, Summary88* __restrict__ out) {
  const int lane = lane_id();
  uint64_t ls = 0;
#pragma unroll
  for (int q = 0; q < 9; ++q) ls += g[q];
  const uint64_t incl = wave_incl_scan(ls);
  const uint64_t excl = incl - ls;
  const uint64_t num = __shfl(incl, 63, 64);
  const double dn = (double)num;

  int my_owner = 0;
  uint64_t my_t = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    uint64_t t;
    if (k == 0)
      t = num ? 1 : 0;
    else if (k == 7)
      t = num;
    else {
      const double p = k == 1 ? 0.50 : k == 2 ? 0.90 : k == 3 ? 0.95 : k == 4 ? 0.99 : k == 5 ? 0.999 : 0.9999;
      t = (uint64_t)java_round_nonneg(__dmul_rn(p, dn));
    }
    const unsigned long long m = __ballot(t != 0 && excl < t && t <= incl);
    const int owner = m ? (__ffsll((long long)m) - 1) : 0;
    if (lane == k) {
      my_owner = owner;
      my_t = t;
    }
  }
  uint64_t acc = __shfl(excl, my_owner, 64);
  int qsel = 0;
  bool done = false;
#pragma unroll
  for (int q = 0; q < 9; ++q) {
    const uint32_t gq = __shfl(g[q], my_owner, 64);
    if (!done) {
      if (acc + gq >= my_t) {
        qsel = q;
        done = true;
      } else {
        acc += gq;
      }
    }
  }
  int64_t res = 0;
  if (lane < 8 && my_t != 0) {
    const int b0 = 28 * my_owner + 4 * qsel;
    const uint4 v = src.get4(b0);
    int b = b0 + 3;
    if (acc + v.x >= my_t)
      b = b0;
    else if (acc + v.x + v.y >= my_t)
      b = b0 + 1;
    else if (acc + v.x + v.y + v.z >= my_t)
      b = b0 + 2;
    res = mid[b];
  }
  // field f of HistogramSummary: count, min(k0), max(k7), sum, p50..p9999(k1..k6), avg
  const int f = lane;
  const int srcl = (f == 1) ? 0 : (f == 2) ? 7 : (f >= 4 && f <= 9) ? (f - 3) : 0;
  const int64_t r = __shfl(res, srcl, 64);
  if (out != nullptr && f < 11) {
    int64_t val;
    if (f == 0)
      val = (int64_t)num;
    else if (f == 3)
      val = total;
    else if (f == 10) {
      const double avg = num == 0 ? 0.0 : __ddiv_rn((double)total, dn);
      val = __double_as_longlong(avg);
    } else
      val = r;
    reinterpret_cast<int64_t*>(out)[f] = val;
  }
}

// Pass over a global row source: group sums + optional dense copy.
template <class Src>
__device__ __forceinline__ void row_pass(const Src& src, uint32_t (&g)[9], int32_t* __restrict__ out_row) {
  const int lane = lane_id();
  const int ng = lane_groups(lane);
#pragma unroll
  for (int q = 0; q < 9; ++q) {
    g[q] = 0;
    if (q < ng) {
      const int b0 = 28 * lane + 4 * q;
      const uint4 v = src.get4(b0);
      g[q] = sum4(v);
      if (out_row) store4_1798(out_row, b0, v);
    }
  }
}

// ------------------------------------------------------------------------
// k_count: tile histogram of one slab of the COO batch, LDS-private.
// table[g][t] = samples of slab g that fall in tile t.
__global__ __launch_bounds__(WG) void k_count(const uint32_t* __restrict__ series, size_t n, size_t per, uint32_t S,
                                              uint32_t F, uint32_t* __restrict__ table, uint32_t* __restrict__ err,
                                              int vec) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint32_t* cnt = smem;
  for (uint32_t t = threadIdx.x; t < F; t += WG) cnt[t] = 0;
  __syncthreads();
  const size_t lo = (size_t)blockIdx.x * per;
  const size_t hi = lo + per < n ? lo + per : n;
  bool bad = false;
  if (lo < hi) {
    if (vec) {  // lo and the base pointer are 16-B aligned
      const size_t nv = (hi - lo) >> 2;
      const uint4* p = reinterpret_cast<const uint4*>(series + lo);
      for (size_t i = threadIdx.x; i < nv; i += WG) {
        const uint4 s = p[i];
        if (s.x < S) atomicAdd(&cnt[s.x >> TILE_SHIFT], 1u); else bad = true;
        if (s.y < S) atomicAdd(&cnt[s.y >> TILE_SHIFT], 1u); else bad = true;
        if (s.z < S) atomicAdd(&cnt[s.z >> TILE_SHIFT], 1u); else bad = true;
        if (s.w < S) atomicAdd(&cnt[s.w >> TILE_SHIFT], 1u); else bad = true;
      }
      for (size_t i = lo + (nv << 2) + threadIdx.x; i < hi; i += WG) {
        const uint32_t s = series[i];
        if (s < S) atomicAdd(&cnt[s >> TILE_SHIFT], 1u); else bad = true;
      }
    } else {
      for (size_t i = lo + threadIdx.x; i < hi; i += WG) {
        const uint32_t s = series[i];
        if (s < S) atomicAdd(&cnt[s >> TILE_SHIFT], 1u); else bad = true;
      }
    }
  }
  if (bad) atomicOr(err, 1u);
  __syncthreads();
  uint32_t* row = table + (size_t)blockIdx.x * F;
  for (uint32_t t = threadIdx.x; t < F; t += WG) row[t] = cnt[t];
}

// k_colscan: per tile, exclusive prefix over slabs (in place) and tile totals.
// WG = 64 tiles x 16 slab groups; G <= 256 slabs.
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

// Block-wide exclusive scan helper for one 1024-thread workgroup.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* lds /*[16]*/, uint32_t* total) {
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) lds[w] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int k = 0; k < 16; ++k) {
      const uint32_t q = lds[k];
      lds[k] = acc;
      acc += q;
    }
    lds[16] = acc;
  }
  __syncthreads();
  const uint32_t r = lds[w] + x - v;
  if (total) *total = lds[16];
  __syncthreads();
  return r;
}

// k_tilescan: tile_base[t] = exclusive prefix of tile totals; tile_base[F] = total.
__global__ __launch_bounds__(1024) void k_tilescan(const uint32_t* __restrict__ tile_tot, uint32_t F,
                                                   uint32_t* __restrict__ tile_base) {
  __shared__ uint32_t lds[17];
  const uint32_t per = (F + 1023) / 1024;
  const uint32_t t0 = threadIdx.x * per;
  uint32_t s = 0;
  for (uint32_t k = 0; k < per; ++k)
    if (t0 + k < F) s += tile_tot[t0 + k];
  uint32_t tot;
  uint32_t acc = block_excl_scan(s, lds, &tot);
  for (uint32_t k = 0; k < per; ++k)
    if (t0 + k < F) {
      tile_base[t0 + k] = acc;
      acc += tile_tot[t0 + k];
    }
  if (threadIdx.x == 0) tile_base[F] = tot;
}

// k_bin: bucketize every sample of slab g and scatter its 4-byte record to the
// slab's exclusive region of its tile.  LDS: limits (8 KB) + one cursor per tile.
__global__ __launch_bounds__(WG) void k_bin(const uint32_t* __restrict__ series, const float* __restrict__ values,
                                            size_t n, size_t per, uint32_t S, uint32_t F,
                                            const uint32_t* __restrict__ table, const uint32_t* __restrict__ tile_base,
                                            const int32_t* __restrict__ lim_pad, uint32_t* __restrict__ records,
                                            int64_t* __restrict__ sumfix, int vec) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  int32_t* lim = reinterpret_cast<int32_t*>(smem);
  uint32_t* cur = smem + LIM_PAD;
  for (int i = threadIdx.x; i < LIM_PAD; i += WG) lim[i] = lim_pad[i];
  const uint32_t* row = table + (size_t)blockIdx.x * F;
  for (uint32_t t = threadIdx.x; t < F; t += WG) cur[t] = tile_base[t] + row[t];
  __syncthreads();
  const size_t lo = (size_t)blockIdx.x * per;
  const size_t hi = lo + per < n ? lo + per : n;
  if (lo >= hi) return;

  auto one = [&](uint32_t s, float f) {
    if (s >= S) return;
    int64_t c;
    const uint32_t b = bucketize(f, lim, c);
    const int64_t base = b ? (int64_t)lim[b - 1] : 0;
    const int64_t off = c - base;
    uint32_t o;
    if ((uint64_t)off < (uint64_t)OFF_ESC) {
      o = (uint32_t)off;
    } else {
      atomicAdd(reinterpret_cast<unsigned long long*>(&sumfix[s]), (unsigned long long)off);
      o = OFF_ESC;
    }
    const uint32_t rec = ((s & (TILE - 1)) << 27) | (b << 16) | o;
    const uint32_t pos = atomicAdd(&cur[s >> TILE_SHIFT], 1u);
    records[pos] = rec;
  };

  if (vec) {
    const size_t nv = (hi - lo) >> 2;
    const uint4* ps = reinterpret_cast<const uint4*>(series + lo);
    const float4* pv = reinterpret_cast<const float4*>(values + lo);
    for (size_t i = threadIdx.x; i < nv; i += WG) {
      const uint4 s = ps[i];
      const float4 f = pv[i];
      one(s.x, f.x);
      one(s.y, f.y);
      one(s.z, f.z);
      one(s.w, f.w);
    }
    for (size_t i = lo + (nv << 2) + threadIdx.x; i < hi; i += WG) one(series[i], values[i]);
  } else {
    for (size_t i = lo + threadIdx.x; i < hi; i += WG) one(series[i], values[i]);
  }
}

// k_plan: one workgroup.  Per tile: records across segments, hot/cold, work
// items; exclusive scans -> item_start[F+1], hot_list, header {items, hot}.
__global__ __launch_bounds__(1024) void k_plan(Segs segs, uint32_t F, int final_mode, uint32_t cold_limit,
                                               uint32_t hot_chunk, Plan plan) {
  __shared__ uint32_t lds_a[17];
  __shared__ uint32_t lds_b[17];
  const uint32_t per = (F + 1023) / 1024;
  const uint32_t t0 = threadIdx.x * per;
  uint32_t items = 0, hot = 0;
  for (uint32_t k = 0; k < per; ++k) {
    const uint32_t t = t0 + k;
    if (t >= F) break;
    uint32_t tot = 0;
    for (int j = 0; j < segs.n; ++j) tot += segs.tbase[j][t + 1] - segs.tbase[j][t];
    plan.tile_tot[t] = tot;
    if (tot > cold_limit) {
      items += 2u * ((tot + hot_chunk - 1) / hot_chunk);
      hot += 1;
    } else if (final_mode || tot > 0) {
      items += 1;
    }
  }
  uint32_t tot_items, tot_hot;
  uint32_t ia = block_excl_scan(items, lds_a, &tot_items);
  uint32_t ha = block_excl_scan(hot, lds_b, &tot_hot);
  for (uint32_t k = 0; k < per; ++k) {
    const uint32_t t = t0 + k;
    if (t >= F) break;
    const uint32_t tot = plan.tile_tot[t];
    plan.item_start[t] = ia;
    if (tot > cold_limit) {
      ia += 2u * ((tot + hot_chunk - 1) / hot_chunk);
      plan.hot_list[ha++] = t;
    } else if (final_mode || tot > 0) {
      ia += 1;
    }
  }
  if (threadIdx.x == 0) {
    plan.item_start[F] = tot_items;
    plan.header[0] = tot_items;
    plan.header[1] = tot_hot;
  }
}

// k_hot_init: split tiles accumulate with global atomics into state rows, so
// clean ones start from zero.
__global__ __launch_bounds__(256) void k_hot_init(const uint32_t* __restrict__ hot_list, State st) {
  const uint32_t t = hot_list[blockIdx.x];
  if (st.dirty[t]) return;
  const uint32_t s0 = t * TILE;
  const uint32_t s1 = min(st.S, s0 + TILE);
  uint4* p = reinterpret_cast<uint4*>(st.counts + (size_t)s0 * ROW);
  const size_t n4 = (size_t)(s1 - s0) * ROW / 4;
  for (size_t i = threadIdx.x; i < n4; i += 256) p[i] = make_uint4(0, 0, 0, 0);
  if (threadIdx.x < s1 - s0) st.total[s0 + threadIdx.x] = 0;
}

__device__ __forceinline__ uint32_t find_tile(const uint32_t* __restrict__ item_start, uint32_t F, uint32_t item) {
  // last t with item_start[t] <= item
  uint32_t lo = 0, hi = F;  // invariant: item_start[lo] <= item < item_start[hi] (item_start[F] = total)
  while (hi - lo > 1) {
    const uint32_t m = (lo + hi) >> 1;
    if (item_start[m] <= item) lo = m; else hi = m;
  }
  return lo;
}

// k_accum: one work item = one tile (cold: <= cold_limit records, 32 series in
// u16-packed LDS bins, fused summary + dense flush) or one (tile, half, chunk)
// of a hot tile (16 series in u32 LDS bins, flushed with global atomics).
__global__ __launch_bounds__(WG) void k_accum(Segs segs, Plan plan, State st, Tables tb, Outputs out,
                                              uint32_t cold_limit, uint32_t hot_chunk, int final_mode, int reset) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t item = blockIdx.x;
  const uint32_t F = st.F;
  const uint32_t t = find_tile(plan.item_start, F, item);
  const uint32_t sub = item - plan.item_start[t];
  const uint32_t tot = plan.tile_tot[t];
  const int lane = lane_id();
  const int w = threadIdx.x >> 6;

  if (tot <= cold_limit) {
    // ---------------- cold tile: single pass ----------------
    uint32_t* hist = smem;                    // [32][900] u16 pairs
    uint32_t* offsum = smem + TILE * CROW;    // [32]
    {
      uint4* p = reinterpret_cast<uint4*>(smem);
      for (int i = threadIdx.x; i < TILE * CROW / 4; i += WG) p[i] = make_uint4(0, 0, 0, 0);
      if (threadIdx.x < TILE) offsum[threadIdx.x] = 0;
    }
    __syncthreads();
    for (int j = 0; j < segs.n; ++j) {
      const uint32_t a = segs.tbase[j][t];
      const uint32_t e = segs.tbase[j][t + 1];
      const uint32_t* __restrict__ r = segs.recs[j];
      for (uint32_t i = a + threadIdx.x; i < e; i += WG) {
        const uint32_t rec = r[i];
        const uint32_t loc = rec >> 27;
        const uint32_t b = (rec >> 16) & 0x7FFu;
        const uint32_t off = rec & 0xFFFFu;
        atomicAdd(&hist[loc * CROW + (b >> 1)], (b & 1u) ? 0x10000u : 1u);
        if (off != 0 && off != OFF_ESC) atomicAdd(&offsum[loc], off);
      }
    }
    __syncthreads();
    const bool dirty = st.dirty[t] != 0;
    const bool keep = !(final_mode && reset);
    const int ng = lane_groups(lane);
    for (int rep = 0; rep < 2; ++rep) {
      const uint32_t loc = w + 16 * rep;
      const uint32_t s = t * TILE + loc;
      if (s >= st.S) continue;
      const uint32_t oi = s - out.first;
      const bool emit = final_mode && s >= out.first && oi < out.count;
      int32_t* orow = (emit && out.counts) ? out.counts + (size_t)oi * NB : nullptr;
      uint32_t* srow = st.counts + (size_t)s * ROW;
      const SrcLds16 lds{hist + loc * CROW};
      uint32_t g[9];
      uint64_t bs = 0;  // sum_b newcount_b * base_b (+ sum(off) below) = exact sum of new samples
      if (!dirty) {
#pragma unroll
        for (int q = 0; q < 9; ++q) {
          g[q] = 0;
          if (q < ng) {
            const int b0 = 28 * lane + 4 * q;
            const uint4 v = lds.get4(b0);
            g[q] = sum4(v);
            bs += dot4(v, tb.base, b0);
            if (orow) store4_1798(orow, b0, v);
            if (keep) store4_state(srow, b0, v);
          }
        }
      } else {
        const SrcRow32 old{srow};
#pragma unroll
        for (int q = 0; q < 9; ++q) {
          g[q] = 0;
          if (q < ng) {
            const int b0 = 28 * lane + 4 * q;
            const uint4 v = lds.get4(b0);
            bs += dot4(v, tb.base, b0);
            const uint4 o = old.get4(b0);
            const uint4 cmb = make_uint4(v.x + o.x, v.y + o.y, v.z + o.z, v.w + o.w);
            g[q] = sum4(cmb);
            if (orow) store4_1798(orow, b0, cmb);
            store4_state(srow, b0, cmb);  // the merged row is also the summary source
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
      }
      bs = wave_sum(bs);
      int64_t total = (int64_t)bs + (int64_t)offsum[loc] + st.sumfix[s];
      if (dirty) total += st.total[s];
      if (lane == 0) {
        st.sumfix[s] = 0;
        if (keep) st.total[s] = total;
      }
      if (emit) {
        Summary88* so = out.summ ? out.summ + oi : nullptr;
        if (dirty)
          wave_summary(g, SrcRow32{srow}, total, tb.mid, so);
        else
          wave_summary(g, lds, total, tb.mid, so);
      }
    }
    if (threadIdx.x == 0) st.dirty[t] = (final_mode && reset) ? 0 : 1;
  } else {
    // ---------------- hot tile: split over (half, chunk) ----------------
    uint32_t* hist = smem;                                                   // [16][1800] u32
    unsigned long long* offsum = reinterpret_cast<unsigned long long*>(smem + 16 * HROW);  // [16]
    const uint32_t half = sub & 1u;
    const uint32_t chunk = sub >> 1;
    {
      uint4* p = reinterpret_cast<uint4*>(smem);
      for (int i = threadIdx.x; i < 16 * HROW / 4; i += WG) p[i] = make_uint4(0, 0, 0, 0);
      if (threadIdx.x < 16) offsum[threadIdx.x] = 0;
    }
    __syncthreads();
    const uint64_t vlo = (uint64_t)chunk * hot_chunk;
    const uint64_t vhi = vlo + hot_chunk < tot ? vlo + hot_chunk : tot;
    uint64_t vbase = 0;
    for (int j = 0; j < segs.n; ++j) {
      const uint32_t a = segs.tbase[j][t];
      const uint32_t e = segs.tbase[j][t + 1];
      const uint64_t len = e - a;
      const uint64_t lo = vlo > vbase ? vlo : vbase;
      const uint64_t hi = vhi < vbase + len ? vhi : vbase + len;
      if (lo < hi) {
        const uint32_t* __restrict__ r = segs.recs[j] + a + (lo - vbase);
        const uint32_t cnt = (uint32_t)(hi - lo);
        for (uint32_t i = threadIdx.x; i < cnt; i += WG) {
          const uint32_t rec = r[i];
          const uint32_t loc = rec >> 27;
          if ((loc >> 4) != half) continue;
          const uint32_t l = loc & 15u;
          const uint32_t b = (rec >> 16) & 0x7FFu;
          const uint32_t off = rec & 0xFFFFu;
          atomicAdd(&hist[l * HROW + b], 1u);
          if (off != 0 && off != OFF_ESC) atomicAdd(&offsum[l], (unsigned long long)off);
        }
      }
      vbase += len;
    }
    __syncthreads();
    const uint32_t s = t * TILE + 16 * half + w;
    if (s < st.S) {
      uint32_t* grow = st.counts + (size_t)s * ROW;
      const uint32_t* hrow = hist + w * HROW;
      uint64_t bs = 0;
      for (int b = lane; b < NB; b += 64) {
        const uint32_t v = hrow[b];
        if (v) {
          bs += (uint64_t)v * (uint64_t)(uint32_t)tb.base[b];
          atomicAdd(&grow[b], v);
        }
      }
      bs = wave_sum(bs);
      if (lane == 0) {
        const uint64_t add = bs + offsum[w];
        if (add) atomicAdd(reinterpret_cast<unsigned long long*>(&st.total[s]), (unsigned long long)add);
      }
    }
  }
}

// k_hot_finish: per (hot tile, half): fold sumfix, summarize the merged rows,
// write outputs, update state/dirty.
__global__ __launch_bounds__(WG) void k_hot_finish(Plan plan, State st, Tables tb, Outputs out, int final_mode,
                                                   int reset) {
  const uint32_t t = plan.hot_list[blockIdx.x >> 1];
  const uint32_t half = blockIdx.x & 1u;
  const int lane = lane_id();
  const int w = threadIdx.x >> 6;
  const uint32_t s = t * TILE + 16 * half + w;
  if (s < st.S) {
    int64_t total = st.total[s] + st.sumfix[s];
    if (final_mode) {
      const uint32_t oi = s - out.first;
      if (s >= out.first && oi < out.count) {
        const SrcRow32 src{st.counts + (size_t)s * ROW};
        uint32_t g[9];
        row_pass(src, g, out.counts ? out.counts + (size_t)oi * NB : nullptr);
        wave_summary(g, src, total, tb.mid, out.summ ? out.summ + oi : nullptr);
      }
    }
    if (lane == 0) {
      st.sumfix[s] = 0;
      st.total[s] = total;
    }
  }
  if (threadIdx.x == 0 && half == 0) st.dirty[t] = (final_mode && reset) ? 0 : 1;
}

// k_rows: one wave per series: summary / dense copy of state rows (range
// snapshot, export) or of external dense rows (fleet merge).
__global__ __launch_bounds__(256) void k_rows(State st, const int32_t* __restrict__ ext,
                                              const int64_t* __restrict__ ext_total, Tables tb, Outputs out, int reset,
                                              int64_t* __restrict__ totals_out) {
  const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= out.count) return;
  const int lane = lane_id();
  uint32_t g[9];
  int32_t* orow = out.counts ? out.counts + (size_t)i * NB : nullptr;
  if (ext) {
    const SrcExt src{ext + (size_t)i * NB};
    const int64_t total = ext_total ? ext_total[i] : 0;
    row_pass(src, g, orow);
    if (out.summ) wave_summary(g, src, total, tb.mid, out.summ + i);
    if (totals_out && lane == 0) totals_out[i] = total;
    return;
  }
  const uint32_t s = out.first + i;
  const bool dirty = st.dirty[s >> TILE_SHIFT] != 0;
  if (dirty) {
    const SrcRow32 src{st.counts + (size_t)s * ROW};
    const int64_t total = st.total[s];
    row_pass(src, g, orow);
    if (out.summ) wave_summary(g, src, total, tb.mid, out.summ + i);
    if (totals_out && lane == 0) totals_out[i] = total;
    if (reset) {
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
      uint32_t* row = st.counts + (size_t)s * ROW;
      const int ng = lane_groups(lane);
#pragma unroll
      for (int q = 0; q < 9; ++q)
        if (q < ng) store4_state(row, 28 * lane + 4 * q, make_uint4(0u, 0u, 0u, 0u));
      if (lane == 0) st.total[s] = 0;
    }
  } else {
#pragma unroll
    for (int q = 0; q < 9; ++q) g[q] = 0;
    if (orow) {
      const int ng = lane_groups(lane);
#pragma unroll
      for (int q = 0; q < 9; ++q)
        if (q < ng) store4_1798(orow, 28 * lane + 4 * q, make_uint4(0u, 0u, 0u, 0u));
    }
    if (out.summ) wave_summary(g, SrcRow32{st.counts}, 0, tb.mid, out.summ + i);  // num == 0: no bin is read
    if (totals_out && lane == 0) totals_out[i] = 0;
  }
}

}  // namespace

// ------------------------------------------------------------------------
hipError_t set_kernel_attributes() {
  hipError_t e;
  const int big = 160 * 1024;
  if ((e = hipFuncSetAttribute((const void*)k_count, hipFuncAttributeMaxDynamicSharedMemorySize, big))) return e;
  if ((e = hipFuncSetAttribute((const void*)k_bin, hipFuncAttributeMaxDynamicSharedMemorySize, big))) return e;
  if ((e = hipFuncSetAttribute((const void*)k_accum, hipFuncAttributeMaxDynamicSharedMemorySize, big))) return e;
  return hipSuccess;
}

hipError_t launch_count(const uint32_t* series, size_t n, size_t per, int G, uint32_t S, uint32_t F,
                        uint32_t* table, uint32_t* err, bool vec, hipStream_t st) {
  const size_t lds = (size_t)F * 4;
  hipLaunchKernelGGL(k_count, dim3(G), dim3(WG), lds, st, series, n, per, S, F, table, err, vec ? 1 : 0);
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
  const size_t lds = (size_t)LIM_PAD * 4 + (size_t)F * 4;
  hipLaunchKernelGGL(k_bin, dim3(G), dim3(WG), lds, st, series, values, n, per, S, F, table, tile_base, tb.lim_pad,
                     records, sumfix, vec ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_plan(Segs segs, uint32_t F, int final_mode, uint32_t cold_limit, uint32_t hot_chunk, Plan plan,
                       hipStream_t st) {
  hipLaunchKernelGGL(k_plan, dim3(1), dim3(1024), 0, st, segs, F, final_mode, cold_limit, hot_chunk, plan);
  return hipGetLastError();
}

hipError_t launch_hot_init(Plan plan, uint32_t num_hot, State state, hipStream_t st) {
  if (num_hot == 0) return hipSuccess;
  hipLaunchKernelGGL(k_hot_init, dim3(num_hot), dim3(256), 0, st, plan.hot_list, state);
  return hipGetLastError();
}

hipError_t launch_accum(Segs segs, Plan plan, uint32_t num_items, State state, Tables tb, Outputs out,
                        uint32_t cold_limit, uint32_t hot_chunk, int final_mode, int reset, hipStream_t st) {
  if (num_items == 0) return hipSuccess;
  hipLaunchKernelGGL(k_accum, dim3(num_items), dim3(WG), ACC_LDS, st, segs, plan, state, tb, out, cold_limit,
                     hot_chunk, final_mode, reset);
  return hipGetLastError();
}

hipError_t launch_hot_finish(Plan plan, uint32_t num_hot, State state, Tables tb, Outputs out, int final_mode,
                             int reset, hipStream_t st) {
  if (num_hot == 0) return hipSuccess;
  hipLaunchKernelGGL(k_hot_finish, dim3(num_hot * 2), dim3(WG), 0, st, plan, state, tb, out, final_mode, reset);
  return hipGetLastError();
}

hipError_t launch_rows(State state, const int32_t* ext, const int64_t* ext_total, Tables tb, Outputs out, int reset,
                       int64_t* totals_out, hipStream_t st) {
  if (out.count == 0) return hipSuccess;
  hipLaunchKernelGGL(k_rows, dim3((out.count + 3) / 4), dim3(256), 0, st, state, ext, ext_total, tb, out, reset,
                     totals_out);
  return hipGetLastError();
}

}  // namespace l5dh
