// l5dh_device.hpp -- device helpers shared by the ingest and snapshot kernels:
// Java numerics, the bucket search, block/wave scans and the wave-cooperative
// HistogramSummary.  Semantics restated from (reference paths relative to the
// linkerd checkout):
//   Metric.Stat.add(Float) -> BucketedHistogram.add(Long)   Metric.scala:30-33
//   Metric.Stat.summary / HistogramSummary                  Metric.scala:53-67,76-88
//   limits                                                  BucketedHistogram.scala:25-46
// and finagle-stats 6.45.0 BucketedHistogram (percentile/min/max/average), as
// written out in SURVEY.md §8a.
#pragma once
#include <type_traits>

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

// DPP lane moves (VALU; no LDS permute): 0x111/0x112/0x114/0x118 = row_shr:1/2/4/8,
// 0x142 = row_bcast:15 (rows 1, 3), 0x143 = row_bcast:31 (rows 2, 3).  Lanes with no
// source (or outside the row mask) read 0.  Whole waves only (EXEC all ones).
template <int CTRL, int ROWS>
__device__ __forceinline__ uint64_t dpp64(uint64_t x) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)x, CTRL, ROWS, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(x >> 32), CTRL, ROWS, 0xF, false);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t wave_incl_scan32(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
  return x;
}

__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t x) {
  x += dpp64<0x111, 0xF>(x);
  x += dpp64<0x112, 0xF>(x);
  x += dpp64<0x114, 0xF>(x);
  x += dpp64<0x118, 0xF>(x);
  x += dpp64<0x142, 0xA>(x);
  x += dpp64<0x143, 0xC>(x);
  return x;
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t x) {  // every lane gets the sum
  x = wave_incl_scan(x);
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)x, 63);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(x >> 32), 63);
  return ((uint64_t)hi << 32) | lo;
}

// ---- bin groups ----------------------------------------------------------
// Lane l of a wave owns bins [28l, 28l+28) = groups q = 0..6 of 4 bins; lane 63
// also owns 1792..1797 (groups 7 and 8; group 8 = bins 1796, 1797 + padding).
__device__ __forceinline__ int lane_groups(int lane) { return lane == 63 ? 9 : 7; }

// Count sources: get4(b0) returns bins b0..b0+3 (b0 % 4 == 0); bins >= 1798 read 0.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
// x.lo + x.hi + c (one v_dot2_u32_u16)
__device__ __forceinline__ uint32_t pair_sum(uint32_t x, uint32_t c) {
  const u16x2 one = {1, 1};
  return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, x), one, c, false);
}
struct SrcLds16 {  // u16-packed row in LDS (cold tile: counts of the new records)
  const uint32_t* row;
  __device__ __forceinline__ uint4 get4(int b0) const {
    const uint2 w = *reinterpret_cast<const uint2*>(row + (b0 >> 1));  // word 899 is zero padding
    return make_uint4(w.x & 0xFFFFu, w.x >> 16, w.y & 0xFFFFu, w.y >> 16);
  }
  __device__ __forceinline__ uint32_t sum4(int b0) const {  // bins b0..b0+3 summed, packed
    const uint2 w = *reinterpret_cast<const uint2*>(row + (b0 >> 1));
    return pair_sum(w.x, pair_sum(w.y, 0u));
  }
};
struct SrcLds32 {  // u32 row in LDS, stride ROW, bins 1798/1799 zero
  const uint32_t* row;
  __device__ __forceinline__ uint4 get4(int b0) const { return *reinterpret_cast<const uint4*>(row + b0); }
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
// SMALL: the row's count is below 2^32 (a cold half-tile: <= 65535 records), so the lane
// prefix, the targets and the owner search are 32-bit (one scan, one readlane, one permute).
template <class Src, bool SMALL = false>
__device__ __forceinline__ void wave_summary(const uint32_t (&g)[9], const Src& src, int64_t total,
                                             const int32_t* __restrict__ mid, Summary88* __restrict__ out) {
  using U = typename std::conditional<SMALL, uint32_t, uint64_t>::type;
  auto rl = [](U x, int k) -> U {  // lane k's value
    if constexpr (SMALL) {
      return (U)__builtin_amdgcn_readlane((uint32_t)x, k);
    } else {
      return ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(x >> 32), k) << 32) |
             __builtin_amdgcn_readlane((uint32_t)x, k);
    }
  };
  const int lane = lane_id();
  U ls = 0;
#pragma unroll
  for (int q = 0; q < 9; ++q) ls += g[q];
  U incl;
  if constexpr (SMALL)
    incl = wave_incl_scan32(ls);
  else
    incl = wave_incl_scan(ls);
  const U excl = incl - ls;
  const U num = rl(incl, 63);
  const double dn = (double)num;

  // lane k < 8 computes target k (min, p50, p90, p95, p99, p999, p9999, max) in
  // parallel; each target's owner lane is then found with one ballot
  U my_t;
  {
    const double p = lane == 1 ? 0.50 : lane == 2 ? 0.90 : lane == 3 ? 0.95 : lane == 4 ? 0.99
                   : lane == 5 ? 0.999 : 0.9999;
    my_t = (U)java_round_nonneg(__dmul_rn(p, dn));
    if (lane == 0) my_t = num ? 1 : 0;
    if (lane >= 7) my_t = num;
  }
  int my_owner = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const U t = rl(my_t, k);
    const unsigned long long m = __ballot(t != 0 && excl < t && t <= incl);
    const int owner = m ? (__ffsll((long long)m) - 1) : 0;
    if (lane == k) my_owner = owner;
  }
  U acc = __shfl(excl, my_owner, 64);
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

constexpr int NB4 = 450;  // groups of 4 bins covering 1798 bins (+2 padding)

// The fleet merge's encoding words of 4 bins (non-empty buckets, + 1 per count >=
// MERGE_CMAX, which takes a second word).
__device__ __forceinline__ uint32_t merge_words4(uint4 v) {
  return (v.x != 0u) + (v.y != 0u) + (v.z != 0u) + (v.w != 0u) + (v.x >= MERGE_CMAX) + (v.y >= MERGE_CMAX) +
         (v.z >= MERGE_CMAX) + (v.w >= MERGE_CMAX);
}

// A dirty row's counts: the new records' (LDS) plus the state row's.
template <class A, class B>
struct SrcSum2 {
  A a;
  B b;
  __device__ __forceinline__ uint4 get4(int b0) const {
    const uint4 x = a.get4(b0), y = b.get4(b0);
    return make_uint4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);
  }
};

// The fleet merge's encoding of one row (one wave): its words, then its entries at
// enc[at..) in bucket order -- bucket << 21 | count, or bucket << 21 | MERGE_CMAX
// followed by the count (l5dh_merge.hip decodes them).  Lane l covers bins 4q..4q+3,
// q = l + 64 k.
template <class Src>
__device__ __forceinline__ uint32_t row_words(const Src& src) {
  const int lane = lane_id();
  uint32_t w = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int q = lane + 64 * k;
    if (q < NB4) w += merge_words4(src.get4(4 * q));
  }
  return (uint32_t)wave_sum((uint64_t)w);
}
template <class Src>
__device__ __forceinline__ void row_encode(const Src& src, uint32_t* __restrict__ enc, uint32_t at) {
  const int lane = lane_id();
#pragma unroll 2
  for (int k = 0; k < 8; ++k) {
    const int q = lane + 64 * k;
    const uint4 v = q < NB4 ? src.get4(4 * q) : make_uint4(0u, 0u, 0u, 0u);
    const uint32_t w = merge_words4(v);
    if (__ballot(w != 0u) == 0ull) continue;  // (wave-uniform) an empty stretch of the row: no scan, no stores
    const uint32_t incl = wave_incl_scan32(w);
    const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
    uint32_t pos = at + incl - w;
    const uint32_t c[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (c[j]) {
        const bool esc = c[j] >= MERGE_CMAX;
        enc[pos++] = ((uint32_t)(4 * q + j) << 21) | (esc ? MERGE_CMAX : c[j]);
        if (esc) enc[pos++] = c[j];
      }
    }
    at += total;
  }
}

// A wave's per-lane word counts -> *out (lane 0), when out is non-null.
__device__ __forceinline__ void put_words(uint32_t w, uint32_t* __restrict__ out) {
  if (out == nullptr) return;
  w = (uint32_t)wave_sum((uint64_t)w);
  if (lane_id() == 0) *out = w;
}

// Pass over a row source: optional dense copy in a coalesced lane order (lane l
// copies groups l, l+64, ...), then the blocked group sums of the summary; with
// words_out, the row's merge-encoding words (counted from the values already read).
template <class Src>
__device__ __forceinline__ void row_pass(const Src& src, uint32_t (&g)[9], int32_t* __restrict__ out_row,
                                         uint32_t* __restrict__ words_out = nullptr) {
  const int lane = lane_id();
  uint32_t w = 0;
  if (out_row) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int q = lane + 64 * k;
      if (q < NB4) {
        const uint4 v = src.get4(4 * q);
        store4_1798(out_row, 4 * q, v);
        w += merge_words4(v);
      }
    }
  }
  const int ng = lane_groups(lane);
#pragma unroll
  for (int q = 0; q < 9; ++q) {
    g[q] = 0u;
    if (q < ng) {
      const uint4 v = src.get4(28 * lane + 4 * q);
      g[q] = sum4(v);
      if (!out_row) w += merge_words4(v);
    }
  }
  put_words(w, words_out);
}

template <int NT = 1024>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* lds /*[NT/64+1]*/, uint32_t* total) {
  constexpr int NW = NT / 64;
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
    for (int k = 0; k < NW; ++k) {
      const uint32_t q = lds[k];
      lds[k] = acc;
      acc += q;
    }
    lds[NW] = acc;
  }
  __syncthreads();
  const uint32_t r = lds[w] + x - v;
  if (total) *total = lds[NW];
  __syncthreads();
  return r;
}

// Four independent exclusive scans in one pass (one set of barriers): v[k] per
// thread -> its exclusive prefix, tot[k] the block totals.  lds: [NT/64 + 1] uint4.
template <int NT = 1024>
__device__ __forceinline__ void block_excl_scan4(uint32_t (&v)[4], uint4* lds, uint32_t (&tot)[4]) {
  constexpr int NW = NT / 64;
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  uint32_t x[4] = {v[0], v[1], v[2], v[3]};
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t y = __shfl_up(x[k], d, 64);
      if (lane >= d) x[k] += y;
    }
  }
  if (lane == 63) lds[w] = make_uint4(x[0], x[1], x[2], x[3]);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint4 acc = make_uint4(0u, 0u, 0u, 0u);
    for (int k = 0; k < NW; ++k) {
      const uint4 q = lds[k];
      lds[k] = acc;
      acc = make_uint4(acc.x + q.x, acc.y + q.y, acc.z + q.z, acc.w + q.w);
    }
    lds[NW] = acc;
  }
  __syncthreads();
  const uint4 b = lds[w], t = lds[NW];
  const uint32_t bb[4] = {b.x, b.y, b.z, b.w};
  const uint32_t tt[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[k] = bb[k] + x[k] - v[k];
    tot[k] = tt[k];
  }
  __syncthreads();
}


// Bucket of a non-negative key v < Int.MaxValue, bit-identical to
// upper_bound(limits, v) (== the Arrays.binarySearch insertion rule of
// BucketedHistogram.add): a 1664-entry LUT indexed by the exponent and the top
// 6 mantissa bits of v brackets the bucket from below (entry bits [10:0]); each
// LUT interval contains at most two limits (checked exhaustively on the host).
// For intervals at most 1024 wide (v < 131072) the entry also holds their
// offsets from the interval start (bits [20:11], [30:21]; 0 = none), so the
// search is one LDS read and two register compares; wider intervals (offset
// field 0x3FF) finish with two compares against the LDS-staged limits.
__device__ __forceinline__ uint32_t bucket_lut(uint32_t v, const uint32_t* __restrict__ lut,
                                               const int32_t* __restrict__ lim) {
  uint32_t idx, start;
  if (v < 64u) {
    idx = v;
    start = v;
  } else {
    const int sh = 25 - __clz((int)v);  // exponent - 6
    idx = 64u + (uint32_t)sh * 64u + ((v >> sh) & 63u);
    start = (v >> sh) << sh;
  }
  const uint32_t x = lut[idx];
  uint32_t b = x & 0x7FFu;
  const uint32_t o1 = (x >> 11) & 0x3FFu;
  const uint32_t o2 = x >> 21;
  if (o1 == 0x3FFu) {
    b += (lim[b] <= (int32_t)v) ? 1u : 0u;
    b += (lim[b] <= (int32_t)v) ? 1u : 0u;
  } else {
    const uint32_t d = v - start;
    b += (o1 != 0u && d >= o1) ? 1u : 0u;
    b += (o2 != 0u && d >= o2) ? 1u : 0u;
  }
  return b;
}

// bucket_lut2 split into its LDS read and its decode, so callers can batch the reads.
__device__ __forceinline__ uint32_t lut2_index(uint32_t v) {
  const bool small = v < 64u;
  const uint32_t sh = small ? 0u : (uint32_t)(25 - __clz((int)v));
  return small ? v : 64u + sh * 64u + ((v >> sh) & 63u);
}
__device__ __forceinline__ uint32_t sel_u32(bool c, uint32_t a, uint32_t b) {  // branch-free select (v_bfi)
  const uint32_t m = 0u - (uint32_t)c;
  return (a & m) | (b & ~m);
}
__device__ __forceinline__ uint32_t lut2_decode(uint32_t v, uint2 x, uint32_t& off) {
  const uint32_t sh = v < 64u ? 0u : (uint32_t)(25 - __clz((int)v));
  const uint32_t d = v & ((1u << sh) - 1u);  // v - interval start
  const uint32_t o1 = x.x & 0xFFFFu, o2 = x.x >> 16;
  const bool k1 = d >= o1, k2 = d >= o2;
  // off = d - o2 | d - o1 | d + p, without branches
  off = d - sel_u32(k2, o2, sel_u32(k1, o1, 0u - (x.y >> 16)));
  return (x.y & 0xFFFFu) + (uint32_t)k1 + (uint32_t)k2;
}

// Exact bucket AND offset from the bucket's lower limit for keys v < 2^21, with one
// 8-byte LDS read and no limit reads.  Interval = [start, start + 2^sh) of the
// same (exponent, 6 mantissa bits) as bucket_lut; entry {o1 | o2 << 16, b0 | p << 16}:
// b0 = bucket(start), o1/o2 = offsets of the (at most two) limits inside the
// interval (0xFFFF = none), p = start - lower limit of b0.
__device__ __forceinline__ uint32_t bucket_lut2(uint32_t v, const uint2* __restrict__ lut2, uint32_t& off) {
  const bool small = v < 64u;
  const uint32_t sh = small ? 0u : (uint32_t)(25 - __clz((int)v));
  const uint32_t idx = small ? v : 64u + sh * 64u + ((v >> sh) & 63u);
  const uint32_t start = (v >> sh) << sh;
  const uint2 x = lut2[idx];
  const uint32_t d = v - start;
  const uint32_t o1 = x.x & 0xFFFFu, o2 = x.x >> 16;
  const bool k1 = d >= o1, k2 = d >= o2;
  off = k2 ? d - o2 : (k1 ? d - o1 : d + (x.y >> 16));
  return (x.y & 0xFFFFu) + (k1 ? 1u : 0u) + (k2 ? 1u : 0u);
}

// Bucket of a binned record (l5dh_kernels.hpp) and its contribution to the
// exact sum: LUT decode of v, or the escaped bucket with contribution 0 (the
// whole contribution is already in sumfix).
__device__ __forceinline__ uint32_t record_bucket(uint32_t rec, const uint2* __restrict__ lut2, uint32_t& v) {
  const uint32_t p = rec & 0x1FFFFFu;
  uint32_t o;
  const uint32_t b = lut2_decode(p, lut2[lut2_index(p)], o);
  const bool esc = p >= V_ESC;
  v = sel_u32(esc, 0u, p);
  return sel_u32(esc, p - V_ESC, b);
}

// Full 11-step search for any int32 key (negative keys come from the Long.toInt
// wrap of negative samples; rare path).
__device__ __forceinline__ uint32_t search_key(int32_t key, const int32_t* __restrict__ lim) {
  int idx = 0;
#pragma unroll
  for (int step = 1024; step > 0; step >>= 1)
    if (lim[idx + step - 1] <= key) idx += step;
  return (uint32_t)(idx < NL ? idx : NL);
}

// upstream BucketedHistogram.add(Long) applied to Metric.Stat.add's
// `value.toLong` (Metric.scala:32): returns the bucket and the sample's
// contribution to `total` (Int.MaxValue for the overflow bucket).
__device__ __forceinline__ uint32_t bucketize(float f, const uint32_t* __restrict__ lut,
                                              const int32_t* __restrict__ lim, int64_t& contrib) {
  if (f >= 0.0f && f < 2147483648.0f) {  // common case: v in [0, 2147483520]
    const uint32_t v = (uint32_t)f;
    contrib = v;
    return bucket_lut(v, lut, lim);
  }
  const int64_t v = java_f2l(f);
  if (v >= (int64_t)INT_MAXV) {
    contrib = INT_MAXV;
    return NL;
  }
  contrib = v;
  const int32_t key = (int32_t)(uint32_t)(uint64_t)v;  // Long.toInt: low 32 bits
  return (key >= 0 && key < INT_MAXV) ? bucket_lut((uint32_t)key, lut, lim) : search_key(key, lim);
}

// Level-1 payload of a sample outside [0, V_ESC): bucketize, add its exact
// contribution to sumfix, return V_ESC + bucket (or the truncated value when it
// lands inside the range after all).  Rare: k_bin1 runs it from a non-unrolled
// loop so one copy of the full search sits in the hot loop's code.
__device__ __forceinline__ uint32_t payload1_slow(uint32_t s, float f, Tables tb,
                                                           int64_t* __restrict__ sumfix) {
  int64_t c;
  const uint32_t b = bucketize(f, tb.lut, tb.lim_pad, c);
  if (c >= 0 && c < (int64_t)V_ESC) return (uint32_t)c;  // e.g. f in (-1, 0) truncates to 0
  // whole contribution (nullptr: a redo pass of the same samples, already added)
  if (sumfix) atomicAdd(reinterpret_cast<unsigned long long*>(&sumfix[s]), (unsigned long long)c);
  return V_ESC + b;
}

__device__ __forceinline__ uint32_t payload1(uint32_t s, float f, Tables tb, int64_t* __restrict__ sumfix) {
  if (f >= 0.0f && f < (float)V_ESC) return (uint32_t)f;
  return payload1_slow(s, f, tb, sumfix);
}

// Number of set bits of m below this lane.
__device__ __forceinline__ uint32_t mask_below(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Wave-aggregated LDS counters for skewed keys (Zipf heads).  Same result as
// every valid lane doing `atomicAdd(&ctr[key], 1)` (the returned ranks are a
// permutation of what that would return), but up to ROUNDS leader rounds merge
// the lanes that share the leading lane's key into one atomic; aggregation stops
// as soon as a leader's key is unique in the wave.  Must be called by the whole
// wave (convergent).
template <int ROUNDS>
__device__ __forceinline__ uint32_t wave_atomic_rank(uint32_t* ctr, uint32_t key, bool valid) {
  unsigned long long active = __ballot(valid);
  uint32_t rank = 0;
  bool done = !valid;
#pragma unroll
  for (int r = 0; r < ROUNDS; ++r) {
    if (!active) break;
    const int leader = __ffsll((long long)active) - 1;
    const uint32_t lk = __builtin_amdgcn_readlane(key, leader);
    const bool mine = !done && key == lk;
    const unsigned long long m = __ballot(mine);
    const uint32_t cnt = (uint32_t)__popcll(m);
    uint32_t base = 0;
    if (lane_id() == leader) base = atomicAdd(&ctr[lk], cnt);
    base = __builtin_amdgcn_readlane(base, leader);
    if (mine) {
      rank = base + mask_below(m);
      done = true;
    }
    active &= ~m;
    if (cnt == 1) break;
  }
  if (!done) rank = atomicAdd(&ctr[key], 1u);
  return rank;
}

template <int ROUNDS>
__device__ __forceinline__ void wave_atomic_inc(uint32_t* ctr, uint32_t key, bool valid) {
  unsigned long long active = __ballot(valid);
  bool done = !valid;
#pragma unroll
  for (int r = 0; r < ROUNDS; ++r) {
    if (!active) break;
    const int leader = __ffsll((long long)active) - 1;
    const uint32_t lk = __builtin_amdgcn_readlane(key, leader);
    const bool mine = !done && key == lk;
    const unsigned long long m = __ballot(mine);
    const uint32_t cnt = (uint32_t)__popcll(m);
    if (lane_id() == leader) atomicAdd(&ctr[lk], cnt);
    if (mine) done = true;
    active &= ~m;
    if (cnt == 1) break;
  }
  if (!done) atomicAdd(&ctr[key], 1u);
}

// Rank of this lane's increment of ctr[key] (like atomicAdd(&ctr[key], 1)); lanes
// whose key is one of the wave-uniform hot keys (Zipf heads, found exactly from
// the count pass) are merged into one atomic per hot key.  Convergent.
__device__ __forceinline__ uint32_t hot_rank(uint32_t* ctr, uint32_t key, bool valid, uint32_t hot0,
                                             uint32_t hot1) {
  uint32_t rank = 0;
  bool handled = !valid;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t hk = h ? hot1 : hot0;
    if (hk != 0xFFFFFFFFu) {
      const bool mine = valid && key == hk;
      const unsigned long long m = __ballot(mine);
      if (m) {
        const int leader = __ffsll((long long)m) - 1;
        uint32_t base = 0;
        if (lane_id() == leader) base = atomicAdd(&ctr[hk], (uint32_t)__popcll(m));
        base = __builtin_amdgcn_readlane(base, leader);
        if (mine) {
          rank = base + mask_below(m);
          handled = true;
        }
      }
    }
  }
  if (!handled) rank = atomicAdd(&ctr[key], 1u);
  return rank;
}

// Batched form of hot_rank over a thread's PT keys (~0u = no key): every lane
// gets the rank atomicAdd(&ctr[key], 1) would give (up to a permutation), but
// the lanes of the HK wave-uniform hot keys (~0u = unused slot) are counted by
// ballots over all PT samples first and then take their ranks from ONE LDS
// atomic per hot key and wave (issued by lanes 0..HK-1 together), so no rank
// waits on an atomic inside the per-sample loop.  Convergent.
template <int HK, int PT>
__device__ __forceinline__ void hot_rank_batch(uint32_t* ctr, const uint32_t (&key)[PT], const uint32_t (&hk)[HK],
                                               uint32_t (&rank)[PT]) {
  uint32_t wcnt[HK];
#pragma unroll
  for (int h = 0; h < HK; ++h) wcnt[h] = 0;
#pragma unroll
  for (int k = 0; k < PT; ++k) {
    bool hot = false;
#pragma unroll
    for (int h = 0; h < HK; ++h) {
      if (hk[h] != 0xFFFFFFFFu) {
        const bool mine = key[k] == hk[h];
        wcnt[h] += (uint32_t)__popcll(__ballot(mine));
        hot |= mine;
      }
    }
    rank[k] = 0;
    if (!hot && key[k] != 0xFFFFFFFFu) rank[k] = atomicAdd(&ctr[key[k]], 1u);
  }
  const int lane = lane_id();
  uint32_t mycnt = 0, mykey = 0xFFFFFFFFu;
#pragma unroll
  for (int h = 0; h < HK; ++h)
    if (lane == h) {
      mycnt = wcnt[h];
      mykey = hk[h];
    }
  uint32_t base = 0;
  if (mycnt != 0 && mykey != 0xFFFFFFFFu) base = atomicAdd(&ctr[mykey], mycnt);
  uint32_t hb[HK];
#pragma unroll
  for (int h = 0; h < HK; ++h) hb[h] = __builtin_amdgcn_readlane(base, h);
#pragma unroll
  for (int k = 0; k < PT; ++k) {
#pragma unroll
    for (int h = 0; h < HK; ++h) {
      if (hk[h] != 0xFFFFFFFFu) {
        const bool mine = key[k] == hk[h];
        const unsigned long long m = __ballot(mine);
        if (mine) rank[k] = hb[h] + mask_below(m);
        hb[h] += (uint32_t)__popcll(m);
      }
    }
  }
}

// Batched hot_inc: ctr[key[k]] += 1 for every key != ~0u, one LDS atomic per
// hot key and wave.  Convergent.
template <int HK, int PT>
__device__ __forceinline__ void hot_inc_batch(uint32_t* ctr, const uint32_t (&key)[PT], const uint32_t (&hk)[HK]) {
  uint32_t wcnt[HK];
#pragma unroll
  for (int h = 0; h < HK; ++h) wcnt[h] = 0;
#pragma unroll
  for (int k = 0; k < PT; ++k) {
    bool hot = false;
#pragma unroll
    for (int h = 0; h < HK; ++h) {
      if (hk[h] != 0xFFFFFFFFu) {
        const bool mine = key[k] == hk[h];
        wcnt[h] += (uint32_t)__popcll(__ballot(mine));
        hot |= mine;
      }
    }
    if (!hot && key[k] != 0xFFFFFFFFu) atomicAdd(&ctr[key[k]], 1u);
  }
  const int lane = lane_id();
  uint32_t mycnt = 0, mykey = 0xFFFFFFFFu;
#pragma unroll
  for (int h = 0; h < HK; ++h)
    if (lane == h) {
      mycnt = wcnt[h];
      mykey = hk[h];
    }
  if (mycnt != 0 && mykey != 0xFFFFFFFFu) atomicAdd(&ctr[mykey], mycnt);
}

// hot_rank for HK wave-uniform hot keys (~0u = unused).  Convergent.
template <int HK>
__device__ __forceinline__ uint32_t hot_rank_n(uint32_t* ctr, uint32_t key, bool valid, const uint32_t (&hk)[HK]) {
  uint32_t rank = 0;
  bool handled = !valid;
#pragma unroll
  for (int h = 0; h < HK; ++h) {
    if (hk[h] != 0xFFFFFFFFu) {
      const bool mine = valid && key == hk[h];
      const unsigned long long m = __ballot(mine);
      if (m) {
        const int leader = __ffsll((long long)m) - 1;
        uint32_t base = 0;
        if (lane_id() == leader) base = atomicAdd(&ctr[hk[h]], (uint32_t)__popcll(m));
        base = __builtin_amdgcn_readlane(base, leader);
        if (mine) {
          rank = base + mask_below(m);
          handled = true;
        }
      }
    }
  }
  if (!handled) rank = atomicAdd(&ctr[key], 1u);
  return rank;
}

// ctr[key] += 1 for every valid lane, with the lanes of up to two wave-uniform
// hot keys merged into one atomic each.  Convergent.
__device__ __forceinline__ void hot_inc(uint32_t* ctr, uint32_t key, bool valid, uint32_t hot0, uint32_t hot1) {
  bool handled = !valid;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t hk = h ? hot1 : hot0;
    if (hk != 0xFFFFFFFFu) {
      const bool mine = valid && key == hk;
      const unsigned long long m = __ballot(mine);
      if (m) {
        if (lane_id() == __ffsll((long long)m) - 1) atomicAdd(&ctr[hk], (uint32_t)__popcll(m));
        handled |= mine;
      }
    }
  }
  if (!handled) atomicAdd(&ctr[key], 1u);
}

// Visit records r[a, e) with 16-B loads, two in flight per thread per step.
template <int NT, class Fn>
__device__ __forceinline__ void for_records(const uint32_t* __restrict__ r, uint32_t a, uint32_t e, Fn&& fn) {
  if (a >= e) return;
  const uint32_t a4 = min(e, (a + 3u) & ~3u);
  if (threadIdx.x < a4 - a) fn(r[a + threadIdx.x]);
  const uint4* __restrict__ p = reinterpret_cast<const uint4*>(r + a4);
  const uint32_t nv = (e - a4) >> 2;
  uint32_t i = threadIdx.x;
  for (; i + NT < nv; i += 2 * NT) {
    const uint4 x = p[i];
    const uint4 y = p[i + NT];
    fn(x.x); fn(x.y); fn(x.z); fn(x.w);
    fn(y.x); fn(y.y); fn(y.z); fn(y.w);
  }
  if (i < nv) {
    const uint4 x = p[i];
    fn(x.x); fn(x.y); fn(x.z); fn(x.w);
  }
  const uint32_t t0 = a4 + (nv << 2);
  if (t0 + threadIdx.x < e) fn(r[t0 + threadIdx.x]);
}

}  // namespace
}  // namespace l5dh
